// mvm_internal.h — helpers shared by the library's translation units (not part
// of the public C ABI).  Errors are recorded per thread for
// mvm_last_error_string().
#pragma once

#include <stdarg.h>

int mvm_fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void mvm_set_error(const char *msg);
void mvm_clear_error();
int mvm_check_launch(const char *what);
int mvm_env_int(const char *name, int dflt);   // tuning knobs: getenv + atoi
