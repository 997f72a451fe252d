// mvm_internal.h — host helpers shared by the library's translation units (not
// part of the public C ABI).  Errors are recorded per thread for
// mvm_last_error_string().
#pragma once

#include <stdarg.h>

#include "mvmatch.h"

int mvm_fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void mvm_set_error(const char *msg);
void mvm_clear_error();
int mvm_check_launch(const char *what);
// *in (NULL = defaults) -> out, every field present; MVM_OK or an error code
int mvm_resolve_options(const mvm_options *in, mvm_options &out);
