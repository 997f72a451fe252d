// mvm_common.hip — library-wide parts of the C ABI (include/mvmatch.h):
// version and status strings, the per-thread error message, option
// resolution, and the HBM write probe bench.py reports next to the roofline.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "mvmatch.h"
#include "mvm_device.h"
#include "mvm_internal.h"

namespace {
thread_local char g_err[512];

// The fastest store stream measured on MI355X: every
// workgroup writes one contiguous 8 KiB block with 16-byte nontemporal stores
// (2 per lane, each wave instruction 1 KiB contiguous), and workgroups are
// remapped so that each XCD writes its own contiguous eighth in order.  The
// other patterns studied (block sizes, cache policies, the kernels' own row
// orders) are in tools/probes/write_probes.hip.
__global__ __launch_bounds__(kThreads) void write_probe_kernel(f32x4 *dst, size_t n16, float val) {
    constexpr int kPerLane = 2;
    const f32x4 v = {val, val, val, val};
    const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blockIdx.x % 8;
    const uint32_t blk = x * q + min(x, r) + blockIdx.x / 8;   // dispatch puts block b on XCD b % 8
    const size_t base = (size_t)blk * (kPerLane * kThreads) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < kPerLane; ++k) {
        const size_t i = base + (size_t)k * kThreads;
        if (i < n16) __builtin_nontemporal_store(v, dst + i);
    }
}
}  // namespace

void mvm_set_error(const char *msg) { snprintf(g_err, sizeof g_err, "%s", msg); }

void mvm_clear_error() { g_err[0] = '\0'; }

int mvm_fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int mvm_check_launch(const char *what) {
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return mvm_fail(MVM_ERR_HIP, "%s: %s", what, hipGetErrorString(err));
    return MVM_OK;
}

int mvm_resolve_options(const mvm_options *in, mvm_options &out) {
    mvm_options_init(&out);
    if (!in) return MVM_OK;
    if (in->size < (int32_t)(2 * sizeof(int32_t)) || (in->size % (int32_t)sizeof(int32_t)) != 0)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "mvm_options.size %d is not a struct size",
                        (int)in->size);
    // a caller built against an older (smaller) struct keeps the defaults of
    // the fields it does not know; a newer caller's extra fields are ignored
    const size_t n = (size_t)in->size < sizeof(mvm_options) ? (size_t)in->size : sizeof(mvm_options);
    memcpy(&out, in, n);
    out.size = (int32_t)sizeof(mvm_options);
    return MVM_OK;
}

extern "C" {

// tools/build_variant.py names its A/B builds (some compute wrong results by design)
#ifdef MVM_VARIANT
const char *mvm_version(void) { return "mvmatch 0.7.0 gfx950 variant " MVM_VARIANT; }
#else
const char *mvm_version(void) { return "mvmatch 0.7.0 gfx950"; }
#endif

const char *mvm_last_error_string(void) { return g_err; }

const char *mvm_status_string(int status) {
    switch (status) {
    case MVM_OK: return "ok";
    case MVM_ERR_INVALID_ARGUMENT: return "invalid argument";
    case MVM_ERR_UNSUPPORTED: return "unsupported configuration";
    case MVM_ERR_WORKSPACE: return "workspace too small";
    case MVM_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
    }
}

void mvm_options_init(mvm_options *opts) {
    if (!opts) return;
    memset(opts, 0, sizeof *opts);
    opts->size = (int32_t)sizeof *opts;
}

int mvm_hbm_write_probe(void *dst_dev, size_t bytes, mvm_stream_t stream) {
    mvm_clear_error();
    if (!dst_dev || (((uintptr_t)dst_dev) & 15) || (bytes & 15))
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "write probe needs a 16-byte aligned buffer/size");
    // one launch per piece of at most kMaxGridBlocks workgroups (~137 GB)
    constexpr size_t kPiece = (size_t)kMaxGridBlocks / 8 * 8 * (2 * kThreads);   // f32x4 per launch
    for (size_t done = 0, n16 = bytes / 16; done < n16; done += kPiece) {
        const size_t n = n16 - done < kPiece ? n16 - done : kPiece;
        const size_t blocks = (n + 2 * kThreads - 1) / (2 * kThreads);
        write_probe_kernel<<<(unsigned)blocks, kThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(
            reinterpret_cast<f32x4 *>(dst_dev) + done, n, 1.0f);
        if (const int st = mvm_check_launch("write_probe_kernel")) return st;
    }
    return MVM_OK;
}

}  // extern "C"
