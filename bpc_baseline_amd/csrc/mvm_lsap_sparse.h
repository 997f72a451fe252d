// mvm_lsap_sparse.h — the candidate-list assignment class (mvm_lsap_sparse.hip),
// shared with mvm_lsap.hip's launcher (not part of the public C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mvmatch.h"

constexpr int kSpMaxCols = 65536;    // long sides up to this (16-bit column ids, 8 KB bitmaps)
constexpr int kSpMaxShort = 1024;    // short sides up to this (4 slots per thread)
constexpr int kSpBlock = 32;         // columns per block minimum
constexpr int kSpTB = 16;            // candidate blocks per row: the list holds >= 16 entries
constexpr int kSpLCap = 128;         // entries per candidate list (more: the row is scanned densely)
constexpr int kSpTileCols = 2048;    // columns per block-minimum workgroup

struct LsapSparseArgs {
    const void *cost;             // float or double (CT)
    const int64_t *cost_offs;
    const int64_t *dims;          // [n][2] rows, cols
    const int64_t *ws_offs;
    unsigned char *ws;
    const int64_t *out_offs;
    int64_t *row_ind;
    int64_t *col_ind;
    int32_t *status;
    int32_t lo;                   // long sides >= lo (> wave_max, <= kSpMaxCols) with short
    int32_t wave_max;             // sides in [1, kSpMaxShort] are this class's
    int32_t s_cap;                // LDS sizing: every short side of the class is <= this
};

__host__ __device__ inline bool lsap_sparse_class(int32_t lo, int32_t wave_max, int64_t R, int64_t K) {
    const int64_t lng = R > K ? R : K, sht = R > K ? K : R;
    return lo > 0 && lng >= lo && lng > wave_max && lng <= kSpMaxCols && sht >= 1 && sht <= kSpMaxShort;
}

// per-problem workspace of the class (inside the plan's region for the problem)
struct SpLayout {
    size_t flags, bm, lcol, lval, ln, theta, total;
};

__host__ __device__ inline SpLayout lsap_sparse_layout(int64_t S, int64_t L, size_t elem) {
    SpLayout y;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return at;
    };
    const int64_t nb = (L + kSpBlock - 1) / kSpBlock, nt = (L + kSpTileCols - 1) / kSpTileCols;
    y.flags = take((size_t)nt * 4);                  // invalid-entry flag per column tile
    y.bm = take((size_t)S * nb * elem);              // ordered keys of the block minima
    y.lcol = take((size_t)S * kSpLCap * 4);
    y.lval = take((size_t)S * kSpLCap * elem);
    y.ln = take((size_t)S * 4);                      // list length (-1: dense row)
    y.theta = take((size_t)S * elem);
    y.total = o;
    return y;
}

// Launch the class's three kernels for cost element type CT (float / double).
int lsap_sparse_launch_f32(const LsapSparseArgs &a, int32_t n, int64_t long_max, hipStream_t s);
int lsap_sparse_launch_f64(const LsapSparseArgs &a, int32_t n, int64_t long_max, hipStream_t s);
