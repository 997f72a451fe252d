// mvm_lsap_sparse.h — the candidate-list assignment class (mvm_lsap_sparse.hip),
// shared with mvm_lsap.hip's launcher (not part of the public C ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mvmatch.h"

constexpr int kSpMaxCols = 65536;    // long sides up to this (16-bit column ids, 8 KB bitmaps)
constexpr int kSpMaxShort = 1024;    // short sides up to this (4 slots per thread)
constexpr int kSpBlock = 32;         // columns per block minimum
constexpr int kSpTB = 16;            // default candidate blocks per row: the list holds >= 16 entries
constexpr int kSpLCap = 128;         // entries per candidate list (more: the row is scanned densely)
constexpr int kSpTileCols = 2048;    // columns per block-minimum workgroup
// default lower bound of the class (mvm_options.lsap_sparse_min_cols): 1000
// problems of 4096 x 64 take 1.29 ms with candidate lists against 1.66 with
// the register-state workgroup; 3136 x 56 1.42 against 1.38, 2304 x 48 1.12
// against 1.03 (tools/bench_lsap.py, profiles/r05/lsap_sparse/)
constexpr int kSparseMinCols = 4096;

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
    // optional: minima of 8 consecutive tall rows per short-side column, as
    // written by mvm_triplet_cost_argmin_bmin8 (problem p's long side is
    // segs[p]-row segments -- a cube's M -- each cut in groups of 8 rows:
    // row g * ceil(seg/8) + j/8 of S keys at bmin8 + bmin8_offs[p])
    const uint16_t *bmin8;
    const int64_t *bmin8_offs;
    const int64_t *segs;
    int32_t tb;                   // candidate blocks per row (mvm_options.lsap_sparse_blocks)
    // optional (mvm_lsap_solve_resid, ABI 7): no cost at all -- problem p is
    // scene p of mvm_triplet_minima, its entries recomputed from the scene's
    // fp64 pair residuals (e12 [N][ld], e13T [P][ld], e23T [P][ld] at
    // resid + p * resid_stride) with the cube's arithmetic (cube_f32)
    const double *resid = nullptr;
    int64_t resid_stride = 0;     // doubles per scene (3 * max_n * ld)
    int32_t resid_ld = 0;
    int32_t resid_rows = 0;       // max_n: e13T starts max_n * ld after e12
    // ... and its block minima as mvm_triplet_minima wrote them (no reduction
    // pass, no block minima in the workspace): row s of problem p at bm32 +
    // bm32_offs[p] + s * ceil(seg/32) * roundup(L/seg, 16), block (jt, g) at
    // jt * roundup(L/seg, 16) + g
    const uint16_t *bm32 = nullptr;                           // 16-bit keys
    const int64_t *bm32_offs = nullptr;
};

// status of a problem that cannot be solved as given (ABI 7): its short side
// exceeds the launch's short_max, its long side the long_max, or -- cube-free
// -- it is outside the candidate-list class
constexpr int32_t kSpStatusBounds = 4;

constexpr int kSpMaxBlocks = 2048;   // block minima per row (32 keys per wave lane)

// problem p's blocks come from bmin8: the segment length (a cube's M), else 0
// (blocks of 32 over the whole long side, from the cost itself)
__host__ __device__ inline int lsap_sparse_seg(const LsapSparseArgs &a, int p, bool tr, int L) {
    if (((!a.bmin8 || !a.bmin8_offs) && !a.bm32) || !a.segs || !tr) return 0;   // 8-row or block minima
    const int64_t seg = a.segs[p];
    if (seg <= 0 || L % seg != 0) return 0;
    return (L / seg) * ((seg + 31) / 32) <= kSpMaxBlocks ? (int)seg : 0;
}

__host__ __device__ inline bool lsap_sparse_class(int32_t lo, int32_t wave_max, int64_t R, int64_t K) {
    const int64_t lng = R > K ? R : K, sht = R > K ? K : R;
    return lo > 0 && lng >= lo && lng > wave_max && lng <= kSpMaxCols && sht >= 1 && sht <= kSpMaxShort;
}

// per-problem workspace of the class (inside the plan's region for the problem)
struct SpLayout {
    size_t stats, flags, bm, lcol, lval, ln, theta, total;
};
// sp_solve_kernel's counters of a solved problem, int32 at the start of its
// workspace region (mvm_lsap_sparse_stats reads them): dense scans for a row's
// free minimum (no list, or no free entry left in it), dense scans for the
// free ties at the sink, rows whose list overflowed kSpLCap, Dijkstra steps
constexpr int kSpStats = 4;

// tr: the problem is tall (transposed, short side = columns); ext_bm: its
// block minima come from outside the workspace (LsapSparseArgs::bm32)
__host__ __device__ inline SpLayout lsap_sparse_layout(int64_t S, int64_t L, size_t elem, bool tr,
                                                       bool ext_bm = false) {
    SpLayout y;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return at;
    };
    // blocks per row: ceil(L/32) over the whole long side; with segments
    // (lsap_sparse_seg, tall problems only) (L/seg) * ceil(seg/32) <=
    // min(kSpMaxBlocks, L) -- reserved only where segments can apply (a wide
    // problem of 24 x 576 would otherwise reserve S * L keys: a copy of its cost)
    const int64_t nbf = (L + kSpBlock - 1) / kSpBlock, nbs = L < kSpMaxBlocks ? L : kSpMaxBlocks;
    const int64_t nb = tr && nbs > nbf ? nbs : nbf;
    const int64_t nt = (L + kSpTileCols - 1) / kSpTileCols;
    y.stats = take(kSpStats * 4);
    y.flags = take((size_t)(nt > 32 ? nt : 32) * 4);   // invalid-entry flag per tile
    y.bm = take(ext_bm ? 0 : (size_t)S * nb * elem);   // ordered keys of the block minima
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
