// mvm_kernels.hip — MI355X (gfx950) kernels of the multi-view epipolar matcher
// and the C ABI declared in include/mvmatch.h.
//
// Hot path of the reference: bpc/inference/epipolar_matching.py
//   epipolar_error (:5-28)  ->  pair residual, factorised into per-detection
//                              normalised epipolar lines (O(n)) + an 8-flop
//                              fp64 point-line evaluation per pair (O(n^2))
//   compute_cost_matrix (:83-98) -> triplet cube over the fp64 pair matrices
//   (new) per-row argmin over the stored float32 values
//
// Arithmetic is float64 throughout and reproduces the reference bit for bit:
// FMAs are placed exactly where numpy/OpenBLAS placed them in the reference
// run (the C oracle in oracle/ is pinned to the reference on the
// golden vectors) and the file is compiled with -ffp-contract=off so no other
// contraction happens.  sqrt and '/' are the IEEE correctly rounded gfx950
// sequences.
//
// Workload shape: HBM-write bound (4 bytes of float32 output per pair, inputs
// O(n)).  Layout per workgroup (256 threads = 4 waves of 64):
//   * the workgroup owns 4*RPW rows of one (scene, pair); wave w owns RPW rows;
//   * columns are processed in chunks of 256: thread t computes the normalised
//     line of column chunk+t once into LDS, then every lane of every wave
//     holds 4 consecutive columns in registers and sweeps its RPW rows, so
//     each row store is one 16-byte-per-lane, 1 KiB-per-wave coalesced store;
//   * the per-row argmin is tracked per lane in registers across chunks and
//     reduced across the wave once per row at the end.
#include <hip/hip_runtime.h>

#include <type_traits>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mvmatch.h"
#include "mvm_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int kWave = 64;
constexpr int kThreads = 256;                  // 4 waves per workgroup
constexpr int kWaves = kThreads / kWave;
constexpr int kColsPerLane = 4;                // one 16-byte store per lane per row
constexpr int kChunk = kWave * kColsPerLane;   // 256 columns per chunk (== kThreads)
constexpr double kDegenerateNorm = 1e-8;       // epipolar_matching.py:20-23
constexpr double kSentinel = 9999.0;           // epipolar_matching.py:25-26
constexpr uint32_t kKeyInvalid = 0xFFFFFFFFu;  // no column (tail / empty row)

// Column / row record states.
constexpr uint32_t kOk = 0;     // non-degenerate line, tame magnitudes
constexpr uint32_t kDeg = 1;    // line norm not > 1e-8: distance is the 9999 sentinel
constexpr uint32_t kNone = 2;   // no detection (chunk tail)
constexpr uint32_t kWild = 3;   // non-degenerate but non-finite / huge: generic path

static_assert(kChunk == kThreads, "one column line per thread per chunk");

// ---------------------------------------------------------------- lines ----
// Row side: l2 = F @ (x, y, 1)   (epipolar_matching.py:13)
__device__ __forceinline__ bool row_line(const double f[9], double x, double y, double &l0,
                                         double &l1, double &l2) {
    l0 = __builtin_fma(f[0], x, f[1] * y) + f[2];
    l1 = __builtin_fma(f[3], x, f[4] * y) + f[5];
    l2 = __builtin_fma(f[6], x, f[7] * y) + f[8];
    const double n = __builtin_sqrt(__builtin_fma(l1, l1, l0 * l0));   // :17-18
    const bool deg = !(n > kDegenerateNorm);                            // :20-23
    if (!deg) {
        l0 = l0 / n;
        l1 = l1 / n;
        l2 = l2 / n;
    }
    return deg;
}

// Column side: l1 = F.T @ (x, y, 1)   (epipolar_matching.py:14)
__device__ __forceinline__ bool col_line(const double f[9], double x, double y, double &l0,
                                         double &l1, double &l2) {
    l0 = __builtin_fma(f[3], y, f[0] * x) + f[6];
    l1 = __builtin_fma(f[4], y, f[1] * x) + f[7];
    l2 = __builtin_fma(f[5], y, f[2] * x) + f[8];
    const double n = __builtin_sqrt(__builtin_fma(l1, l1, l0 * l0));
    const bool deg = !(n > kDegenerateNorm);
    if (!deg) {
        l0 = l0 / n;
        l1 = l1 / n;
        l2 = l2 / n;
    }
    return deg;
}

// |l . (x, y, 1)|  (epipolar_matching.py:25-26, numpy ddot order)
__device__ __forceinline__ double line_dist(double l0, double l1, double l2, double x, double y) {
    return __builtin_fabs(__builtin_fma(l1, y, l0 * x) + l2);
}

// Magnitude guard for the branch-free fast path: with |x|,|y| <= 2^40 and
// |l2| <= 2^60 no intermediate can overflow, so a non-degenerate pair value is
// finite and its float32 bit pattern orders like the value.
__device__ __forceinline__ bool tame(double l2, double x, double y) {
    return __builtin_fabs(x) <= 0x1p40 && __builtin_fabs(y) <= 0x1p40 &&
           __builtin_fabs(l2) <= 0x1p60;
}

// -------------------------------------------------------------- argmin ----
// Ordering key of a stored float32 (values are >= +0 or NaN): NaN -> 0 (the
// smallest, np.argmin semantics), otherwise bits + 1.  kKeyInvalid marks
// "no column".  Lanes scan their columns in ascending order with a strict
// '<', so each lane keeps the lowest index among its equal minima.
__device__ __forceinline__ uint32_t key_of(float v) {
    return (v != v) ? 0u : (__float_as_uint(v) + 1u);
}

__device__ __forceinline__ float value_of_key(uint32_t k) {
    return (k == 0u || k == kKeyInvalid) ? __uint_as_float(0x7FC00000u) : __uint_as_float(k - 1u);
}

// DPP min step: v = min(v, v from the lane DPP control CTRL selects).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_min(uint32_t v) {
    // old = UINT_MAX (umin's identity) lets the DPP-combine pass fold the move
    // into the min (one v_min_u32_dpp per step)
    const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, 0xF, 0xF, false);
    return o < v ? o : v;
}

// Minimum over the wave, returned as a uniform (SGPR) value: four DPP steps
// reduce each 16-lane row in registers (quad_perm [1,0,3,2], quad_perm
// [2,3,0,1], row_half_mirror, row_mirror), then the four row minima are read
// with v_readlane and combined on the scalar unit.  No LDS round trips.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = dpp_min<0xB1>(v);
    v = dpp_min<0x4E>(v);
    v = dpp_min<0x141>(v);
    v = dpp_min<0x140>(v);
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    const uint32_t ab = a < b ? a : b, cd = c < d ? c : d;
    return ab < cd ? ab : cd;
}

// Reduce (key, idx) over the wave: minimum key, then the lowest column index
// among the lanes holding it (exact np.argmin tie rule).  A unique minimum
// (the common case) costs one ballot + one readlane; ties fall back to a
// second reduction over the candidates' indices.
__device__ __forceinline__ void wave_argmin(uint32_t key, int32_t idx, uint32_t &kmin,
                                            int32_t &imin) {
    kmin = wave_min_u32(key);
    const uint64_t hit = __ballot(key == kmin);
    if (__builtin_popcountll(hit) == 1) {
        imin = __builtin_amdgcn_readlane(idx, (int)__builtin_ctzll(hit));
    } else {
        imin = (int32_t)wave_min_u32(key == kmin ? (uint32_t)idx : 0x7FFFFFFFu);
    }
}

// ----------------------------------------------------------- stores ----
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// 4 consecutive outputs of one lane: one 16-byte store (float) or two (double)
__device__ __forceinline__ void store4_nt(float *dst, const double e[4]) {
    const f32x4 v = {(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(dst));
}
typedef f32x4 __attribute__((address_space(1))) g_f32x4;   // global (AS 1) pointee

// Row store from a scalar (SGPR) row address + a 32-bit per-lane byte offset:
// lowers to `global_store_dwordx4 v_off, v_data, s_base nt` (saddr form, no
// per-row 64-bit VALU address arithmetic).
// Store policy POL: 1 nt (default of the residual kernels), 0 default policy,
// 2 sc1, 3 sc0 sc1 (the last two through inline asm: no builtin exposes them;
// they drop the line from the XCD's L2 instead of keeping it)
template <int POL = 1>
__device__ __forceinline__ void store4_nt_row(uint64_t row_base, uint32_t byte_off,
                                              const float v4[4]) {
    const f32x4 v = {v4[0], v4[1], v4[2], v4[3]};
    if constexpr (POL == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<g_f32x4 *>(row_base + byte_off));
    else if constexpr (POL == 0)
        *reinterpret_cast<g_f32x4 *>(row_base + byte_off) = v;
    else if constexpr (POL == 2)
        asm volatile("global_store_dwordx4 %0, %1, %2 sc1" ::"v"(byte_off), "v"(v), "s"(row_base) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, %2 sc0 sc1" ::"v"(byte_off), "v"(v), "s"(row_base) : "memory");
}
__device__ __forceinline__ void store4_nt(double *dst, const double e[4]) {
    const f64x2 lo = {e[0], e[1]}, hi = {e[2], e[3]};
    __builtin_nontemporal_store(lo, reinterpret_cast<f64x2 *>(dst));
    __builtin_nontemporal_store(hi, reinterpret_cast<f64x2 *>(dst + 2));
}

// ------------------------------------------------------- pairwise kernel ----
struct PairArgs {
    const double *pts;
    const int64_t *cam_offs;
    const double *F;
    const int64_t *dist_offs;   // null -> (s*P + p) * mat_stride
    const int64_t *row_offs;    // null -> no argmin output
    void *dist;                 // float* or double*; null -> not written
    int32_t *argmin;
    float *minval;
    int64_t mat_stride;
    int64_t ld;                 // row stride of each matrix; 0 -> n_b
    int32_t n_cams, n_pairs, row_blocks;
    int32_t rows_per_wg;        // kWaves * RPW * row groups
    int32_t col_tile;           // columns whose lines are resident in LDS (multiple of kChunk)
    int32_t lane_results;       // 1: one RPW-lane store per group; 0: one store per row
    int32_t xcd_remap;          // 1: each XCD takes a contiguous range of the logical grid
    int32_t interleave;         // 1: a matrix's row blocks interleave in units of 4*RPW rows
    int32_t stagger;            // 1: workgroups start their row groups at different offsets
    int32_t lazy;               // 1: lazy argmin in clean row groups (chunk tracked, column recovered)
    int32_t pair_a[MVM_MAX_PAIRS];
    int32_t pair_b[MVM_MAX_PAIRS];
};

struct ColRegs {
    double l0[kColsPerLane], l1[kColsPerLane], l2[kColsPerLane];
    double x[kColsPerLane], y[kColsPerLane];
    uint32_t state[kColsPerLane];   // kOk / kDeg / kNone / kWild
};

// Row stores of the argmin / min of rows r0..r0+RPW-1: lane r holds row r's
// result (one store instruction with RPW active lanes instead of RPW stores).
// With a row rotation r_rot, slot r holds row (r + r_rot) mod RPW.
template <int RPW>
__device__ __forceinline__ void store_row_results(const uint32_t (&kmin)[RPW],
                                                  const int32_t (&imin)[RPW], int nrows, int lane,
                                                  int r_rot, int32_t *argmin, float *minval,
                                                  int64_t row0) {
    uint32_t k = kKeyInvalid;
    int32_t ix = 0;
    const int slot = (lane - r_rot) & (RPW - 1);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        k = (slot == r) ? kmin[r] : k;
        ix = (slot == r) ? imin[r] : ix;
    }
    if (lane < nrows) {
        if (argmin) argmin[row0 + lane] = (k == kKeyInvalid) ? -1 : ix;
        if (minval) minval[row0 + lane] = value_of_key(k);
    }
}

// The partner lane's value under DPP control CTRL (every lane has a partner).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_from(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Argmin of 8 rows over the wave when every lane's column indices exceed
// those of the lanes below it (one k-chunk of the cube: lane l holds columns
// 4l..4l+3, idx = its first minimum).  A transposing butterfly reduces the 8
// rows' keys together: after the xor-1/2/4 steps each lane holds one row
// (r = 4*b0 + 2*b1 + b2 of its lane bits) reduced over its 8-lane group, and
// the xor-8/16/32 steps finish it -- ~32 VALU for the 8 rows instead of 8
// per-row DPP chains.  The winner of row r is then the lowest lane holding
// its minimum (ballot + ff1): the lowest column, np.argmin's rule.  Lane
// dst0 + r returns row r's key and index (dst0 = 0: store_row_results' layout).
template <int N>
__device__ __forceinline__ void wave_argmin8_transposed(const uint32_t (&key)[N],
                                                        const int32_t (&idx)[N], int lane,
                                                        uint32_t &my_k, int32_t &my_i,
                                                        int dst0 = 0) {
    static_assert(N == 8, "8 rows");
    const bool b0 = lane & 1, b1 = lane & 2, b2 = lane & 4;
    uint32_t w[4], x[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // xor 1: keep rows 4*b0 + i
        const uint32_t send = b0 ? key[i] : key[i + 4], keep = b0 ? key[i + 4] : key[i];
        w[i] = umin(keep, dpp_from<0xB1>(send));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {   // xor 2: keep rows 4*b0 + 2*b1 + i
        const uint32_t send = b1 ? w[i] : w[i + 2], keep = b1 ? w[i + 2] : w[i];
        x[i] = umin(keep, dpp_from<0x4E>(send));
    }
    uint32_t y;
    {                               // xor 4 (swizzle, bit mode): keep row 4*b0 + 2*b1 + b2
        const uint32_t send = b2 ? x[0] : x[1], keep = b2 ? x[1] : x[0];
        y = umin(keep, (uint32_t)__builtin_amdgcn_ds_swizzle((int)send, 0x1F | (4 << 10)));
    }
    y = umin(y, dpp_from<0x128>(y));                                                  // xor 8 (row_ror:8)
    y = umin(y, (uint32_t)__builtin_amdgcn_ds_swizzle((int)y, 0x1F | (16 << 10)));      // xor 16
    y = umin(y, (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, (int)y));      // xor 32
    my_k = kKeyInvalid;
    my_i = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        // a lane whose row is r: bits (b0, b1, b2) = (r >> 2, r >> 1, r) & 1
        const int lr = ((r >> 2) & 1) | (((r >> 1) & 1) << 1) | ((r & 1) << 2);
        const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)y, lr);
        const uint64_t hit = __ballot(key[r] == k);
        const int32_t ix = __builtin_amdgcn_readlane(idx[r], (int)__builtin_ctzll(hit));
        my_k = (lane == dst0 + r) ? k : my_k;
        my_i = (lane == dst0 + r) ? ix : my_i;
    }
}

// 0.5 * s for s >= +0 finite, as bits, EXACT after the float32 cast: the
// saturating decrement of the exponent field halves every s >= 2^-1021
// exactly, maps +0 to +0, and maps s < 2^-1021 to some fp64 value below
// 2^-1021 -- which, like the true s/2 < 2^-1022, rounds to float32 +0.
// One 32-bit op instead of an fp64 multiply.  Used only where the result is
// consumed as float32 (the f64 output path multiplies by 0.5).
__device__ __forceinline__ double half_for_f32(double s) {
    const uint64_t b = (uint64_t)__double_as_longlong(s);
    const uint32_t hi = __builtin_elementwise_sub_sat((uint32_t)(b >> 32), 0x00100000u);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | (uint32_t)b));
}

// Running argmin of one row within one lane: best float32 value + its
// column.  bidx == 0x7FFFFFFF means "no column yet".  Fast-path values are
// finite, so `v < best` (strict: first occurrence wins) is the whole rule.
struct Best {
    float v;
    int32_t j;
};

__device__ __forceinline__ void best_update_fast(Best &b, float v, int32_t j) {
    const bool lt = v < b.v;
    b.v = lt ? v : b.v;
    b.j = lt ? j : b.j;
}

// Generic rule (np.argmin): a NaN beats everything and the first NaN wins;
// otherwise strict '<'; the first valid column always replaces "none".
__device__ __forceinline__ void best_update_safe(Best &b, float v, int32_t j) {
    const bool lt = (b.j == 0x7FFFFFFF) || ((v != v) ? (b.v == b.v) : (v < b.v));
    b.v = lt ? v : b.v;
    b.j = lt ? j : b.j;
}

__device__ __forceinline__ uint32_t best_key(const Best &b) {
    if (b.j == 0x7FFFFFFF) return kKeyInvalid;
    return key_of(b.v);
}

// One row x 4 columns of one lane, clean case: 7 fp64 ops + 1 int op + 1 cvt
// per pair, one 16-byte store, 3 int ops of argmin per pair.
// MASK: the tail chunk of an aligned matrix (n_b % 4 == 0): a lane's 4 columns
// are all in the view or all past it (state kNone), and only the former store.
template <bool ARGMIN, bool STORE, typename OutT, int NT = 1, bool MASK = false>
__device__ __forceinline__ void row_fast(const ColRegs &c, double rl0, double rl1, double rl2,
                                         double rx, double ry, OutT *drow, int jbase, Best &best) {
    double e[kColsPerLane];
    float v[kColsPerLane];
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        const double d1 = __builtin_fma(c.l1[q], ry, c.l0[q] * rx) + c.l2[q];      // l1 . p1
        const double d2 = __builtin_fma(rl1, c.y[q], rl0 * c.x[q]) + rl2;         // l2 . p2
        const double sum = __builtin_fabs(d1) + __builtin_fabs(d2);
        if constexpr (sizeof(OutT) == 4) {
            v[q] = (float)half_for_f32(sum);
        } else {
            e[q] = 0.5 * sum;
        }
    }
    if constexpr (sizeof(OutT) == 4) {
        if (MASK && c.state[0] == kNone) return;
        if (STORE) store4_nt_row<NT>(reinterpret_cast<uint64_t>(drow), (uint32_t)jbase * 4u, v);
        if (ARGMIN) {
#pragma unroll
            for (int q = 0; q < kColsPerLane; ++q) best_update_fast(best, v[q], jbase + q);
        }
    } else {
        if (STORE) store4_nt(drow + jbase, e);
    }
}

// Clean row of a matrix whose rows are not 16-byte aligned (n_b % 4 != 0):
// the lane holds columns jbase + 64q, so each of the 4 dword stores writes 256
// contiguous bytes.  Default store policy: a row's first and last lines are
// shared with its neighbours and L2 merges them (nontemporal partial lines
// reach HBM as masked writes, ~3.7x slower).
// Also the tail chunk of any float32 matrix: columns past the view (kNone) are
// skipped per lane.  drow == nullptr: association only.
template <bool ARGMIN>
__device__ __forceinline__ void row_fast_strided(const ColRegs &c, double rl0, double rl1,
                                                 double rl2, double rx, double ry, float *drow,
                                                 int jbase, Best &best) {
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        const double d1 = __builtin_fma(c.l1[q], ry, c.l0[q] * rx) + c.l2[q];
        const double d2 = __builtin_fma(rl1, c.y[q], rl0 * c.x[q]) + rl2;
        const float v = (float)half_for_f32(__builtin_fabs(d1) + __builtin_fabs(d2));
        if (c.state[q] != kNone) {
            if (drow) drow[jbase + kWave * q] = v;
            if (ARGMIN) best_update_fast(best, v, jbase + kWave * q);
        }
    }
}

// Generic row: degenerate lines (9999 sentinel), non-finite or huge values,
// tails, unaligned rows, no output buffer.  Column of slot q: jbase + q*jstep.
template <bool ARGMIN, typename OutT>
__device__ __forceinline__ void row_safe(const ColRegs &c, double rl0, double rl1, double rl2,
                                         double rx, double ry, bool rdeg, OutT *drow, int jbase,
                                         int jstep, Best &best) {
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        double d1 = line_dist(c.l0[q], c.l1[q], c.l2[q], rx, ry);
        d1 = (c.state[q] == kDeg) ? kSentinel : d1;
        const double d2 = rdeg ? kSentinel : line_dist(rl0, rl1, rl2, c.x[q], c.y[q]);
        const double e = 0.5 * (d1 + d2);                                            // :28
        const bool valid = c.state[q] != kNone;
        const int j = jbase + q * jstep;
        if (drow && valid) drow[j] = (OutT)e;   // default policy: L2 merges partial lines
        if (ARGMIN && valid) best_update_safe(best, (float)e, j);
    }
}

// ---- lazy argmin (clean row groups) ----
// In a row group whose rows and columns are all clean (finite, non-degenerate,
// one column tile), a lane keeps per row only the float32 bits of its minimum
// (non-negative finite floats order like their bits) and the CHUNK it came
// from: two v_min3_u32 + one compare + one select per 4 pairs instead of a
// compare and two selects per pair.  The column inside the chunk is recovered
// once per group (lane r recomputes the 4 values of row r's winning lane and
// chunk, `lazy_recover`), so the result is exactly np.argmin's: the earliest
// chunk wins inside a lane (strict '<'), the lowest q inside a chunk, and
// rows whose minimum sits in several lanes take the tie path.
__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t ab = a < b ? a : b;   // -> v_min3_u32
    return ab < c ? ab : c;
}

// float32 bits of the 4 stored values of one lane for one row (row_fast's arithmetic)
__device__ __forceinline__ void pair_bits4(const ColRegs &c, double rl0, double rl1, double rl2,
                                           double rx, double ry, float v[kColsPerLane]) {
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        const double d1 = __builtin_fma(c.l1[q], ry, c.l0[q] * rx) + c.l2[q];
        const double d2 = __builtin_fma(rl1, c.y[q], rl0 * c.x[q]) + rl2;
        v[q] = (float)half_for_f32(__builtin_fabs(d1) + __builtin_fabs(d2));
    }
}

template <bool STORE, int NT>
__device__ __forceinline__ void row_fast_lazy(const ColRegs &c, double rl0, double rl1, double rl2,
                                              double rx, double ry, float *drow, int jbase,
                                              uint32_t &bbits, int32_t &bchunk, int32_t cidx) {
    float v[kColsPerLane];
    pair_bits4(c, rl0, rl1, rl2, rx, ry, v);
    if (STORE) store4_nt_row<NT>(reinterpret_cast<uint64_t>(drow), (uint32_t)jbase * 4u, v);
    const uint32_t m = min3_u32(min3_u32(__float_as_uint(v[0]), __float_as_uint(v[1]),
                                         __float_as_uint(v[2])),
                                __float_as_uint(v[3]), bbits);
    bchunk = (m < bbits) ? cidx : bchunk;
    bbits = m;
}

// Column (within the tile) of the first of the 4 values of columns jj0..jj0+3
// against row line/point `rl`/`rx,ry` whose bits equal `k` (4 if none).
__device__ __forceinline__ int lazy_first_q(const double *s_l0, const double *s_l1,
                                            const double *s_l2, const double *s_x,
                                            const double *s_y, int jj0, double rl0, double rl1,
                                            double rl2, double rx, double ry, uint32_t k) {
    ColRegs c;
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        c.l0[q] = s_l0[jj0 + q];
        c.l1[q] = s_l1[jj0 + q];
        c.l2[q] = s_l2[jj0 + q];
        c.x[q] = s_x[jj0 + q];
        c.y[q] = s_y[jj0 + q];
    }
    float v[kColsPerLane];
    pair_bits4(c, rl0, rl1, rl2, rx, ry, v);
    int q = kColsPerLane;
#pragma unroll
    for (int p = kColsPerLane - 1; p >= 0; --p) q = (__float_as_uint(v[p]) == k) ? p : q;
    return q;
}

// ---- transposed lazy reduction (lazy == 2, the default) ----
// Minimum over the LPR = 64 / RPW consecutive lanes that share one row slot.
// Quad xor steps, then row_half_mirror / row_mirror: every lane of the group
// ends with the group minimum.
template <int RPW>
__device__ __forceinline__ uint32_t group_min_u32(uint32_t v) {
    constexpr int LPR = kWave / RPW;
    if constexpr (LPR >= 2) v = dpp_min<0xB1>(v);
    if constexpr (LPR >= 4) v = dpp_min<0x4E>(v);
    if constexpr (LPR >= 8) v = dpp_min<0x141>(v);
    if constexpr (LPR >= 16) v = dpp_min<0x140>(v);
    return v;
}

// The RPW lane minima of row slot `rs` that segment `seg` owns, from the
// wave's [RPW][64] LDS scratch (16-byte reads; RPW is a multiple of 4).
template <int RPW>
__device__ __forceinline__ void read_segment(const uint32_t *red, int rs, int seg,
                                             uint32_t (&v)[RPW]) {
    const uint32_t *src = red + rs * kWave + seg * RPW;
#pragma unroll
    for (int i = 0; i < RPW; i += 4) {
        const uint4 q = *reinterpret_cast<const uint4 *>(src + i);
        v[i] = q.x;
        v[i + 1] = q.y;
        v[i + 2] = q.z;
        v[i + 3] = q.w;
    }
}

// End of a clean (lazy) row group.  Lane L holds, per row slot r, the float32
// bits of its minimum bbits[r] and the chunk it first reached it in,
// bchunk[r].  The per-row wave reductions (RPW x (4 DPP + 4 readlane + ballot
// + selects)) become one transpose through LDS: lane L takes row slot
// rs = L / LPR and the RPW lanes [seg*RPW, seg*RPW + RPW) of that row
// (seg = L % LPR), reduces them in registers, and finishes over its LPR lanes
// with DPP.  The winner is the lowest (chunk, lane) holding the row minimum k
// -- the lowest column, since column = chunk*256 + 4*lane + q.  Returns k and
// the winner's lane and chunk, uniform over the LPR lanes of the row slot.
template <int RPW>
__device__ __forceinline__ void lazy_reduce_transposed(uint32_t *red, const uint32_t (&bbits)[RPW],
                                                       const int32_t (&bchunk)[RPW], bool multi,
                                                       int lane, uint32_t &k, int &w, int &c) {
    constexpr int LPR = kWave / RPW;
    const int rs = lane / LPR, seg = lane % LPR;
#pragma unroll
    for (int r = 0; r < RPW; ++r) red[r * kWave + lane] = bbits[r];
    // the same wave reads them back: LDS executes one wave's ops in order
    uint32_t v[RPW];
    read_segment<RPW>(red, rs, seg, v);
    uint32_t m = v[0];
#pragma unroll
    for (int i = 1; i < RPW; ++i) m = v[i] < m ? v[i] : m;
    k = group_min_u32<RPW>(m);
    uint32_t key = 0xFFFFFFFFu;
    if (!multi) {   // one chunk: the first lane of the segment holding k
        uint32_t pos = RPW;
#pragma unroll
        for (int i = RPW - 1; i >= 0; --i) pos = (v[i] == k) ? (uint32_t)i : pos;
        key = (pos < (uint32_t)RPW) ? (uint32_t)(seg * RPW) + pos : key;
    } else {        // several chunks: lowest (chunk, lane) among the lanes holding k
#pragma unroll
        for (int r = 0; r < RPW; ++r) red[r * kWave + lane] = (uint32_t)bchunk[r];
        uint32_t ch[RPW];
        read_segment<RPW>(red, rs, seg, ch);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const uint32_t ki = (ch[i] << 6) | (uint32_t)(seg * RPW + i);
            const uint32_t cand = (v[i] == k) ? ki : 0xFFFFFFFFu;
            key = cand < key ? cand : key;
        }
    }
    key = group_min_u32<RPW>(key);
    w = (int)(key & 63u);
    c = (int)(key >> 6);
}

// Workgroup = 4 waves owning rows_per_wg rows of one (scene, pair).  The
// normalised lines of (up to col_tile) columns are computed ONCE per
// workgroup into LDS; each wave then sweeps groups of RPW rows: per 256-column
// chunk every lane holds 4 consecutive columns in registers and walks the
// RPW rows, one coalesced 16-byte store per lane per row.
// occupancy: 3 waves/SIMD (<= 168 VGPRs) at RPW 16, 4 (<= 128) below;
// -DMVM_PAIRWISE_WAVES16=4 builds the RPW-16 form at 4 (A/B builds only)
#ifndef MVM_PAIRWISE_WAVES16
#define MVM_PAIRWISE_WAVES16 3
#endif
template <int RPW, bool ARGMIN, typename OutT, int NT = 1>
__global__ __launch_bounds__(kThreads, RPW >= 16 ? MVM_PAIRWISE_WAVES16 : 4) void pairwise_kernel(PairArgs args) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    const int T = args.col_tile;
    double *s_l0 = reinterpret_cast<double *>(s_dyn);
    double *s_l1 = s_l0 + T;
    double *s_l2 = s_l1 + T;
    double *s_x = s_l2 + T;
    double *s_y = s_x + T;
    // per wave: the row lines of up to 64 rows (all its groups when they fit)
    double(*s_row)[kWave][6] = reinterpret_cast<double(*)[kWave][6]>(s_y + T);
    double *s_rpt = s_y + T + kWaves * kWave * 6;            // row centroids of the workgroup
    uint32_t *s_cst = reinterpret_cast<uint32_t *>(s_rpt + 2 * args.rows_per_wg);
    // lazy == 2: per wave an [RPW][64] u32 scratch for the transposed reduction
    uint32_t *s_red = s_cst + T;

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);   // uniform by construction
    const int lane = t % kWave;
    // dispatch places workgroup b on XCD b % 8; with xcd_remap each XCD walks a
    // contiguous range of (scene, pair, row block)s, so a (scene, pair)'s row
    // blocks share one L2 and its output region stays contiguous per XCD
    uint32_t blk = blockIdx.x;
    if (args.xcd_remap) {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const int rb = (int)(blk % (uint32_t)args.row_blocks);
    const int sp = (int)(blk / (uint32_t)args.row_blocks);
    const int s = sp / args.n_pairs;
    const int p = sp - s * args.n_pairs;
    const int cam_a = args.pair_a[p], cam_b = args.pair_b[p];
    const int64_t oa = args.cam_offs[(int64_t)s * args.n_cams + cam_a];
    const int na = (int)(args.cam_offs[(int64_t)s * args.n_cams + cam_a + 1] - oa);
    const int64_t ob = args.cam_offs[(int64_t)s * args.n_cams + cam_b];
    const int nb = (int)(args.cam_offs[(int64_t)s * args.n_cams + cam_b + 1] - ob);
    // rows of the workgroup: contiguous [row0, row0 + rows_per_wg), or with
    // `interleave` units of U = 4*RPW rows dealt round-robin over the matrix's
    // row blocks (at any time a matrix's workgroups write adjacent units)
    constexpr int U = kWaves * RPW;
    const bool ilv = args.interleave != 0;
    const int row0 = ilv ? rb * U : rb * args.rows_per_wg;
    if (row0 >= na) return;   // uniform over the workgroup
    auto grow_of = [&](int x) {   // local row index -> matrix row
        return ilv ? ((x / U) * args.row_blocks + rb) * U + (x % U) : row0 + x;
    };

    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = args.F[(int64_t)sp * 9 + k];

    const int64_t doff = args.dist_offs ? args.dist_offs[sp] : (int64_t)sp * args.mat_stride;
    // first association row of this matrix, loaded before any store (a vector
    // load issued after the stores would wait for all of them: vmcnt is in order)
    const int64_t row_off0 = args.row_offs ? args.row_offs[sp] : 0;
    const int64_t ld = args.ld ? args.ld : nb;
    OutT *const dbase = args.dist ? reinterpret_cast<OutT *>(args.dist) + doff : nullptr;
    const bool vec_ok = dbase && ((doff & 3) == 0) && ((ld & 3) == 0);
    // unaligned float32 rows: lanes take strided columns (coalesced dword stores)
    const bool strided = dbase && !vec_ok && sizeof(OutT) == 4;

    // column lines of columns [c0, c0 + T) -> LDS (threads stride the tile)
    auto load_tile = [&](int c0) {
        for (int jj = t; jj < T; jj += kThreads) {
            const int j = c0 + jj;
            uint32_t st = kNone;
            double l0 = 0, l1 = 0, l2 = 0, x = 0, y = 0;
            if (j < nb) {
                x = args.pts[2 * (ob + j)];
                y = args.pts[2 * (ob + j) + 1];
                st = col_line(f, x, y, l0, l1, l2) ? kDeg : (tame(l2, x, y) ? kOk : kWild);
            }
            s_l0[jj] = l0;
            s_l1[jj] = l1;
            s_l2[jj] = l2;
            s_x[jj] = x;
            s_y[jj] = y;
            s_cst[jj] = st;
        }
    };
    // every global load of the workgroup's rows happens here, before the first
    // store (on CDNA vmcnt orders loads behind earlier stores)
    for (int x = t; x < args.rows_per_wg; x += kThreads) {
        const int i = grow_of(x);
        const f64x2 v = (i < na) ? *reinterpret_cast<const f64x2 *>(args.pts + 2 * (oa + i))
                                 : f64x2{0.0, 0.0};
        *reinterpret_cast<f64x2 *>(s_rpt + 2 * x) = v;
    }
    const int n_tiles = (nb + T - 1) / T;
    if (n_tiles == 1) load_tile(0);
    // lazy argmin needs every column of the (single) tile clean
    bool my_clean = n_tiles == 1;
    if (ARGMIN && sizeof(OutT) == 4 && args.lazy && n_tiles == 1)
        for (int jj = t; jj < T; jj += kThreads) my_clean &= (s_cst[jj] == kOk);
    const bool tile_clean = __syncthreads_and(my_clean) != 0;

    const int n_groups = ilv ? min(args.rows_per_wg / U,
                                   (na - row0 + args.row_blocks * U - 1) / (args.row_blocks * U))
                             : (min(args.rows_per_wg, na - row0) + U - 1) / U;   // uniform over the WG
    // with `stagger`, concurrently running workgroups sit at different row
    // offsets of their blocks (their stores are not 1 MiB-strided in lockstep)
    const int g_rot = (args.stagger && n_groups > 0) ? (int)(blk % (uint32_t)n_groups) : 0;
    // group g's geometry: first local row, matrix row, rows, and (stagger >= 2)
    // the rotation inside a full group -- slot r holds row (r + r_rot) mod RPW
    auto group_rows = [&](int g, int &xw, int &grow0, int &nrows, int &r_rot) {
        xw = (g * kWaves + wave) * RPW;
        grow0 = grow_of(xw);
        nrows = min(RPW, na - grow0);                          // may be <= 0
        r_rot = (args.stagger >= 2 && nrows == RPW)
                    ? (int)((blk * 5u + (uint32_t)g * 3u) & (uint32_t)(RPW - 1)) : 0;
    };
    // line of local row xw + row into slot `slot` of the wave's LDS rows
    auto put_row_line = [&](int slot, int xw, int row, int nrows) {
        double l0 = 0, l1 = 0, l2 = 0, x = 0, y = 0;
        bool deg = true;
        if (row < nrows) {
            x = s_rpt[2 * (xw + row)];
            y = s_rpt[2 * (xw + row) + 1];
            deg = row_line(f, x, y, l0, l1, l2);
        }
        s_row[wave][slot][0] = l0;
        s_row[wave][slot][1] = l1;
        s_row[wave][slot][2] = l2;
        s_row[wave][slot][3] = x;
        s_row[wave][slot][4] = y;
        s_row[wave][slot][5] = (double)(deg ? kDeg : (tame(l2, x, y) ? kOk : kWild));
    };
    // all of the wave's groups fit in 64 rows: one lane per row computes every
    // row line up front (one pass instead of one 16-lane pass per group)
    const bool pre = RPW * n_groups <= kWave;   // uniform
    if (pre && lane < RPW * n_groups) {
        int xw, grow0, nrows, r_rot;
        const int g = lane / RPW, slot = lane % RPW;
        group_rows(g, xw, grow0, nrows, r_rot);
        put_row_line(lane, xw, (slot + r_rot) & (RPW - 1), nrows);
    }
    for (int g_it = 0; g_it < n_groups; ++g_it) {
        const int g = (g_it + g_rot < n_groups) ? g_it + g_rot : g_it + g_rot - n_groups;
        int xw, grow0, nrows, r_rot;
        group_rows(g, xw, grow0, nrows, r_rot);
        double(*rowp)[6] = s_row[wave] + (pre ? g * RPW : 0);   // this group's slots
        if (!pre && lane < RPW)   // row lines of this wave's group (wave-private LDS slots)
            put_row_line((lane - r_rot) & (RPW - 1), xw, lane, nrows);
        // the same wave reads them back (LDS executes one wave's ops in order)
        const bool rows_fast =
            (nrows == RPW) && __all(lane >= RPW || rowp[lane % RPW][5] == 0.0);

        Best best[RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) best[r] = Best{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
        // uniform: the whole group takes the lazy argmin (clean rows and tile)
        const bool lazy = ARGMIN && sizeof(OutT) == 4 && args.lazy && args.row_offs &&
                          tile_clean && rows_fast && (vec_ok || !dbase);
        if (lazy) {
            uint32_t bbits[RPW];
            int32_t bchunk[RPW];
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                bbits[r] = 0x7F800000u;
                bchunk[r] = 0;
            }
            for (int c0 = 0, cidx = 0; c0 < nb; c0 += kChunk, ++cidx) {
                ColRegs c;
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) {
                    const int jj = c0 + kColsPerLane * lane + q;
                    c.l0[q] = s_l0[jj];
                    c.l1[q] = s_l1[jj];
                    c.l2[q] = s_l2[jj];
                    c.x[q] = s_x[jj];
                    c.y[q] = s_y[jj];
                }
                const int jbase = c0 + kColsPerLane * lane;
                if (dbase) {
                    const uint64_t rstep = (uint64_t)ld * sizeof(OutT);
                    const uint64_t rbase = reinterpret_cast<uint64_t>(dbase + (int64_t)grow0 * ld);
                    uint64_t rp = rbase + (uint64_t)r_rot * rstep;
                    const uint64_t rwrap = rbase + (uint64_t)RPW * rstep;
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        row_fast_lazy<true, NT>(c, rowp[r][0], rowp[r][1],
                                                rowp[r][2], rowp[r][3],
                                                rowp[r][4], reinterpret_cast<float *>(rp),
                                                jbase, bbits[r], bchunk[r], cidx);
                        rp += rstep;
                        rp = (rp == rwrap) ? rbase : rp;
                        __asm__ volatile("" : "+s"(rp));
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < RPW; ++r)
                        row_fast_lazy<false, NT>(c, rowp[r][0], rowp[r][1],
                                                 rowp[r][2], rowp[r][3],
                                                 rowp[r][4], nullptr, jbase, bbits[r],
                                                 bchunk[r], cidx);
                }
            }
            if (args.lazy >= 2) {
                constexpr int LPR = kWave / RPW;
                uint32_t k;
                int w, cw;
                lazy_reduce_transposed<RPW>(s_red + wave * (RPW * kWave), bbits, bchunk,
                                            nb > kChunk, lane, k, w, cw);
                // the LPR lanes of row slot rs recompute the winner's 4 values
                // (lane seg takes q = seg % 4) and keep the first equal to k
                const int rs = lane / LPR, q = (lane % LPR) & (kColsPerLane - 1);
                const int jj = cw * kChunk + kColsPerLane * w + q;
                const double *rl = rowp[rs];
                const double d1 = __builtin_fma(s_l1[jj], rl[4], s_l0[jj] * rl[3]) + s_l2[jj];
                const double d2 = __builtin_fma(rl[1], s_y[jj], rl[0] * s_x[jj]) + rl[2];
                const uint32_t b =
                    __float_as_uint((float)half_for_f32(__builtin_fabs(d1) + __builtin_fabs(d2)));
                const uint32_t qm = group_min_u32<RPW>((b == k) ? (uint32_t)q : 0xFFFFFFFFu);
                if (lane % LPR == 0) {
                    const int64_t row = row_off0 + grow0 + ((rs + r_rot) & (RPW - 1));
                    if (args.argmin) args.argmin[row] = jj - q + (int)qm;
                    if (args.minval) args.minval[row] = __uint_as_float(k);
                }
                continue;
            }
            // per row: wave minimum, its lane and chunk; lane r gathers row r's
            uint32_t my_k = 0;
            int32_t my_l = 0, my_c = 0;
            uint32_t ties = 0;   // rows whose minimum sits in several lanes
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const uint32_t k = wave_min_u32(bbits[r]);
                const uint64_t hit = __ballot(bbits[r] == k);
                const int wl = (int)__builtin_ctzll(hit);
                ties |= (__builtin_popcountll(hit) > 1) ? (1u << r) : 0u;
                const int wc = __builtin_amdgcn_readlane(bchunk[r], wl);
                my_k = (lane == r) ? k : my_k;
                my_l = (lane == r) ? wl : my_l;
                my_c = (lane == r) ? wc : my_c;
            }
            int32_t my_j = 0;
            if (lane < RPW) {   // lane r recovers the column of row slot r
                const int jj0 = my_c * kChunk + kColsPerLane * my_l;
                my_j = jj0 + lazy_first_q(s_l0, s_l1, s_l2, s_x, s_y, jj0, rowp[lane][0],
                                          rowp[lane][1], rowp[lane][2],
                                          rowp[lane][3], rowp[lane][4], my_k);
            }
            if (ties) {
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    if (!(ties & (1u << r))) continue;   // uniform
                    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)my_k, r);
                    uint32_t cand = 0x7FFFFFFFu;
                    if (bbits[r] == k) {   // every lane holding the minimum finds its first column
                        const int jj0 = bchunk[r] * kChunk + kColsPerLane * lane;
                        cand = (uint32_t)(jj0 + lazy_first_q(s_l0, s_l1, s_l2, s_x, s_y, jj0,
                                                             rowp[r][0], rowp[r][1],
                                                             rowp[r][2], rowp[r][3],
                                                             rowp[r][4], k));
                    }
                    const int32_t jt = (int32_t)wave_min_u32(cand);
                    my_j = (lane == r) ? jt : my_j;
                }
            }
            if (lane < nrows) {
                const int64_t row = row_off0 + grow0 + ((lane + r_rot) & (RPW - 1));
                if (args.argmin) args.argmin[row] = my_j;
                if (args.minval) args.minval[row] = __uint_as_float(my_k);
            }
            continue;
        }

        for (int tile = 0; tile < n_tiles; ++tile) {
            if (n_tiles > 1) {   // large views: stream the column lines tile by tile
                __syncthreads();
                load_tile(tile * T);
                __syncthreads();
            }
            const int tile_cols = min(T, nb - tile * T);
            if (nrows <= 0) continue;
            for (int c0 = 0; c0 < tile_cols; c0 += kChunk) {
                // strided columns for unaligned rows; an aligned matrix's tail chunk
                // keeps 16-byte stores, masked per lane
                const bool str = strided;
                const bool tail = sizeof(OutT) == 4 && c0 + kChunk > tile_cols;
                ColRegs c;
                bool clean = true, clean_m = true;
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) {
                    const int jj = str ? c0 + lane + kWave * q : c0 + kColsPerLane * lane + q;
                    c.l0[q] = s_l0[jj];
                    c.l1[q] = s_l1[jj];
                    c.l2[q] = s_l2[jj];
                    c.x[q] = s_x[jj];
                    c.y[q] = s_y[jj];
                    c.state[q] = s_cst[jj];
                    clean &= (c.state[q] == kOk);
                    clean_m &= (c.state[q] == kOk || c.state[q] == kNone);
                }
                const int jbase = tile * T + c0 + (str ? lane : kColsPerLane * lane);
                const int jstep = str ? kWave : 1;
                const bool fast = rows_fast && __all(clean);   // wave-uniform
                if (str && rows_fast && __all(clean_m)) {   // clean rows: unaligned output or tail
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        const int rr = (r + r_rot) & (RPW - 1);
                        row_fast_strided<ARGMIN>(c, rowp[r][0], rowp[r][1],
                                                 rowp[r][2], rowp[r][3],
                                                 rowp[r][4],
                                                 dbase ? reinterpret_cast<float *>(dbase + (int64_t)(grow0 + rr) * ld)
                                                       : nullptr,
                                                 jbase, best[r]);
                    }
                } else if (tail && vec_ok && rows_fast && __all(clean_m)) {   // aligned tail chunk
                    const uint64_t rstep = (uint64_t)ld * sizeof(OutT);
                    const uint64_t rbase = reinterpret_cast<uint64_t>(dbase + (int64_t)grow0 * ld);
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        const int rr = (r + r_rot) & (RPW - 1);
                        row_fast<ARGMIN, true, OutT, NT, true>(
                            c, rowp[r][0], rowp[r][1], rowp[r][2],
                            rowp[r][3], rowp[r][4],
                            reinterpret_cast<OutT *>(rbase + (uint64_t)rr * rstep), jbase, best[r]);
                    }
                } else if (fast && vec_ok) {   // the common case: clean rows, aligned output
                    const uint64_t rstep = (uint64_t)ld * sizeof(OutT);
                    const uint64_t rbase = reinterpret_cast<uint64_t>(dbase + (int64_t)grow0 * ld);
                    uint64_t rp = rbase + (uint64_t)r_rot * rstep;
                    const uint64_t rwrap = rbase + (uint64_t)RPW * rstep;
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        row_fast<ARGMIN, true, OutT, NT>(c, rowp[r][0], rowp[r][1],
                                               rowp[r][2], rowp[r][3],
                                               rowp[r][4], reinterpret_cast<OutT *>(rp),
                                               jbase, best[r]);
                        rp += rstep;
                        rp = (rp == rwrap) ? rbase : rp;
                        // keep the row address a running scalar: stops LICM
                        // hoisting all RPW row bases out of the chunk loop
                        // (they would be spilled to VGPR lanes)
                        __asm__ volatile("" : "+s"(rp));
                    }
                } else if (fast && !dbase) {   // association only, no matrix output
#pragma unroll
                    for (int r = 0; r < RPW; ++r)
                        row_fast<ARGMIN, false, OutT>(c, rowp[r][0], rowp[r][1],
                                                      rowp[r][2], rowp[r][3],
                                                      rowp[r][4], nullptr, jbase, best[r]);
                } else {
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        if (r < nrows) {
                            const int rr = (r + r_rot) & (RPW - 1);
                            OutT *drow = dbase ? dbase + (int64_t)(grow0 + rr) * ld : nullptr;
                            const bool rdeg = __builtin_amdgcn_readfirstlane(
                                                  (int)rowp[r][5]) == (int)kDeg;
                            row_safe<ARGMIN>(c, rowp[r][0], rowp[r][1],
                                             rowp[r][2], rowp[r][3],
                                             rowp[r][4], rdeg, drow, jbase, jstep, best[r]);
                        }
                    }
                }
            }
        }

        if (ARGMIN && args.row_offs && nrows > 0) {
            uint32_t kmin[RPW];
            int32_t imin[RPW];
#pragma unroll
            for (int r = 0; r < RPW; ++r) {   // independent DPP chains interleave
                kmin[r] = kKeyInvalid;
                imin[r] = 0;
                if (r < nrows) wave_argmin(best_key(best[r]), best[r].j, kmin[r], imin[r]);
            }
            if (args.lane_results) {
                store_row_results<RPW>(kmin, imin, nrows, lane, r_rot, args.argmin, args.minval,
                                       row_off0 + grow0);
            } else if (lane == 0) {
                for (int r = 0; r < nrows; ++r) {
                    const int64_t row = row_off0 + grow0 + ((r + r_rot) & (RPW - 1));
                    if (args.argmin) args.argmin[row] = (kmin[r] == kKeyInvalid) ? -1 : imin[r];
                    if (args.minval) args.minval[row] = value_of_key(kmin[r]);
                }
            }
        }
    }
}

// --------------------------------------------------------- triplet kernel ----
struct CubeArgs {
    const int64_t *cam_offs;    // [S*3 + 1]
    const double *e;            // fp64 pair matrices (e12, e13, e23 per scene)
    int64_t mat_stride;         // elements between consecutive matrices
    int64_t ld;                 // row stride of every matrix (multiple of 4)
    const int64_t *cube_offs;
    const int64_t *row_offs;
    float *cube;
    int32_t *argmin;
    float *minval;
    int32_t i_count;            // max_n (grid i extent)
    int32_t j_blocks;
};

// ((e12 + e13) + e23) / 3 -> float32  (epipolar_matching.py:78-81, :96)
__device__ __forceinline__ double triple_cost(double e12, double e13, double e23) {
    return ((e12 + e13) + e23) / 3.0;
}

template <int RPW>
__global__ __launch_bounds__(kThreads) void triplet_kernel(CubeArgs args) {
    const int t = threadIdx.x;
    const int wave = t / kWave;
    const int lane = t % kWave;
    const int jb = (int)(blockIdx.x % (uint32_t)args.j_blocks);
    const int si = (int)(blockIdx.x / (uint32_t)args.j_blocks);
    const int s = si / args.i_count;
    const int i = si - s * args.i_count;
    const int64_t o1 = args.cam_offs[3 * (int64_t)s];
    const int N = (int)(args.cam_offs[3 * (int64_t)s + 1] - o1);
    const int M = (int)(args.cam_offs[3 * (int64_t)s + 2] - args.cam_offs[3 * (int64_t)s + 1]);
    const int P = (int)(args.cam_offs[3 * (int64_t)s + 3] - args.cam_offs[3 * (int64_t)s + 2]);
    const int j0 = jb * kWaves * RPW + wave * RPW;
    if (i >= N || j0 >= M) return;   // uniform over the wave (no barriers below)

    const double *e12 = args.e + (int64_t)(3 * s + 0) * args.mat_stride;
    const double *e13 = args.e + (int64_t)(3 * s + 1) * args.mat_stride + (int64_t)i * args.ld;
    const double *e23 = args.e + (int64_t)(3 * s + 2) * args.mat_stride;
    const int64_t coff = args.cube_offs[s];
    const bool vec_ok = ((coff & 3) == 0) && ((P & 3) == 0);

    uint32_t bkey[RPW];
    int32_t bidx[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        bkey[r] = kKeyInvalid;
        bidx[r] = 0x7FFFFFFF;
    }

    for (int c0 = 0; c0 < P; c0 += kChunk) {
        const int kbase = c0 + kColsPerLane * lane;
        const bool full = vec_ok && (c0 + kChunk <= P);
        double a13[kColsPerLane];
#pragma unroll
        for (int q = 0; q < kColsPerLane; ++q) a13[q] = (kbase + q < P) ? e13[kbase + q] : 0.0;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int j = j0 + r;
            if (j >= M) break;
            const double v12 = e12[(int64_t)i * args.ld + j];
            const double *e23r = e23 + (int64_t)j * args.ld;
            double e[kColsPerLane];
#pragma unroll
            for (int q = 0; q < kColsPerLane; ++q) {
                const double v23 = (kbase + q < P) ? e23r[kbase + q] : 0.0;
                e[q] = triple_cost(v12, a13[q], v23);
            }
            float *crow = args.cube ? args.cube + coff + ((int64_t)i * M + j) * P : nullptr;
            if (crow) {
                if (full) {
                    store4_nt(crow + kbase, e);
                } else {
#pragma unroll
                    for (int q = 0; q < kColsPerLane; ++q)
                        if (kbase + q < P) crow[kbase + q] = (float)e[q];   // L2 merges strided dwords
                }
            }
#pragma unroll
            for (int q = 0; q < kColsPerLane; ++q) {
                const uint32_t k = (kbase + q < P) ? key_of((float)e[q]) : kKeyInvalid;
                if (k < bkey[r]) {
                    bkey[r] = k;
                    bidx[r] = kbase + q;
                }
            }
        }
    }

    const int64_t roff = args.row_offs[s];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int j = j0 + r;
        if (j >= M) break;
        uint32_t kmin;
        int32_t imin;
        wave_argmin(bkey[r], bidx[r], kmin, imin);
        if (lane == 0) {
            const int64_t row = roff + (int64_t)i * M + j;
            if (args.argmin) args.argmin[row] = (kmin == kKeyInvalid) ? -1 : imin;
            if (args.minval) args.minval[row] = value_of_key(kmin);
        }
    }
}

// ------------------------------------------------- fast triplet kernel ----
// float32(RN(x / 3)) for x >= +0 without an IEEE division in the common case
// (third_fast_ok: the -DMVM_CUBE_THIRD_CHECK=1 form; the default is third_q below).
// q0 = RN(x * RN(1/3)) is within one ulp of RN(x / 3) (RN(1/3) = (1 - 2^-54)/3,
// so |x*RN(1/3) - x/3| <= ulp/2, plus the product's own rounding).  Their
// float32 roundings can differ only if a float32 rounding midpoint -- an fp64
// value whose low 29 mantissa bits are exactly 2^28 -- lies within one ulp of
// q0, or if the result leaves the float32 normal range.  Those (rare) lanes
// take the correctly rounded division; tests/test_host_logic.py checks the
// rule on random and adversarial near-midpoint inputs.
constexpr double kThird = 1.0 / 3.0;
// residual bound under which a sum of three is finite (tile-wide fast path)
constexpr double kTameResidual = 0x1p1020;

// 4 consecutive doubles at a 16-byte aligned address (two dwordx4 loads);
// lanes past the view's end read zeros.
__device__ __forceinline__ void load4(const double *p, int valid, double out[4]) {
    if (valid >= 4) {
        const f64x2 lo = *reinterpret_cast<const f64x2 *>(p);
        const f64x2 hi = *reinterpret_cast<const f64x2 *>(p + 2);
        out[0] = lo.x;
        out[1] = lo.y;
        out[2] = hi.x;
        out[3] = hi.y;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) out[q] = q < valid ? p[q] : 0.0;
    }
}

__device__ __forceinline__ bool third_fast_ok(double q0) {
    const uint64_t b = (uint64_t)__double_as_longlong(q0);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    const uint32_t low29 = lo & 0x1FFFFFFFu;
    const bool near_mid = (low29 - ((1u << 28) - 3u)) <= 6u;      // |low29 - 2^28| <= 3
    const bool in_range = ((hi >> 20) - (1023u - 126u)) <= 252u;   // 2^-126 <= q0 < 2^127
    return !near_mid && in_range;                                  // NaN/inf/negative: false
}

// RN(s / 3) by one Markstein correction (the default): with y = RN(1/3) and
// q0 = RN(s * y) within one ulp of s/3, r = fma(-q0, 3, s) is exact and
// q1 = fma(r, y, q0) is the correctly rounded quotient -- for every finite s
// (checked against the IEEE division on 1.1e9 random, binade-edge,
// subnormal and near-midpoint inputs, tools/probes/third_markstein.c, and in
// tests/test_host_logic.py).  Three fp64 ops and a finiteness test instead
// of the product plus third_fast_ok's midpoint/range test (~8 ops); only
// non-finite sums (inf: q1 = NaN) take the division.  A sum of residuals is
// never -0, the one input whose sign the correction would not keep.
// -DMVM_CUBE_THIRD_CHECK=1 restores the product + third_fast_ok form (A/B).
#ifndef MVM_CUBE_THIRD_CHECK
#define MVM_CUBE_THIRD_CHECK 0
#endif
__device__ __forceinline__ double third_q(double s) {
#if MVM_CUBE_THIRD_CHECK
    return s * kThird;
#else
    const double q0 = s * kThird;
    return __builtin_fma(__builtin_fma(-q0, 3.0, s), kThird, q0);
#endif
}

// true: third_q(s) == RN(s / 3); false: the caller divides
__device__ __forceinline__ bool third_ok(double q) {
#if MVM_CUBE_THIRD_CHECK
    return third_fast_ok(q);
#else
    return __builtin_isfinite(q);
#endif
}

// ------------------------------------------- tiled triplet kernel (v3) ----
// The 3-camera cube for P <= 256 from the fp64 workspace: a workgroup owns
// (scene, 16 consecutive j, IB consecutive i).  Its prologue loads everything
// the tile needs -- e23 rows into registers, the e13[i-block][:] and
// e12[i-block][j-block] tiles into LDS -- with ONE wait; the main loop then
// issues only LDS reads, VALU work and stores.  This matters on CDNA, where
// vmcnt counts loads and stores together in issue order: a global load
// issued after a row store waits for that store's acknowledgement, so loads
// inside a store-streaming loop stall it.

struct Cube3Args {
    const int64_t *cam_offs;
    const double *e;
    int64_t mat_stride;
    int64_t ld;
    const int64_t *cube_offs;
    const int64_t *row_offs;
    float *cube;
    int32_t *argmin;
    float *minval;
    int32_t j_blocks, i_blocks;
};

template <int kCubeIB, int kCubeRPW>   // i rows per tile, j rows per wave
__global__ __launch_bounds__(kThreads) void triplet_tile_kernel(Cube3Args args) {
    __shared__ __attribute__((aligned(16))) double s13[kCubeIB][kChunk];              // 32 KiB
    __shared__ __attribute__((aligned(16))) double s12[kCubeIB][kWaves * kCubeRPW];   // 2 KiB

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);
    const int lane = t % kWave;
    const uint32_t per_scene = (uint32_t)(args.j_blocks * args.i_blocks);
    const int s = (int)(blockIdx.x / per_scene);
    const int rem = (int)(blockIdx.x % per_scene);
    const int jb = rem % args.j_blocks;
    const int ib = rem / args.j_blocks;
    const int64_t c0 = args.cam_offs[3 * (int64_t)s];
    const int N = (int)(args.cam_offs[3 * (int64_t)s + 1] - c0);
    const int M = (int)(args.cam_offs[3 * (int64_t)s + 2] - args.cam_offs[3 * (int64_t)s + 1]);
    const int P = (int)(args.cam_offs[3 * (int64_t)s + 3] - args.cam_offs[3 * (int64_t)s + 2]);
    const int jw0 = jb * kWaves * kCubeRPW;            // first j of the workgroup
    const int i0 = ib * kCubeIB;
    if (jw0 >= M || i0 >= N || P == 0) return;         // uniform over the workgroup
    const int ni = min(kCubeIB, N - i0);
    const int j0 = jw0 + wave * kCubeRPW;              // this wave's first j
    const int nrows = min(kCubeRPW, M - j0);           // may be <= 0 (scalar)

    const double *e12 = args.e + (int64_t)(3 * s + 0) * args.mat_stride;
    const double *e13 = args.e + (int64_t)(3 * s + 1) * args.mat_stride;
    const double *e23 = args.e + (int64_t)(3 * s + 2) * args.mat_stride;
    const int kb = kColsPerLane * lane;
    const int kvalid = P - kb;
    const int64_t coff = args.cube_offs[s];
    const int64_t roff = args.row_offs[s];
    // vector rows: every lane's 4 k valid or none (P % 4 == 0), 16-byte aligned
    const bool full = ((P & 3) == 0) && ((coff & 3) == 0) && args.cube;
    const bool act = kvalid > 0;

    // ---- prologue: all loads of the tile, then one barrier ----------------
    double a23[kCubeRPW][kColsPerLane];
#pragma unroll
    for (int r = 0; r < kCubeRPW; ++r)
        load4(e23 + (int64_t)(j0 + max(0, min(r, nrows - 1))) * args.ld + kb, kvalid, a23[r]);
    for (int x = t; x < kCubeIB * (kChunk / 2); x += kThreads) {   // e13 tile, 16 B per load
        const int r = x / (kChunk / 2), c = 2 * (x % (kChunk / 2));
        f64x2 v = {0.0, 0.0};
        if (r < ni && c < P) {
            if (c + 1 < P) {
                v = *reinterpret_cast<const f64x2 *>(e13 + (int64_t)(i0 + r) * args.ld + c);
            } else {
                v.x = e13[(int64_t)(i0 + r) * args.ld + c];
            }
        }
        *reinterpret_cast<f64x2 *>(&s13[r][c]) = v;
    }
    for (int x = t; x < kCubeIB * kWaves * kCubeRPW; x += kThreads) {
        const int r = x / (kWaves * kCubeRPW), c = x % (kWaves * kCubeRPW);
        s12[r][c] = (r < ni && jw0 + c < M) ? e12[(int64_t)(i0 + r) * args.ld + jw0 + c] : 0.0;
    }
    __syncthreads();
    if (nrows <= 0) return;   // after the barrier: no more barriers below

    for (int ii = 0; ii < ni; ++ii) {
        const int i = i0 + ii;
        double a13[kColsPerLane];
        {
            const f64x2 lo = *reinterpret_cast<const f64x2 *>(&s13[ii][kb]);
            const f64x2 hi = *reinterpret_cast<const f64x2 *>(&s13[ii][kb + 2]);
            a13[0] = lo.x; a13[1] = lo.y; a13[2] = hi.x; a13[3] = hi.y;
        }
        uint32_t key[kCubeRPW];
        int32_t idx[kCubeRPW];
#pragma unroll
        for (int r = 0; r < kCubeRPW; ++r) {
            key[r] = kKeyInvalid;
            idx[r] = 0x7FFFFFFF;
            if (r >= nrows) continue;   // uniform
            const double v12 = s12[ii][wave * kCubeRPW + r];
            double sum[kColsPerLane], q0[kColsPerLane];
            bool ok = true;
#pragma unroll
            for (int q = 0; q < kColsPerLane; ++q) {
                sum[q] = (v12 + a13[q]) + a23[r][q];          // (e12 + e13) + e23, :81
                q0[q] = third_q(sum[q]);
                ok &= third_ok(q0[q]);
            }
            float v[kColsPerLane];
            const int64_t row = (int64_t)i * M + j0 + r;
            if (full && __all(ok || !act)) {
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) v[q] = (float)q0[q];
                if (act) {
                    store4_nt_row(reinterpret_cast<uint64_t>(args.cube + coff + row * P),
                                  (uint32_t)kb * 4u, v);
                }
                Best b{v[0], kb};
#pragma unroll
                for (int q = 1; q < kColsPerLane; ++q) best_update_fast(b, v[q], kb + q);
                key[r] = act ? __float_as_uint(b.v) + 1u : kKeyInvalid;
                idx[r] = act ? b.j : 0x7FFFFFFF;
            } else {
                Best b{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
                // the IEEE division only when some lane needs it (uniform branch)
                double qq[kColsPerLane];
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) qq[q] = q0[q];
                if (!__all(ok || !act)) {
#pragma unroll
                    for (int q = 0; q < kColsPerLane; ++q)
                        qq[q] = third_ok(q0[q]) ? q0[q] : sum[q] / 3.0;
                }
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) {
                    v[q] = (float)qq[q];
                    if (q < kvalid) {
                        if (args.cube)
                            args.cube[coff + row * P + kb + q] = v[q];   // L2 merges the 4 strided dword stores
                        best_update_safe(b, v[q], kb + q);
                    }
                }
                key[r] = best_key(b);
                idx[r] = b.j;
            }
        }
        uint32_t kmin[kCubeRPW];
        int32_t imin[kCubeRPW];
#pragma unroll
        for (int r = 0; r < kCubeRPW; ++r) {
            kmin[r] = kKeyInvalid;
            imin[r] = 0;
            if (r < nrows) wave_argmin(key[r], idx[r], kmin[r], imin[r]);
        }
        store_row_results<kCubeRPW>(kmin, imin, nrows, lane, 0, args.argmin, args.minval,
                                    roff + (int64_t)i * M + j0);
    }
}

// ------------------------------------------- fused tiled cube (v4) ----
// triplet_tile_kernel without the fp64 workspace: the prologue computes the
// tile's pair residuals from the centroids and F directly (exactly row_safe's
// arithmetic) instead of loading them -- e23 for the wave's RPW j rows and the
// lane's 4 k into registers, e13 [IB][P] and e12 [IB][4*RPW] into LDS -- so
// the cube costs one launch and no workspace write + read (the
// workspace was ~10% of the cube's HBM traffic at 256^3).
struct CubeFusedArgs {
    const double *pts;
    const int64_t *cam_offs;
    const double *F;            // [S*3, 9]: F12, F13, F23
    const int64_t *cube_offs;
    const int64_t *row_offs;
    float *cube;
    int32_t *argmin;
    float *minval;
    int32_t j_blocks, i_blocks;
    int32_t xcd_remap;          // as PairArgs::xcd_remap
};

struct LineRec {
    double l0, l1, l2;
    double deg;                 // 1.0: degenerate line (9999 sentinel)
};

__device__ __forceinline__ double pair_e(const LineRec &col, const LineRec &row, double rx,
                                         double ry, double cx, double cy) {
    const double d1 = col.deg != 0.0 ? kSentinel : line_dist(col.l0, col.l1, col.l2, rx, ry);
    const double d2 = row.deg != 0.0 ? kSentinel : line_dist(row.l0, row.l1, row.l2, cx, cy);
    return 0.5 * (d1 + d2);                                                       // :28
}

__device__ __forceinline__ void load_f(const double *F, double f[9]) {
#pragma unroll
    for (int q = 0; q < 9; ++q) f[q] = F[q];
}

// SPLIT 2 / 4 (views of <= 128 / <= 64 detections, kCubeRPW == 8): the wave
// splits into SPLIT lane groups of 64/SPLIT lanes, each taking one (i, j) row
// with lanes along k (4 k per lane), so a wave instruction covers SPLIT rows
// and no lane idles past P <= 256/SPLIT; a lane computes wave rows
// r + (8/SPLIT)*(its group).  The argmin of the 8 rows is the transposed
// butterfly over keys that are invalid outside each row's group.
template <int kCubeIB, int kCubeRPW, int SPLIT = 1>
__global__ __launch_bounds__(kThreads, kCubeIB <= 16 ? 4 : 2) void triplet_fused_kernel(CubeFusedArgs args) {
    constexpr bool HALF = SPLIT > 1;   // split mapping
    static_assert(SPLIT == 1 || (kCubeRPW == 8 && (SPLIT == 2 || SPLIT == 4)), "8 rows in 2 or 4 groups");
    constexpr int kLaneRows = kCubeRPW / SPLIT;   // rows a lane computes
    constexpr int kLPR = kWave / SPLIT;           // lanes per row
    constexpr int kJ = kWaves * kCubeRPW;                                          // j per workgroup
    __shared__ __attribute__((aligned(16))) double s13[kCubeIB][kChunk];           // 32 KiB
    __shared__ __attribute__((aligned(16))) double s12[kCubeIB][kJ];
    __shared__ LineRec s_r13[kCubeIB], s_r12[kCubeIB], s_c12[kJ], s_r23[kJ];
    __shared__ double s_p0[kCubeIB][2], s_p1[kJ][2];

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);
    const int lane = t % kWave;
    uint32_t blk = blockIdx.x;
    if (args.xcd_remap) {       // each XCD walks a contiguous range of tiles
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const uint32_t per_scene = (uint32_t)(args.j_blocks * args.i_blocks);
    const int s = (int)(blk / per_scene);
    const int rem = (int)(blk % per_scene);
    const int jb = rem % args.j_blocks;
    const int ib = rem / args.j_blocks;
    const int64_t *co = args.cam_offs + 3 * (int64_t)s;
    const int64_t c0 = co[0], c1 = co[1], c2 = co[2];
    const int N = (int)(c1 - c0), M = (int)(c2 - c1), P = (int)(co[3] - c2);
    const int jw0 = jb * kJ;
    const int i0 = ib * kCubeIB;
    if (jw0 >= M || i0 >= N || P == 0) return;         // uniform over the workgroup
    const int ni = min(kCubeIB, N - i0);
    const int j0 = jw0 + wave * kCubeRPW;
    const int nrows = min(kCubeRPW, M - j0);
    const int hl = lane / kLPR;                                      // row group of the lane
    const int kb = kColsPerLane * (lane % kLPR);
    const int kvalid = P - kb;
    const int64_t coff = args.cube_offs[s];
    const int64_t roff = args.row_offs[s];
    // vector rows: every lane's 4 k valid or none (P % 4 == 0), 16-byte aligned
    const bool full = ((P & 3) == 0) && ((coff & 3) == 0) && args.cube;
    const bool act_k = kvalid > 0;
    const double *F12 = args.F + (3 * (int64_t)s + 0) * 9;
    const double *F13 = args.F + (3 * (int64_t)s + 1) * 9;
    const double *F23 = args.F + (3 * (int64_t)s + 2) * 9;

    // ---- prologue 1: the tile's view-0 rows and view-1 rows/columns --------
    if (t < kCubeIB) {
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (t < ni) {
            double f[9];
            px = args.pts[2 * (c0 + i0 + t)];
            py = args.pts[2 * (c0 + i0 + t) + 1];
            load_f(F13, f);
            a.deg = row_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F12, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        s_r13[t] = a;
        s_r12[t] = b;
        s_p0[t][0] = px;
        s_p0[t][1] = py;
    } else if (t >= kWave && t < kWave + kJ) {
        const int jj = t - kWave;
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (jw0 + jj < M) {
            double f[9];
            px = args.pts[2 * (c1 + jw0 + jj)];
            py = args.pts[2 * (c1 + jw0 + jj) + 1];
            load_f(F12, f);
            a.deg = col_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F23, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        s_c12[jj] = a;
        s_r23[jj] = b;
        s_p1[jj][0] = px;
        s_p1[jj][1] = py;
    }
    __syncthreads();
    // ---- prologue 2: the tile's pair residuals (row_safe's arithmetic) -------
    bool tame_in = true;   // every residual this thread produced is <= kTameResidual
    {
        const int k = t;                                   // kThreads == kChunk: one column each
        if (k < P) {
            double f[9];
            load_f(F13, f);
            const double x = args.pts[2 * (c2 + k)], y = args.pts[2 * (c2 + k) + 1];
            LineRec cl{0.0, 0.0, 0.0, 0.0};
            cl.deg = col_line(f, x, y, cl.l0, cl.l1, cl.l2) ? 1.0 : 0.0;
#pragma unroll 4
            for (int r = 0; r < kCubeIB; ++r) {
                const double e = r < ni ? pair_e(cl, s_r13[r], s_p0[r][0], s_p0[r][1], x, y) : 0.0;
                s13[r][k] = e;
                tame_in &= e <= kTameResidual;
            }
        } else {
            for (int r = 0; r < kCubeIB; ++r) s13[r][k] = 0.0;
        }
    }
    for (int x = t; x < kCubeIB * kJ; x += kThreads) {
        const int r = x / kJ, jj = x % kJ;
        const double e = (r < ni && jw0 + jj < M)
                             ? pair_e(s_c12[jj], s_r12[r], s_p0[r][0], s_p0[r][1], s_p1[jj][0], s_p1[jj][1])
                             : 0.0;
        s12[r][jj] = e;
        tame_in &= e <= kTameResidual;
    }
    double a23[kLaneRows][kColsPerLane];
    {
        double f[9];
        load_f(F23, f);
#pragma unroll
        for (int q = 0; q < kColsPerLane; ++q) {
            LineRec cl{0.0, 0.0, 0.0, 0.0};
            double x = 0.0, y = 0.0;
            if (q < kvalid) {
                x = args.pts[2 * (c2 + kb + q)];
                y = args.pts[2 * (c2 + kb + q) + 1];
                cl.deg = col_line(f, x, y, cl.l0, cl.l1, cl.l2) ? 1.0 : 0.0;
            }
#pragma unroll
            for (int r = 0; r < kLaneRows; ++r) {
                const int rr = r + hl * kLaneRows;            // the wave row
                const int jj = wave * kCubeRPW + rr;
                a23[r][q] = (rr < nrows && q < kvalid)
                                ? pair_e(cl, s_r23[jj], s_p1[jj][0], s_p1[jj][1], x, y)
                                : 0.0;
                tame_in &= a23[r][q] <= kTameResidual;
            }
        }
    }
    // every sum of the tile is finite when its three residuals are <= 2^1020
    // (NaN fails the compare): then third_q is RN(s/3) for all of them and the
    // main loop needs no per-row check (a loop without the fallback path)
    const bool tile_fast = __syncthreads_and(tame_in) != 0 && full && !MVM_CUBE_THIRD_CHECK;
    if (nrows <= 0) return;   // after the barrier: no more barriers below

    auto main_loop = [&](auto fast_tag) {
        constexpr bool FAST = decltype(fast_tag)::value;
        for (int ii = 0; ii < ni; ++ii) {
            const int i = i0 + ii;
            double a13[kColsPerLane];
            {
                const f64x2 lo = *reinterpret_cast<const f64x2 *>(&s13[ii][kb]);
                const f64x2 hi = *reinterpret_cast<const f64x2 *>(&s13[ii][kb + 2]);
                a13[0] = lo.x; a13[1] = lo.y; a13[2] = hi.x; a13[3] = hi.y;
            }
            uint32_t key[kLaneRows];
            int32_t idx[kLaneRows];
#pragma unroll
            for (int r = 0; r < kLaneRows; ++r) {
                key[r] = kKeyInvalid;
                idx[r] = 0x7FFFFFFF;
                if (r >= nrows) continue;   // uniform (the lower half's row is the smaller)
                const int rr = r + hl * kLaneRows;                 // the wave row
                const bool act = act_k && rr < nrows;              // HALF: the upper row may not exist
                const double v12 = s12[ii][wave * kCubeRPW + rr];
                double sum[kColsPerLane], q0[kColsPerLane];
                bool ok = true;
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) {
                    sum[q] = (v12 + a13[q]) + a23[r][q];          // (e12 + e13) + e23, :81
                    q0[q] = third_q(sum[q]);
                    if (!FAST) ok &= third_ok(q0[q]);
                }
                float v[kColsPerLane];
                const int64_t row = (int64_t)i * M + j0 + rr;
                if (FAST || (full && __all(ok || !act))) {
#pragma unroll
                    for (int q = 0; q < kColsPerLane; ++q) v[q] = (float)q0[q];
                    if (act) {
                        store4_nt_row(reinterpret_cast<uint64_t>(args.cube + coff + row * P),
                                      (uint32_t)kb * 4u, v);
                    }
                    Best b{v[0], kb};
#pragma unroll
                    for (int q = 1; q < kColsPerLane; ++q) best_update_fast(b, v[q], kb + q);
                    key[r] = act ? __float_as_uint(b.v) + 1u : kKeyInvalid;
                    idx[r] = act ? b.j : 0x7FFFFFFF;
                } else {
                    Best b{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
                    // the IEEE division only when some lane needs it (uniform branch)
                    double qq[kColsPerLane];
#pragma unroll
                    for (int q = 0; q < kColsPerLane; ++q) qq[q] = q0[q];
                    if (!__all(ok || !act)) {
#pragma unroll
                        for (int q = 0; q < kColsPerLane; ++q)
                            qq[q] = third_ok(q0[q]) ? q0[q] : sum[q] / 3.0;
                    }
#pragma unroll
                    for (int q = 0; q < kColsPerLane; ++q) {
                        v[q] = (float)qq[q];
                        if (act && q < kvalid) {
                            if (args.cube)
                                args.cube[coff + row * P + kb + q] = v[q];   // L2 merges the 4 strided dword stores
                            best_update_safe(b, v[q], kb + q);
                        }
                    }
                    key[r] = best_key(b);
                    idx[r] = b.j;
                }
            }
            if constexpr (HALF) {   // SPLIT rows share a wave: keys of the other groups are invalid
                uint32_t key8[kCubeRPW];
                int32_t idx8[kCubeRPW];
#pragma unroll
                for (int r = 0; r < kCubeRPW; ++r) {
                    const bool mine = (r / kLaneRows) == hl;
                    key8[r] = mine ? key[r % kLaneRows] : kKeyInvalid;
                    idx8[r] = mine ? idx[r % kLaneRows] : 0x7FFFFFFF;
                }
                uint32_t mk;
                int32_t mi;
                wave_argmin8_transposed(key8, idx8, lane, mk, mi);
                if (lane < nrows) {
                    const int64_t row = roff + (int64_t)i * M + j0 + lane;
                    if (args.argmin) args.argmin[row] = (mk == kKeyInvalid) ? -1 : mi;
                    if (args.minval) args.minval[row] = value_of_key(mk);
                }
            } else if constexpr (FAST && kCubeRPW == 8) {   // finite keys, one k-chunk
                uint32_t mk;
                int32_t mi;
                wave_argmin8_transposed(key, idx, lane, mk, mi);
                if (lane < nrows) {
                    const int64_t row = roff + (int64_t)i * M + j0 + lane;
                    if (args.argmin) args.argmin[row] = (mk == kKeyInvalid) ? -1 : mi;
                    if (args.minval) args.minval[row] = value_of_key(mk);
                }
            } else {
                uint32_t kmin[kCubeRPW];
                int32_t imin[kCubeRPW];
#pragma unroll
                for (int r = 0; r < kCubeRPW; ++r) {
                    kmin[r] = kKeyInvalid;
                    imin[r] = 0;
                    if (r < nrows) wave_argmin(key[r], idx[r], kmin[r], imin[r]);
                }
                store_row_results<kCubeRPW>(kmin, imin, nrows, lane, 0, args.argmin, args.minval,
                                            roff + (int64_t)i * M + j0);
            }
        }
    };
    if (tile_fast) main_loop(std::integral_constant<bool, true>{});
    else main_loop(std::integral_constant<bool, false>{});
}

// ------------------------------------ fused tiled cube, any P (v5) ----
// triplet_fused_kernel for views of more than 256 detections: the k axis is
// walked in chunks of 256.  Per chunk the prologue computes that chunk's
// e13 [IB][256] (LDS) and the wave's e23 [RPW j][4 k] (registers) exactly as
// the single-chunk kernel does; the tile's view-0 / view-1 lines and e12 are
// computed once.  Each (i, j) row's argmin runs across chunks in two lane-
// distributed registers (row x = ii*RPW + r lives in lane x % 64, slot x / 64):
// a chunk's wave minimum replaces the running one only if strictly smaller,
// so the earliest chunk wins ties (np.argmin's first index).
template <int kCubeIB, int kCubeRPW>
__global__ __launch_bounds__(kThreads, 3) void triplet_fused_chunked_kernel(CubeFusedArgs args) {
    constexpr int kJ = kWaves * kCubeRPW;
    constexpr int kRows = kCubeIB * kCubeRPW;                                      // (i, j) rows per wave
    constexpr int kSlots = (kRows + kWave - 1) / kWave;
    __shared__ __attribute__((aligned(16))) double s13[kCubeIB][kChunk];           // 32 KiB
    __shared__ __attribute__((aligned(16))) double s12[kCubeIB][kJ];
    __shared__ LineRec s_r13[kCubeIB], s_r12[kCubeIB], s_c12[kJ], s_r23[kJ];
    __shared__ double s_p0[kCubeIB][2], s_p1[kJ][2];

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);
    const int lane = t % kWave;
    uint32_t blk = blockIdx.x;
    if (args.xcd_remap) {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const uint32_t per_scene = (uint32_t)(args.j_blocks * args.i_blocks);
    const int s = (int)(blk / per_scene);
    const int rem = (int)(blk % per_scene);
    const int jb = rem % args.j_blocks;
    const int ib = rem / args.j_blocks;
    const int64_t *co = args.cam_offs + 3 * (int64_t)s;
    const int64_t c0 = co[0], c1 = co[1], c2 = co[2];
    const int N = (int)(c1 - c0), M = (int)(c2 - c1), P = (int)(co[3] - c2);
    const int jw0 = jb * kJ;
    const int i0 = ib * kCubeIB;
    if (jw0 >= M || i0 >= N || P == 0) return;         // uniform over the workgroup
    const int ni = min(kCubeIB, N - i0);
    const int j0 = jw0 + wave * kCubeRPW;
    const int nrows = min(kCubeRPW, M - j0);
    const int kb = kColsPerLane * lane;
    const int64_t coff = args.cube_offs[s];
    const int64_t roff = args.row_offs[s];
    const double *F12 = args.F + (3 * (int64_t)s + 0) * 9;
    const double *F13 = args.F + (3 * (int64_t)s + 1) * 9;
    const double *F23 = args.F + (3 * (int64_t)s + 2) * 9;

    // ---- once per tile: view-0 rows, view-1 rows/columns, e12 ---------------
    if (t < kCubeIB) {
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (t < ni) {
            double f[9];
            px = args.pts[2 * (c0 + i0 + t)];
            py = args.pts[2 * (c0 + i0 + t) + 1];
            load_f(F13, f);
            a.deg = row_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F12, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        s_r13[t] = a;
        s_r12[t] = b;
        s_p0[t][0] = px;
        s_p0[t][1] = py;
    } else if (t >= kWave && t < kWave + kJ) {
        const int jj = t - kWave;
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (jw0 + jj < M) {
            double f[9];
            px = args.pts[2 * (c1 + jw0 + jj)];
            py = args.pts[2 * (c1 + jw0 + jj) + 1];
            load_f(F12, f);
            a.deg = col_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F23, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        s_c12[jj] = a;
        s_r23[jj] = b;
        s_p1[jj][0] = px;
        s_p1[jj][1] = py;
    }
    __syncthreads();
    bool tame12 = true;   // as triplet_fused_kernel's tame_in, for this thread's e12
    for (int x = t; x < kCubeIB * kJ; x += kThreads) {
        const int r = x / kJ, jj = x % kJ;
        const double e = (r < ni && jw0 + jj < M)
                             ? pair_e(s_c12[jj], s_r12[r], s_p0[r][0], s_p0[r][1], s_p1[jj][0], s_p1[jj][1])
                             : 0.0;
        s12[r][jj] = e;
        tame12 &= e <= kTameResidual;
    }
    uint32_t run_k[kSlots];
    int32_t run_i[kSlots];
#pragma unroll
    for (int z = 0; z < kSlots; ++z) {
        run_k[z] = kKeyInvalid;
        run_i[z] = 0;
    }

    for (int kc = 0; kc < P; kc += kChunk) {
        const int Pc = min(kChunk, P - kc);
        const int kvalid = Pc - kb;
        if (kc > 0) __syncthreads();   // every wave is done with the previous chunk's s13
        bool tame_in = tame12;
        {   // e13 of this chunk: one column per thread
            const int k = t;
            double f13[9];
            load_f(F13, f13);
            if (k < Pc) {
                const double x = args.pts[2 * (c2 + kc + k)], y = args.pts[2 * (c2 + kc + k) + 1];
                LineRec cl{0.0, 0.0, 0.0, 0.0};
                cl.deg = col_line(f13, x, y, cl.l0, cl.l1, cl.l2) ? 1.0 : 0.0;
#pragma unroll 4
                for (int r = 0; r < kCubeIB; ++r) {
                    const double e = r < ni ? pair_e(cl, s_r13[r], s_p0[r][0], s_p0[r][1], x, y) : 0.0;
                    s13[r][k] = e;
                    tame_in &= e <= kTameResidual;
                }
            } else {
                for (int r = 0; r < kCubeIB; ++r) s13[r][k] = 0.0;
            }
        }
        double a23[kCubeRPW][kColsPerLane];
        double f23[9];
        load_f(F23, f23);
#pragma unroll
        for (int q = 0; q < kColsPerLane; ++q) {
            LineRec cl{0.0, 0.0, 0.0, 0.0};
            double x = 0.0, y = 0.0;
            if (q < kvalid) {
                x = args.pts[2 * (c2 + kc + kb + q)];
                y = args.pts[2 * (c2 + kc + kb + q) + 1];
                cl.deg = col_line(f23, x, y, cl.l0, cl.l1, cl.l2) ? 1.0 : 0.0;
            }
#pragma unroll
            for (int r = 0; r < kCubeRPW; ++r) {
                const int jj = wave * kCubeRPW + r;
                a23[r][q] = (r < nrows && q < kvalid)
                                ? pair_e(cl, s_r23[jj], s_p1[jj][0], s_p1[jj][1], x, y)
                                : 0.0;
                tame_in &= a23[r][q] <= kTameResidual;
            }
        }
        const bool full = ((P & 3) == 0) && ((coff & 3) == 0) && args.cube;
        // every sum of this chunk finite: the loop without the per-row vote
        const bool chunk_fast = __syncthreads_and(tame_in) != 0 && full && !MVM_CUBE_THIRD_CHECK;
        if (nrows <= 0) continue;   // uniform; the barriers above are still reached

        const bool act = kvalid > 0;
        auto chunk_loop = [&](auto fast_tag) {
            constexpr bool FAST = decltype(fast_tag)::value;
            for (int ii = 0; ii < ni; ++ii) {
                const int i = i0 + ii;
                double a13[kColsPerLane];
                {
                    const f64x2 lo = *reinterpret_cast<const f64x2 *>(&s13[ii][kb]);
                    const f64x2 hi = *reinterpret_cast<const f64x2 *>(&s13[ii][kb + 2]);
                    a13[0] = lo.x; a13[1] = lo.y; a13[2] = hi.x; a13[3] = hi.y;
                }
                uint32_t key[kCubeRPW];
                int32_t idx[kCubeRPW];
#pragma unroll
                for (int r = 0; r < kCubeRPW; ++r) {
                    key[r] = kKeyInvalid;
                    idx[r] = 0x7FFFFFFF;
                    if (r >= nrows) continue;   // uniform
                    const double v12 = s12[ii][wave * kCubeRPW + r];
                    double sum[kColsPerLane], q0[kColsPerLane];
                    bool ok = true;
#pragma unroll
                    for (int q = 0; q < kColsPerLane; ++q) {
                        sum[q] = (v12 + a13[q]) + a23[r][q];          // (e12 + e13) + e23, :81
                        q0[q] = third_q(sum[q]);
                        if (!FAST) ok &= third_ok(q0[q]);
                    }
                    float v[kColsPerLane];
                    const int64_t row = (int64_t)i * M + j0 + r;
                    if (FAST || (full && __all(ok || !act))) {
#pragma unroll
                        for (int q = 0; q < kColsPerLane; ++q) v[q] = (float)q0[q];
                        if (act) {
                            store4_nt_row(reinterpret_cast<uint64_t>(args.cube + coff + row * P + kc),
                                          (uint32_t)kb * 4u, v);
                        }
                        Best b{v[0], kb};
#pragma unroll
                        for (int q = 1; q < kColsPerLane; ++q) best_update_fast(b, v[q], kb + q);
                        key[r] = act ? __float_as_uint(b.v) + 1u : kKeyInvalid;
                        idx[r] = act ? b.j : 0x7FFFFFFF;
                    } else {
                        Best b{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
                        // the IEEE division only when some lane needs it (uniform branch)
                        double qq[kColsPerLane];
#pragma unroll
                        for (int q = 0; q < kColsPerLane; ++q) qq[q] = q0[q];
                        if (!__all(ok || !act)) {
#pragma unroll
                            for (int q = 0; q < kColsPerLane; ++q)
                                qq[q] = third_ok(q0[q]) ? q0[q] : sum[q] / 3.0;
                        }
#pragma unroll
                        for (int q = 0; q < kColsPerLane; ++q) {
                            v[q] = (float)qq[q];
                            if (q < kvalid) {
                                if (args.cube)
                                    args.cube[coff + row * P + kc + kb + q] = v[q];
                                best_update_safe(b, v[q], kb + q);
                            }
                        }
                        key[r] = best_key(b);
                        idx[r] = b.j;
                    }
                }
                if constexpr (FAST && kCubeRPW == 8 && kWave % 8 == 0) {
                    // rows x = ii*8 + r land in lanes x % 64 of slot x / 64 directly
                    const int x0 = ii * kCubeRPW;   // uniform
                    uint32_t km;
                    int32_t im;
                    wave_argmin8_transposed(key, idx, lane, km, im, x0 % kWave);
                    const bool mine = lane - x0 % kWave >= 0 && lane - x0 % kWave < nrows;
#pragma unroll
                    for (int z = 0; z < kSlots; ++z) {
                        if (z != x0 / kWave) continue;   // uniform
                        const bool take = mine && km < run_k[z];
                        run_k[z] = take ? km : run_k[z];
                        run_i[z] = take ? kc + im : run_i[z];
                    }
                    continue;
                }
#pragma unroll
                for (int r = 0; r < kCubeRPW; ++r) {
                    if (r >= nrows) continue;
                    uint32_t km;
                    int32_t im;
                    wave_argmin(key[r], idx[r], km, im);
                    const int x = ii * kCubeRPW + r;   // uniform
                    const bool mine = lane == (x % kWave);
#pragma unroll
                    for (int z = 0; z < kSlots; ++z) {
                        if (z != x / kWave) continue;   // uniform
                        const bool take = mine && km < run_k[z];
                        run_k[z] = take ? km : run_k[z];
                        run_i[z] = take ? kc + im : run_i[z];
                    }
                }
            }
        };
        if (chunk_fast) chunk_loop(std::integral_constant<bool, true>{});
        else chunk_loop(std::integral_constant<bool, false>{});
    }
    if (nrows <= 0) return;
#pragma unroll
    for (int z = 0; z < kSlots; ++z) {
        const int x = z * kWave + lane;
        const int ii = x / kCubeRPW, r = x % kCubeRPW;
        if (x < kRows && ii < ni && r < nrows) {
            const int64_t row = roff + (int64_t)(i0 + ii) * M + j0 + r;
            if (args.argmin) args.argmin[row] = (run_k[z] == kKeyInvalid) ? -1 : run_i[z];
            if (args.minval) args.minval[row] = value_of_key(run_k[z]);
        }
    }
}

// ------------------------------------------------- small-scene cube ----
// Scenes whose views hold at most kSmallMaxN detections (the IPD regime: a
// few to a few dozen objects per image) are too small for the tiled kernel's
// 16 x 32 tiles and its fp64 workspace pass.  A workgroup owns (scene, block
// of `ib` rows i): it stages the three views' centroids, the six line sets,
// e23 [M][P] and its rows of e12 [ib][M], e13 [ib][P] in LDS (exactly the
// residuals of row_safe: sentinel, 0.5 * (d1 + d2)), then streams its
// contiguous slice of the cube in flattened order -- 16-byte nontemporal
// stores, indices advanced incrementally (no divisions in the loop), every
// wave instruction 1 KiB contiguous whatever P is -- and finally one thread
// per (i, j) row recomputes the row from LDS for the argmin over k.
constexpr int kSmallMaxN = 64;
// default switch-over to the fused kernel's four-rows-per-wave form: measured
// per 1000 scenes, small vs fused: 24^3 0.041 vs 0.064 ms, 32^3 0.095 vs
// 0.072, 40^3 0.138 vs 0.173, 48^3 0.220 vs 0.193, 56^3 0.417 vs 0.261
// (the fused tiles are 32 j wide: M = 40 leaves 3/8 of them empty)
constexpr int kSmallAutoMaxN = 44;

struct CubeSmallArgs {
    const double *pts;
    const int64_t *cam_offs;
    const double *F;            // [S*3, 9]: F12, F13, F23
    const int64_t *cube_offs;
    const int64_t *row_offs;
    float *cube;
    int32_t *argmin;
    float *minval;
    int32_t max_n;
    int32_t ib;                 // rows i per workgroup
    int32_t i_blocks;           // ceil(max_n / ib)
};

__host__ __device__ inline size_t small_lds_bytes(int nmax, int ib) {
    return ((size_t)24 * nmax + 2 * (size_t)ib * nmax + (size_t)nmax * nmax) * sizeof(double) +
           6 * (size_t)nmax;
}

__device__ __forceinline__ float cube_f32(double e12, double e13, double e23) {
    const double sum = (e12 + e13) + e23;
    double q = third_q(sum);
    if (!third_ok(q)) {   // non-finite sum: the IEEE division, skipped when no lane needs it
        double s2 = sum;
        __asm__ volatile("" : "+v"(s2));   // keeps the division inside the branch (no if-conversion)
        q = s2 / 3.0;
    }
    return (float)q;
}

__global__ __launch_bounds__(kThreads) void triplet_small_kernel(CubeSmallArgs args) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    const int nmax = args.max_n, IB = args.ib;
    double *sp = reinterpret_cast<double *>(s_dyn);         // [3][nmax][2] centroids
    double *sl = sp + 6 * nmax;                              // [3 pairs][2 sides][nmax][3] lines
    double *s12 = sl + 18 * nmax;                            // [ib][M]
    double *s13 = s12 + IB * nmax;                           // [ib][P]
    double *s23 = s13 + IB * nmax;                           // [M][P]
    unsigned char *sdeg = reinterpret_cast<unsigned char *>(s23 + nmax * nmax);  // [3][2][nmax]

    const int s = blockIdx.x / args.i_blocks, t = threadIdx.x;
    const int i0 = (blockIdx.x - s * args.i_blocks) * IB;
    const int64_t *co = args.cam_offs + 3 * (int64_t)s;
    const int64_t o0 = co[0];
    const int n[3] = {(int)(co[1] - co[0]), (int)(co[2] - co[1]), (int)(co[3] - co[2])};
    const int N = n[0], M = n[1], P = n[2];
    if (i0 >= N || M == 0) return;                           // no (i, j) rows in this block
    const int nb = min(IB, N - i0);
    const int64_t roff = args.row_offs[s];

    for (int v = 0; v < 3; ++v) {
        const int64_t ov = co[v] - o0;
        for (int q = t; q < 2 * n[v]; q += kThreads) sp[(v * nmax) * 2 + q] = args.pts[2 * (o0 + ov) + q];
    }
    __syncthreads();
    // pair p = (a, b): row lines of view a with F_p, column lines of view b
    const int pa[3] = {0, 0, 1}, pb[3] = {1, 2, 2};
    for (int w = t; w < 6 * nmax; w += kThreads) {
        const int p = w / (2 * nmax), side = (w / nmax) & 1, i = w % nmax;
        const int v = side ? pb[p] : pa[p];
        if (i >= n[v]) continue;
        double f[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) f[q] = args.F[(3 * (int64_t)s + p) * 9 + q];
        const double x = sp[(v * nmax + i) * 2], y = sp[(v * nmax + i) * 2 + 1];
        double l0, l1, l2;
        const bool deg = side ? col_line(f, x, y, l0, l1, l2) : row_line(f, x, y, l0, l1, l2);
        double *L = sl + ((p * 2 + side) * nmax + i) * 3;
        L[0] = l0;
        L[1] = l1;
        L[2] = l2;
        sdeg[(p * 2 + side) * nmax + i] = deg;
    }
    __syncthreads();
    // e_ab(i, j) of row_safe: pairs (0,1) and (0,2) for this block's rows, (1,2) whole
    const int rows_of[3] = {nb, nb, M}, first_of[3] = {i0, i0, 0};
    double *dst_of[3] = {s12, s13, s23};
    for (int p = 0; p < 3; ++p) {
        const int na = rows_of[p], nbb = n[pb[p]], r0 = first_of[p];
        double *E = dst_of[p];
        for (int w = t; w < na * nbb; w += kThreads) {
            const int il = w / nbb, j = w - il * nbb, i = r0 + il;
            const double *R = sl + ((p * 2 + 0) * nmax + i) * 3;
            const double *C = sl + ((p * 2 + 1) * nmax + j) * 3;
            const double rx = sp[(pa[p] * nmax + i) * 2], ry = sp[(pa[p] * nmax + i) * 2 + 1];
            const double cx = sp[(pb[p] * nmax + j) * 2], cy = sp[(pb[p] * nmax + j) * 2 + 1];
            const double d1 = sdeg[(p * 2 + 1) * nmax + j] ? kSentinel : line_dist(C[0], C[1], C[2], rx, ry);
            const double d2 = sdeg[(p * 2 + 0) * nmax + i] ? kSentinel : line_dist(R[0], R[1], R[2], cx, cy);
            E[w] = 0.5 * (d1 + d2);                                                   // :28
        }
    }
    __syncthreads();

    if (args.cube && P > 0) {
        const int MP = M * P, total = nb * MP;
        const int64_t gbase = args.cube_offs[s] + (int64_t)i0 * MP;
        float *cb = args.cube + gbase;
        const int head = min(total, (int)((4 - (gbase & 3)) & 3));   // to a 16-byte boundary
        const int body = (total - head) / 4;                          // float4 groups
        if (t < head) {
            const int il = t / MP, r = t - il * MP, j = r / P, k = r - j * P;
            __builtin_nontemporal_store(cube_f32(s12[il * M + j], s13[il * P + k], s23[j * P + k]), cb + t);
        }
        const int tail0 = head + 4 * body;
        if (t < total - tail0) {
            const int f = tail0 + t;
            const int il = f / MP, r = f - il * MP, j = r / P, k = r - j * P;
            __builtin_nontemporal_store(cube_f32(s12[il * M + j], s13[il * P + k], s23[j * P + k]), cb + f);
        }
        if (t < body) {
            // element f = head + 4g for group g = t + 256 * iter; advance by 1024 elements
            int f = head + 4 * t;
            int il = f / MP, r = f - il * MP, j = r / P, k = r - j * P;
            constexpr int kStep = 4 * kThreads;
            const int dk = kStep % P, q = kStep / P, dj = q % M, dil = q / M;
            for (int g = t; g < body; g += kThreads) {
                float v4[4];
                int a = il, b = j, c = k;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v4[e] = cube_f32(s12[a * M + b], s13[a * P + c], s23[b * P + c]);
                    if (++c == P) {
                        c = 0;
                        if (++b == M) {
                            b = 0;
                            ++a;
                        }
                    }
                }
                const f32x4 vv = {v4[0], v4[1], v4[2], v4[3]};
                __builtin_nontemporal_store(vv, reinterpret_cast<f32x4 *>(cb + head) + g);
                k += dk;
                const int ck = k >= P;
                k -= ck ? P : 0;
                j += dj + ck;
                const int cj = j >= M;
                j -= cj ? M : 0;
                il += dil + cj;
            }
        }
    }
    for (int w = t; w < nb * M; w += kThreads) {
        const int il = w / M, j = w - il * M;
        uint32_t bk = kKeyInvalid;
        int32_t bi = -1;
        const double a = s12[w];
        for (int k = 0; k < P; ++k) {
            const uint32_t key = key_of(cube_f32(a, s13[il * P + k], s23[j * P + k]));
            if (key < bk) {
                bk = key;
                bi = k;
            }
        }
        const int64_t row = roff + (int64_t)i0 * M + w;
        if (args.argmin) args.argmin[row] = bi;
        if (args.minval) args.minval[row] = value_of_key(bk);
    }
}

// ------------------------------------------------------- write probe ----
// Speed-of-light reference for the roofline: every workgroup writes one
// contiguous 16 KiB block with 16-byte nontemporal stores (4 per lane, each
// wave instruction 1 KiB contiguous) -- the store form of the residual kernels.
template <int PER_LANE, bool NT, bool XCD = false, bool SCRAMBLE = false>
__global__ __launch_bounds__(kThreads) void write_probe_kernel(f32x4 *dst, size_t n16, float val) {
    const f32x4 v = {val, val, val, val};
    uint32_t blk = blockIdx.x;
    if (XCD) {                  // each XCD writes a contiguous eighth
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        uint32_t k = blk / 8;
        const uint32_t cnt = q + (x < r ? 1u : 0u);
        if (SCRAMBLE) k = (uint32_t)(((uint64_t)k * 2654435761ull) % cnt);   // odd multiplier:
        blk = x * q + min(x, r) + k;                                         // a permutation when gcd = 1
    }
    const size_t base = (size_t)blk * (PER_LANE * kThreads) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PER_LANE; ++k) {
        const size_t i = base + (size_t)k * kThreads;
        if (i < n16) {
            if (NT) __builtin_nontemporal_store(v, dst + i);
            else dst[i] = v;
        }
    }
}

// cache-policy variants of the 16 KiB/WG stream (inline asm: the builtins
// expose only nt); POL 1 = sc1, 2 = sc0 sc1, 3 = nt sc1
template <int POL>
__global__ __launch_bounds__(kThreads) void write_probe_pol_kernel(f32x4 *dst, size_t n16, float val) {
    const f32x4 v = {val, val, val, val};
    const size_t base = (size_t)blockIdx.x * (4 * kThreads) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t i = base + (size_t)k * kThreads;
        if (i < n16) {
            const uint64_t ptr = reinterpret_cast<uint64_t>(dst + i);
            if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ptr), "v"(v) : "memory");
            if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(ptr), "v"(v) : "memory");
            if (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(ptr), "v"(v) : "memory");
        }
    }
}

// the pairwise kernel's store ORDER on a 256 KiB block per workgroup: 64 rows
// of 4 KiB, wave w owns rows 16w..16w+15 and walks chunk-outer / row-inner
// (consecutive stores of a wave are 4 KiB apart); ROWMAJOR = 1 walks each
// row's 4 chunks first (consecutive stores contiguous)
template <bool ROWMAJOR, bool XCD = false>
__global__ __launch_bounds__(kThreads) void write_probe_rows_kernel(f32x4 *dst, size_t n16, float val) {
    const f32x4 v = {val, val, val, val};
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    uint32_t blk = blockIdx.x;
    if (XCD) {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const size_t base = (size_t)blk * (64 * 256);         // 16-byte units: 64 rows x 256
    for (int a = 0; a < 16; ++a) {
        for (int b = 0; b < 4; ++b) {
            const int row = wave * 16 + (ROWMAJOR ? a : (a % 4) * 4 + b) ;
            const int chunk = ROWMAJOR ? b : a / 4;
            const size_t i = base + (size_t)row * 256 + chunk * 64 + lane;
            if (i < n16) __builtin_nontemporal_store(v, dst + i);
        }
    }
}

// store-shape model of a residual kernel: workgroups own `rpw * rg` (OWN 1)
// or `4 * rpw * rg` (OWN 0) rows of 4 KiB, XCD-sequential; OWN 0: wave w owns
// rpw rows of each group and walks chunk-outer / row-inner (the pairwise
// kernel, rpw rows open per wave); OWN 1: wave w owns 1-KiB chunk w of every
// row of the group (the workgroup's 4 waves share rpw open rows)
// `pace` s_sleep(1) (~64 clocks) after each store stands in for the residual
// arithmetic between a real kernel's stores
template <int OWN>
__global__ __launch_bounds__(kThreads) void write_probe_shape_kernel(f32x4 *dst, size_t n16,
                                                                     int rpw, int rg, int pace,
                                                                     float val) {
    const f32x4 v = {val, val, val, val};
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    uint32_t blk = blockIdx.x;
    {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const int rows_wg = (OWN == 0 ? 4 : 1) * rpw * rg;
    const size_t base = (size_t)blk * rows_wg * 256;       // 16-byte units, 256 per row
    for (int g = 0; g < rg; ++g) {
        if (OWN == 0) {
            const int r0 = g * 4 * rpw + wave * rpw;
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < rpw; ++r) {
                    const size_t i = base + (size_t)(r0 + r) * 256 + c * 64 + lane;
                    if (i < n16) __builtin_nontemporal_store(v, dst + i);
                    for (int z = 0; z < pace; ++z) __builtin_amdgcn_s_sleep(1);
                }
        } else {
            const int r0 = g * rpw;
            for (int r = 0; r < rpw; ++r) {
                const size_t i = base + (size_t)(r0 + r) * 256 + wave * 64 + lane;
                if (i < n16) __builtin_nontemporal_store(v, dst + i);
                for (int z = 0; z < pace; ++z) __builtin_amdgcn_s_sleep(1);
            }
        }
    }
}

// model of a "16-row unit" decomposition: a persistent grid, workgroup k of
// XCD x walks units k, k+W, ... of that XCD's eighth; per unit it reads a
// 44 KiB line block (from a 4 MiB L2-resident region) and writes 64 KiB
// (16 rows of 4 KiB, 4 waves x 4 rows)
__global__ __launch_bounds__(kThreads) void write_probe_units_kernel(f32x4 *dst, size_t n16,
                                                                     const f32x4 *lines) {
    const uint32_t W = gridDim.x / 8, x = blockIdx.x % 8, k = blockIdx.x / 8;
    const size_t n_units = n16 / 4096;                        // 64 KiB = 4096 x 16 B
    const size_t u0 = n_units * x / 8, u1 = n_units * (x + 1) / 8;
    const int t = threadIdx.x;
    for (size_t u = u0 + k; u < u1; u += W) {
        const f32x4 *lb = lines + (u % 90) * 2816;            // 44 KiB = 2816 x 16 B
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 11; ++q) acc += lb[t + 256 * q];
        f32x4 *ob = dst + u * 4096;
#pragma unroll
        for (int q = 0; q < 16; ++q) __builtin_nontemporal_store(acc, ob + t + 256 * q);
    }
}

// grid-stride variant: a fixed grid of `waves per CU` x 256 CUs workgroups
template <bool NT>
__global__ __launch_bounds__(kThreads) void write_probe_stride_kernel(f32x4 *dst, size_t n16,
                                                                      float val) {
    const f32x4 v = {val, val, val, val};
    const size_t step = (size_t)gridDim.x * kThreads * 4;
    for (size_t b = (size_t)blockIdx.x * kThreads * 4 + threadIdx.x; b < n16; b += step) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t i = b + (size_t)k * kThreads;
            if (i < n16) {
                if (NT) __builtin_nontemporal_store(v, dst + i);
                else dst[i] = v;
            }
        }
    }
}

// ------------------------------------------------------------ host side ----
constexpr int kRowsPerWave = 16;       // pairwise default: 64 rows per workgroup
constexpr int kTripletRowsPerWave = 8; // generic triplet: 32 (i, j) rows per workgroup

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...);

int check_launch(const char *what) { return mvm_check_launch(what); }

int fill_pairs(PairArgs &a, const int32_t *pair_a, const int32_t *pair_b, int n_pairs,
               int n_cams) {
    if (n_cams < 2 || n_cams > MVM_MAX_CAMS)
        return fail(MVM_ERR_UNSUPPORTED, "n_cams=%d outside [2, %d]", n_cams, MVM_MAX_CAMS);
    if (n_pairs < 1 || n_pairs > MVM_MAX_PAIRS)
        return fail(MVM_ERR_UNSUPPORTED, "n_pairs=%d outside [1, %d]", n_pairs, MVM_MAX_PAIRS);
    if (!pair_a || !pair_b) return fail(MVM_ERR_INVALID_ARGUMENT, "null pair list");
    for (int p = 0; p < n_pairs; ++p) {
        if (pair_a[p] < 0 || pair_a[p] >= n_cams || pair_b[p] < 0 || pair_b[p] >= n_cams ||
            pair_a[p] == pair_b[p])
            return fail(MVM_ERR_INVALID_ARGUMENT, "pair %d = (%d, %d) invalid for %d cameras", p,
                        pair_a[p], pair_b[p], n_cams);
        a.pair_a[p] = pair_a[p];
        a.pair_b[p] = pair_b[p];
    }
    a.n_cams = n_cams;
    a.n_pairs = n_pairs;
    return MVM_OK;
}

// Tuning knobs (read per launch; defaults tuned on MI355X):
//   MVM_PAIRWISE_LANE_RESULTS  1: argmin rows stored by RPW lanes at once
//   MVM_TRIPLET_VARIANT  3: tiled/fused cube kernels (default), 1: generic
//   MVM_PAIRWISE_RPW  rows per wave per group (4 / 8 / 16)
//   MVM_PAIRWISE_RG   row groups per wave (1..16)
//   MVM_PAIRWISE_NT   row store policy: 1 nt (default), 0 default, 2 sc1, 3 sc0 sc1
//   MVM_TRIPLET_SMALL one-workgroup-per-scene cube: unset = views of <= 44, 1 = < 64, 0 = off
//   MVM_TRIPLET_FUSED 1: tiled cube with in-prologue pair residuals (<= 256)
//   MVM_LSAP_WAVE_MAX_COLS  long-side limit of the one-wave LSAP (mvm_lsap.hip)
int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}

constexpr int kMaxColTile = 1024;   // column lines resident in LDS per workgroup

template <int RPW>
size_t pairwise_lds_bytes(int col_tile, int rows_per_wg, bool transposed_reduction) {
    return (size_t)col_tile * (5 * sizeof(double) + sizeof(uint32_t)) +
           (size_t)kWaves * kWave * 6 * sizeof(double) + (size_t)rows_per_wg * 2 * sizeof(double) +
           (transposed_reduction ? (size_t)kWaves * RPW * kWave * sizeof(uint32_t) : 0);
}

// Launch with `lds` bytes of dynamic LDS (above 64 KiB the kernel must opt in).
template <typename Kernel>
void launch_lds(Kernel kern, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
                const PairArgs &a) {
    if (lds > 65536)
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<grid, block, lds, stream>>>(a);
}

template <int RPW>
void launch_pairwise_rpw(PairArgs &a, int64_t sp_count, int max_rows, int max_cols,
                         int row_groups, bool argmin, bool f64, hipStream_t stream) {
    a.col_tile = min(kMaxColTile, max(kChunk, (max_cols + kChunk - 1) / kChunk * kChunk));
    a.lane_results = env_int("MVM_PAIRWISE_LANE_RESULTS", 1);
    a.xcd_remap = env_int("MVM_PAIRWISE_XCD", 1);   // MI355X C3: 4.63 vs 4.72 ms per launch
    a.interleave = env_int("MVM_PAIRWISE_INTERLEAVE", 0);
    a.stagger = env_int("MVM_PAIRWISE_STAGGER", 0);
    // 2: transposed reduction (default); 1: per-row DPP reductions; 0: eager argmin
    a.lazy = env_int("MVM_PAIRWISE_LAZY", 2);
    a.rows_per_wg = kWaves * RPW * row_groups;
    a.row_blocks = (max_rows + a.rows_per_wg - 1) / a.rows_per_wg;
    const dim3 grid((unsigned)(sp_count * a.row_blocks)), block(kThreads);
    // MVM_PAIRWISE_LDS_PAD (experiments): unused LDS per workgroup, to cap the
    // resident workgroups per CU
    const size_t lds = pairwise_lds_bytes<RPW>(a.col_tile, a.rows_per_wg,
                                               argmin && !f64 && a.lazy >= 2) +
                       (size_t)max(0, env_int("MVM_PAIRWISE_LDS_PAD", 0));
    if (f64) {
        launch_lds(pairwise_kernel<RPW, false, double>, grid, block, lds, stream, a);
    } else {
        // nontemporal stores for whole-line rows; rows that end mid-line share
        // that line with the next row, and L2 must merge it (default policy)
        switch (env_int("MVM_PAIRWISE_NT", (max_cols % 32 == 0) ? 1 : 0)) {
        case 0:
            if (argmin) launch_lds(pairwise_kernel<RPW, true, float, 0>, grid, block, lds, stream, a);
            else launch_lds(pairwise_kernel<RPW, false, float, 0>, grid, block, lds, stream, a);
            break;
        case 2:
            if (argmin) launch_lds(pairwise_kernel<RPW, true, float, 2>, grid, block, lds, stream, a);
            else launch_lds(pairwise_kernel<RPW, false, float, 2>, grid, block, lds, stream, a);
            break;
        case 3:
            if (argmin) launch_lds(pairwise_kernel<RPW, true, float, 3>, grid, block, lds, stream, a);
            else launch_lds(pairwise_kernel<RPW, false, float, 3>, grid, block, lds, stream, a);
            break;
        default:
            if (argmin) launch_lds(pairwise_kernel<RPW, true, float, 1>, grid, block, lds, stream, a);
            else launch_lds(pairwise_kernel<RPW, false, float, 1>, grid, block, lds, stream, a);
            break;
        }
    }
}


int launch_pairwise_common(PairArgs &a, int32_t n_scenes, int32_t max_rows, int32_t max_cols,
                           bool argmin, bool f64, hipStream_t stream) {
    if (n_scenes < 0 || max_rows < 0 || max_cols < 0)
        return fail(MVM_ERR_INVALID_ARGUMENT, "negative n_scenes/max_rows/max_cols");
    if (n_scenes == 0 || max_rows == 0) return MVM_OK;
    int rpw = env_int("MVM_PAIRWISE_RPW", kRowsPerWave);
    if (rpw != 4 && rpw != 8 && rpw != 16) rpw = kRowsPerWave;
    // enough row groups to amortise the column lines over >= ~256 rows, but
    // never more than the rows a view has
    const int groups_needed = (max_rows + kWaves * rpw - 1) / (kWaves * rpw);
    int rg = env_int("MVM_PAIRWISE_RG", 0);
    if (rg <= 0) rg = max(1, min(groups_needed, 256 / (kWaves * rpw)));
    rg = max(1, min(rg, 16));
    const int64_t sp_count = (int64_t)n_scenes * a.n_pairs;
    const int64_t rows_per_wg = (int64_t)kWaves * rpw * rg;
    const int64_t blocks = sp_count * ((max_rows + rows_per_wg - 1) / rows_per_wg);
    if (blocks > 0x7FFFFFFFLL)
        return fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                    (long long)blocks);
    switch (rpw) {
    case 4: launch_pairwise_rpw<4>(a, sp_count, max_rows, max_cols, rg, argmin, f64, stream); break;
    case 8: launch_pairwise_rpw<8>(a, sp_count, max_rows, max_cols, rg, argmin, f64, stream); break;
    default: launch_pairwise_rpw<16>(a, sp_count, max_rows, max_cols, rg, argmin, f64, stream); break;
    }
    return check_launch("pairwise_kernel");
}

}  // namespace

// ============================================================ internals ====
namespace {
thread_local char g_err[512];
}

void mvm_set_error(const char *msg) {
    snprintf(g_err, sizeof g_err, "%s", msg);
}

void mvm_clear_error() { mvm_clear_error(); }

int mvm_fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int mvm_env_int(const char *name, int dflt) { return env_int(name, dflt); }

int mvm_check_launch(const char *what) {
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return mvm_fail(MVM_ERR_HIP, "%s: %s", what, hipGetErrorString(err));
    return MVM_OK;
}

namespace {
int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char buf[512];
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    mvm_set_error(buf);
    return code;
}
}  // namespace

// ================================================================ C ABI ====
extern "C" {

const char *mvm_version(void) { return "mvmatch 0.1.0 gfx950"; }

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

int mvm_pairwise_residual_argmin(const double *pts_dev, const int64_t *cam_offs_dev,
                                 const double *F_dev, const int32_t *pair_a,
                                 const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                 int32_t n_pairs, int32_t max_n, const int64_t *dist_offs_dev,
                                 const int64_t *row_offs_dev, float *dist_dev,
                                 int32_t *argmin_dev, float *minval_dev, mvm_stream_t stream) {
    mvm_clear_error();
    PairArgs a{};
    int st = fill_pairs(a, pair_a, pair_b, n_pairs, n_cams);
    if (st) return st;
    if (n_scenes > 0 && max_n > 0 && (!pts_dev || !cam_offs_dev || !F_dev))
        return fail(MVM_ERR_INVALID_ARGUMENT, "null input pointer");
    if (dist_dev && !dist_offs_dev) return fail(MVM_ERR_INVALID_ARGUMENT, "dist without dist_offs");
    if ((argmin_dev || minval_dev) && !row_offs_dev)
        return fail(MVM_ERR_INVALID_ARGUMENT, "argmin/minval without row_offs");
    a.pts = pts_dev;
    a.cam_offs = cam_offs_dev;
    a.F = F_dev;
    a.dist_offs = dist_offs_dev;
    a.row_offs = row_offs_dev;
    a.dist = dist_dev;
    a.argmin = argmin_dev;
    a.minval = minval_dev;
    a.ld = 0;
    const bool want_argmin = argmin_dev || minval_dev;
    return launch_pairwise_common(a, n_scenes, max_n, max_n, want_argmin, false,
                                  reinterpret_cast<hipStream_t>(stream));
}

int mvm_pairwise_residual_f64(const double *pts_dev, const int64_t *cam_offs_dev,
                              const double *F_dev, const int32_t *pair_a, const int32_t *pair_b,
                              int32_t n_scenes, int32_t n_cams, int32_t n_pairs,
                              int32_t max_n, int64_t mat_stride, int64_t ld, double *e_dev,
                              mvm_stream_t stream) {
    mvm_clear_error();
    PairArgs a{};
    int st = fill_pairs(a, pair_a, pair_b, n_pairs, n_cams);
    if (st) return st;
    if (n_scenes > 0 && max_n > 0 && (!pts_dev || !cam_offs_dev || !F_dev || !e_dev))
        return fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (ld <= 0 || mat_stride < 0)
        return fail(MVM_ERR_INVALID_ARGUMENT, "ld must be > 0 and mat_stride >= 0");
    a.pts = pts_dev;
    a.cam_offs = cam_offs_dev;
    a.F = F_dev;
    a.dist = e_dev;
    a.mat_stride = mat_stride;
    a.ld = ld;
    return launch_pairwise_common(a, n_scenes, max_n, max_n, false, true,
                                  reinterpret_cast<hipStream_t>(stream));
}

int mvm_hbm_write_probe(void *dst_dev, size_t bytes, mvm_stream_t stream) {
    mvm_clear_error();
    if (!dst_dev || (((uintptr_t)dst_dev) & 15) || (bytes & 15))
        return fail(MVM_ERR_INVALID_ARGUMENT, "write probe needs a 16-byte aligned buffer/size");
    const size_t n16 = bytes / 16;
    // MVM_PROBE_MODE (experiments): 0 nt 16 KiB/WG (the residual kernels' form),
    // 1 plain 16 KiB/WG, 2 nt 64 KiB/WG, 3 plain 64 KiB/WG, 4 nt grid-stride, 5 plain grid-stride,
    // 6 sc1, 7 sc0 sc1, 8 nt sc1 (16 KiB/WG), 9 / 10 the pairwise kernel's row order
    // (chunk-outer / row-major) on 256 KiB per WG
    // default 17: the fastest store stream measured on MI355X (XCD-sequential
    // 8 KiB blocks, 6.7 TB/s) -- the achievable ceiling bench.py reports
    const int mode = env_int("MVM_PROBE_MODE", 17);
    const int per = (mode == 2 || mode == 3) ? 16 : 4;
    const size_t blocks = (n16 + per * kThreads - 1) / (per * kThreads);
    if (blocks == 0) return MVM_OK;
    if (blocks > 0x7FFFFFFFull) return fail(MVM_ERR_UNSUPPORTED, "write probe buffer too large");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    f32x4 *d = reinterpret_cast<f32x4 *>(dst_dev);
    const unsigned stride_grid = (unsigned)env_int("MVM_PROBE_GRID", 256 * 8);
    // MVM_PROBE_LDS: unused dynamic LDS per workgroup (modes 12, 17) to cap the
    // resident workgroups per CU like a real kernel's footprint does
    const size_t plds = (size_t)env_int("MVM_PROBE_LDS", 0);
    switch (mode) {
        case 1: write_probe_kernel<4, false><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 2: write_probe_kernel<16, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 3: write_probe_kernel<16, false><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 4: write_probe_stride_kernel<true><<<stride_grid, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 5: write_probe_stride_kernel<false><<<stride_grid, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 6: write_probe_pol_kernel<1><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 7: write_probe_pol_kernel<2><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 8: write_probe_pol_kernel<3><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 11: write_probe_kernel<4, true, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 12: write_probe_rows_kernel<false, true><<<(unsigned)((n16 + 16383) / 16384), kThreads, plds, s>>>(d, n16, 1.0f); break;
        case 13: write_probe_kernel<4, false, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 14: write_probe_kernel<4, true, true, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 15: write_probe_kernel<8, true, true><<<(unsigned)((n16 + 8 * kThreads - 1) / (8 * kThreads)), kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 16: write_probe_kernel<16, true, true><<<(unsigned)((n16 + 16 * kThreads - 1) / (16 * kThreads)), kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 17: write_probe_kernel<2, true, true><<<(unsigned)((n16 + 2 * kThreads - 1) / (2 * kThreads)), kThreads, plds, s>>>(d, n16, 1.0f); break;
        case 18: {
            // lines region: the last 4 MiB of the buffer (units stop before it)
            const size_t reserve = (4u << 20) / 16;
            if (n16 <= reserve + 4096) return fail(MVM_ERR_INVALID_ARGUMENT, "buffer too small");
            const unsigned grid = (unsigned)env_int("MVM_PROBE_GRID", 8 * 96);
            write_probe_units_kernel<<<grid, kThreads, 0, s>>>(d, n16 - reserve, d + (n16 - reserve));
            break;
        }
        case 20:
        case 21: {
            const int rpw = env_int("MVM_PROBE_RPW", 16), rg = env_int("MVM_PROBE_RG", 4);
            const int pace = env_int("MVM_PROBE_PACE", 0);
            const size_t rows_wg = (size_t)(mode == 20 ? 4 : 1) * rpw * rg;
            const unsigned g = (unsigned)((n16 + rows_wg * 256 - 1) / (rows_wg * 256));
            if (mode == 20) write_probe_shape_kernel<0><<<g, kThreads, plds, s>>>(d, n16, rpw, rg, pace, 1.0f);
            else write_probe_shape_kernel<1><<<g, kThreads, plds, s>>>(d, n16, rpw, rg, pace, 1.0f);
            break;
        }
        case 9: write_probe_rows_kernel<false><<<(unsigned)((n16 + 16383) / 16384), kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 10: write_probe_rows_kernel<true><<<(unsigned)((n16 + 16383) / 16384), kThreads, 0, s>>>(d, n16, 1.0f); break;
        default: write_probe_kernel<4, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
    }
    return check_launch("write_probe_kernel");
}

size_t mvm_triplet_workspace_bytes(int32_t n_scenes, int32_t max_n) {
    if (n_scenes <= 0 || max_n <= 0) return 0;
    const int64_t ld = ((int64_t)max_n + 3) / 4 * 4;
    return (size_t)n_scenes * 3 * (size_t)max_n * (size_t)ld * sizeof(double);
}

int mvm_triplet_cost_argmin(const double *pts_dev, const int64_t *cam_offs_dev,
                            const double *F_dev, int32_t n_scenes, int32_t max_n,
                            const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                            float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                            void *workspace_dev, size_t workspace_bytes, mvm_stream_t stream) {
    mvm_clear_error();
    if (n_scenes < 0 || max_n < 0) return fail(MVM_ERR_INVALID_ARGUMENT, "negative sizes");
    if (n_scenes == 0 || max_n == 0) return MVM_OK;
    if (!pts_dev || !cam_offs_dev || !F_dev || !row_offs_dev)
        return fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (cube_dev && !cube_offs_dev) return fail(MVM_ERR_INVALID_ARGUMENT, "cube without cube_offs");
    const size_t need = mvm_triplet_workspace_bytes(n_scenes, max_n);
    if (!workspace_dev || workspace_bytes < need)
        return fail(MVM_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
    if (((uintptr_t)workspace_dev & 15) != 0)
        return fail(MVM_ERR_INVALID_ARGUMENT, "workspace not 16-byte aligned");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int variant = env_int("MVM_TRIPLET_VARIANT", 3);   // 3 tiled / fused, 1 generic
    // the small kernel up to 63 detections; at 64 the fused tiles are ~10% faster
    // (0.75 vs 0.84 ms per 1000 scenes; below 64 the small kernel wins by 1.1-2.4x)
    // MVM_TRIPLET_SMALL: unset = views of <= kSmallAutoMaxN, 1 = up to the
    // kernel's limit (< kSmallMaxN), 0 = never
    const int small_env = env_int("MVM_TRIPLET_SMALL", -1);
    const bool small = small_env < 0 ? max_n <= kSmallAutoMaxN : (small_env != 0 && max_n < kSmallMaxN);
    if (small && variant == 3) {
        // one workgroup per scene, everything in LDS, no workspace pass
        CubeSmallArgs c{};
        c.pts = pts_dev;
        c.cam_offs = cam_offs_dev;
        c.F = F_dev;
        c.cube_offs = cube_offs_dev;
        c.row_offs = row_offs_dev;
        c.cube = cube_dev;
        c.argmin = argmin_dev;
        c.minval = minval_dev;
        c.max_n = max_n;
        // MVM_TRIPLET_SMALL_IB: rows i per workgroup.  Default: the whole scene up
        // to 32 detections, then 16-row blocks (measured on MI355X: 1.2-1.6 TB/s
        // from 16 to 64 detections, 2-10x the tiled path; tools/gpu_cube_small.sh)
        c.ib = env_int("MVM_TRIPLET_SMALL_IB", max_n <= 32 ? max_n : 16);
        c.ib = c.ib < 1 ? 1 : (c.ib > max_n ? max_n : c.ib);
        c.i_blocks = (max_n + c.ib - 1) / c.ib;
        const size_t lds = small_lds_bytes(max_n, c.ib);
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute(reinterpret_cast<const void *>(&triplet_small_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
        const int64_t blocks = (int64_t)n_scenes * c.i_blocks;
        if (blocks > 0x7FFFFFFFLL)
            return fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                        (long long)blocks);
        triplet_small_kernel<<<dim3((unsigned)blocks), dim3(kThreads), lds, s>>>(c);
        return check_launch("triplet_small_kernel");
    }
    if (max_n <= kChunk && variant == 3 && env_int("MVM_TRIPLET_FUSED", 1)) {
        // tiles of 16 i x 32 j whose pair residuals are computed in the prologue
        CubeFusedArgs c{};
        c.pts = pts_dev;
        c.cam_offs = cam_offs_dev;
        c.F = F_dev;
        c.cube_offs = cube_offs_dev;
        c.row_offs = row_offs_dev;
        c.cube = cube_dev;
        c.argmin = argmin_dev;
        c.minval = minval_dev;
        c.xcd_remap = env_int("MVM_TRIPLET_XCD", 0);
        // MVM_TRIPLET_TILE: 3 = 16 i x 32 j (default), 4 = 32 i x 32 j, 2 = 8 i x 32 j, 0 = 16 i x 16 j
        const int tile = env_int("MVM_TRIPLET_TILE", 3);
        const int ib = tile == 4 ? 32 : (tile == 2 ? 8 : 16);
        const int rpw = tile == 0 ? 4 : 8;
        c.j_blocks = (max_n + kWaves * rpw - 1) / (kWaves * rpw);
        c.i_blocks = (max_n + ib - 1) / ib;
        const int64_t blocks = (int64_t)n_scenes * c.j_blocks * c.i_blocks;
        if (blocks > 0x7FFFFFFFLL)
            return fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                        (long long)blocks);
        const dim3 grid((unsigned)blocks), block(kThreads);
        // views of <= 128 / <= 64: two / four rows per wave instruction
        // (MVM_TRIPLET_HALF=0: off, 2: at most two)
        const int split_env = env_int("MVM_TRIPLET_HALF", 1);
        if (tile == 3 && split_env && max_n <= kChunk / 4 && split_env != 2) {
            triplet_fused_kernel<16, 8, 4><<<grid, block, 0, s>>>(c);
            return check_launch("triplet_fused_kernel");
        }
        if (tile == 3 && split_env && max_n <= kChunk / 2) {
            triplet_fused_kernel<16, 8, 2><<<grid, block, 0, s>>>(c);
            return check_launch("triplet_fused_kernel");
        }
        switch (tile) {
        case 4: triplet_fused_kernel<32, 8><<<grid, block, 0, s>>>(c); break;
        case 2: triplet_fused_kernel<8, 8><<<grid, block, 0, s>>>(c); break;
        case 0: triplet_fused_kernel<16, 4><<<grid, block, 0, s>>>(c); break;
        default: triplet_fused_kernel<16, 8><<<grid, block, 0, s>>>(c); break;
        }
        return check_launch("triplet_fused_kernel");
    }
    if (max_n > kChunk && variant == 3 && env_int("MVM_TRIPLET_CHUNKED", 1)) {
        // views of more than 256: fused tiles walking k in chunks of 256
        CubeFusedArgs c{};
        c.pts = pts_dev;
        c.cam_offs = cam_offs_dev;
        c.F = F_dev;
        c.cube_offs = cube_offs_dev;
        c.row_offs = row_offs_dev;
        c.cube = cube_dev;
        c.argmin = argmin_dev;
        c.minval = minval_dev;
        c.xcd_remap = env_int("MVM_TRIPLET_XCD", 0);
        c.j_blocks = (max_n + kWaves * 8 - 1) / (kWaves * 8);
        c.i_blocks = (max_n + 16 - 1) / 16;
        const int64_t blocks = (int64_t)n_scenes * c.j_blocks * c.i_blocks;
        if (blocks > 0x7FFFFFFFLL)
            return fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                        (long long)blocks);
        triplet_fused_chunked_kernel<16, 8><<<dim3((unsigned)blocks), dim3(kThreads), 0, s>>>(c);
        return check_launch("triplet_fused_chunked_kernel");
    }
    const int64_t ld = ((int64_t)max_n + 3) / 4 * 4;
    const int64_t mat_stride = (int64_t)max_n * ld;
    // pairs (0,1), (0,2), (1,2): F12, F13, F23 (process_pose.py:157-159)
    const int32_t pa[3] = {0, 0, 1}, pb[3] = {1, 2, 2};
    int st = mvm_pairwise_residual_f64(pts_dev, cam_offs_dev, F_dev, pa, pb, n_scenes, 3, 3,
                                       max_n, mat_stride, ld, (double *)workspace_dev, stream);
    if (st) return st;
    if (max_n <= kChunk && variant == 3) {
        // tile shape knob MVM_TRIPLET_TILE: 3 = 16i x 32j (default, fastest on
        // MI355X), 0 = 16i x 16j, 1 = 8i x 16j, 2 = 8i x 32j
        const int tile = env_int("MVM_TRIPLET_TILE", 3);
        const int ib = (tile == 1 || tile == 2) ? 8 : 16;
        const int rpw = (tile == 2 || tile == 3) ? 8 : 4;
        Cube3Args c{};
        c.cam_offs = cam_offs_dev;
        c.e = (const double *)workspace_dev;
        c.mat_stride = mat_stride;
        c.ld = ld;
        c.cube_offs = cube_offs_dev;
        c.row_offs = row_offs_dev;
        c.cube = cube_dev;
        c.argmin = argmin_dev;
        c.minval = minval_dev;
        c.j_blocks = (max_n + kWaves * rpw - 1) / (kWaves * rpw);
        c.i_blocks = (max_n + ib - 1) / ib;
        const int64_t blocks = (int64_t)n_scenes * c.j_blocks * c.i_blocks;
        if (blocks > 0x7FFFFFFFLL)
            return fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                        (long long)blocks);
        const dim3 grid((unsigned)blocks), block(kThreads);
        switch (tile) {
        case 1: triplet_tile_kernel<8, 4><<<grid, block, 0, s>>>(c); break;
        case 2: triplet_tile_kernel<8, 8><<<grid, block, 0, s>>>(c); break;
        case 0: triplet_tile_kernel<16, 4><<<grid, block, 0, s>>>(c); break;
        default: triplet_tile_kernel<16, 8><<<grid, block, 0, s>>>(c); break;
        }
        return check_launch("triplet_tile_kernel");
    }
    CubeArgs c{};
    c.cam_offs = cam_offs_dev;
    c.e = (const double *)workspace_dev;
    c.mat_stride = mat_stride;
    c.ld = ld;
    c.cube_offs = cube_offs_dev;
    c.row_offs = row_offs_dev;
    c.cube = cube_dev;
    c.argmin = argmin_dev;
    c.minval = minval_dev;
    c.i_count = max_n;
    const int rows_per_wg = kWaves * kTripletRowsPerWave;
    c.j_blocks = (max_n + rows_per_wg - 1) / rows_per_wg;
    const int64_t blocks = (int64_t)n_scenes * max_n * c.j_blocks;
    if (blocks > 0x7FFFFFFFLL)
        return fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                    (long long)blocks);
    triplet_kernel<kTripletRowsPerWave><<<dim3((unsigned)blocks), dim3(kThreads), 0, s>>>(c);
    return check_launch("triplet_kernel");
}

}  // extern "C"
