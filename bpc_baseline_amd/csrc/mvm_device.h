// mvm_device.h — device-side building blocks shared by the matcher's kernels
// (mvm_pairwise.hip, mvm_cube.hip): the reference's line / distance
// arithmetic, the np.argmin ordering keys and wave reductions, and the
// store forms.  Internal to the library (not part of the C ABI).
//
// Arithmetic is float64 and reproduces the reference bit for bit: FMAs are
// placed exactly where numpy/OpenBLAS placed them in the reference run
// (the C oracle in oracle/ is pinned to the reference on the
// golden vectors) and every translation unit is compiled with
// -ffp-contract=off (plus the pragma below) so no other contraction happens.
// sqrt and '/' are the IEEE correctly rounded gfx950 sequences.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#pragma clang fp contract(off)

namespace {

constexpr int kWave = 64;
constexpr int kThreads = 256;                  // 4 waves per workgroup
// A dispatch packet counts work-items in 32 bits per dimension: a 1-D grid of
// 256-thread workgroups holds at most this many (larger launches must split)
constexpr long long kMaxGridBlocks = 0xFFFFFFFFLL / kThreads;
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
// per-row 64-bit VALU address arithmetic).  NT 1: nontemporal (whole-line
// rows), 0: default policy (rows that end mid-line: L2 merges the shared line).
template <int NT = 1>
__device__ __forceinline__ void store4_nt_row(uint64_t row_base, uint32_t byte_off,
                                              const float v4[4]) {
    const f32x4 v = {v4[0], v4[1], v4[2], v4[3]};
    if constexpr (NT == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<g_f32x4 *>(row_base + byte_off));
    else
        *reinterpret_cast<g_f32x4 *>(row_base + byte_off) = v;
}
// The same 16-byte row store for rows that are only 4-byte aligned (cube rows
// whose P is not a multiple of 4): gfx950 takes a dword-aligned dwordx4, and
// the instruction is the same one the aligned form issues.
typedef f32x4 __attribute__((address_space(1), aligned(4))) g_f32x4a4;
template <int NT = 1>
__device__ __forceinline__ void store4_row_a4(uint64_t row_base, uint32_t byte_off, const float v4[4]) {
    const f32x4 v = {v4[0], v4[1], v4[2], v4[3]};
    if constexpr (NT == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<g_f32x4a4 *>(row_base + byte_off));
    else
        *reinterpret_cast<g_f32x4a4 *>(row_base + byte_off) = v;
}

// 3 consecutive outputs of one lane (rows of 3-k lanes): `global_store_dwordx3`,
// saddr form, 4-byte aligned
typedef float f32x3 __attribute__((ext_vector_type(3)));
typedef f32x3 __attribute__((address_space(1), aligned(4))) g_f32x3;
template <int NT = 1>
__device__ __forceinline__ void store3_row(uint64_t row_base, uint32_t byte_off, const float v3[3]) {
    const f32x3 v = {v3[0], v3[1], v3[2]};
    if constexpr (NT == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<g_f32x3 *>(row_base + byte_off));
    else
        *reinterpret_cast<g_f32x3 *>(row_base + byte_off) = v;
}
__device__ __forceinline__ void store4_nt(double *dst, const double e[4]) {
    const f64x2 lo = {e[0], e[1]}, hi = {e[2], e[3]};
    __builtin_nontemporal_store(lo, reinterpret_cast<f64x2 *>(dst));
    __builtin_nontemporal_store(hi, reinterpret_cast<f64x2 *>(dst + 2));
}

// Row stores of the argmin / min of rows r0..r0+RPW-1: lane r holds row r's
// result (one store instruction with RPW active lanes instead of RPW stores).
template <int RPW>
__device__ __forceinline__ void store_row_results(const uint32_t (&kmin)[RPW],
                                                  const int32_t (&imin)[RPW], int nrows, int lane,
                                                  int32_t *argmin, float *minval,
                                                  int64_t row0) {
    uint32_t k = kKeyInvalid;
    int32_t ix = 0;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        k = (lane == r) ? kmin[r] : k;
        ix = (lane == r) ? imin[r] : ix;
    }
    if (lane < nrows) {
        if (argmin) argmin[row0 + lane] = (k == kKeyInvalid) ? -1 : ix;
        if (minval) minval[row0 + lane] = value_of_key(k);
    }
}
// Minimum over aligned groups of L lanes, in every lane of the group: L = 16
// is one DPP row (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror,
// row_mirror), L = 8 its first three steps, L = 32 joins two rows with an
// xor-16 swizzle.
template <int L>
__device__ __forceinline__ uint32_t lane_group_min(uint32_t v) {
    static_assert(L == 8 || L == 16 || L == 32, "8-, 16- or 32-lane groups");
    v = dpp_min<0xB1>(v);
    v = dpp_min<0x4E>(v);
    v = dpp_min<0x141>(v);
    if constexpr (L == 8) return v;
    v = dpp_min<0x140>(v);
    if constexpr (L == 32) {
        const uint32_t o = (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (16 << 10));
        v = o < v ? o : v;
    }
    return v;
}

// The partner lane's value under DPP control CTRL (every lane has a partner).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_from(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t ab = a < b ? a : b;   // -> v_min3_u32
    return ab < c ? ab : c;
}

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

// ------------------------------------------------------- the cube value ----
constexpr double kThird = 1.0 / 3.0;
// residual bound under which a sum of three is finite (tile-wide fast path)
constexpr double kTameResidual = 0x1p1020;

// RN(s / 3) by one Markstein correction (the default): with y = RN(1/3) and
// q0 = RN(s * y) within one ulp of s/3, r = fma(-q0, 3, s) is exact and
// q1 = fma(r, y, q0) is the correctly rounded quotient -- for every finite s
// (checked against the IEEE division on 1.1e9 random, binade-edge,
// subnormal and near-midpoint inputs, tools/probes/third_markstein.c, and in
// tests/test_host_logic.py).  Three fp64 ops and a finiteness test instead
// of a product plus a float32-midpoint/range test (~8 ops, measured 12%
// slower at 256^3); only non-finite sums (inf: q1 = NaN) take the division.
// A sum of residuals is never -0, the one input whose sign the correction
// would not keep.
__device__ __forceinline__ double third_q(double s) {
    const double q0 = s * kThird;
    return __builtin_fma(__builtin_fma(-q0, 3.0, s), kThird, q0);
}

// true: third_q(s) == RN(s / 3); false: the caller divides
__device__ __forceinline__ bool third_ok(double q) { return __builtin_isfinite(q); }

// One cube entry: float32(((e12 + e13) + e23) / 3) (epipolar_matching.py:78-81,
// :96) for any residuals, NaN / inf included.  Every cube kernel computes
// exactly this (the fused loops inline it); the cube-free consumers of the
// assignment (mvm_lsap_sparse.hip, select_triangulate) recompute entries with
// this function from the fp64 pair residuals, so they read the same bits the
// cube would hold.
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

}  // namespace
