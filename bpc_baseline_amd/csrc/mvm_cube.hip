// mvm_cube.hip — the three-camera cost cube (compute_cost_matrix) and its C ABI.
//
// Reference: bpc/inference/epipolar_matching.py
//   compute_cost_matrix (:83-98)  cube[i][j][k] = float32(epipolar_error_full)
//   epipolar_error_full (:73-81)  ((e12 + e13) + e23) / 3 in fp64
//   (new)          per-(i, j) argmin over k of the stored float32
//
// HBM-write bound: 4 bytes per triple out, O(n) in.  Four kernels, picked by
// the batch's largest view: a one-workgroup-per-scene
// kernel for IPD-sized views, fused 16 i x 32 j tiles whose pair residuals
// are computed in the prologue (k-chunked above 256), and a workspace form
// (fp64 pair matrices, then tiles or one row per wave) kept as the exact
// generic path.
#include <algorithm>
#include <hip/hip_runtime.h>

#include <type_traits>

#include <stdint.h>

#include "mvmatch.h"
#include "mvm_device.h"
#include "mvm_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int kTripletRowsPerWave = 8;   // generic kernel: 32 (i, j) rows per workgroup

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
// (third_q / third_ok / cube_f32 / kTameResidual: mvm_device.h)

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

// One lane's 16 bytes of a cube row.  `lined`: every row starts on a 128-byte
// line (P and the scene's offset multiples of 32) -> nontemporal; otherwise a
// row's first and last lines are shared with its neighbours and the default
// policy lets L2 merge them (nontemporal partial lines reach HBM as masked
// writes: 200^3 1.91 -> 1.57 ms, 100^3 1.11 -> 1.06 ms per launch on the same
// buffers, profiles/r03/ab/cube_partial_lines_*.log).  Uniform per launch.
template <int KPL = kColsPerLane>
__device__ __forceinline__ void cube_row_store(uint64_t base, uint32_t off, const float v[KPL],
                                               bool lined) {
    static_assert(KPL == 3 || KPL == 4, "3 or 4 k per lane (5-8: two panels, row_store_n)");
    if constexpr (KPL == 4) {   // rows may be only 4-byte aligned (P % 4 != 0)
        if (lined) store4_row_a4<1>(base, off, v);
        else store4_row_a4<0>(base, off, v);
    } else {
        if (lined) store3_row<1>(base, off, v);
        else store3_row<0>(base, off, v);
    }
}

// 1-4 consecutive outputs of a lane (the second panel of 5-8 k per lane)
template <int K>
__device__ __forceinline__ void row_store_n(uint64_t base, uint32_t off, const float *v, bool lined) {
    static_assert(K >= 1 && K <= 4, "1 to 4 k");
    if constexpr (K >= 3) {
        cube_row_store<K>(base, off, v, lined);
    } else if constexpr (K == 2) {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        typedef f32x2 __attribute__((address_space(1), aligned(4))) g_f32x2a4;
        const f32x2 w = {v[0], v[1]};
        if (lined) __builtin_nontemporal_store(w, reinterpret_cast<g_f32x2a4 *>(base + off));
        else *reinterpret_cast<g_f32x2a4 *>(base + off) = w;
    } else {
        typedef float __attribute__((address_space(1))) g_f32;
        if (lined) __builtin_nontemporal_store(v[0], reinterpret_cast<g_f32 *>(base + off));
        else *reinterpret_cast<g_f32 *>(base + off) = v[0];
    }
}

// A scene whose third view is empty (P == 0) has no cube entries, but its
// (i, j) rows still get the association result "no column": argmin -1, minimum
// NaN (value_of_key(kKeyInvalid); the small and generic kernels' result for
// such rows, and the oracle's).  Rows i = i_first + i_step * ii (ii < ni) and
// j in [j0, j0 + nj) of a workgroup's tile; every thread takes a share.
__device__ __forceinline__ void empty_k_rows(int32_t *argmin, float *minval, int64_t roff, int M,
                                             int i_first, int i_step, int ni, int j0, int nj) {
    for (int x = threadIdx.x; x < ni * nj; x += kThreads) {
        const int ii = x / nj, jj = x - ii * nj;
        const int64_t row = roff + (int64_t)(i_first + i_step * ii) * M + j0 + jj;
        if (argmin) argmin[row] = -1;
        if (minval) minval[row] = value_of_key(kKeyInvalid);
    }
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
    if (jw0 >= M || i0 >= N) return;                   // uniform over the workgroup
    if (P == 0) {
        empty_k_rows(args.argmin, args.minval, args.row_offs[s], M, i0, 1, min(kCubeIB, N - i0),
                     jw0, min(kWaves * kCubeRPW, M - jw0));
        return;
    }
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
                    cube_row_store(reinterpret_cast<uint64_t>(args.cube + coff + row * P),
                                  (uint32_t)kb * 4u, v, ((P | coff) & 31) == 0);
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
        store_row_results<kCubeRPW>(kmin, imin, nrows, lane, args.argmin, args.minval,
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
    // optional (BM8 instantiations): per (scene, i, group of 8 j rows) the
    // minimum over the group of every k, as the upper 16 bits of its
    // order-preserving key (bm8_key): row (i * ceil(M/8) + j/8) of P keys at
    // bmin8 + bmin8_offs[s].  The candidate-list assignment
    // (mvm_lsap_sparse.hip) reduces these instead of reading the cube once
    // more; 16 bits are a lower bound of the minimum good to 1/128, enough to
    // choose the candidates, whose costs it then reads exactly.
    uint16_t *bmin8;
    const int64_t *bmin8_offs;
};

// order-preserving key of a cube value (>= +0 or +inf) for bmin8; NaN -> 0,
// below every value's key, so one NaN entry shows in its group's minimum
// (scipy rejects a cost with any NaN; a large NaN key would hide behind the
// group's finite entries -- a NaN j point makes one NaN row of eight)
constexpr uint32_t kBm8NaN = 0u;
__device__ __forceinline__ uint32_t bm8_key(float v) {
    return v != v ? kBm8NaN : (__float_as_uint(v) | 0x80000000u);
}

// minimum over the SPLIT lane groups of a split-form wave (lanes l, l + L,
// l + 2L, ... with L = 64 / SPLIT hold the same k): xor 8 (DPP row_ror:8),
// xor 16 (swizzle), xor 32 (bpermute)
template <int SPLIT>
__device__ __forceinline__ uint32_t min_across_groups(uint32_t v, int lane) {
    if constexpr (SPLIT >= 8) v = umin(v, dpp_from<0x128>(v));
    if constexpr (SPLIT >= 4) v = umin(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (16 << 10)));
    if constexpr (SPLIT >= 2) v = umin(v, (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, (int)v));
    return v;
}

// one lane's KPL keys of an 8-row group (k = kb .. kb + KPL - 1, kvalid of
// them in the view), stored as their upper halves; vec: 8-byte aligned row
template <int KPL>
__device__ __forceinline__ void bm8_store(uint16_t *row, int kb, int kvalid, const uint32_t (&k)[KPL],
                                          bool vec) {
    if (KPL == 4 && vec && kvalid >= 4) {
        *reinterpret_cast<uint2 *>(row + kb) = make_uint2((k[0] >> 16) | (k[1] & 0xFFFF0000u),
                                                          (k[2] >> 16) | (k[KPL - 1] & 0xFFFF0000u));
    } else {
#pragma unroll
        for (int q = 0; q < KPL; ++q)
            if (q < kvalid) row[kb + q] = (uint16_t)(k[q] >> 16);
    }
}

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
// r + (8/SPLIT)*(its group).  A row's argmin is reduced inside its lane
// group (lane_group_min: DPP within 16-lane rows, an xor-16 swizzle for 32):
// per row-step 10-12 VALU instead of the 8-row transposed butterfly over the
// whole wave, which cost more than the row-steps themselves at P <= 64
// (same buffers: 48^3 2.96 -> 2.26 ms, 64^3 1.92 -> 1.56 ms per 8 GB launch,
// profiles/r03/ab/cube_group_argmin_*.log).
// KPL: k per lane.  3 where the view fits 3 * (64 / SPLIT) k (48 / 96 / 192):
// a quarter fewer VALU per row step than 4 k per lane, whose last quarter of
// lanes would hold no k there; rows are stored with `global_store_dwordx3`.
// 5-8 (split forms only): a view of, e.g., 130 at two rows per instruction
// with 5 k on each of a row's 32 lanes (81% of the lanes busy) instead of one
// row per instruction with 3 k (68%): cube_lane_shape picks the form.
// workgroups per CU of triplet_fused_kernel: the VGPR budget's (more than 128
// VGPRs for 12-row waves, the 8-row minima at 4 k per lane, and 6-8 k per
// lane at two rows per instruction) or the static LDS's, whichever is less
constexpr int fused_occupancy(int ib, int rpw, int split, int kpl, bool bm8) {
    const int w13 = (kWave / split) * kpl < kChunk ? (kWave / split) * kpl : kChunk;
    const int kj = kWaves * rpw;
    const int lds = 8 * ib * w13 + 8 * ib * kj + 64 * (ib + kj) + 16 * (ib + kj) + 1024;
    const int by_vgpr = (rpw > 8 || (bm8 && kpl == 4) || (split == 2 && kpl >= 6)) ? 3 : 4;
    const int by_lds = 160 * 1024 / lds;
    return by_lds < by_vgpr ? (by_lds > 1 ? by_lds : 1) : by_vgpr;
}

template <int kCubeIB, int kCubeRPW, int SPLIT = 1, int KPL = kColsPerLane, bool BM8 = false>
// kCubeIB: i rows per tile, 16 or (split forms, mvm_options.cube_tile_rows) 32.
__global__ __launch_bounds__(kThreads, fused_occupancy(kCubeIB, kCubeRPW, SPLIT, KPL, BM8))
void triplet_fused_kernel(CubeFusedArgs args) {
    static_assert(!BM8 || kCubeRPW == 8, "8-row minima: 8 rows per wave (one 8-row group)");
    constexpr bool HALF = SPLIT > 1;   // split mapping
    static_assert(SPLIT == 1 || ((kCubeRPW == 8 || kCubeRPW == 12) && (SPLIT == 2 || SPLIT == 4)) ||
                      (kCubeRPW == 8 && SPLIT == 8 && KPL <= 4),
                  "8 or 12 rows in 2 or 4 groups, or 8 rows in 8 groups of 3-4 k per lane");
    static_assert(kCubeRPW % SPLIT == 0, "whole rows per lane group");
    static_assert(KPL >= 3 && KPL <= 8 && (KPL <= 4 || SPLIT > 1),
                  "3 or 4 k per lane; 5-8 in the split forms (views of 65-256 at 2 or 4 rows per "
                  "instruction)");
    constexpr int kLaneRows = kCubeRPW / SPLIT;   // rows a lane computes
    constexpr int kLPR = kWave / SPLIT;           // lanes per row
    constexpr int kJ = kWaves * kCubeRPW;                                          // j per workgroup
    // k columns a row's lanes hold: the e13 rows' width (a split form's view
    // is <= kLPR * KPL, so 32 i rows at 4 rows per instruction take the LDS
    // of 16 at one)
    constexpr int kW13 = kLPR * KPL < kChunk ? kLPR * KPL : kChunk;
    static_assert(kCubeIB <= kWave, "the tile's i rows: one thread of wave 0 each");
    __shared__ __attribute__((aligned(16))) double s13[kCubeIB][kW13];             // <= 32 KiB
    __shared__ __attribute__((aligned(16))) double s12[kCubeIB][kJ];
    __shared__ LineRec s_r13[kCubeIB], s_r12[kCubeIB], s_c12[kJ], s_r23[kJ];
    __shared__ double s_p0[kCubeIB][2], s_p1[kJ][2];

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);
    const int lane = t % kWave;
    // Write order.  Dispatch puts workgroup b on XCD b % 8; the remap gives
    // each XCD a contiguous range of tiles, so one XCD holds all the tiles of
    // a scene at once.  A tile owns the i rows ib, ib + IB', ib + 2 IB', ...
    // (IB' = the scene's i tile count: interleaved, not 16 consecutive rows), so at its
    // step ii the scene's tiles write the ADJACENT rows ii * IB' .. ii * IB' +
    // IB' - 1 -- one contiguous band of the cube per XCD, moving through it as
    // ii advances, instead of 16 bands 16 rows apart.
    uint32_t blk = blockIdx.x;
    {
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
    // tile rows: ib + i_stride * ii, over THIS scene's i tiles: a view of
    // N < max_n rows fills ceil(N / IB) tiles (the rest exit) instead of
    // spreading N rows thinly over all i_blocks tiles of the grid
    const int i_stride = min(args.i_blocks, (N + kCubeIB - 1) / kCubeIB);
    if (jw0 >= M || ib >= i_stride) return;             // uniform over the workgroup
    const int ni = min(kCubeIB, (N - ib + i_stride - 1) / i_stride);
    if (P == 0) {
        empty_k_rows(args.argmin, args.minval, args.row_offs[s], M, ib, i_stride, ni, jw0,
                     min(kJ, M - jw0));
        return;
    }
    const int j0 = jw0 + wave * kCubeRPW;
    const int nrows = min(kCubeRPW, M - j0);
    const int hl = lane / kLPR;                                      // row group of the lane
    const int gl = lane % kLPR;                                      // lane within its row
    // The lane's k.  3 or 4 per lane: k = KPL gl .. KPL gl + KPL - 1, one
    // dwordx3/x4 store per row.  5-8 per lane: two panels, k = 4 gl .. 4 gl + 3
    // (the row's first 4 kLPR k) and k = 4 kLPR + K2 gl .. (K2 = KPL - 4), so
    // each of the row's two store instructions writes one dense contiguous
    // span -- a lane's 5-8 consecutive k would make both sparse (16 of every
    // 4 KPL bytes, then the rest), measured 0.59-0.70 of the write probe
    constexpr int K2 = KPL > 4 ? KPL - 4 : 0;
    const int kb = (K2 ? 4 : KPL) * gl;                              // the lane's first k
    auto kpos = [&](int q) -> int {
        if constexpr (K2 > 0) return q < 4 ? kb + q : 4 * kLPR + K2 * gl + (q - 4);
        return kb + q;
    };
    const int kvalid = P - kb;                                       // 3-4 k: valid k of the lane
    const int64_t coff = args.cube_offs[s];
    const int64_t roff = args.row_offs[s];
    // vector rows for any P: a lane stores its k with one dwordx3/x4 per
    // panel (dword-aligned: gfx950 takes it), except the lane a row ends in,
    // which stores its remaining k alone
    const bool full = args.cube != nullptr;
    const bool act_k = kvalid > 0;
    const double *F12 = args.F + (3 * (int64_t)s + 0) * 9;
    const double *F13 = args.F + (3 * (int64_t)s + 1) * 9;
    const double *F23 = args.F + (3 * (int64_t)s + 2) * 9;

    // ---- prologue 1: the tile's view-0 rows, view-1 rows/columns, and the
    // k columns' lines (one column per thread: kThreads == kChunk).  The F23
    // column lines are shared by the 4 waves: they go to the s13 storage as
    // scratch (read back in prologue 2, before e13 overwrites it) instead of
    // every wave recomputing them
    struct ColRec {
        LineRec l;
        double x, y;
    };
    static_assert(sizeof(ColRec) * kW13 <= sizeof(s13), "F23 column scratch fits s13");
    ColRec *s_c23 = reinterpret_cast<ColRec *>(&s13[0][0]);
    bool any_deg = false;   // a degenerate line among this thread's (9999 sentinel)
    if (t < kCubeIB) {
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (t < ni) {
            double f[9];
            px = args.pts[2 * (c0 + ib + i_stride * t)];
            py = args.pts[2 * (c0 + ib + i_stride * t) + 1];
            load_f(F13, f);
            a.deg = row_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F12, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        any_deg |= (a.deg != 0.0) || (b.deg != 0.0);
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
        any_deg |= (a.deg != 0.0) || (b.deg != 0.0);
        s_c12[jj] = a;
        s_r23[jj] = b;
        s_p1[jj][0] = px;
        s_p1[jj][1] = py;
    }
    LineRec cl13{0.0, 0.0, 0.0, 0.0};   // column k = t, F13 (registers, for e13)
    double kx = 0.0, ky = 0.0;
    {
        ColRec c23{{0.0, 0.0, 0.0, 0.0}, 0.0, 0.0};
        if (t < P) {
            double f[9];
            kx = args.pts[2 * (c2 + t)];
            ky = args.pts[2 * (c2 + t) + 1];
            load_f(F13, f);
            cl13.deg = col_line(f, kx, ky, cl13.l0, cl13.l1, cl13.l2) ? 1.0 : 0.0;
            load_f(F23, f);
            c23.l.deg = col_line(f, kx, ky, c23.l.l0, c23.l.l1, c23.l.l2) ? 1.0 : 0.0;
            c23.x = kx;
            c23.y = ky;
            any_deg |= (cl13.deg != 0.0) || (c23.l.deg != 0.0);
        }
        if (t < kW13) s_c23[t] = c23;
    }
    // uniform: no line of the tile is degenerate, so every residual is
    // 0.5 * (|l1 . p1| + |l2 . p2|) without the sentinel selects
    const bool no_deg = __syncthreads_and(!any_deg) != 0;
    auto pair = [&](const LineRec &col, const LineRec &row, double rx, double ry, double cx,
                    double cy) {
        if (no_deg)
            return 0.5 * (line_dist(col.l0, col.l1, col.l2, rx, ry) +
                          line_dist(row.l0, row.l1, row.l2, cx, cy));   // :28
        return pair_e(col, row, rx, ry, cx, cy);
    };
    // ---- prologue 2: the wave's e23 rows into registers ---------------------
    bool tame_in = true;   // every residual this thread produced is <= kTameResidual
    double a23[kLaneRows][KPL];
#pragma unroll
    for (int q = 0; q < KPL; ++q) {
        const ColRec cl = s_c23[min(kpos(q), kW13 - 1)];
#pragma unroll
        for (int r = 0; r < kLaneRows; ++r) {
            const int rr = r + hl * kLaneRows;            // the wave row
            const int jj = wave * kCubeRPW + rr;
            a23[r][q] = (rr < nrows && kpos(q) < P)
                            ? pair(cl.l, s_r23[jj], s_p1[jj][0], s_p1[jj][1], cl.x, cl.y)
                            : 0.0;
            tame_in &= a23[r][q] <= kTameResidual;
        }
    }
    __syncthreads();   // every wave has its F23 columns: s13 is free for e13
    // ---- prologue 3: the tile's e13 / e12 (row_safe's arithmetic) -----------
    if (t < P) {
#pragma unroll 4
        for (int r = 0; r < kCubeIB; ++r) {
            const double e = r < ni ? pair(cl13, s_r13[r], s_p0[r][0], s_p0[r][1], kx, ky) : 0.0;
            s13[r][t] = e;
            tame_in &= e <= kTameResidual;
        }
    } else if (t < kW13) {
        for (int r = 0; r < kCubeIB; ++r) s13[r][t] = 0.0;
    }
    for (int x = t; x < kCubeIB * kJ; x += kThreads) {
        const int r = x / kJ, jj = x % kJ;
        const double e = (r < ni && jw0 + jj < M)
                             ? pair(s_c12[jj], s_r12[r], s_p0[r][0], s_p0[r][1], s_p1[jj][0], s_p1[jj][1])
                             : 0.0;
        s12[r][jj] = e;
        tame_in &= e <= kTameResidual;
    }
    // every sum of the tile is finite when its three residuals are <= 2^1020
    // (NaN fails the compare): then third_q is RN(s/3) for all of them and the
    // main loop needs no per-row check (a loop without the fallback path)
    const bool tile_fast = __syncthreads_and(tame_in) != 0 && full;
    if (nrows <= 0) return;   // after the barrier: no more barriers below

    // Row stores from a uniform row address: the wave's row r at step ii
    // starts at cube + coff + ((i M + j0 + r) P) floats (scalar), and a lane
    // of row group hl writes row r + hl * kLaneRows from its k = kb on, a
    // loop-invariant 32-bit byte offset -- the saddr form, no per-row 64-bit
    // address arithmetic on the VALU
    const uint32_t lane_off = (uint32_t)((hl * kLaneRows * P + kb) * 4);
    const uint32_t lane_off2 = (uint32_t)((hl * kLaneRows * P + (K2 ? 4 * kLPR + K2 * gl : 0)) * 4);
    const uint64_t cube_base = reinterpret_cast<uint64_t>(args.cube) + (uint64_t)coff * 4u;
    const bool lined = ((P | coff) & 31) == 0;
    auto main_loop = [&](auto fast_tag) {
        constexpr bool FAST = decltype(fast_tag)::value;
        for (int ii = 0; ii < ni; ++ii) {
            const int i = ib + i_stride * ii;
            const uint64_t row_i = cube_base + (uint64_t)((int64_t)i * M + j0) * (uint64_t)P * 4u;
            double a13[KPL];
            if constexpr (KPL >= 4) {   // 4 k at kb (16-byte aligned), then panel 2's
                const f64x2 lo = *reinterpret_cast<const f64x2 *>(&s13[ii][kb]);
                const f64x2 hi = *reinterpret_cast<const f64x2 *>(&s13[ii][kb + 2]);
                a13[0] = lo.x; a13[1] = lo.y; a13[2] = hi.x; a13[3] = hi.y;
#pragma unroll
                for (int q = 4; q < KPL; ++q) a13[q] = s13[ii][min(kpos(q), kW13 - 1)];
            } else {
#pragma unroll
                for (int q = 0; q < KPL; ++q) a13[q] = s13[ii][min(kb + q, kW13 - 1)];
            }
            uint32_t key[kLaneRows];
            int32_t idx[kLaneRows];
            uint32_t bmk[KPL];                                   // BM8: the 8 rows' minima per k
#pragma unroll
            for (int q = 0; q < KPL; ++q) bmk[q] = 0xFFFFFFFFu;
#pragma unroll
            for (int r = 0; r < kLaneRows; ++r) {
                key[r] = kKeyInvalid;
                idx[r] = 0x7FFFFFFF;
                if (r >= nrows) continue;   // uniform (the lower half's row is the smaller)
                const int rr = r + hl * kLaneRows;                 // the wave row
                const bool act = act_k && rr < nrows;              // HALF: the upper row may not exist
                const double v12 = s12[ii][wave * kCubeRPW + rr];
                double sum[KPL], q0[KPL];
                bool ok = true;
#pragma unroll
                for (int q = 0; q < KPL; ++q) {
                    sum[q] = (v12 + a13[q]) + a23[r][q];          // (e12 + e13) + e23, :81
                    q0[q] = third_q(sum[q]);
                    if (!FAST) ok &= third_ok(q0[q]);
                }
                float v[KPL];
                const int64_t row = (int64_t)i * M + j0 + rr;
                if (FAST || (full && __all(ok || !act))) {
#pragma unroll
                    for (int q = 0; q < KPL; ++q) v[q] = (float)q0[q];
                    const bool whole = kvalid >= KPL;   // the lane's k all in the row
                    if (act) {
                        const uint64_t row_r = row_i + (uint64_t)r * (uint64_t)P * 4u;   // uniform
                        uint32_t off = lane_off;
                        __asm__ volatile("" : "+v"(off));   // a 32-bit lane offset at the store: saddr form
                        using gfloat = float __attribute__((address_space(1)));
                        if constexpr (K2 == 0) {
                            if (whole) {
                                cube_row_store<KPL>(row_r, off, v, lined);
                            } else {   // the row's last lane (P % KPL != 0)
                                gfloat *rp = reinterpret_cast<gfloat *>(row_r + off);
#pragma unroll
                                for (int q = 0; q < KPL - 1; ++q)
                                    if (q < kvalid) rp[q] = v[q];
                            }
                        } else {   // two panels, each one dense span per instruction
                            if (kb + 3 < P) {
                                cube_row_store<4>(row_r, off, v, lined);
                            } else {
                                gfloat *rp = reinterpret_cast<gfloat *>(row_r + off);
#pragma unroll
                                for (int q = 0; q < 3; ++q)
                                    if (kb + q < P) rp[q] = v[q];
                            }
                            uint32_t off2 = lane_off2;
                            __asm__ volatile("" : "+v"(off2));
                            if (kpos(KPL - 1) < P) {
                                row_store_n<K2>(row_r, off2, v + 4, lined);
                            } else {
                                gfloat *rp = reinterpret_cast<gfloat *>(row_r + off2);
#pragma unroll
                                for (int q = 4; q < KPL - 1; ++q)
                                    if (kpos(q) < P) rp[q - 4] = v[q];
                            }
                        }
                    }
                    if constexpr (BM8) {
#pragma unroll
                        for (int q = 0; q < KPL; ++q)
                            if (act && (K2 ? kpos(q) < P : (whole || q < kvalid)))
                                bmk[q] = umin(bmk[q], bm8_key(v[q]));
                    }
                    Best b{v[0], kb};
#pragma unroll
                    for (int q = 1; q < KPL; ++q)
                        if (K2 ? kpos(q) < P : (whole || q < kvalid)) best_update_fast(b, v[q], kpos(q));
                    key[r] = act ? __float_as_uint(b.v) + 1u : kKeyInvalid;
                    idx[r] = act ? b.j : 0x7FFFFFFF;
                } else {
                    Best b{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
                    // the IEEE division only when some lane needs it (uniform branch)
                    double qq[KPL];
#pragma unroll
                    for (int q = 0; q < KPL; ++q) qq[q] = q0[q];
                    if (!__all(ok || !act)) {
#pragma unroll
                        for (int q = 0; q < KPL; ++q)
                            qq[q] = third_ok(q0[q]) ? q0[q] : sum[q] / 3.0;
                    }
#pragma unroll
                    for (int q = 0; q < KPL; ++q) {
                        v[q] = (float)qq[q];
                        if (act && kpos(q) < P) {
                            if (args.cube)
                                args.cube[coff + row * P + kpos(q)] = v[q];   // L2 merges the strided dword stores
                            best_update_safe(b, v[q], kpos(q));
                            if constexpr (BM8) bmk[q] = umin(bmk[q], bm8_key(v[q]));
                        }
                    }
                    key[r] = best_key(b);
                    idx[r] = b.j;
                }
            }
            if constexpr (BM8) {
                uint16_t *brow = args.bmin8 + args.bmin8_offs[s] + ((int64_t)i * ((M + 7) / 8) + j0 / 8) * P;
                if constexpr (HALF) {
                    // the wave's 8 rows lie on SPLIT lane groups holding the
                    // same k: the minimum across the groups (lane strides of
                    // kLPR), then group 0 stores the keys
#pragma unroll
                    for (int q = 0; q < KPL; ++q) bmk[q] = min_across_groups<SPLIT>(bmk[q], lane);
                    if (hl == 0 && act_k) {
                        if constexpr (K2 == 0) {
                            bm8_store<KPL>(brow, kb, kvalid, bmk, (P & 3) == 0 && (args.bmin8_offs[s] & 3) == 0);
                        } else {
#pragma unroll
                            for (int q = 0; q < KPL; ++q)
                                if (kpos(q) < P) brow[kpos(q)] = (uint16_t)(bmk[q] >> 16);
                        }
                    }
                } else if (act_k) {
                    bm8_store<KPL>(brow, kb, kvalid, bmk, (P & 3) == 0 && (args.bmin8_offs[s] & 3) == 0);
                }
            }
            if constexpr (HALF) {
                // each row lies on one group of kLPR lanes: reduce inside the
                // groups (key, then the lowest index holding it), then lane g
                // of group hl stores the group's row g
                const int g = lane % kLPR;
                uint32_t mk = kKeyInvalid;
                int32_t mi = 0x7FFFFFFF;
#pragma unroll
                for (int r = 0; r < kLaneRows; ++r) {
                    const uint32_t gk = lane_group_min<kLPR>(key[r]);
                    const uint32_t gi =
                        lane_group_min<kLPR>(key[r] == gk ? (uint32_t)idx[r] : 0x7FFFFFFFu);
                    mk = (g == r) ? gk : mk;
                    mi = (g == r) ? (int32_t)gi : mi;
                }
                const int rr = g + hl * kLaneRows;
                if (g < kLaneRows && rr < nrows) {
                    const int64_t row0 = roff + (int64_t)i * M + j0;   // uniform
                    if (args.argmin) (args.argmin + row0)[rr] = (mk == kKeyInvalid) ? -1 : mi;
                    if (args.minval) (args.minval + row0)[rr] = value_of_key(mk);
                }
            } else if constexpr (FAST && kCubeRPW == 8) {   // finite keys, one k-chunk
                uint32_t mk;
                int32_t mi;
                // the lane id as a fresh value: the row address below is then
                // computed here, not hoisted out of the tile loop and spilled
                // (its reload after the row stores waited for all of them:
                // vmcnt is in order)
                int lz = lane;
                __asm__ volatile("" : "+v"(lz));
                wave_argmin8_transposed(key, idx, lz, mk, mi);
                if (lz < nrows) {
                    const int64_t row = roff + (int64_t)i * M + j0 + lz;
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
                int lz = lane;   // fresh per row group (see above)
                __asm__ volatile("" : "+v"(lz));
                store_row_results<kCubeRPW>(kmin, imin, nrows, lz, args.argmin, args.minval,
                                            roff + (int64_t)i * M + j0);
            }
        }
    };
    // Full tiles (every lane's 4 k inside the view, all 8 wave rows present:
    // the whole 256^3 regime): the fast loop without per-row existence tests
    // or exec masking, rows stored from one running scalar address, and the
    // in-lane argmin from unsigned minima of the float32 bits (the values are
    // finite and non-negative here, so they order like their bits) -- the
    // first q holding the minimum is np.argmin's first index within the lane.
    auto full_loop = [&](auto) {   // generic: instantiated only where called (4 k per lane)
        constexpr uint64_t kRowBytes = kChunk * sizeof(float);
        uint64_t rp = reinterpret_cast<uint64_t>(args.cube + coff) +
                      (uint64_t)((int64_t)ib * M + j0) * kRowBytes;
        const uint64_t i_step = (uint64_t)i_stride * M * kRowBytes;
        for (int ii = 0; ii < ni; ++ii) {
            double a13[kColsPerLane];
            {
                const f64x2 lo = *reinterpret_cast<const f64x2 *>(&s13[ii][kb]);
                const f64x2 hi = *reinterpret_cast<const f64x2 *>(&s13[ii][kb + 2]);
                a13[0] = lo.x; a13[1] = lo.y; a13[2] = hi.x; a13[3] = hi.y;
            }
            double v12s[kCubeRPW];   // the 8 rows' e12, read together (4 x 16 B)
#pragma unroll
            for (int r = 0; r < kCubeRPW; r += 2) {
                const f64x2 w = *reinterpret_cast<const f64x2 *>(&s12[ii][wave * kCubeRPW + r]);
                v12s[r] = w.x;
                v12s[r + 1] = w.y;
            }
            uint32_t key[kCubeRPW];
            int32_t idx[kCubeRPW];
            uint32_t bmk[kColsPerLane];                          // BM8: the 8 rows' minima per k
#pragma unroll
            for (int q = 0; q < kColsPerLane; ++q) bmk[q] = 0xFFFFFFFFu;
            uint64_t p = rp;
#pragma unroll
            for (int r = 0; r < kCubeRPW; ++r) {
                const double v12 = v12s[r];
                float v[kColsPerLane];
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q)
                    v[q] = (float)third_q((v12 + a13[q]) + a23[r][q]);   // (e12 + e13) + e23, :81
                uint32_t off = (uint32_t)kb * 4u;
                __asm__ volatile("" : "+v"(off));   // a 32-bit lane offset at the store: saddr form
                store4_nt_row(p, off, v);
                p += kRowBytes;
                __asm__ volatile("" : "+s"(p));     // one running scalar row address
                const uint32_t b0 = __float_as_uint(v[0]), b1 = __float_as_uint(v[1]);
                const uint32_t b2 = __float_as_uint(v[2]), b3 = __float_as_uint(v[3]);
                const uint32_t m = umin(min3_u32(b0, b1, b2), b3);
                if constexpr (BM8) {                             // finite, >= +0: the bits order
                    bmk[0] = umin(bmk[0], b0);
                    bmk[1] = umin(bmk[1], b1);
                    bmk[2] = umin(bmk[2], b2);
                    bmk[3] = umin(bmk[3], b3);
                }
                int q = (b2 == m) ? 2 : 3;
                q = (b1 == m) ? 1 : q;
                q = (b0 == m) ? 0 : q;
                key[r] = m;                       // the bits themselves: no NaN / invalid here
                idx[r] = kb + q;
            }
            if constexpr (BM8) {
                uint32_t kk[kColsPerLane];
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) kk[q] = bmk[q] | 0x80000000u;
                bm8_store<kColsPerLane>(args.bmin8 + args.bmin8_offs[s] +
                                            ((int64_t)(ib + i_stride * ii) * ((M + 7) / 8) + j0 / 8) * P,
                                        kb, kColsPerLane, kk, (args.bmin8_offs[s] & 3) == 0);
            }
            uint32_t mk;
            int32_t mi;
            wave_argmin8_transposed(key, idx, lane, mk, mi);
            if (lane < kCubeRPW) {
                const int64_t row = roff + (int64_t)(ib + i_stride * ii) * M + j0 + lane;
                if (args.argmin) args.argmin[row] = mi;
                if (args.minval) args.minval[row] = __uint_as_float(mk);
            }
            rp += i_step;
        }
    };
    if constexpr (SPLIT == 1 && KPL == kColsPerLane) {
        if (tile_fast && nrows == kCubeRPW && P == kChunk) {   // uniform
            full_loop(0);
            return;
        }
    }
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
    const uint32_t blk = blockIdx.x;
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
    if (jw0 >= M || i0 >= N) return;                   // uniform over the workgroup
    const int ni = min(kCubeIB, N - i0);
    if (P == 0) {
        empty_k_rows(args.argmin, args.minval, args.row_offs[s], M, i0, 1, ni, jw0, min(kJ, M - jw0));
        return;
    }
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
        // the chunk's column points from a uniform base and 32-bit lane
        // offsets (saddr loads): no 64-bit per-lane address to keep
        const double *pk = args.pts + 2 * (c2 + kc);
        if (kc > 0) __syncthreads();   // every wave is done with the previous chunk's s13
        bool tame_in = tame12;
        {   // e13 of this chunk: one column per thread
            const int k = t;
            double f13[9];
            load_f(F13, f13);
            if (k < Pc) {
                const double x = pk[2 * k], y = pk[2 * k + 1];
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
                x = pk[2 * (kb + q)];
                y = pk[2 * (kb + q) + 1];
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
        const bool full = args.cube != nullptr;   // any P: see triplet_fused_kernel
        // every sum of this chunk finite: the loop without the per-row vote
        const bool chunk_fast = __syncthreads_and(tame_in) != 0 && full;
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
                        const bool whole = kvalid >= kColsPerLane;
                        if (act) {
                            if (whole) {
                                cube_row_store(reinterpret_cast<uint64_t>(args.cube + coff + row * P + kc),
                                               (uint32_t)kb * 4u, v, ((P | coff) & 31) == 0);
                            } else {   // the row's last lane (P % 4 != 0)
#pragma unroll
                                for (int q = 0; q < kColsPerLane - 1; ++q)
                                    if (q < kvalid) args.cube[coff + row * P + kc + kb + q] = v[q];
                            }
                        }
                        Best b{v[0], kb};
#pragma unroll
                        for (int q = 1; q < kColsPerLane; ++q)
                            if (whole || q < kvalid) best_update_fast(b, v[q], kb + q);
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
                if constexpr (kCubeRPW == 8 && kWave % 8 == 0) {
                    // rows x = ii*8 + r land in lanes x % 64 of slot x / 64 directly;
                    // keys are ordered like np.argmin's rule (NaN 0, no column
                    // kKeyInvalid) and a lane's columns follow its lane id, so
                    // the lowest lane holding the minimum has the lowest index
                    // -- also on the generic chunk path (fewer live registers
                    // than eight per-row wave reductions)
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
// default switch-over to the fused kernel: measured on 2 GB launches, the
// same buffers (profiles/r05/cube/small/), ms per launch, small vs fused at
// eight rows per instruction with tiles of 32 i rows (up to 32) or four rows
// per instruction (above): 16^3 0.974 vs 1.063, 24^3 0.787 vs 0.571, 32^3
// 1.162 vs 0.426, 40^3 0.850 vs 0.581, 44^3 0.921 vs 0.500 (round 1 had set
// 44 against the fused kernel of its time)
constexpr int kSmallAutoMaxN = 16;

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

// CubeFusedArgs::bmin8 read back from a finished cube, for the kernel paths
// that do not emit the 8-row minima themselves: one workgroup per (scene,
// block of `ir` rows i), ir chosen so a workgroup has >= ~1,024 items; its
// threads take the (i, 8-row group, k) items in turn -- four k per item with
// 16-byte loads where the rows allow, the group's 8 rows loaded together (the
// round-4 form walked k alone for one i, with 8 dependent loads)
__global__ __launch_bounds__(kThreads) void bmin8_from_cube_kernel(const int64_t *cam_offs,
                                                                   const int64_t *cube_offs,
                                                                   const float *cube, uint16_t *bmin8,
                                                                   const int64_t *bmin8_offs, int i_blocks,
                                                                   int ir) {
    const int s = (int)(blockIdx.x / (unsigned)i_blocks);
    const int i0 = (int)(blockIdx.x % (unsigned)i_blocks) * ir;
    const int64_t *co = cam_offs + 3 * (int64_t)s;
    const int N = (int)(co[1] - co[0]), M = (int)(co[2] - co[1]), P = (int)(co[3] - co[2]);
    if (i0 >= N || M == 0 || P == 0) return;
    const int ni = min(ir, N - i0);
    const int g8 = (M + 7) / 8;
    const int64_t cb = cube_offs[s] + (int64_t)i0 * M * P, ob = bmin8_offs[s] + (int64_t)i0 * g8 * P;
    const float *base = cube + cb;                 // row i0's (j, k) block; row i0 + ii at + ii M P
    uint16_t *out = bmin8 + ob;                    // ... at + ii g8 P
    if ((P & 3) == 0 && (cb & 3) == 0 && (ob & 3) == 0) {
        const int P4 = P / 4, per_i = g8 * P4, items = ni * per_i;
        for (int x = threadIdx.x; x < items; x += kThreads) {
            const int ii = x / per_i, y = x - ii * per_i, jg = y / P4, k = 4 * (y - jg * P4);
            const float *bi = base + (int64_t)ii * M * P;
            f32x4 v[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int j = 8 * jg + r;
                v[r] = j < M ? *reinterpret_cast<const f32x4 *>(bi + (int64_t)j * P + k)
                             : f32x4{INFINITY, INFINITY, INFINITY, INFINITY};
            }
            uint32_t m[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                if (8 * jg + r >= M) continue;
                m[0] = umin(m[0], bm8_key(v[r].x));
                m[1] = umin(m[1], bm8_key(v[r].y));
                m[2] = umin(m[2], bm8_key(v[r].z));
                m[3] = umin(m[3], bm8_key(v[r].w));
            }
            *reinterpret_cast<uint2 *>(out + (int64_t)ii * g8 * P + (int64_t)jg * P + k) =
                make_uint2((m[0] >> 16) | (m[1] & 0xFFFF0000u), (m[2] >> 16) | (m[3] & 0xFFFF0000u));
        }
        return;
    }
    const int per_i = g8 * P, items = ni * per_i;
    for (int x = threadIdx.x; x < items; x += kThreads) {
        const int ii = x / per_i, y = x - ii * per_i, jg = y / P, k = y - jg * P;
        const float *bi = base + (int64_t)ii * M * P;
        float v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int j = 8 * jg + r;
            v[r] = j < M ? bi[(int64_t)j * P + k] : INFINITY;
        }
        uint32_t m = 0xFFFFFFFFu;
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (8 * jg + r < M) m = umin(m, bm8_key(v[r]));
        out[(int64_t)ii * g8 * P + (int64_t)jg * P + k] = (uint16_t)(m >> 16);
    }
}

// --------------------------------------- cube-free 8-row minima (ABI 7) ----
// For an assignment that never reads the cube itself (match_captures with
// keep_cube=False, bench.py c2match), everything it needs instead of the cube:
//   bmin8  the 16-bit 8-row minima the fused kernel writes next to the cube
//          (CubeFusedArgs::bmin8), bit for bit;
//   bm32   the 32-column block minima the candidate-list kernels start from,
//          as upper bounds ((h << 16) | 0xFFFF of the block's smallest 16-bit
//          key h, capped at +inf's key; sp_bmin8_reduce_kernel's values): per
//          scene P rows of nb = ceil(M/32) * npad keys, npad = roundup(N, 16),
//          block (jt, i) at jt * npad + i (rows i >= N: 0xFFFFFFFF, never a
//          candidate), rows at bm32 + bm32_offs[s] + k * nb;
//   resid  every scene's fp64 pair residuals, from which the assignment's
//          kernels recompute the few entries they read (cube_f32):
//            e12  [N][ld]  at resid + s * stride                  (i, j)
//            e13T [P][ld]  at resid + s * stride + max_n * ld     (k, i)
//            e23T [P][ld]  at resid + s * stride + 2 * max_n * ld (k, j)
//          stride = 3 * max_n * ld, ld = roundup(max_n, 4).
// RN(s / 3) and the float32 cast are monotone, so the minimum over a group's
// 8 j of float32(third(s_j)) is float32(third(min_j s_j)): where every
// residual is <= 2^1020 (finite sums) a triple costs two fp64 adds and one
// fp64 min, and the third runs once per (group, k) -- a quarter of the fused
// kernel's VALU per triple and none of its 4 B/triple of stores.  Elsewhere
// every entry is computed exactly (third_q, the division for non-finite sums)
// and the minimum taken over the keys (NaN -> key 0), as the fused kernel does.
// A workgroup owns (scene, one 32-column block jb of j); thread t takes the
// short-side column k = t (P <= 256) for all 32 j of the block, so a block's
// minimum (four 8-row groups) is one thread's, and e13[i][k] is the thread's
// own value: per chunk of IB rows i only the chunk's row lines and its e12
// [IB][32] tile go through LDS.  The e23 column (32 j) sits in the thread's
// registers for the whole scene.  Workgroups of block 0 write e13T, every
// workgroup its e23T rows and e12 columns.
// the approximate minima (triplet_minima_kernel): residuals up to 2^64 (their
// float32 images and sums finite), the lower 16 bits of a float32 cost at
// least kApproxMargin from a carry either way, costs >= 2^-100 (normal
// float32 throughout)
constexpr double kApproxResidual = 0x1p64;
constexpr uint32_t kApproxMargin = 8;
constexpr uint32_t kApproxTiny = 0x0D800000u;   // the bits of 2^-100
constexpr float kThirdF = 1.0f / 3.0f;

struct MinimaArgs {
    const double *pts;
    const int64_t *cam_offs;
    const double *F;            // [S*3, 9]: F12, F13, F23
    uint16_t *bmin8;
    const int64_t *bmin8_offs;
    uint16_t *bm32;                 // 16-bit keys
    const int64_t *bm32_offs;
    double *resid;
    int64_t stride;             // doubles per scene
    int32_t ld;                 // row stride of e12 / e13T / e23T (multiple of 4)
    int32_t max_n;
    int32_t j_blocks;
};

template <int IB, bool G8>   // G8: the 8-row minima too (else the block minima only)
__global__ __launch_bounds__(kThreads, 4) void triplet_minima_kernel(MinimaArgs args) {
    constexpr int kJ = 32;                     // j per workgroup: four 8-row groups
    static_assert(IB == 16, "the chunk's block minima leave as one 64-byte run per k");
    __shared__ __attribute__((aligned(16))) double s12[IB][kJ];
    __shared__ __attribute__((aligned(16))) float s12f[IB][kJ];
    // every row's lines (thread t: row i = t, once per workgroup) and each
    // chunk's degenerate flag
    __shared__ LineRec s_r13[kThreads], s_r12[kThreads], s_c12[kJ], s_r23[kJ];
    __shared__ double s_p0[kThreads][2], s_p1[kJ][2];
    __shared__ int32_t s_degc[kThreads / IB];
    __shared__ __attribute__((aligned(16))) uint16_t s_bm[IB][kThreads];   // the chunk's block minima (16-bit)

    const int t = threadIdx.x;
    uint32_t blk = blockIdx.x;   // each XCD a contiguous range of (scene, j block)s
    {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const int s = (int)(blk / (uint32_t)args.j_blocks);
    const int jb = (int)(blk % (uint32_t)args.j_blocks);
    const int64_t *co = args.cam_offs + 3 * (int64_t)s;
    const int64_t c0 = co[0], c1 = co[1], c2 = co[2];
    const int N = (int)(c1 - c0), M = (int)(c2 - c1), P = (int)(co[3] - c2);
    const int jw0 = jb * kJ;
    if (jw0 >= M || N == 0 || P == 0) return;   // uniform; an empty problem reads no cost
    const int nj = min(kJ, M - jw0);             // j rows of this block (uniform)
    const int k = t;
    const bool kv = k < P;
    const double *F12 = args.F + (3 * (int64_t)s + 0) * 9;
    const double *F13 = args.F + (3 * (int64_t)s + 1) * 9;
    const double *F23 = args.F + (3 * (int64_t)s + 2) * 9;
    const int ld = args.ld;
    double *E12 = args.resid + (int64_t)s * args.stride;
    double *E13T = E12 + (int64_t)args.max_n * ld;
    double *E23T = E13T + (int64_t)args.max_n * ld;
    const int g8 = (M + 7) / 8;
    uint16_t *B8 = args.bmin8 ? args.bmin8 + args.bmin8_offs[s] : nullptr;   // optional
    const int npad = (N + 15) & ~15;
    const int nbk = ((M + 31) / 32) * npad;
    uint16_t *BM = args.bm32 + args.bm32_offs[s] + (int64_t)k * nbk + (int64_t)jb * npad;

    // ---- once per workgroup: the block's j lines, this thread's k lines -----
    bool any_deg = false;
    if (t < kJ) {
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (t < nj) {
            double f[9];
            px = args.pts[2 * (c1 + jw0 + t)];
            py = args.pts[2 * (c1 + jw0 + t) + 1];
            load_f(F12, f);
            a.deg = col_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F23, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        any_deg |= (a.deg != 0.0) || (b.deg != 0.0);
        s_c12[t] = a;
        s_r23[t] = b;
        s_p1[t][0] = px;
        s_p1[t][1] = py;
    }
    LineRec cl13{0.0, 0.0, 0.0, 0.0}, c23{0.0, 0.0, 0.0, 0.0};
    double kx = 0.0, ky = 0.0;
    if (kv) {
        double f[9];
        kx = args.pts[2 * (c2 + k)];
        ky = args.pts[2 * (c2 + k) + 1];
        load_f(F13, f);
        cl13.deg = col_line(f, kx, ky, cl13.l0, cl13.l1, cl13.l2) ? 1.0 : 0.0;
        load_f(F23, f);
        c23.deg = col_line(f, kx, ky, c23.l0, c23.l1, c23.l2) ? 1.0 : 0.0;
        any_deg |= (cl13.deg != 0.0) || (c23.deg != 0.0);
    }
    {   // row i = t's lines; a chunk (16 rows of one wave) is degenerate when
        // any of its rows is
        LineRec a{0.0, 0.0, 0.0, 0.0}, b{0.0, 0.0, 0.0, 0.0};
        double px = 0.0, py = 0.0;
        if (t < N) {
            double f[9];
            px = args.pts[2 * (c0 + t)];
            py = args.pts[2 * (c0 + t) + 1];
            load_f(F13, f);
            a.deg = row_line(f, px, py, a.l0, a.l1, a.l2) ? 1.0 : 0.0;
            load_f(F12, f);
            b.deg = row_line(f, px, py, b.l0, b.l1, b.l2) ? 1.0 : 0.0;
        }
        s_r13[t] = a;
        s_r12[t] = b;
        s_p0[t][0] = px;
        s_p0[t][1] = py;
        static_assert(kWave % IB == 0, "a wave's rows: whole chunks");
        const uint64_t dm = __ballot((a.deg != 0.0) || (b.deg != 0.0));
        if (t % kWave < kWave / IB)
            s_degc[t / kWave * (kWave / IB) + t % kWave] = ((dm >> (IB * (t % kWave))) & ((1ull << IB) - 1)) != 0;
    }
    // uniform: no j / k line of the workgroup is degenerate (the rows' lines
    // are judged per chunk: s_degc)
    const bool deg_fixed = __syncthreads_or(any_deg) != 0;
    auto pair = [&](bool nd, const LineRec &col, const LineRec &row, double rx, double ry, double cx,
                    double cy) {
        if (nd)
            return 0.5 * (line_dist(col.l0, col.l1, col.l2, rx, ry) +
                          line_dist(row.l0, row.l1, row.l2, cx, cy));   // :28
        return pair_e(col, row, rx, ry, cx, cy);
    };
    // e23[j][k] of the block's 32 j, in float32 for the approximate minima
    // (rows past the view +inf: never a group's minimum); the fp64 values go
    // to e23T and are recomputed where an exact minimum is needed
    auto e23_at = [&](int jj) {
        return jj >= nj ? (double)INFINITY
               : kv     ? pair(!deg_fixed, c23, s_r23[jj], s_p1[jj][0], s_p1[jj][1], kx, ky)
                        : 0.0;
    };
    bool near = true;                            // every residual <= kApproxResidual
    float f23[kJ];
    {
        double *dst = E23T + (int64_t)k * ld + jw0;
#pragma unroll
        for (int jj = 0; jj < kJ; jj += 2) {
            const double a0 = e23_at(jj), a1 = e23_at(jj + 1);
            near &= (jj >= nj || a0 <= kApproxResidual) && (jj + 1 >= nj || a1 <= kApproxResidual);
            f23[jj] = (float)a0;
            f23[jj + 1] = (float)a1;
            if (kv) {                            // e23T row k: the block's j (256 contiguous bytes)
                if (nj == kJ) {
                    *reinterpret_cast<f64x2 *>(dst + jj) = f64x2{a0, a1};
                } else {
                    if (jj < nj) dst[jj] = a0;
                    if (jj + 1 < nj) dst[jj + 1] = a1;
                }
            }
        }
    }

    // ---- the scene's i rows, IB at a time --------------------------------------
    for (int i0 = 0; i0 < N; i0 += IB) {
        const int ni = min(IB, N - i0);
        // (every wave past the previous chunk's reads of s12 / s12f)
        __syncthreads();
        const bool deg_chunk = s_degc[i0 / IB] != 0;
        const bool nd = !deg_fixed && !deg_chunk;
        bool near_c = near;
        for (int x = t; x < IB * kJ; x += kThreads) {
            const int r = x / kJ, jj = x % kJ;
            const bool v = r < ni && jj < nj;
            const double e = v ? pair(nd, s_c12[jj], s_r12[i0 + r], s_p0[i0 + r][0], s_p0[i0 + r][1],
                                      s_p1[jj][0], s_p1[jj][1])
                               : 0.0;
            s12[r][jj] = e;
            s12f[r][jj] = (float)e;
            near_c &= e <= kApproxResidual;
            if (v) E12[(int64_t)(i0 + r) * ld + jw0 + jj] = e;
        }
        // block minima of a whole chunk: this thread's 16 e13 first (their
        // fp64 lines and e13T stores together, float32 kept in registers),
        // then the 16 rows unrolled so the LDS reads of one row overlap the
        // sums of another
        const bool whole = !G8 && ni == IB;      // uniform
        float f13r[IB];
        if (whole) {
#pragma unroll
            for (int ii = 0; ii < IB; ii += 2) {
                const double a0 = kv ? pair(nd, cl13, s_r13[i0 + ii], s_p0[i0 + ii][0], s_p0[i0 + ii][1], kx, ky) : 0.0;
                const double a1 =
                    kv ? pair(nd, cl13, s_r13[i0 + ii + 1], s_p0[i0 + ii + 1][0], s_p0[i0 + ii + 1][1], kx, ky) : 0.0;
                near_c &= a0 <= kApproxResidual && a1 <= kApproxResidual;
                f13r[ii] = (float)a0;
                f13r[ii + 1] = (float)a1;
                if (jb == 0 && kv) *reinterpret_cast<f64x2 *>(E13T + (int64_t)k * ld + i0 + ii) = f64x2{a0, a1};
            }
        }
        const bool chunk_near = __syncthreads_and(near_c) != 0;
        if (whole && chunk_near) {
#pragma unroll
            for (int ii = 0; ii < IB; ++ii) {
                float v[kJ];
#pragma unroll
                for (int r = 0; r < kJ; r += 4) {
                    const f32x4 w = *reinterpret_cast<const f32x4 *>(&s12f[ii][r]);
                    v[r] = w.x + f23[r];
                    v[r + 1] = w.y + f23[r + 1];
                    v[r + 2] = w.z + f23[r + 2];
                    v[r + 3] = w.w + f23[r + 3];
                }
#pragma unroll
                for (int w = kJ / 2; w >= 1; w /= 2)
#pragma unroll
                    for (int r = 0; r < w; ++r) v[r] = __builtin_fminf(v[r], v[r + w]);
                uint32_t b = __float_as_uint((v[0] + f13r[ii]) * kThirdF);
                const bool ok = !kv || ((b & 0xFFFFu) - kApproxMargin < 0x10000u - 2 * kApproxMargin &&
                                        b >= kApproxTiny);
                if (!ok) {                               // exact: 32 fp64 sums (see the row loop below)
                    const double e13 = pair(nd, cl13, s_r13[i0 + ii], s_p0[i0 + ii][0], s_p0[i0 + ii][1], kx, ky);
                    const double *e23r = E23T + (int64_t)k * ld + jw0;
                    double sm = (double)INFINITY;
#pragma unroll 4
                    for (int jj = 0; jj < kJ; ++jj)
                        sm = fmin(sm, (s12[ii][jj] + e13) + (jj < nj ? e23r[jj] : (double)INFINITY));   // :81
                    b = __float_as_uint((float)third_q(sm));
                }
                s_bm[ii][t] = (uint16_t)((b | 0x80000000u) >> 16);
            }
        }
        for (int ii = 0; ii < ni && !(whole && chunk_near); ++ii) {
            const int i = i0 + ii;
            const double e13 =
                kv ? pair(nd, cl13, s_r13[i], s_p0[i][0], s_p0[i][1], kx, ky) : 0.0;
            if (jb == 0 && kv) E13T[(int64_t)k * ld + i] = e13;
            // every residual of the wave's rows <= kApproxResidual (wave-uniform)
            const bool fast = chunk_near && __all(e13 <= kApproxResidual);
            // the four groups' keys (a group past the view -- all its e23
            // +inf -- is computed and ignored below)
            uint32_t key[kJ / 8];
            uint32_t hmin = 0xFFFFu;             // the block's smallest 16-bit key
            if (!G8 && fast) {
                // the block's minimum over its 32 j at once, the same float32
                // sums and recheck as the groups' below
                const float f13 = (float)e13;
                float v[kJ];
#pragma unroll
                for (int r = 0; r < kJ; r += 4) {
                    const f32x4 w = *reinterpret_cast<const f32x4 *>(&s12f[ii][r]);
                    v[r] = w.x + f23[r];
                    v[r + 1] = w.y + f23[r + 1];
                    v[r + 2] = w.z + f23[r + 2];
                    v[r + 3] = w.w + f23[r + 3];
                }
#pragma unroll
                for (int w = kJ / 2; w >= 1; w /= 2)
#pragma unroll
                    for (int r = 0; r < w; ++r) v[r] = __builtin_fminf(v[r], v[r + w]);
                uint32_t b = __float_as_uint((v[0] + f13) * kThirdF);
                const bool ok = !kv || ((b & 0xFFFFu) - kApproxMargin < 0x10000u - 2 * kApproxMargin &&
                                        b >= kApproxTiny);
                if (!ok) {                               // exact: 32 fp64 sums, e23 from this thread's e23T row
                    const double *e23r = E23T + (int64_t)k * ld + jw0;
                    double sm = (double)INFINITY;
#pragma unroll 4
                    for (int jj = 0; jj < kJ; ++jj)
                        sm = fmin(sm, (s12[ii][jj] + e13) + (jj < nj ? e23r[jj] : (double)INFINITY));   // :81
                    b = __float_as_uint((float)third_q(sm));
                }
                hmin = (b | 0x80000000u) >> 16;
            } else if (fast) {
                const float f13 = (float)e13;
#pragma unroll
                for (int g = 0; g < kJ / 8; ++g) {
                    // float32 sums, each within 3 units of 2^-24 of the exact
                    // (nonnegative) sum: their minimum, + e13 and / 3 lands
                    // within 6 units in the last place of the float32 cost of
                    // the exact minimum.  Its upper 16 bits are
                    // the key's unless the lower 16 lie within kApproxMargin of
                    // a carry, or the value is tiny (subnormal inputs): then
                    // this lane's group is computed exactly below
                    float v[8];
#pragma unroll
                    for (int r = 0; r < 8; r += 4) {
                        const f32x4 w = *reinterpret_cast<const f32x4 *>(&s12f[ii][8 * g + r]);
                        v[r] = w.x + f23[8 * g + r];
                        v[r + 1] = w.y + f23[8 * g + r + 1];
                        v[r + 2] = w.z + f23[8 * g + r + 2];
                        v[r + 3] = w.w + f23[8 * g + r + 3];
                    }
                    const float m = __builtin_fminf(
                        __builtin_fminf(__builtin_fminf(v[0], v[1]), __builtin_fminf(v[2], v[3])),
                        __builtin_fminf(__builtin_fminf(v[4], v[5]), __builtin_fminf(v[6], v[7])));
                    const uint32_t b = __float_as_uint((m + f13) * kThirdF);
                    const bool ok = !kv || 8 * g >= nj ||
                                    ((b & 0xFFFFu) - kApproxMargin < 0x10000u - 2 * kApproxMargin &&
                                     b >= kApproxTiny);
                    key[g] = b | 0x80000000u;
                    if (!ok) {                           // exact: eight fp64 sums
                        double sm = (double)INFINITY;
#pragma unroll 1
                        for (int r = 0; r < 8; ++r) {
                            const int jj = 8 * g + r;
                            sm = fmin(sm, (s12[ii][jj] + e13) + e23_at(jj));   // (e12 + e13) + e23, :81
                        }
                        key[g] = __float_as_uint((float)third_q(sm)) | 0x80000000u;
                    }
                }
            } else {   // a huge / non-finite residual: every entry exactly
#pragma unroll 1
                for (int g = 0; g < kJ / 8; ++g) {
                    uint32_t kk = 0xFFFFFFFFu;
#pragma unroll 1
                    for (int r = 0; r < 8; ++r) {
                        const int jj = 8 * g + r;
                        const double sum = (s12[ii][jj] + e13) + e23_at(jj);
                        double qv = third_q(sum);
                        qv = third_ok(qv) ? qv : sum / 3.0;
                        kk = umin(kk, bm8_key((float)qv));
                    }
                    key[g] = kk;
                }
            }
            if (G8 || !fast) {
#pragma unroll
                for (int g = 0; g < kJ / 8; ++g) {
                    if (8 * g < nj) {            // uniform
                        const uint32_t h = key[g] >> 16;
                        hmin = umin(hmin, h);
                        if (G8 && kv) B8[((int64_t)i * g8 + 4 * jb + g) * P + k] = (uint16_t)h;
                    }
                }
            }
            s_bm[ii][t] = (uint16_t)hmin;
        }
        // the chunk's 16 block minima of column k: one 32-byte run of 16-bit
        // keys (rows past the view 0xFFFF, never a candidate)
        if (kv) {
            uint32_t v[IB / 2];
#pragma unroll
            for (int ii = 0; ii < IB; ii += 2)
                v[ii / 2] = (ii < ni ? (uint32_t)s_bm[ii][t] : 0xFFFFu) |
                            ((ii + 1 < ni ? (uint32_t)s_bm[ii + 1][t] : 0xFFFFu) << 16);
#pragma unroll
            for (int w = 0; w < IB / 2; w += 4)
                *reinterpret_cast<uint4 *>(BM + i0 + 2 * w) = make_uint4(v[w], v[w + 1], v[w + 2], v[w + 3]);
        }
    }
}

int cube_launch(const double *pts_dev, const int64_t *cam_offs_dev, const double *F_dev,
                int32_t n_scenes, int32_t max_n, const int64_t *cube_offs_dev,
                const int64_t *row_offs_dev, float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev, void *workspace_dev,
                size_t workspace_bytes, const mvm_options *opts, hipStream_t s, bool &emitted);

int grid_check(int64_t blocks) {
    if (blocks > kMaxGridBlocks)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                        (long long)blocks);
    return MVM_OK;
}

CubeFusedArgs fused_args(const double *pts, const int64_t *cam_offs, const double *F,
                         const int64_t *cube_offs, const int64_t *row_offs, float *cube,
                         int32_t *argmin, float *minval, int max_n, int ib, int rpw = 8) {
    CubeFusedArgs c{};
    c.pts = pts;
    c.cam_offs = cam_offs;
    c.F = F;
    c.cube_offs = cube_offs;
    c.row_offs = row_offs;
    c.cube = cube;
    c.argmin = argmin;
    c.minval = minval;
    c.j_blocks = (max_n + kWaves * rpw - 1) / (kWaves * rpw);
    c.i_blocks = (max_n + ib - 1) / ib;
    return c;
}

}  // namespace

// ================================================================ C ABI ====
extern "C" {

size_t mvm_triplet_workspace_bytes(int32_t n_scenes, int32_t max_n) {
    if (n_scenes <= 0 || max_n <= 0) return 0;
    const int64_t ld = ((int64_t)max_n + 3) / 4 * 4;
    return (size_t)n_scenes * 3 * (size_t)max_n * (size_t)ld * sizeof(double);
}

int mvm_triplet_cost_argmin_bmin8(const double *pts_dev, const int64_t *cam_offs_dev,
                                  const double *F_dev, int32_t n_scenes, int32_t max_n,
                                  const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                                  float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                                  uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev,
                                  void *workspace_dev, size_t workspace_bytes,
                                  const mvm_options *opts, mvm_stream_t stream) {
    mvm_clear_error();
    if (bmin8_dev && (!bmin8_offs_dev || !cube_dev || !cube_offs_dev))
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "bmin8 needs its offsets and the cube");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    bool emitted = false;
    int st = cube_launch(pts_dev, cam_offs_dev, F_dev, n_scenes, max_n, cube_offs_dev, row_offs_dev,
                         cube_dev, argmin_dev, minval_dev, bmin8_dev, bmin8_offs_dev, workspace_dev,
                         workspace_bytes, opts, s, emitted);
    if (st || !bmin8_dev || emitted || n_scenes == 0 || max_n == 0) return st;
    // rows i per workgroup: >= ~1,024 (i, group, 4 k) items at the largest view
    const int64_t per_i = (int64_t)((max_n + 7) / 8) * ((max_n + 3) / 4);
    const int ir = (int)std::min<int64_t>(max_n, std::max<int64_t>(1, (1024 + per_i - 1) / per_i));
    const int i_blocks = (max_n + ir - 1) / ir;
    const int64_t blocks = (int64_t)n_scenes * i_blocks;
    if ((st = grid_check(blocks))) return st;
    bmin8_from_cube_kernel<<<dim3((unsigned)blocks), dim3(kThreads), 0, s>>>(
        cam_offs_dev, cube_offs_dev, cube_dev, bmin8_dev, bmin8_offs_dev, i_blocks, ir);
    return mvm_check_launch("bmin8_from_cube_kernel");
}

int mvm_triplet_cost_argmin_ex(const double *pts_dev, const int64_t *cam_offs_dev,
                               const double *F_dev, int32_t n_scenes, int32_t max_n,
                               const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                               float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                               void *workspace_dev, size_t workspace_bytes,
                               const mvm_options *opts, mvm_stream_t stream) {
    return mvm_triplet_cost_argmin_bmin8(pts_dev, cam_offs_dev, F_dev, n_scenes, max_n, cube_offs_dev,
                                         row_offs_dev, cube_dev, argmin_dev, minval_dev, nullptr, nullptr,
                                         workspace_dev, workspace_bytes, opts, stream);
}

int mvm_triplet_minima(const double *pts_dev, const int64_t *cam_offs_dev, const double *F_dev,
                       int32_t n_scenes, int32_t max_n, uint16_t *bmin8_dev,
                       const int64_t *bmin8_offs_dev, uint16_t *bm32_dev, const int64_t *bm32_offs_dev,
                       double *resid_dev, size_t resid_bytes, const mvm_options *opts,
                       mvm_stream_t stream) {
    mvm_clear_error();
    mvm_options o;
    int st = mvm_resolve_options(opts, o);
    if (st) return st;
    if (n_scenes < 0 || max_n < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative sizes");
    if (max_n > kChunk)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "mvm_triplet_minima: views of at most %d detections "
                        "(%d given)", kChunk, (int)max_n);
    if (n_scenes == 0 || max_n == 0) return MVM_OK;
    if (!pts_dev || !cam_offs_dev || !F_dev || (bmin8_dev && !bmin8_offs_dev) || !bm32_dev ||
        !bm32_offs_dev || !resid_dev)   // (the 8-row minima are optional)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (((uintptr_t)bm32_dev & 15) != 0)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "bm32 not 16-byte aligned");
    const size_t need = mvm_triplet_workspace_bytes(n_scenes, max_n);
    if (resid_bytes < need)
        return mvm_fail(MVM_ERR_WORKSPACE, "residual workspace %zu bytes < required %zu", resid_bytes, need);
    if (((uintptr_t)resid_dev & 15) != 0)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "residual workspace not 16-byte aligned");
    MinimaArgs a{};
    a.pts = pts_dev;
    a.cam_offs = cam_offs_dev;
    a.F = F_dev;
    a.bmin8 = bmin8_dev;
    a.bmin8_offs = bmin8_offs_dev;
    a.bm32 = bm32_dev;
    a.bm32_offs = bm32_offs_dev;
    a.resid = resid_dev;
    a.ld = (max_n + 3) / 4 * 4;
    a.max_n = max_n;
    a.stride = (int64_t)3 * max_n * a.ld;
    a.j_blocks = (max_n + 31) / 32;
    const int64_t blocks = (int64_t)n_scenes * a.j_blocks;
    if ((st = grid_check(blocks))) return st;
    if (bmin8_dev)
        triplet_minima_kernel<16, true><<<dim3((unsigned)blocks), dim3(kThreads), 0,
                                          reinterpret_cast<hipStream_t>(stream)>>>(a);
    else
        triplet_minima_kernel<16, false><<<dim3((unsigned)blocks), dim3(kThreads), 0,
                                           reinterpret_cast<hipStream_t>(stream)>>>(a);
    return mvm_check_launch("triplet_minima_kernel");
}

}  // extern "C"

namespace {

// the fused kernel at two / four / eight rows per instruction, tiles of IB i
// rows; BM8: it also writes the 8-row minima (not the 48-j tiles' 12-row waves)
template <int IB, bool BM8 = false>
void launch_split(int split, int kpl, bool j48, dim3 grid, dim3 block, hipStream_t s, const CubeFusedArgs &c) {
    if (split == 8) {   // views of <= 32: eight rows per instruction
        if (kpl == 3) triplet_fused_kernel<IB, 8, 8, 3, BM8><<<grid, block, 0, s>>>(c);
        else triplet_fused_kernel<IB, 8, 8, 4, BM8><<<grid, block, 0, s>>>(c);
        return;
    }
    if constexpr (BM8 && IB == 32) {   // not launched (the host's bm8 rule): not instantiated
        return;
    } else if (split == 4) {
        if (j48 && !BM8) {
            triplet_fused_kernel<IB, 12, 4, 3><<<grid, block, 0, s>>>(c);
            return;
        }
        switch (kpl) {
        case 3: triplet_fused_kernel<IB, 8, 4, 3, BM8><<<grid, block, 0, s>>>(c); break;
        case 4: triplet_fused_kernel<IB, 8, 4, 4, BM8><<<grid, block, 0, s>>>(c); break;
        case 5: triplet_fused_kernel<IB, 8, 4, 5, BM8><<<grid, block, 0, s>>>(c); break;
        case 6: triplet_fused_kernel<IB, 8, 4, 6, BM8><<<grid, block, 0, s>>>(c); break;
        case 7: triplet_fused_kernel<IB, 8, 4, 7, BM8><<<grid, block, 0, s>>>(c); break;
        default: triplet_fused_kernel<IB, 8, 4, 8, BM8><<<grid, block, 0, s>>>(c); break;
        }
    } else {
        switch (kpl) {
        case 3: triplet_fused_kernel<IB, 8, 2, 3, BM8><<<grid, block, 0, s>>>(c); break;
        case 4: triplet_fused_kernel<IB, 8, 2, 4, BM8><<<grid, block, 0, s>>>(c); break;
        case 5: triplet_fused_kernel<IB, 8, 2, 5, BM8><<<grid, block, 0, s>>>(c); break;
        case 6: triplet_fused_kernel<IB, 8, 2, 6, BM8><<<grid, block, 0, s>>>(c); break;
        case 7: triplet_fused_kernel<IB, 8, 2, 7, BM8><<<grid, block, 0, s>>>(c); break;
        default: triplet_fused_kernel<IB, 8, 2, 8, BM8><<<grid, block, 0, s>>>(c); break;
        }
    }
}

// every cube path; `emitted`: the launched kernel wrote bmin8 itself
int cube_launch(const double *pts_dev, const int64_t *cam_offs_dev, const double *F_dev,
                int32_t n_scenes, int32_t max_n, const int64_t *cube_offs_dev,
                const int64_t *row_offs_dev, float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev, void *workspace_dev,
                size_t workspace_bytes, const mvm_options *opts, hipStream_t s, bool &emitted) {
    mvm_options o;
    int st = mvm_resolve_options(opts, o);
    if (st) return st;
    if (n_scenes < 0 || max_n < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative sizes");
    if (o.cube_kernel < MVM_CUBE_DEFAULT || o.cube_kernel > MVM_CUBE_GENERIC)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_kernel %d", (int)o.cube_kernel);
    if (o.cube_rows_per_instr != 0 && o.cube_rows_per_instr != 1 && o.cube_rows_per_instr != 2 &&
        o.cube_rows_per_instr != 4 && o.cube_rows_per_instr != 8)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_rows_per_instr %d not 0, 1, 2, 4 or 8",
                        (int)o.cube_rows_per_instr);
    if (o.cube_cols_per_lane != 0 && (o.cube_cols_per_lane < 3 || o.cube_cols_per_lane > 8))
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_cols_per_lane %d not 0 or 3..8",
                        (int)o.cube_cols_per_lane);
    if (o.cube_tile_rows != 0 && o.cube_tile_rows != 16 && o.cube_tile_rows != 32)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_tile_rows %d not 0, 16 or 32", (int)o.cube_tile_rows);
    if (n_scenes == 0 || max_n == 0) return MVM_OK;
    if (!pts_dev || !cam_offs_dev || !F_dev || !row_offs_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (cube_dev && !cube_offs_dev) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube without cube_offs");
    const size_t need = mvm_triplet_workspace_bytes(n_scenes, max_n);
    if (!workspace_dev || workspace_bytes < need)
        return mvm_fail(MVM_ERR_WORKSPACE, "workspace %zu bytes < required %zu", workspace_bytes, need);
    if (((uintptr_t)workspace_dev & 15) != 0)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "workspace not 16-byte aligned");
    const int kernel = o.cube_kernel;

    // the one-workgroup-per-scene kernel: by default up to kSmallAutoMaxN
    // (measured crossover vs the fused four-rows-per-wave form), on request
    // up to its limit; everything in LDS, no workspace pass
    const bool small = kernel == MVM_CUBE_DEFAULT ? max_n <= kSmallAutoMaxN
                                                  : (kernel == MVM_CUBE_SMALL && max_n < kSmallMaxN);
    if (small) {
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
        // rows i per workgroup: the whole scene up to 32 detections, then
        // 16-row blocks (tools/gpu_cube_small.sh)
        c.ib = max_n <= 32 ? max_n : 16;
        c.i_blocks = (max_n + c.ib - 1) / c.ib;
        const size_t lds = small_lds_bytes(max_n, c.ib);
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute(reinterpret_cast<const void *>(&triplet_small_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
        const int64_t blocks = (int64_t)n_scenes * c.i_blocks;
        if ((st = grid_check(blocks))) return st;
        triplet_small_kernel<<<dim3((unsigned)blocks), dim3(kThreads), lds, s>>>(c);
        return mvm_check_launch("triplet_small_kernel");
    }
    if (kernel == MVM_CUBE_DEFAULT || kernel == MVM_CUBE_SMALL || kernel == MVM_CUBE_FUSED) {
        // tiles of 16 (32) i x 32 j; views of <= 32 / <= 64 / <= 128 put
        // eight / four / two (i, j) rows in every wave instruction; 3 k per
        // lane where the view fits them (<= 24 / 48 / 96 / 192 at eight / four
        // / two / one rows per instruction)
        const int want = o.cube_rows_per_instr ? o.cube_rows_per_instr : 8;
        int split = (want >= 8 && max_n <= 4 * (kWave / 8)) ? 8
                  : (want >= 4 && max_n <= kChunk / 4) ? 4 : (want >= 2 && max_n <= kChunk / 2) ? 2 : 1;
        if (o.cube_cols_per_lane == 3) {
            // 3 k per lane forced: fewer rows per instruction until a row's
            // 64 / split lanes hold the view (unless those are forced too);
            // views of more than 256 run the k-chunked kernel, 4 k per lane only
            if (max_n > kChunk)
                return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_cols_per_lane 3: views of %d detections "
                                "take the k-chunked kernel (4 k per lane)", (int)max_n);
            while (split > 1 && max_n > 3 * (kWave / split) && !o.cube_rows_per_instr) split /= 2;
            if (max_n > 3 * (kWave / split))
                return mvm_fail(MVM_ERR_INVALID_ARGUMENT,
                                "cube_cols_per_lane 3: views of %d detections exceed %d k per row",
                                (int)max_n, 3 * (kWave / split));
        }
        int kpl = o.cube_cols_per_lane ? o.cube_cols_per_lane : (max_n <= 3 * (kWave / split) ? 3 : 4);
        if (o.cube_cols_per_lane >= 5) {
            // 5-8 k per lane forced: the split forms only (2 or 4 rows per
            // instruction), the most rows per instruction whose lanes hold the view
            if (max_n > kChunk)
                return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_cols_per_lane %d: views of %d detections "
                                "take the k-chunked kernel (4 k per lane)", kpl, (int)max_n);
            split = 0;
            for (int sp = 4; sp >= 2 && !split; sp /= 2)
                if ((!o.cube_rows_per_instr || o.cube_rows_per_instr == sp) && (kWave / sp) * kpl >= max_n)
                    split = sp;
            if (!split)
                return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cube_cols_per_lane %d: no 2 or 4 rows per "
                                "instruction hold views of %d detections", kpl, (int)max_n);
        } else if (!o.cube_cols_per_lane && !o.cube_rows_per_instr && max_n <= kChunk) {
            // a split form with 5-8 k per lane when it keeps >= 8 % more of the
            // lanes busy than the 3 / 4 k shape (e.g. 130: 2 rows x 5 k, 81%,
            // against 1 row x 3 k, 68%; 100: 4 rows x 7 k, 89%, against 78%)
            double best = (double)max_n / ((kWave / split) * kpl);
            for (int sp = 4; sp >= 2; sp /= 2) {
                const int lpr = kWave / sp, k = (max_n + lpr - 1) / lpr;
                const double u = (double)max_n / (lpr * k);
                if (k >= 5 && k <= 8 && u >= best + 0.08) {
                    best = u;
                    split = sp;
                    kpl = k;
                }
            }
        }
        // views of 33-48 at four rows per instruction and 3 k per lane: tiles
        // of 48 j (12 rows per wave), so a view of 48 fills one tile instead of
        // leaving half of a second 32-wide tile empty
        // (not when the 8-row minima are wanted: the 8-row waves write them,
        // the 12-row ones would leave them to a pass over the cube)
        const bool j48 = split == 4 && kpl == 3 && max_n > kWaves * 8 && !bmin8_dev;
        // i rows per tile: 32 on request in the split forms (ABI 6), and by
        // default at eight rows per instruction (views of <= 32: a tile of
        // 16 i rows of such a view is mostly prologue; 24^3 0.663 -> 0.571,
        // 32^3 0.456 -> 0.426 ms per 2 GB launch)
        const int tile_rows =
            split > 1 && (o.cube_tile_rows == 32 || (o.cube_tile_rows == 0 && split == 8)) ? 32 : 16;
        CubeFusedArgs c = fused_args(pts_dev, cam_offs_dev, F_dev, cube_offs_dev, row_offs_dev,
                                     cube_dev, argmin_dev, minval_dev, max_n, tile_rows, j48 ? 12 : 8);
        c.bmin8 = bmin8_dev;
        c.bmin8_offs = bmin8_offs_dev;
        const int64_t blocks = (int64_t)n_scenes * c.j_blocks * c.i_blocks;
        if ((st = grid_check(blocks))) return st;
        const dim3 grid((unsigned)blocks), block(kThreads);
        if (max_n > kChunk) {
            // views of more than 256: fused tiles walking k in chunks of 256
            triplet_fused_chunked_kernel<16, 8><<<grid, block, 0, s>>>(c);
            return mvm_check_launch("triplet_fused_chunked_kernel");
        }
        if (split > 1) {
            // the 8-row minima from the same kernel, but for the 48-j tiles
            // (12 rows per wave); tiles of 32 i rows at eight rows per
            // instruction, 16 otherwise (the shapes the defaults take)
            const bool bm8 = bmin8_dev && !j48 && tile_rows == (split == 8 ? 32 : 16);
            if (bm8) {
                if (tile_rows == 32) launch_split<32, true>(split, kpl, j48, grid, block, s, c);
                else launch_split<16, true>(split, kpl, j48, grid, block, s, c);
                emitted = true;
            } else if (tile_rows == 32) {
                launch_split<32>(split, kpl, j48, grid, block, s, c);
            } else {
                launch_split<16>(split, kpl, j48, grid, block, s, c);
            }
        } else if (bmin8_dev) {                  // the 8-row minima from the same kernel
            if (kpl == 3) triplet_fused_kernel<16, 8, 1, 3, true><<<grid, block, 0, s>>>(c);
            else triplet_fused_kernel<16, 8, 1, kColsPerLane, true><<<grid, block, 0, s>>>(c);
            emitted = true;
        } else {
            if (kpl == 3) triplet_fused_kernel<16, 8, 1, 3><<<grid, block, 0, s>>>(c);
            else triplet_fused_kernel<16, 8><<<grid, block, 0, s>>>(c);
        }
        return mvm_check_launch("triplet_fused_kernel");
    }
    // workspace forms: the fp64 pair matrices e12, e13, e23 of every scene
    // (pairs (0,1), (0,2), (1,2): F12, F13, F23, process_pose.py:157-159)
    const int64_t ld = ((int64_t)max_n + 3) / 4 * 4;
    const int64_t mat_stride = (int64_t)max_n * ld;
    const int32_t pa[3] = {0, 0, 1}, pb[3] = {1, 2, 2};
    st = mvm_pairwise_residual_f64(pts_dev, cam_offs_dev, F_dev, pa, pb, n_scenes, 3, 3, max_n,
                                   mat_stride, ld, (double *)workspace_dev, reinterpret_cast<mvm_stream_t>(s));
    if (st) return st;
    if (kernel == MVM_CUBE_WORKSPACE && max_n <= kChunk) {
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
        c.j_blocks = (max_n + kWaves * 8 - 1) / (kWaves * 8);
        c.i_blocks = (max_n + 16 - 1) / 16;
        const int64_t blocks = (int64_t)n_scenes * c.j_blocks * c.i_blocks;
        if ((st = grid_check(blocks))) return st;
        triplet_tile_kernel<16, 8><<<dim3((unsigned)blocks), dim3(kThreads), 0, s>>>(c);
        return mvm_check_launch("triplet_tile_kernel");
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
    if ((st = grid_check(blocks))) return st;
    triplet_kernel<kTripletRowsPerWave><<<dim3((unsigned)blocks), dim3(kThreads), 0, s>>>(c);
    return mvm_check_launch("triplet_kernel");
}

}  // namespace

extern "C" int mvm_triplet_cost_argmin(const double *pts_dev, const int64_t *cam_offs_dev,
                                       const double *F_dev, int32_t n_scenes, int32_t max_n,
                                       const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                                       float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                                       void *workspace_dev, size_t workspace_bytes, mvm_stream_t stream) {
    return mvm_triplet_cost_argmin_ex(pts_dev, cam_offs_dev, F_dev, n_scenes, max_n, cube_offs_dev,
                                      row_offs_dev, cube_dev, argmin_dev, minval_dev, workspace_dev,
                                      workspace_bytes, nullptr, stream);
}
