// mvm_lsap.hip — batched rectangular linear-sum assignment on MI355X.
//
// Replaces the reference's association step: match_objects
// (bpc/inference/epipolar_matching.py:100-116) calls
// scipy.optimize.linear_sum_assignment on the (N*M, P) flattened cost cube.
// scipy (pinned 1.14.0) implements Crouse's shortest-augmenting-path
// algorithm; this kernel reproduces it decision for decision (oracle/lsap.py
// restates it and is pinned to scipy and to the reference's golden matches):
//   * a tall matrix is transposed (rows = the short side);
//   * per short-side row, one Dijkstra-like search over the remaining
//     columns, whose scan order is an array initialised in REVERSE column
//     order and shrunk by swap-with-last removal;
//   * per step: r = ((minVal + C[i][j]) - u[i]) - v[j] in fp64 (no FMA),
//     spc[j] = min(spc[j], r); among the columns with the smallest spc the
//     scan keeps the first one in scan order unless a later equal one is
//     unassigned (then the LAST such one);
//   * dual updates u[SR] += minVal - spc[col4row[.]], v[SC] -= minVal - spc[.].
//
// MI355X mapping: one 1024-thread workgroup per problem (scene).  The tall
// cost is transposed once through LDS tiles into the workspace; per-column
// state (spc, v f64; row4col, path, scan position i32) lives in the
// workspace, indexed by column so every scan is a coalesced stream, and the
// scan position array turns the sequential tie rule into an order-free
// reduction: winner = max scan position among the unassigned minima if any,
// else the min scan position among the minima.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "mvmatch.h"
#include "mvm_internal.h"
#include "mvm_lsap_sparse.h"

#pragma clang fp contract(off)

namespace {

constexpr int kLsapThreads = 1024;
constexpr int kLsapWaves = kLsapThreads / 64;
constexpr int kTile = 64;   // transpose tile
constexpr int kScanU = 4;   // columns per thread whose loads are batched in a Dijkstra scan

struct LsapArgs {
    const void *cost;           // float or double (the kernels' CT)
    const int64_t *cost_offs;   // element offset of each problem's matrix
    const int64_t *dims;        // [n][2]: rows, cols (row-major, ld = cols)
    const int64_t *ws_offs;     // byte offset of each problem's workspace
    unsigned char *ws;
    const int64_t *out_offs;    // offset of each problem's min(rows, cols) output pairs
    int64_t *row_ind;
    int64_t *col_ind;
    int32_t *status;            // 0 ok, 1 invalid entries (NaN / -inf), 2 infeasible
    int32_t wave_max_cols;      // problems with max(rows, cols) <= this run in lsap_wave_kernel
    int32_t multi_g;            // > 1: larger problems run in lsap_multi_kernel, G workgroups each
    int32_t mid_max_cols;       // long sides in (wave_max_cols, this]: 256-thread lsap_kernel
    unsigned char *sync;        // per-problem barrier + reduction slots (multi kernel)
    int32_t lds_max_cols;       // long sides in (wave_max_cols, this]: column state in LDS
    int32_t lds_small_cols;     // ... of which those up to this: 256-thread LDS kernel
    int32_t reg_max_cols;       // long sides in (wave_max_cols, this] with short sides <=
                                // kRegMaxShort: lsap_reg_kernel (column state in VGPRs)
    int32_t reg_nc_cap, reg_nr_cap;   // its dynamic LDS sizing (columns, rows)
    int32_t mreg_g;             // > 0: long sides in (mreg_lo, mreg_max_cols] with short sides
                                // <= kRegMaxShort run in lsap_mreg_kernel, mreg_g workgroups each
    int32_t mreg_slots;         // ... in this many co-resident groups of workgroups
    int32_t mreg_lo, mreg_max_cols, mreg_nr_cap;
    int32_t sparse_lo;          // > 0: long sides >= this (lsap_sparse_class) are solved by
                                // the candidate-list kernels (mvm_lsap_sparse.hip)
    const uint16_t *bmin8;      // optional inputs of those kernels (LsapSparseArgs)
    const int64_t *bmin8_offs;
    const int64_t *segs;
};

__device__ __forceinline__ bool in_sparse_class(const LsapArgs &a, int64_t R, int64_t K) {
    return lsap_sparse_class(a.sparse_lo, a.wave_max_cols, R, K);
}

// lsap_reg_kernel's class: short sides up to this (its row state is in LDS)
constexpr int kRegMaxShort = 1024;
constexpr int kRegMaxCols = 4096;      // 512 threads x 8 columns, or 1024 x 4
// (kSparseMinCols, the candidate-list class's default lower bound: mvm_lsap_sparse.h)

__device__ __forceinline__ bool in_reg_class(const LsapArgs &a, int64_t R, int64_t K) {
    const int64_t lng = R > K ? R : K, sht = R > K ? K : R;
    return a.reg_max_cols > 0 && lng > a.wave_max_cols && lng <= a.reg_max_cols &&
           sht <= kRegMaxShort && !in_sparse_class(a, R, K);
}

__device__ __forceinline__ bool in_mreg_class(const LsapArgs &a, int64_t R, int64_t K) {
    const int64_t lng = R > K ? R : K, sht = R > K ? K : R;
    return a.mreg_g > 0 && lng > a.mreg_lo && lng <= a.mreg_max_cols && sht > 0 && sht <= kRegMaxShort &&
           !in_sparse_class(a, R, K);
}

// Column state of lsap_kernel<.., true> in LDS: spc, v (f64), path, row4col,
// pos, rem (i32) = 32 bytes per long-side column.
constexpr int kLdsStateBytes = 32;
constexpr int kLdsMaxCols = 4096;   // 128 KiB + the transpose tile fit the CU's 160 KiB

struct Red {
    double m;      // smallest shortest-path cost seen
    int32_t first; // smallest scan position holding m
    int32_t last_free;   // largest scan position holding m with an unassigned column (-1: none)
};

__device__ __forceinline__ Red red_combine(Red a, Red b) {
    if (b.m < a.m) return b;
    if (a.m < b.m) return a;
    a.first = min(a.first, b.first);
    a.last_free = max(a.last_free, b.last_free);
    return a;
}

// Wave reduction with DPP: four row-local steps (quad_perm [1,0,3,2],
// quad_perm [2,3,0,1], row_half_mirror, row_mirror) leave every lane of a
// 16-lane row with the row's result; the four rows are then combined on the
// scalar unit from v_readlane.  No LDS round trips (a shuffle is a bpermute).
template <int CTRL>
__device__ __forceinline__ Red red_dpp_step(Red r) {
    const uint64_t mb = (uint64_t)__double_as_longlong(r.m);
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)mb, (int)(uint32_t)mb, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(mb >> 32), (int)(uint32_t)(mb >> 32), CTRL,
                                               0xF, 0xF, false);
    Red o;
    o.m = __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
    o.first = __builtin_amdgcn_update_dpp(r.first, r.first, CTRL, 0xF, 0xF, false);
    o.last_free = __builtin_amdgcn_update_dpp(r.last_free, r.last_free, CTRL, 0xF, 0xF, false);
    return red_combine(r, o);
}

__device__ __forceinline__ Red red_readlane(const Red &r, int l) {
    const uint64_t mb = (uint64_t)__double_as_longlong(r.m);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mb, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mb >> 32), l);
    Red o;
    o.m = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    o.first = __builtin_amdgcn_readlane(r.first, l);
    o.last_free = __builtin_amdgcn_readlane(r.last_free, l);
    return o;
}

__device__ __forceinline__ Red red_wave_dpp(Red r) {
    r = red_dpp_step<0xB1>(r);
    r = red_dpp_step<0x4E>(r);
    r = red_dpp_step<0x141>(r);
    r = red_dpp_step<0x140>(r);
    Red a = red_readlane(r, 0);
    a = red_combine(a, red_readlane(r, 16));
    a = red_combine(a, red_readlane(r, 32));
    return red_combine(a, red_readlane(r, 48));
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Layout {
    size_t ct, spc, v, path, row4col, pos, rem, u, col4row, sr, sc, total;
};

__host__ __device__ inline Layout lsap_layout(int64_t nr, int64_t nc, bool transpose, size_t elem) {
    Layout L;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return at;
    };
    L.ct = take(transpose ? (size_t)nr * nc * elem : 0);
    L.spc = take(nc * sizeof(double));
    L.v = take(nc * sizeof(double));
    L.path = take(nc * sizeof(int32_t));
    L.row4col = take(nc * sizeof(int32_t));
    L.pos = take(nc * sizeof(int32_t));
    L.rem = take(nc * sizeof(int32_t));
    L.u = take(nr * sizeof(double));
    L.col4row = take(nr * sizeof(int32_t));
    L.sr = take((nr + 1) * sizeof(int32_t));
    L.sc = take((nr + 1) * sizeof(int32_t));
    L.total = o;
    return L;
}

// LDS: the per-column state lives in LDS instead of the workspace (long
// sides up to kLdsMaxCols): every Dijkstra scan then reads LDS, not L2/MALL.
template <typename CT, int NT, bool LDS = false>
__global__ __launch_bounds__(NT) void lsap_kernel(LsapArgs a) {
    constexpr int kNW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char s_state[];
    constexpr int kU = NT >= 1024 ? kScanU : 2 * kScanU;   // batched loads per thread (VGPR budget)
    constexpr int kT = kTile * 4 / (int)sizeof(CT);        // the same tile bytes for float / double
    __shared__ CT s_tile[kT][kT + 1];
    __shared__ Red s_red[kNW];
    __shared__ int s_flag;
    __shared__ int s_i, s_sink, s_nrem, s_nsr, s_nsc;
    __shared__ double s_min;

    const int t = threadIdx.x;
    const int lane = t % 64, wave = t / 64;
    const int p = blockIdx.x;
    const int64_t R = a.dims[2 * p], K = a.dims[2 * p + 1];
    if (R == 0 || K == 0) {
        if (t == 0) a.status[p] = 0;
        return;
    }
    if ((R > K ? R : K) <= a.wave_max_cols) return;   // solved by lsap_wave_kernel
    if (a.multi_g > 1) return;                         // solved by lsap_multi_kernel
    if (in_reg_class(a, R, K)) return;                 // solved by lsap_reg_kernel
    if (in_mreg_class(a, R, K)) return;                // solved by lsap_mreg_kernel
    if (in_sparse_class(a, R, K)) return;              // solved by the candidate-list kernels
    const int64_t longside = R > K ? R : K;
    // class of the problem: LDS state with 256 threads (long side <= lds_small)
    // or 1024 threads, then workspace state with 256 or 1024 threads
    const int cls = longside <= a.lds_max_cols
                        ? (longside <= a.lds_small_cols ? 0 : 1)
                        : (longside <= a.mid_max_cols ? 2 : 3);
    if (cls != (LDS ? 0 : 2) + (NT < kLsapThreads ? 0 : 1)) return;   // another kernel's
    const bool transpose = K < R;
    const int64_t nr = transpose ? K : R, nc = transpose ? R : K;
    const Layout L = lsap_layout(nr, nc, transpose, sizeof(CT));
    unsigned char *w = a.ws + a.ws_offs[p];
    const CT *C0 = reinterpret_cast<const CT *>(a.cost) + a.cost_offs[p];
    double *spc = reinterpret_cast<double *>(LDS ? s_state : w + L.spc);
    double *v = LDS ? spc + nc : reinterpret_cast<double *>(w + L.v);
    int32_t *path = reinterpret_cast<int32_t *>(LDS ? reinterpret_cast<unsigned char *>(v + nc)
                                                     : w + L.path);
    int32_t *row4col = LDS ? path + nc : reinterpret_cast<int32_t *>(w + L.row4col);
    int32_t *pos = LDS ? row4col + nc : reinterpret_cast<int32_t *>(w + L.pos);
    int32_t *rem = LDS ? pos + nc : reinterpret_cast<int32_t *>(w + L.rem);
    double *u = reinterpret_cast<double *>(w + L.u);
    int32_t *col4row = reinterpret_cast<int32_t *>(w + L.col4row);
    int32_t *sr = reinterpret_cast<int32_t *>(w + L.sr);
    int32_t *sc = reinterpret_cast<int32_t *>(w + L.sc);
    const CT *Ct = transpose ? reinterpret_cast<const CT *>(w + L.ct) : C0;

    // ---- validate (NaN / -inf, as scipy) and transpose a tall matrix -------
    if (t == 0) s_flag = 0;
    __syncthreads();
    int bad = 0;
    if (transpose) {
        CT *Ctw = reinterpret_cast<CT *>(w + L.ct);   // [nr][nc] = C0^T
        for (int64_t r0 = 0; r0 < R; r0 += kT) {
            for (int64_t c0 = 0; c0 < K; c0 += kT) {
                for (int x = t; x < kT * kT; x += NT) {
                    const int rr = x / kT, cc = x % kT;
                    CT val = 0;
                    if (r0 + rr < R && c0 + cc < K) {
                        val = C0[(r0 + rr) * K + c0 + cc];
                        bad |= (val != val) || (val == -INFINITY);
                    }
                    s_tile[rr][cc] = val;
                }
                __syncthreads();
                for (int x = t; x < kT * kT; x += NT) {
                    const int cc = x / kT, rr = x % kT;
                    if (r0 + rr < R && c0 + cc < K) Ctw[(c0 + cc) * nc + r0 + rr] = s_tile[rr][cc];
                }
                __syncthreads();
            }
        }
    } else {
        for (int64_t x = t; x < R * K; x += NT) {
            const CT val = C0[x];
            bad |= (val != val) || (val == -INFINITY);
        }
    }
    if (bad) atomicOr(&s_flag, 1);
    for (int64_t j = t; j < nc; j += NT) {
        v[j] = 0.0;
        row4col[j] = -1;
        path[j] = -1;
    }
    for (int64_t i = t; i < nr; i += NT) {
        u[i] = 0.0;
        col4row[i] = -1;
    }
    __syncthreads();
    if (s_flag) {
        if (t == 0) a.status[p] = 1;
        return;
    }

    // ---- one shortest augmenting path per short-side row --------------------
    for (int cur = 0; cur < nr; ++cur) {
        for (int64_t j = t; j < nc; j += NT) {
            spc[j] = INFINITY;
            pos[j] = (int32_t)(nc - 1 - j);   // scan array starts in reverse column order
            rem[nc - 1 - j] = (int32_t)j;
        }
        if (t == 0) {
            s_i = cur;
            s_sink = -1;
            s_nrem = (int)nc;
            s_nsr = 0;
            s_nsc = 0;
            s_min = 0.0;
        }
        __syncthreads();
        while (true) {
            const int i = s_i;
            const double min_val = s_min;
            const double ui = u[i];
            const CT *Ci = Ct + (int64_t)i * nc;
            Red best{INFINITY, 0x7FFFFFFF, -1};
            // kU columns per thread per batch: all their loads are issued
            // before any is used (a load-use chain per column would serialise
            // the L2 latency)
            for (int64_t jb = t; jb < nc; jb += (int64_t)NT * kU) {
                int32_t pj[kU], r4[kU];
                CT cj[kU];
                double vj[kU], sj[kU];
#pragma unroll
                for (int q = 0; q < kU; ++q) {
                    const int64_t j = jb + (int64_t)q * NT;
                    const int64_t jc = j < nc ? j : jb;
                    pj[q] = pos[jc];
                    cj[q] = Ci[jc];
                    vj[q] = v[jc];
                    sj[q] = spc[jc];
                    r4[q] = row4col[jc];
                    if (j >= nc) pj[q] = -1;
                }
#pragma unroll
                for (int q = 0; q < kU; ++q) {
                    if (pj[q] < 0) continue;   // already visited (removed from the scan)
                    const int64_t j = jb + (int64_t)q * NT;
                    const double r = ((min_val + (double)cj[q]) - ui) - vj[q];
                    double sq = sj[q];
                    if (r < sq) {
                        path[j] = i;
                        spc[j] = r;
                        sq = r;
                    }
                    const bool free_col = r4[q] == -1;
                    if (sq < best.m) {
                        best.m = sq;
                        best.first = pj[q];
                        best.last_free = free_col ? pj[q] : -1;
                    } else if (sq == best.m) {
                        best.first = min(best.first, pj[q]);
                        if (free_col) best.last_free = max(best.last_free, pj[q]);
                    }
                }
            }
            best = red_wave_dpp(best);   // 6% faster than a shuffle butterfly at 576 x 24
            if (lane == 0) s_red[wave] = best;
            __syncthreads();
            if (t == 0) {
                Red r = s_red[0];
                for (int k = 1; k < kNW; ++k) r = red_combine(r, s_red[k]);
                sr[s_nsr++] = i;
                if (r.m == INFINITY) {
                    s_flag = 2;   // infeasible (scipy: "cost matrix is infeasible")
                } else {
                    const int index = r.last_free >= 0 ? r.last_free : r.first;
                    const int j = rem[index];
                    s_min = r.m;
                    if (row4col[j] == -1) {
                        s_sink = j;
                    } else {
                        s_i = row4col[j];
                    }
                    sc[s_nsc++] = j;
                    const int last = rem[--s_nrem];
                    rem[index] = last;
                    pos[last] = index;
                    pos[j] = -1;
                }
            }
            __syncthreads();
            if (s_flag || s_sink >= 0) break;
        }
        if (s_flag) {
            if (t == 0) a.status[p] = 2;
            return;
        }
        // dual updates (each entry independent: order-free)
        const double min_val = s_min;
        for (int k = t; k < s_nsr; k += NT) {
            const int i = sr[k];
            if (i != cur) u[i] += min_val - spc[col4row[i]];
        }
        for (int k = t; k < s_nsc; k += NT) {
            const int j = sc[k];
            v[j] -= min_val - spc[j];
        }
        __syncthreads();
        if (t == 0) {
            u[cur] += min_val;
            int j = s_sink;
            while (true) {   // augment along the path
                const int i = path[j];
                row4col[j] = i;
                const int prev = col4row[i];
                col4row[i] = j;
                j = prev;
                if (i == cur) break;
            }
        }
        __syncthreads();
    }

    // ---- output pairs in scipy's order ------------------------------------
    const int64_t o = a.out_offs[p];
    if (transpose) {
        // (col4row[k], k) sorted by col4row[k] (distinct): rank by counting
        for (int64_t k = t; k < nr; k += NT) {
            const int32_t rk = col4row[k];
            int64_t rank = 0;
            for (int64_t k2 = 0; k2 < nr; ++k2) rank += col4row[k2] < rk;
            a.row_ind[o + rank] = rk;
            a.col_ind[o + rank] = k;
        }
    } else {
        for (int64_t i = t; i < nr; i += NT) {
            a.row_ind[o + i] = i;
            a.col_ind[o + i] = col4row[i];
        }
    }
    if (t == 0) a.status[p] = 0;
}

// ------------------------------------------------ one wave per problem ----
// Problems whose long side fits 64 * kWaveMaxK columns (every scene of a few
// dozen detections: (N*M) x P = 576 x 24 at 24 per view) are solved by ONE
// wave with no workgroup barriers: lane l keeps the per-column state of
// columns l, l + 64, ... in registers (spc, v, path, row4col, scan
// position, SC flag), the row duals u and col4row sit in the wave's LDS slice,
// and every decision is a wave-wide reduction.  Same algorithm and tie rule
// as lsap_kernel (and scipy): the row dual update is driven from the columns
// -- a visited row i != cur is row4col[j] of exactly one visited column j, and
// col4row[i] == j -- so no SR list is needed.
constexpr int kWaveMaxK = 16;              // columns per lane -> long side <= 1024
constexpr int kWaveProblems = 4;           // waves (problems) per workgroup
constexpr int kWaveMaxCols = 64 * kWaveMaxK;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename CT, int K>
__device__ __forceinline__ void lsap_wave_solve(const LsapArgs &a, int p, int64_t R, int64_t Kc, double *u,
                                int32_t *c4r, int lane) {
    const bool transpose = Kc < R;
    const int nr = (int)(transpose ? Kc : R), nc = (int)(transpose ? R : Kc);
    const Layout L = lsap_layout(nr, nc, transpose, sizeof(CT));
    unsigned char *w = a.ws + a.ws_offs[p];
    const CT *C0 = reinterpret_cast<const CT *>(a.cost) + a.cost_offs[p];
    const CT *Ct = transpose ? reinterpret_cast<const CT *>(w + L.ct) : C0;

    // validate (NaN / -inf, as scipy) and transpose a tall matrix
    int bad = 0;
    {
        // kTL loads per lane in flight (32 for the wide classes: 1000 x (576 x 24)
        // 0.195 -> 0.192 ms, 1000 x (900 x 30) 0.316 -> 0.303 ms against 8,
        // profiles/r03/lsap/wave_transpose_loads.log), 32-bit index
        // arithmetic (R * Kc <= 2^20)
        constexpr int kTL = K >= 8 ? 32 : 8;
        CT *Ctw = reinterpret_cast<CT *>(w + L.ct);   // [nr][nc] = C0^T
        const uint32_t total = (uint32_t)(R * Kc), kc = (uint32_t)Kc;
        for (uint32_t x0 = lane; x0 < total; x0 += 64 * kTL) {
            CT val[kTL];
#pragma unroll
            for (int q = 0; q < kTL; ++q) {
                const uint32_t x = x0 + 64u * q;
                val[q] = x < total ? C0[x] : (CT)0;
            }
#pragma unroll
            for (int q = 0; q < kTL; ++q) {
                const uint32_t x = x0 + 64u * q;
                if (x < total) {
                    bad |= (val[q] != val[q]) || (val[q] == -INFINITY);
                    if (transpose) {
                        const uint32_t j = x / kc, i = x - j * kc;
                        Ctw[(int64_t)i * nc + j] = val[q];
                    }
                }
            }
        }
    }
    if (__ballot(bad)) {
        if (lane == 0) a.status[p] = 1;
        return;
    }
    for (int i = lane; i < nr; i += 64) {
        u[i] = 0.0;
        c4r[i] = -1;
    }
    double spc[K], v[K];
    int32_t path[K], r4c[K], pos[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        v[q] = 0.0;
        path[q] = -1;
        r4c[q] = -1;
    }
    wave_sync();

    for (int cur = 0; cur < nr; ++cur) {
        uint32_t insc = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const int j = lane + 64 * q;
            spc[q] = INFINITY;
            pos[q] = j < nc ? nc - 1 - j : -1;   // scan array starts in reverse column order
        }
        int i = cur, nrem = nc, sink = -1;
        double min_val = 0.0;
        while (sink < 0) {
            const double ui = u[i];
            const CT *Ci = Ct + (int64_t)i * nc;
            // all K cost loads first (a load per slot behind the slot's branch
            // would serialise K L2 round trips per step)
            CT cq[K];
#pragma unroll
            for (int q = 0; q < K; ++q) cq[q] = Ci[min(lane + 64 * q, nc - 1)];
            Red best{INFINITY, 0x7FFFFFFF, -1};
#pragma unroll
            for (int q = 0; q < K; ++q) {
                if (pos[q] < 0) continue;
                const double r = ((min_val + (double)cq[q]) - ui) - v[q];
                if (r < spc[q]) {
                    path[q] = i;
                    spc[q] = r;
                }
                const double sj = spc[q];
                const bool free_col = r4c[q] == -1;
                if (sj < best.m) {
                    best.m = sj;
                    best.first = pos[q];
                    best.last_free = free_col ? pos[q] : -1;
                } else if (sj == best.m) {
                    best.first = min(best.first, pos[q]);
                    if (free_col) best.last_free = max(best.last_free, pos[q]);
                }
            }
            best = red_wave_dpp(best);   // 6% faster than a shuffle butterfly at 576 x 24
            if (!(best.m < INFINITY)) {
                if (lane == 0) a.status[p] = 2;   // infeasible
                return;
            }
            const int index = best.last_free >= 0 ? best.last_free : best.first;
            --nrem;
            // the chosen column (scan position index) and the scan array's last
            // one, as per-lane slot masks: data-driven selects only, so the
            // register arrays are never indexed dynamically (no scratch)
            uint32_t jm = 0, lm = 0;
            int32_t r4 = -1, jcol = -1;
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const bool hit = pos[q] == index;
                jm |= hit ? 1u << q : 0u;
                lm |= pos[q] == nrem ? 1u << q : 0u;
                r4 = hit ? r4c[q] : r4;
                jcol = hit ? lane + 64 * q : jcol;
            }
            const int jl = (int)__builtin_ctzll(__ballot(jm != 0));
            const int j = __builtin_amdgcn_readlane(jcol, jl);
            r4 = __builtin_amdgcn_readlane(r4, jl);
            min_val = best.m;
#pragma unroll
            for (int q = 0; q < K; ++q) {
                if (lm & (1u << q)) pos[q] = index;   // remaining[index] = remaining[nrem]
                if (jm & (1u << q)) pos[q] = -1;      // (after: last == j leaves j removed)
            }
            insc |= jm;
            if (r4 == -1) sink = j;
            else i = r4;
        }
        // dual updates
        if (lane == 0) u[cur] += min_val;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            if (insc & (1u << q)) {
                if (r4c[q] != -1) u[r4c[q]] += min_val - spc[q];
                v[q] -= min_val - spc[q];
            }
        }
        wave_sync();
        // augment along the path
        int j = sink;
        while (true) {
            int32_t pj = -1;
#pragma unroll
            for (int q = 0; q < K; ++q) pj = (lane + 64 * q == j) ? path[q] : pj;
            const int i2 = __builtin_amdgcn_readlane(pj, j % 64);
#pragma unroll
            for (int q = 0; q < K; ++q) r4c[q] = (lane + 64 * q == j) ? i2 : r4c[q];
            const int prev = c4r[i2];
            wave_sync();
            if (lane == 0) c4r[i2] = j;
            wave_sync();
            j = prev;
            if (i2 == cur) break;
        }
    }

    // output pairs in scipy's order
    const int64_t o = a.out_offs[p];
    if (transpose) {
        for (int k = lane; k < nr; k += 64) {
            const int32_t rk = c4r[k];
            int rank = 0;
            for (int k2 = 0; k2 < nr; ++k2) rank += c4r[k2] < rk;
            a.row_ind[o + rank] = rk;
            a.col_ind[o + rank] = k;
        }
    } else {
        for (int i = lane; i < nr; i += 64) {
            a.row_ind[o + i] = i;
            a.col_ind[o + i] = c4r[i];
        }
    }
    if (lane == 0) a.status[p] = 0;
}

template <typename CT, int K, int LO = (K > 1 ? 32 * K : 0)>
__global__ __launch_bounds__(64 * kWaveProblems) void lsap_wave_kernel(LsapArgs a, int32_t n) {
    __shared__ double s_u[kWaveProblems][64 * K];      // rows <= long side <= 64 K
    __shared__ int32_t s_c4r[kWaveProblems][64 * K];
    const int lane = threadIdx.x % 64;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const int p = blockIdx.x * kWaveProblems + wave;
    if (p >= n) return;
    const int64_t R = a.dims[2 * p], Kc = a.dims[2 * p + 1];
    const int64_t nc = R > Kc ? R : Kc;
    if (R == 0 || Kc == 0) {               // empty (every kernel class writes the same 0)
        if (lane == 0) a.status[p] = 0;
        return;
    }
    if (nc > a.wave_max_cols) return;
    // each instantiation owns the long sides (LO, 64K]: its own register budget
    if (nc > 64 * K || nc <= LO) return;
    lsap_wave_solve<CT, K>(a, p, R, Kc, s_u[wave], s_c4r[wave], lane);
}


// -------------------------- one workgroup per problem, state in VGPRs ----
// Long sides of 1,025 .. 4,096 columns (the flattened cubes of 33-64
// detections per view: 4096 x 64) with short sides <= kRegMaxShort.  The
// wave kernel's layout over a whole workgroup: thread t keeps the state of
// columns t, t + NT, ... (K of them: spc, v, path, row4col, scan position)
// in registers, so a Dijkstra step reads no column state from memory, only
// the current cost row (coalesced).  Per step every wave reduces its
// candidates with the tie rule (mred_wave: the winner's column and row4col
// travel with it), publishes one record, and after ONE barrier every wave
// combines the NT/64 records in the same order -- no serial thread-0 stage,
// no second barrier (the records alternate between two buffers).  The swap-
// with-last removal is done by the owners of the chosen column and of the
// column at the last scan position.  Row duals and col4row live in LDS;
// augmentation walks the path through an LDS copy of the visited columns'
// path entries, marking each path column with its new row, which the owners
// read back.  Against the LDS-state kernel it needs ~20 B of LDS per column
// instead of 32 B of state read and written every step, and no rem array.
template <typename CT, int NT>
__device__ __forceinline__ bool validate_transpose(const LsapArgs &a, const CT *C0, CT *Ctw,
                                                   int64_t R, int64_t K, int64_t nc, bool transpose,
                                                   CT (*s_tile)[kTile * 4 / sizeof(CT) + 1],
                                                   int *s_flag) {
    constexpr int kT = kTile * 4 / (int)sizeof(CT);
    const int t = threadIdx.x;
    if (t == 0) *s_flag = 0;
    __syncthreads();
    int bad = 0;
    if (transpose) {
        for (int64_t r0 = 0; r0 < R; r0 += kT) {
            for (int64_t c0 = 0; c0 < K; c0 += kT) {
                for (int x = t; x < kT * kT; x += NT) {
                    const int rr = x / kT, cc = x % kT;
                    CT val = 0;
                    if (r0 + rr < R && c0 + cc < K) {
                        val = C0[(r0 + rr) * K + c0 + cc];
                        bad |= (val != val) || (val == -INFINITY);
                    }
                    s_tile[rr][cc] = val;
                }
                __syncthreads();
                for (int x = t; x < kT * kT; x += NT) {
                    const int cc = x / kT, rr = x % kT;
                    if (r0 + rr < R && c0 + cc < K) Ctw[(c0 + cc) * nc + r0 + rr] = s_tile[rr][cc];
                }
                __syncthreads();
            }
        }
    } else {
        for (int64_t x = t; x < R * K; x += NT) {
            const CT val = C0[x];
            bad |= (val != val) || (val == -INFINITY);
        }
    }
    if (bad) atomicOr(s_flag, 1);
    __syncthreads();
    return *s_flag == 0;
}

// --------------------------------------- G workgroups per problem ----
// For few large problems (a single 256^3 scene: 65,536 columns) one CU
// streaming all the column state per Dijkstra step is the bottleneck.  Here G
// co-resident workgroups (cooperative launch) split the columns; each owns a
// contiguous range and its state (spc, v, path, pos, and its SC list).  Per
// step every workgroup scans its range, publishes one reduction record, meets
// the others at a per-problem barrier, and combines the G records in the same
// fixed order, so all keep identical copies of the uniform state (current
// row, minVal, remaining count, sink).  The record also carries what the
// sequential algorithm would read from other columns: the winner's column
// and row4col, and the column holding the last scan position (the
// swap-with-last removal), so pos stays owner-local and no rem array exists.
// Cross-workgroup data (records, u, path, row4col) is published with
// agent-scope fences around the barrier.  Barrier waits are bounded: a
// timeout reports status 3 instead of hanging.
constexpr int kMultiMaxG = 16;
constexpr size_t kSyncBytes = 2304;     // lsap_multi_kernel: counter + flags + 2 x kMultiMaxG
                                        // records; lsap_mreg_kernel: flag + 2 x kMultiMaxG x 8 granules

struct MRed {
    double m;
    int32_t first, first_col, first_r4;   // smallest scan position holding m (+ its column, row4col)
    int32_t last_free, last_free_col;     // largest free scan position holding m (+ column)
    int32_t last_col;                     // column at scan position nrem - 1 (-1: not here)
};

__device__ __forceinline__ MRed mred_combine(MRed a, const MRed &b) {
    const int32_t lc = max(a.last_col, b.last_col);
    if (b.m < a.m) {
        a = b;
    } else if (!(a.m < b.m)) {
        if (b.first < a.first) {
            a.first = b.first;
            a.first_col = b.first_col;
            a.first_r4 = b.first_r4;
        }
        if (b.last_free > a.last_free) {
            a.last_free = b.last_free;
            a.last_free_col = b.last_free_col;
        }
    }
    a.last_col = lc;
    return a;
}

__device__ __forceinline__ MRed mred_wave(MRed r) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        MRed o;
        o.m = __shfl_xor(r.m, off, 64);
        o.first = __shfl_xor(r.first, off, 64);
        o.first_col = __shfl_xor(r.first_col, off, 64);
        o.first_r4 = __shfl_xor(r.first_r4, off, 64);
        o.last_free = __shfl_xor(r.last_free, off, 64);
        o.last_free_col = __shfl_xor(r.last_free_col, off, 64);
        o.last_col = __shfl_xor(r.last_col, off, 64);
        r = mred_combine(r, o);
    }
    return r;
}

struct SyncBlock {
    unsigned int counter;
    int flag;          // 1: invalid entries, 2: infeasible, 3: barrier timeout
    int pad[14];
    MRed slot[2][kMultiMaxG];
};
static_assert(sizeof(SyncBlock) <= kSyncBytes, "sync block too large");
static_assert(kSyncBytes % 256 == 0, "sync blocks stay 256-byte aligned");

// all G workgroups of a problem; returns false on timeout (flag set to 3)
__device__ bool group_barrier(SyncBlock *sb, unsigned int target) {
    __shared__ int s_ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        // agent-scope release (L2 write-back) then arrive; after the wait an
        // agent-scope acquire (this CU's L1 invalidated): one of each, not two
        // full __threadfence()s
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        atomicAdd(&sb->counter, 1u);
        int ok = 1;
        for (long spins = 0;; ++spins) {
            const unsigned int c =
                __hip_atomic_load(&sb->counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c >= target) break;
            if (__hip_atomic_load(&sb->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3 ||
                spins > (1L << 24)) {
                atomicExch(&sb->flag, 3);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_ok = ok;
    }
    __syncthreads();
    return s_ok;
}

// OCC: waves per SIMD to fit (512 threads: 4 -> two workgroups per CU at <= 128 VGPRs)
template <typename CT, int NT, int K, int OCC = (NT == 512 ? 4 : 1)>
__global__ __launch_bounds__(NT, OCC) void lsap_reg_kernel(LsapArgs a) {
    constexpr int kNW = NT / 64;
    constexpr int kT = kTile * 4 / (int)sizeof(CT);
    __shared__ CT s_tile[kT][kT + 1];
    __shared__ Red s_rec[2][kNW];
    __shared__ int s_flag;
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    static_assert(NT * K <= 4096, "scan keys hold 12-bit positions and columns");

    const int t = threadIdx.x, lane = t % 64, wave = t / 64;
    const int p = blockIdx.x;
    const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
    if (R == 0 || Kd == 0) {
        if (t == 0) a.status[p] = 0;
        return;
    }
    if (a.multi_g > 1 || !in_reg_class(a, R, Kd)) return;   // another kernel's problem
    const bool transpose = Kd < R;
    const int nr = (int)(transpose ? Kd : R), nc = (int)(transpose ? R : Kd);
    const Layout L = lsap_layout(nr, nc, transpose, sizeof(CT));
    unsigned char *w = a.ws + a.ws_offs[p];
    const CT *C0 = reinterpret_cast<const CT *>(a.cost) + a.cost_offs[p];
    const CT *Ct = transpose ? reinterpret_cast<const CT *>(w + L.ct) : C0;
    // LDS: row duals and col4row [reg_nr_cap], per column path and row4col [reg_nc_cap]
    double *u = reinterpret_cast<double *>(s_dyn);
    int32_t *c4r = reinterpret_cast<int32_t *>(u + a.reg_nr_cap);
    int32_t *s_path = c4r + a.reg_nr_cap;
    int32_t *s_r4c = s_path + a.reg_nc_cap;

    if (!validate_transpose<CT, NT>(a, C0, reinterpret_cast<CT *>(w + L.ct), R, Kd, nc, transpose,
                                    s_tile, &s_flag)) {
        if (t == 0) a.status[p] = 1;
        return;
    }
    for (int i = t; i < nr; i += NT) {
        u[i] = 0.0;
        c4r[i] = -1;
    }
    for (int j = t; j < nc; j += NT) s_r4c[j] = -1;
    // per column, in registers: spc, v, scan position; bit q of `freem`:
    // column t + NT*q has no row yet (row4col == -1)
    double spc[K], v[K];
    int32_t pos[K];
    uint32_t freem = (1u << K) - 1;
#pragma unroll
    for (int q = 0; q < K; ++q) v[q] = 0.0;
    int par = 0;
    for (int cur = 0; cur < nr; ++cur) {
        uint32_t insc = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const int j = t + NT * q;
            spc[q] = INFINITY;
            pos[q] = j < nc ? nc - 1 - j : -1;   // scan array starts in reverse column order
        }
        int i = cur, sink = -1, nrem = nc;
        double min_val = 0.0;
        __syncthreads();                          // u / c4r / s_r4c of the previous row are in place
        while (sink < 0) {
            const double ui = u[i];
            const CT *Ci = Ct + (int64_t)i * nc;
            CT cq[K];
#pragma unroll
            for (int q = 0; q < K; ++q) cq[q] = Ci[min(t + NT * q, nc - 1)];   // all loads first
            // candidates keyed (scan position << 12 | column): positions are
            // unique, so the smallest key is the first minimum in scan order
            // and the largest free key the last free one -- the wave kernel's
            // Red and its DPP reduction carry the columns along
            Red best{INFINITY, 0x7FFFFFFF, -1};
#pragma unroll
            for (int q = 0; q < K; ++q) {
                if (pos[q] < 0) continue;         // visited, or past the columns
                const int32_t j = t + NT * q;
                const double r = ((min_val + (double)cq[q]) - ui) - v[q];
                if (r < spc[q]) {
                    s_path[j] = i;
                    spc[q] = r;
                }
                const double sq = spc[q];
                const int32_t key = (pos[q] << 12) | j;
                const bool fr = (freem >> q) & 1u;
                if (sq < best.m) {
                    best.m = sq;
                    best.first = key;
                    best.last_free = fr ? key : -1;
                } else if (sq == best.m) {
                    best.first = min(best.first, key);
                    if (fr) best.last_free = max(best.last_free, key);
                }
            }
            best = red_wave_dpp(best);
            if (lane == 0) s_rec[par][wave] = best;
            __syncthreads();
            // every wave combines the kNW records: lane k < kNW reads record k,
            // DPP steps over those lanes (the combine is commutative and
            // associative), so every wave holds the same result
            Red r{INFINITY, 0x7FFFFFFF, -1};
            if (lane < kNW) r = s_rec[par][lane];
            r = red_dpp_step<0xB1>(r);
            r = red_dpp_step<0x4E>(r);
            if (kNW > 4) r = red_dpp_step<0x141>(r);
            if (kNW > 8) r = red_dpp_step<0x140>(r);
            r = red_readlane(r, 0);
            par ^= 1;
            if (!(r.m < INFINITY)) {              // uniform over the workgroup
                if (t == 0) a.status[p] = 2;      // infeasible
                return;
            }
            const int32_t key = r.last_free >= 0 ? r.last_free : r.first;
            const int32_t index = key >> 12, j = key & 0xFFF;
            const int32_t r4 = r.last_free >= 0 ? -1 : s_r4c[j];
            --nrem;
#pragma unroll
            for (int q = 0; q < K; ++q) {         // swap-with-last removal, by the owners
                if (pos[q] == nrem) pos[q] = index;   // the last scan position moves to index
                if (t + NT * q == j) {                // (after: last == j leaves j removed)
                    pos[q] = -1;
                    insc |= 1u << q;
                }
            }
            min_val = r.m;
            if (r4 == -1) sink = j;
            else i = r4;
        }
        // dual updates, column-driven: a visited row i != cur is row4col[j] of
        // exactly one visited column j; cur itself has no column yet
#pragma unroll
        for (int q = 0; q < K; ++q) {
            if (insc & (1u << q)) {
                const int32_t ri = s_r4c[t + NT * q];
                if (ri != -1) u[ri] += min_val - spc[q];
                v[q] -= min_val - spc[q];
            }
        }
        if (t == 0) u[cur] += min_val;
        __syncthreads();
        if (t == 0) {                             // augment along the path
            int j = sink;
            while (true) {
                const int i2 = s_path[j];
                s_r4c[j] = i2;
                const int prev = c4r[i2];
                c4r[i2] = j;
                j = prev;
                if (i2 == cur) break;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < K; ++q)               // path columns (all visited) now have rows
            if ((insc >> q) & 1u) freem &= s_r4c[t + NT * q] == -1 ? ~0u : ~(1u << q);
    }
    __syncthreads();
    // output pairs in scipy's order
    const int64_t o = a.out_offs[p];
    if (transpose) {
        for (int k = t; k < nr; k += NT) {
            const int32_t rk = c4r[k];
            int rank = 0;
            for (int k2 = 0; k2 < nr; ++k2) rank += c4r[k2] < rk;
            a.row_ind[o + rank] = rk;
            a.col_ind[o + rank] = k;
        }
    } else {
        for (int k = t; k < nr; k += NT) {
            a.row_ind[o + k] = k;
            a.col_ind[o + k] = c4r[k];
        }
    }
    if (t == 0) a.status[p] = 0;
}

template <typename CT>
__global__ __launch_bounds__(kLsapThreads) void lsap_multi_kernel(LsapArgs a, int32_t n) {
    constexpr int kT = kTile * 4 / (int)sizeof(CT);
    __shared__ CT s_tile[kT][kT + 1];
    __shared__ MRed s_red[kLsapWaves];
    __shared__ MRed s_win;
    __shared__ int s_bad;
    __shared__ int s_nsc;
    __shared__ int32_t s_sc[4096];           // this workgroup's visited columns (SC)

    const int G = a.multi_g;
    // keep a problem's G workgroups on one XCD (dispatch order round-robins
    // workgroups over the 8 XCDs): p's workgroups are b = xcd + 8 * (q*G + g)
    const int b = blockIdx.x, xcd = b % 8, qg = b / 8;
    const int p = xcd + 8 * (qg / G), g = qg % G;
    if (p >= n) return;
    const int t = threadIdx.x, lane = t % 64, wave = t / 64;
    const int64_t R = a.dims[2 * p], K = a.dims[2 * p + 1];
    if (R == 0 || K == 0 || (R > K ? R : K) <= a.wave_max_cols) return;
    if (in_mreg_class(a, R, K)) return;                // solved by lsap_mreg_kernel
    if (in_sparse_class(a, R, K)) return;              // solved by the candidate-list kernels
    const bool transpose = K < R;
    const int64_t nr = transpose ? K : R, nc = transpose ? R : K;
    const int64_t c0 = nc * g / G, c1 = nc * (g + 1) / G;   // owned columns [c0, c1)
    const Layout L = lsap_layout(nr, nc, transpose, sizeof(CT));
    unsigned char *w = a.ws + a.ws_offs[p];
    const CT *C0 = reinterpret_cast<const CT *>(a.cost) + a.cost_offs[p];
    double *spc = reinterpret_cast<double *>(w + L.spc);
    double *v = reinterpret_cast<double *>(w + L.v);
    int32_t *path = reinterpret_cast<int32_t *>(w + L.path);
    int32_t *row4col = reinterpret_cast<int32_t *>(w + L.row4col);
    int32_t *pos = reinterpret_cast<int32_t *>(w + L.pos);
    double *u = reinterpret_cast<double *>(w + L.u);
    int32_t *col4row = reinterpret_cast<int32_t *>(w + L.col4row);
    const CT *Ct = transpose ? reinterpret_cast<const CT *>(w + L.ct) : C0;
    SyncBlock *sb = reinterpret_cast<SyncBlock *>(a.sync + (size_t)p * kSyncBytes);
    unsigned int gen = 0;

    // ---- validate, transpose the owned columns, init owned state ----------
    if (t == 0) s_bad = 0;
    __syncthreads();
    int bad = 0;
    if (transpose) {
        CT *Ctw = reinterpret_cast<CT *>(w + L.ct);   // [nr][nc] = C0^T
        for (int64_t r0 = c0; r0 < c1; r0 += kT) {             // rows of C0 = owned columns
            for (int64_t cc0 = 0; cc0 < K; cc0 += kT) {
                for (int x = t; x < kT * kT; x += kLsapThreads) {
                    const int rr = x / kT, cc = x % kT;
                    CT val = 0;
                    if (r0 + rr < c1 && cc0 + cc < K) {
                        val = C0[(r0 + rr) * K + cc0 + cc];
                        bad |= (val != val) || (val == -INFINITY);
                    }
                    s_tile[rr][cc] = val;
                }
                __syncthreads();
                for (int x = t; x < kT * kT; x += kLsapThreads) {
                    const int cc = x / kT, rr = x % kT;
                    if (r0 + rr < c1 && cc0 + cc < K) Ctw[(cc0 + cc) * nc + r0 + rr] = s_tile[rr][cc];
                }
                __syncthreads();
            }
        }
    } else {
        for (int64_t i = 0; i < R; ++i)
            for (int64_t j = c0 + t; j < c1; j += kLsapThreads) {
                const CT val = C0[i * K + j];
                bad |= (val != val) || (val == -INFINITY);
            }
    }
    if (bad) atomicOr(&s_bad, 1);
    for (int64_t j = c0 + t; j < c1; j += kLsapThreads) {
        v[j] = 0.0;
        row4col[j] = -1;
        path[j] = -1;
    }
    if (g == 0)
        for (int64_t i = t; i < nr; i += kLsapThreads) {
            u[i] = 0.0;
            col4row[i] = -1;
        }
    __syncthreads();
    if (t == 0 && s_bad) atomicOr(&sb->flag, 1);
    if (!group_barrier(sb, (++gen) * G)) goto timeout;
    if (__hip_atomic_load(&sb->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
        if (g == 0 && t == 0) a.status[p] = 1;
        return;
    }

    for (int cur = 0; cur < nr; ++cur) {
        for (int64_t j = c0 + t; j < c1; j += kLsapThreads) {
            spc[j] = INFINITY;
            pos[j] = (int32_t)(nc - 1 - j);   // scan array starts in reverse column order
        }
        if (t == 0) s_nsc = 0;
        int i = cur, sink = -1, step = 0;
        int64_t nrem = nc;
        double min_val = 0.0;
        __syncthreads();
        while (sink < 0) {
            const double ui = u[i];
            const CT *Ci = Ct + (int64_t)i * nc;
            MRed best{INFINITY, 0x7FFFFFFF, -1, -1, -1, -1, -1};
            for (int64_t jb = c0 + t; jb < c1; jb += (int64_t)kLsapThreads * kScanU) {
                int32_t pj[kScanU], r4[kScanU];
                CT cj[kScanU];
                double vj[kScanU], sj[kScanU];
#pragma unroll
                for (int q = 0; q < kScanU; ++q) {     // all loads first
                    const int64_t j = jb + (int64_t)q * kLsapThreads;
                    const int64_t jc = j < c1 ? j : jb;
                    pj[q] = pos[jc];
                    cj[q] = Ci[jc];
                    vj[q] = v[jc];
                    sj[q] = spc[jc];
                    r4[q] = row4col[jc];
                    if (j >= c1) pj[q] = -1;
                }
#pragma unroll
                for (int q = 0; q < kScanU; ++q) {
                    if (pj[q] < 0) continue;
                    const int64_t j = jb + (int64_t)q * kLsapThreads;
                    if (pj[q] == nrem - 1) best.last_col = (int32_t)j;
                    const double r = ((min_val + (double)cj[q]) - ui) - vj[q];
                    double sq = sj[q];
                    if (r < sq) {
                        path[j] = i;
                        spc[j] = r;
                        sq = r;
                    }
                    if (sq < best.m) {
                        best.m = sq;
                        best.first = pj[q];
                        best.first_col = (int32_t)j;
                        best.first_r4 = r4[q];
                        best.last_free = r4[q] == -1 ? pj[q] : -1;
                        best.last_free_col = r4[q] == -1 ? (int32_t)j : -1;
                    } else if (sq == best.m) {
                        if (pj[q] < best.first) {
                            best.first = pj[q];
                            best.first_col = (int32_t)j;
                            best.first_r4 = r4[q];
                        }
                        if (r4[q] == -1 && pj[q] > best.last_free) {
                            best.last_free = pj[q];
                            best.last_free_col = (int32_t)j;
                        }
                    }
                }
            }
            best = mred_wave(best);
            if (lane == 0) s_red[wave] = best;
            __syncthreads();
            if (t == 0) {
                MRed r = s_red[0];
                for (int k = 1; k < kLsapWaves; ++k) r = mred_combine(r, s_red[k]);
                sb->slot[step & 1][g] = r;
            }
            if (!group_barrier(sb, (++gen) * G)) goto timeout;
            if (t == 0) {
                MRed r = sb->slot[step & 1][0];
                for (int k = 1; k < G; ++k) r = mred_combine(r, sb->slot[step & 1][k]);
                s_win = r;
            }
            __syncthreads();
            const MRed r = s_win;
            ++step;
            if (!(r.m < INFINITY)) {
                if (g == 0 && t == 0) a.status[p] = 2;   // infeasible
                return;
            }
            const bool use_free = r.last_free >= 0;
            const int32_t index = use_free ? r.last_free : r.first;
            const int32_t j = use_free ? r.last_free_col : r.first_col;
            const int32_t r4 = use_free ? -1 : r.first_r4;
            --nrem;
            if (t == 0) {
                // swap-with-last removal, owner-local; when last == j, j ends removed
                if (r.last_col >= c0 && r.last_col < c1) pos[r.last_col] = index;
                if (j >= c0 && j < c1) {
                    pos[j] = -1;
                    if (s_nsc < 4096) s_sc[s_nsc] = j;
                    ++s_nsc;
                }
            }
            min_val = r.m;
            if (r4 == -1) sink = j;
            else i = r4;
            __syncthreads();
        }
        // dual updates, column-driven: a visited row i != cur is row4col[j] of
        // exactly one visited column j, and col4row[i] == j
        const int nsc = s_nsc;
        if (nsc > 4096) {                      // SC list overflow: cannot happen for nr <= 4096
            if (t == 0) atomicExch(&sb->flag, 3);
            goto timeout;
        }
        for (int k = t; k < nsc; k += kLsapThreads) {
            const int32_t j = s_sc[k];
            const int32_t ri = row4col[j];
            if (ri != -1) u[ri] += min_val - spc[j];
            v[j] -= min_val - spc[j];
        }
        if (g == 0 && t == 0) u[cur] += min_val;
        if (!group_barrier(sb, (++gen) * G)) goto timeout;
        if (g == 0 && t == 0) {      // augment along the path
            int j = sink;
            while (true) {
                const int i2 = path[j];
                row4col[j] = i2;
                const int prev = col4row[i2];
                col4row[i2] = j;
                j = prev;
                if (i2 == cur) break;
            }
        }
        if (!group_barrier(sb, (++gen) * G)) goto timeout;
    }

    if (g == 0) {   // output pairs in scipy's order
        const int64_t o = a.out_offs[p];
        if (transpose) {
            for (int64_t k = t; k < nr; k += kLsapThreads) {
                const int32_t rk = col4row[k];
                int64_t rank = 0;
                for (int64_t k2 = 0; k2 < nr; ++k2) rank += col4row[k2] < rk;
                a.row_ind[o + rank] = rk;
                a.col_ind[o + rank] = k;
            }
        } else {
            for (int64_t i = t; i < nr; i += kLsapThreads) {
                a.row_ind[o + i] = i;
                a.col_ind[o + i] = col4row[i];
            }
        }
        if (t == 0) a.status[p] = 0;
    }
    return;
timeout:
    if (g == 0 && t == 0) a.status[p] = 3;
}

// ------------------ G workgroups per problem, column state in VGPRs ----
// The flattened cubes of 65-256 detections per view (8,192 .. 65,536 x 256):
// lsap_reg_kernel's register layout spread over G co-resident workgroups of
// 512 threads x 8 columns (cooperative launch), persistent over the batch:
// slot s (G workgroups on one XCD) solves the class's problems s, s + slots,
// ...  What the sequential algorithm reads across columns reaches every
// workgroup through ONE exchange per Dijkstra step: each workgroup publishes
// its best candidate record -- keys (scan position << 16 | column), plus the
// row4col and the path STEP of its candidate columns -- and after one
// barrier every wave combines the G records in the same order, so the
// decisions are uniform over the slot.  Each workgroup keeps the step lists
// (row, column, path step, minimum) of the search, so both the row-dual
// update (u[i_k] += minVal - m_(k-1): the chosen column's spc IS the step's
// minimum) and the augmentation walk (path[j_k] = i_(ps_k), col4row[i_s] =
// j_(s-1)) are local replays over replicated row duals and col4row in LDS:
// no global row state, no per-search barrier, no path array in memory.
// Keys: positions and columns below 65,536.  `first` none is ~0u (column 0
// is the only one that can sit at position 65,535); `last_free` none is 0
// (key 0 as the last free minimum is also the first minimum and free: the
// same column and sink either way).
constexpr int kMregNT = 512, kMregK = 8;
constexpr int kMregCols = kMregNT * kMregK;              // columns per workgroup
constexpr int kMregMaxCols = kMultiMaxG * kMregCols;     // 65,536

struct URed {
    double m;
    uint32_t first, last_free;
};

__device__ __forceinline__ URed ured_combine(URed a, const URed &b) {
    if (b.m < a.m) return b;
    if (a.m < b.m) return a;
    a.first = b.first < a.first ? b.first : a.first;
    a.last_free = b.last_free > a.last_free ? b.last_free : a.last_free;
    return a;
}

template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)b, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(b >> 32), (int)(uint32_t)(b >> 32), CTRL,
                                               0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ URed ured_dpp_step(URed r) {
    URed o{dpp64<CTRL>(r.m), dpp32<CTRL>(r.first), dpp32<CTRL>(r.last_free)};
    return ured_combine(r, o);
}

__device__ __forceinline__ URed ured_readlane(const URed &r, int l) {
    const uint64_t mb = (uint64_t)__double_as_longlong(r.m);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mb, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mb >> 32), l);
    return URed{__longlong_as_double((long long)(((uint64_t)hi << 32) | lo)),
                (uint32_t)__builtin_amdgcn_readlane((int)r.first, l),
                (uint32_t)__builtin_amdgcn_readlane((int)r.last_free, l)};
}

__device__ __forceinline__ URed ured_wave(URed r) {
    r = ured_dpp_step<0xB1>(r);
    r = ured_dpp_step<0x4E>(r);
    r = ured_dpp_step<0x141>(r);
    r = ured_dpp_step<0x140>(r);
    URed a = ured_readlane(r, 0);
    a = ured_combine(a, ured_readlane(r, 16));
    a = ured_combine(a, ured_readlane(r, 32));
    return ured_combine(a, ured_readlane(r, 48));
}

// one workgroup's record; ps = path step of `first` | of `last_free` << 16
struct alignas(16) XRed {
    double m;
    uint32_t first, last_free;
    int32_t first_r4;
    uint32_t ps;
    uint32_t pad[2];
};

__device__ __forceinline__ XRed xred_combine(XRed a, const XRed &b) {
    if (b.m < a.m) return b;
    if (a.m < b.m) return a;
    if (b.first < a.first) {
        a.first = b.first;
        a.first_r4 = b.first_r4;
        a.ps = (a.ps & 0xFFFF0000u) | (b.ps & 0xFFFFu);
    }
    if (b.last_free > a.last_free) {
        a.last_free = b.last_free;
        a.ps = (a.ps & 0xFFFFu) | (b.ps & 0xFFFF0000u);
    }
    return a;
}

template <int CTRL>
__device__ __forceinline__ XRed xred_dpp_step(XRed r) {
    XRed o = r;
    o.m = dpp64<CTRL>(r.m);
    o.first = dpp32<CTRL>(r.first);
    o.last_free = dpp32<CTRL>(r.last_free);
    o.first_r4 = (int32_t)dpp32<CTRL>((uint32_t)r.first_r4);
    o.ps = dpp32<CTRL>(r.ps);
    return xred_combine(r, o);
}

// Records travel as tagged granules (MI355X_MICROARCH.md, hand-off R2): each
// 32-bit field is one naturally aligned 8-byte {tag = exchange number, value}
// written by one relaxed agent-scope (sc1, write-through) store; readers poll
// with sc1 loads until every tag matches.  The data is its own flag: no
// counter, no release (L2 write-back) or acquire (L1 invalidate) fence.  Two
// buffers alternate: a workgroup republishes a buffer only after reading the
// records of the exchange in between, which every other workgroup publishes
// only after reading this buffer's.
struct XSync {
    int flag;          // 3: a workgroup timed out waiting for the others
    int pad[63];
    unsigned long long gran[2][kMultiMaxG][8];
};
static_assert(sizeof(XSync) <= kSyncBytes, "sync block too large");
constexpr int kXFields = 6;    // m (2 words), first, last_free, first_r4, ps
constexpr long kSpinLimit = 1L << 24;

// lanes < G of a wave: wait for and read workgroup `lane`'s record of exchange tag
__device__ __forceinline__ bool xsync_read(XSync *sb, int par, int lane, int G, uint32_t tag,
                                           uint32_t (&v)[kXFields]) {
    bool ok = true;
    if (lane < G) {
        unsigned long long *q = &sb->gran[par][lane][0];
        for (long spins = 0;; ++spins) {
            bool all = true;
#pragma unroll
            for (int e = 0; e < kXFields; ++e) {
                const unsigned long long x = __hip_atomic_load(q + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v[e] = (uint32_t)x;
                all &= (uint32_t)(x >> 32) == tag;
            }
            if (all) break;
            if (spins > kSpinLimit ||
                __hip_atomic_load(&sb->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3) {
                atomicExch(&sb->flag, 3);
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return __ballot(!ok) == 0;
}

// lanes e < kXFields of ONE wave: publish field e (one store instruction)
__device__ __forceinline__ void xsync_publish(XSync *sb, int par, int g, int lane, uint32_t tag, uint32_t val) {
    if (lane < kXFields)
        __hip_atomic_store(&sb->gran[par][g][lane], ((unsigned long long)tag << 32) | val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// dynamic LDS of lsap_mreg_kernel for short sides up to cap
__host__ __device__ constexpr size_t mreg_lds_bytes(int cap) {
    return (size_t)kMregCols * 4 + (size_t)cap * 8 + (size_t)(cap + 1) * 8 + (size_t)cap * 4 +
           (size_t)(cap + 1) * 8 + (size_t)(cap + 1) * 2 + (size_t)kMregCols * 2;
}

// C0 rows [r_lo, r_hi) of ncols columns (row-major) -> Ctw[c * ld_out + r]
// through LDS tiles, D tiles' loads in flight at once (the one-tile loop waits
// a full memory latency per 16 KB tile: 0.85 ms of a 256^3 problem on 16
// workgroups).  Returns this thread's invalid-entry flag (NaN / -inf).
template <typename CT, int NT, int D>
__device__ __forceinline__ int transpose_rows(const CT *C0, CT *Ctw, int r_lo, int r_hi, int ncols,
                                              int64_t ld_out, CT (*s_tile)[kTile * 4 / sizeof(CT) + 1]) {
    constexpr int kT = kTile * 4 / (int)sizeof(CT), E = kT * kT / NT;
    static_assert(E * NT == kT * kT, "a tile is E elements per thread");
    const int ntc = (ncols + kT - 1) / kT, ntiles = (r_hi - r_lo + kT - 1) / kT * ntc;
    int bad = 0;
    for (int tb = 0; tb < ntiles; tb += D) {
        // the per-element tile coordinates are recomputed per group (cheap), not
        // hoisted out of the caller's problem loop into spilled registers
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        CT val[D][E];
#pragma unroll
        for (int d = 0; d < D; ++d) {                        // all D tiles' loads first
            const int tt = tb + d;
            const int r0 = r_lo + (tt / ntc) * kT, cc0 = (tt % ntc) * kT;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int x = t + NT * e, rr = x / kT, cc = x % kT;
                val[d][e] = tt < ntiles && r0 + rr < r_hi && cc0 + cc < ncols
                                ? C0[(int64_t)(r0 + rr) * ncols + cc0 + cc] : (CT)0;
            }
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int tt = tb + d;
            if (tt >= ntiles) break;                         // uniform
            const int r0 = r_lo + (tt / ntc) * kT, cc0 = (tt % ntc) * kT;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int x = t + NT * e, rr = x / kT, cc = x % kT;
                bad |= (val[d][e] != val[d][e]) || (val[d][e] == -INFINITY);
                s_tile[rr][cc] = val[d][e];
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int x = t + NT * e, cc = x / kT, rr = x % kT;
                if (r0 + rr < r_hi && cc0 + cc < ncols) Ctw[(int64_t)(cc0 + cc) * ld_out + r0 + rr] = s_tile[rr][cc];
            }
            __syncthreads();
        }
    }
    return bad;
}

template <typename CT>
__global__ __launch_bounds__(kMregNT, 4) void lsap_mreg_kernel(LsapArgs a, int32_t n) {
    constexpr int NT = kMregNT, K = kMregK, kNW = NT / 64;
    constexpr int kT = kTile * 4 / (int)sizeof(CT);
    __shared__ CT s_tile[kT][kT + 1];
    __shared__ URed s_rec[kNW];
    __shared__ int s_flag;
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];

    const int G = a.mreg_g, slots = a.mreg_slots, cap = a.mreg_nr_cap;
    // a slot's G workgroups on one XCD (dispatch round-robins workgroups over the 8)
    const int b = blockIdx.x, xcd = b % 8, qg = b / 8;
    const int slot = xcd + 8 * (qg / G), g = qg % G;
    if (slot >= slots) return;
    const int t = threadIdx.x, lane = t % 64, wave = t / 64;
    // LDS: per owned column row4col and path step; replicated row duals and
    // col4row; the search's step lists (row, column, path step, minimum)
    int32_t *s_r4c = reinterpret_cast<int32_t *>(s_dyn);   // [kMregCols]
    double *s_u = reinterpret_cast<double *>(s_r4c + kMregCols);   // [cap]
    double *s_m = s_u + cap;                                 // [cap + 1]
    int32_t *c4r = reinterpret_cast<int32_t *>(s_m + cap + 1);   // [cap]
    int32_t *s_i = c4r + cap;                                // [cap + 1]
    int32_t *s_j = s_i + cap + 1;                            // [cap + 1]
    uint16_t *s_pk = reinterpret_cast<uint16_t *>(s_j + cap + 1);   // [cap + 1]
    uint16_t *s_ps = s_pk + cap + 1;                         // [kMregCols]
    XSync *sb = reinterpret_cast<XSync *>(a.sync + (size_t)slot * kSyncBytes);
    uint32_t gen = 0;                                        // exchanges so far (the tags)
    int par = 0, kth = 0;
#ifdef MVM_LSAP_PROF   // diagnostic build only: phase times of slot 0's workgroup 0 (100 MHz clock)
    uint64_t pf[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt0 = 0, pt = 0;
    int pst = 0;
#define MREG_PT(k) do { if (t == 0) { const uint64_t n_ = wall_clock64(); pf[k] += n_ - pt; pt = n_; } } while (0)
#else
#define MREG_PT(k) do { } while (0)
#endif

    for (int p = 0; p < n; ++p) {
        const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
        if (!in_mreg_class(a, R, Kd)) continue;
        if (kth++ % slots != slot) continue;
        const bool transpose = Kd < R;
        const int nr = (int)(transpose ? Kd : R), nc = (int)(transpose ? R : Kd);
        const int c0 = (int)((int64_t)nc * g / G), c1 = (int)((int64_t)nc * (g + 1) / G);
        const int own = c1 - c0;
        const Layout L = lsap_layout(nr, nc, transpose, sizeof(CT));
        unsigned char *w = a.ws + a.ws_offs[p];
        const CT *C0 = reinterpret_cast<const CT *>(a.cost) + a.cost_offs[p];
        const CT *Ct = transpose ? reinterpret_cast<const CT *>(w + L.ct) : C0;

        // ---- validate and transpose the owned columns; init --------------
        __syncthreads();                                     // the previous problem's output is read
#ifdef MVM_LSAP_PROF
        if (t == 0) { pt0 = pt = wall_clock64(); pst = 0; for (int z = 0; z < 8; ++z) pf[z] = 0; }
#endif
        if (t == 0) s_flag = 0;
        __syncthreads();
        int bad = 0;
        if (transpose) {                                     // rows of C0 = owned columns
            bad = transpose_rows<CT, NT, (sizeof(CT) == 4 ? 4 : 8)>(C0, reinterpret_cast<CT *>(w + L.ct), c0, c1, nr, nc, s_tile);
        } else {
            for (int i = 0; i < nr; ++i)
                for (int j = c0 + t; j < c1; j += NT) {
                    const CT val = C0[(int64_t)i * nc + j];
                    bad |= (val != val) || (val == -INFINITY);
                }
        }
        if (bad) atomicOr(&s_flag, 1);
        for (int i = t; i < nr; i += NT) {
            s_u[i] = 0.0;
            c4r[i] = -1;
        }
        for (int jl = t; jl < kMregCols; jl += NT) s_r4c[jl] = -1;
        double spc[K], v[K];
        int32_t pos[K];
        uint32_t freem = 0;                                  // bit q: column c0 + t + NT q has no row
#pragma unroll
        for (int q = 0; q < K; ++q) {
            v[q] = 0.0;
            freem |= t + NT * q < own ? 1u << q : 0u;
        }
        __syncthreads();
        {                                                    // any workgroup's entries invalid?
            const uint32_t tag = ++gen;
            if (wave == 0) xsync_publish(sb, par, g, lane, tag, (uint32_t)s_flag);
            uint32_t f[kXFields];
            if (!xsync_read(sb, par, lane, G, tag, f)) goto timeout;
            par ^= 1;
            if (__ballot(lane < G && f[0] != 0u)) {
                if (g == 0 && t == 0) a.status[p] = 1;
                continue;
            }
        }

        // ---- one shortest augmenting path per short-side row -------------
        MREG_PT(0);                                          // validate + transpose + first exchange
        // the next cost row's loads are issued as soon as the row is known: after
        // a step's decision, and for the next search's first row before this
        // search's end work (duals, walk, barrier), which then hides their latency
        CT cq[K];
        auto load_row = [&](int row) {
            const CT *Ci = Ct + (int64_t)row * nc + c0;
            int lim = __builtin_amdgcn_readfirstlane(own > 0 ? own - 1 : 0);   // c0 < nc
            asm volatile("" : "+s"(lim));
#pragma unroll
            for (int q = 0; q < K; ++q) cq[q] = Ci[min(t + NT * q, lim)];
        };
        if (nr > 0) load_row(0);
        for (int cur = 0; cur < nr; ++cur) {
            uint32_t insc = 0;
            // per-search and per-step uniforms are laundered through an SGPR so
            // their per-lane derivatives are recomputed, not held in VGPRs for the
            // whole problem (that hoisting spilled 8 VGPRs)
            int base = __builtin_amdgcn_readfirstlane(nc - 1 - c0);
            asm volatile("" : "+s"(base));
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const int jl = t + NT * q;
                spc[q] = INFINITY;
                pos[q] = jl < own ? base - jl : -1;   // reverse column order
            }
            int i = cur, nrem = nc, k = 0, sink = -1;
            double min_val = 0.0;
            // (the previous row's replay is in place: the barrier after the walk)
            while (true) {
                const double ui = s_u[i];
                URed best{INFINITY, ~0u, 0u};
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    if (pos[q] < 0) continue;                // visited, or past the owned columns
                    const int jl = t + NT * q;
                    const double r = ((min_val + (double)cq[q]) - ui) - v[q];
                    if (r < spc[q]) {
                        s_ps[jl] = (uint16_t)k;
                        spc[q] = r;
                    }
                    const double sq = spc[q];
                    const uint32_t key = ((uint32_t)pos[q] << 16) | (uint32_t)(c0 + jl);
                    const bool fr = (freem >> q) & 1u;
                    if (sq < best.m) {
                        best.m = sq;
                        best.first = key;
                        best.last_free = fr ? key : 0u;
                    } else if (sq == best.m) {
                        best.first = key < best.first ? key : best.first;
                        if (fr && key > best.last_free) best.last_free = key;
                    }
                }
                best = ured_wave(best);
                MREG_PT(1);                                  // row load + scan + wave reduction
                if (lane == 0) s_rec[wave] = best;
                __syncthreads();
                MREG_PT(2);                                  // workgroup barrier
                const uint32_t tag = ++gen;
                if (wave == 0) {                             // publish this workgroup's record
                    URed w{INFINITY, ~0u, 0u};
                    if (lane < kNW) w = s_rec[lane];
                    w = ured_dpp_step<0xB1>(w);
                    w = ured_dpp_step<0x4E>(w);
                    w = ured_dpp_step<0x141>(w);
                    w = ured_readlane(w, 0);
                    uint32_t f_r4 = ~0u, ps = 0u;            // row4col -1 when no candidate
                    if (w.first != ~0u) {
                        const int jl = (int)(w.first & 0xFFFFu) - c0;
                        f_r4 = (uint32_t)s_r4c[jl];
                        ps = s_ps[jl];
                    }
                    if (w.last_free != 0u) ps |= (uint32_t)s_ps[(int)(w.last_free & 0xFFFFu) - c0] << 16;
                    const uint64_t mb = (uint64_t)__double_as_longlong(w.m);
                    const uint32_t val = lane == 0 ? (uint32_t)mb : lane == 1 ? (uint32_t)(mb >> 32)
                                       : lane == 2 ? w.first : lane == 3 ? w.last_free : lane == 4 ? f_r4 : ps;
                    xsync_publish(sb, par, g, lane, tag, val);
                }
                MREG_PT(3);                                  // workgroup record + publish
                // every wave reads and combines the G records: lane l < G holds record l
                uint32_t f[kXFields];
                if (!xsync_read(sb, par, lane, G, tag, f)) goto timeout;
                MREG_PT(4);                                  // waiting for the slot's records
#ifdef MVM_LSAP_PROF
                ++pst;
#endif
                XRed r{INFINITY, ~0u, 0u, -1, 0u, {0u, 0u}};
                if (lane < G) {
                    r.m = __longlong_as_double((long long)(((uint64_t)f[1] << 32) | f[0]));
                    r.first = f[2];
                    r.last_free = f[3];
                    r.first_r4 = (int32_t)f[4];
                    r.ps = f[5];
                }
                r = xred_dpp_step<0xB1>(r);
                r = xred_dpp_step<0x4E>(r);
                if (G > 4) r = xred_dpp_step<0x141>(r);
                if (G > 8) r = xred_dpp_step<0x140>(r);
                {
                    const uint64_t mb = (uint64_t)__double_as_longlong(r.m);
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)mb);
                    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(mb >> 32));
                    r.m = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
                    r.first = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.first);
                    r.last_free = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.last_free);
                    r.first_r4 = __builtin_amdgcn_readfirstlane(r.first_r4);
                    r.ps = (uint32_t)__builtin_amdgcn_readfirstlane((int)r.ps);
                }
                par ^= 1;
                if (!(r.m < INFINITY)) break;                // infeasible (uniform over the slot)
                const bool use_free = r.last_free != 0u;
                const uint32_t key = use_free ? r.last_free : r.first;
                const int index = (int)(key >> 16), j = (int)(key & 0xFFFFu);
                const int r4 = use_free ? -1 : r.first_r4;
                const int psk = (int)(use_free ? r.ps >> 16 : r.ps & 0xFFFFu);
                --nrem;
#pragma unroll
                for (int q = 0; q < K; ++q) {                // swap-with-last removal, by the owners
                    if (pos[q] == nrem) pos[q] = index;
                    if (c0 + t + NT * q == j) {              // (after: last == j leaves j removed)
                        pos[q] = -1;
                        insc |= 1u << q;
                    }
                }
                if (t == 0) {
                    s_i[k] = i;
                    s_j[k] = j;
                    s_pk[k] = (uint16_t)psk;
                    s_m[k] = r.m;
                }
                min_val = r.m;
                if (r4 == -1) {
                    sink = j;
                    break;
                }
                i = r4;
                load_row(i);
                MREG_PT(5);                                  // combine + decision
                if (++k > nr) {                              // a step list overflow cannot happen
                    if (t == 0) atomicExch(&sb->flag, 3);
                    goto timeout;
                }
            }
            if (sink < 0) break;                             // infeasible
            if (cur + 1 < nr) load_row(cur + 1);
#pragma unroll
            for (int q = 0; q < K; ++q) {
                if ((insc >> q) & 1u) v[q] -= min_val - spc[q];
                // the only free column a search visits is its sink, now assigned
                if (c0 + t + NT * q == sink) freem &= ~(1u << q);
            }
            // row duals: u[cur] += minVal; u[i_k] += minVal - spc[col4row[i_k]]
            // with col4row[i_k] = j_(k-1), whose spc is step k-1's minimum (rows
            // distinct: one lane each)
            if (wave == 0)
                for (int kk = 1 + lane; kk <= k; kk += 64) s_u[s_i[kk]] += min_val - s_m[kk - 1];
            if (t == 0) {
                s_u[cur] += min_val;
                // augment: path[j_kk] = i_s (s = its path step); col4row[i_s] was j_(s-1)
                int kk = k;
                while (true) {
                    const int s = s_pk[kk], i2 = s_i[s], jj = s_j[kk];
                    c4r[i2] = jj;
                    if (jj >= c0 && jj < c1) s_r4c[jj - c0] = i2;
                    if (s == 0) break;
                    kk = s - 1;
                }
            }
            __syncthreads();
            MREG_PT(6);                                      // search end: duals, walk
        }
        __syncthreads();
        MREG_PT(7);
#ifdef MVM_LSAP_PROF
        if (t == 0 && g == 0 && slot == 0)
            printf("mreg p=%d G=%d steps=%d total=%lu prep=%lu scan=%lu wgbar=%lu pub=%lu wait=%lu dec=%lu end=%lu\n",
                   p, G, pst, (unsigned long)(pt - pt0), (unsigned long)pf[0], (unsigned long)pf[1],
                   (unsigned long)pf[2], (unsigned long)pf[3], (unsigned long)pf[4], (unsigned long)pf[5],
                   (unsigned long)pf[6]);
#endif
        if (g == 0) {
            bool feasible = true;
            for (int r = 0; r < nr; ++r) feasible &= c4r[r] >= 0;   // uniform LDS reads
            if (!feasible) {
                if (t == 0) a.status[p] = 2;                 // infeasible
                continue;
            }
            const int64_t o = a.out_offs[p];                 // output pairs in scipy's order
            if (transpose) {
                for (int kk = t; kk < nr; kk += NT) {
                    const int32_t rk = c4r[kk];
                    int rank = 0;
                    for (int k2 = 0; k2 < nr; ++k2) rank += c4r[k2] < rk;
                    a.row_ind[o + rank] = rk;
                    a.col_ind[o + rank] = kk;
                }
            } else {
                for (int kk = t; kk < nr; kk += NT) {
                    a.row_ind[o + kk] = kk;
                    a.col_ind[o + kk] = c4r[kk];
                }
            }
            if (t == 0) a.status[p] = 0;
        }
    }
    return;
timeout:
    if (g == 0 && t == 0) {                                  // this and the slot's later problems
        int idx = 0;
        for (int p = 0; p < n; ++p) {
            const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
            if (!in_mreg_class(a, R, Kd)) continue;
            const int me = idx++;
            if (me % slots == slot && me >= kth - 1) a.status[p] = 3;
        }
    }
}

// Launch every kernel class of the batch for cost element type CT.
template <typename CT>
int lsap_launch(LsapArgs a, int32_t n_problems, size_t sync_bytes, int64_t long_min,
                int64_t long_max, int64_t short_max, const mvm_options &o, hipStream_t s) {
    // long sides up to wave_max: the one-wave-per-problem kernel (default
    // 1024, -1 = never, capped at 1024)
    int wave_max = o.lsap_wave_max_cols == 0 ? kWaveMaxCols : o.lsap_wave_max_cols;
    wave_max = wave_max < 0 ? 0 : (wave_max > kWaveMaxCols ? kWaveMaxCols : wave_max);
    a.wave_max_cols = wave_max;
    // long_min / long_max bound max(rows, cols) over the non-empty problems
    // (long_max 0: all empty): kernel classes that cannot have work are not
    // launched.  Every class writes status 0 for empty problems.
    if (long_max < 1) {
        long_min = long_max = 0;
    }
    auto overlaps = [&](int64_t lo, int64_t hi) { return long_max >= lo && long_min <= hi; };
    // candidate-list kernels (mvm_lsap_sparse.hip) for wide problems: long
    // sides >= lsap_sparse_min_cols (default kSparseMinCols), <= 65,536, short
    // sides <= 1,024.  They also write status 0 for the empty problems.
    bool empty_done = false, sparse_all = false;
    {
        const int sp_lo = o.lsap_sparse_min_cols == 0 ? kSparseMinCols
                                                      : (o.lsap_sparse_min_cols < 0 ? 0 : o.lsap_sparse_min_cols);
        const int64_t s_max = short_max < long_max ? short_max : long_max;
        if (sp_lo > 0 && long_max >= sp_lo && long_max > wave_max && s_max >= 1) {
            a.sparse_lo = sp_lo;
            LsapSparseArgs sa{a.cost, a.cost_offs, a.dims, a.ws_offs, a.ws, a.out_offs, a.row_ind,
                              a.col_ind, a.status, sp_lo, wave_max,
                              (int32_t)(s_max < kSpMaxShort ? s_max : kSpMaxShort),
                              a.bmin8, a.bmin8_offs, a.segs,
                              o.lsap_sparse_blocks ? o.lsap_sparse_blocks : kSpTB};
            const int st = sizeof(CT) == 8 ? lsap_sparse_launch_f64(sa, n_problems, long_max, s)
                                            : lsap_sparse_launch_f32(sa, n_problems, long_max, s);
            if (st != MVM_OK) return st;
            empty_done = true;
            // every non-empty problem is the class's: no other class has work
            sparse_all = long_min >= sp_lo && long_min > wave_max && long_max <= kSpMaxCols &&
                         short_max <= kSpMaxShort;
        }
    }
    const dim3 wgrid((unsigned)((n_problems + kWaveProblems - 1) / kWaveProblems));
    const dim3 wblock(64 * kWaveProblems);
    if (wave_max > 0) {
        if (overlaps(0, 64) || (long_max == 0 && !empty_done)) {
            lsap_wave_kernel<CT, 1><<<wgrid, wblock, 0, s>>>(a, n_problems);
            empty_done = true;
        }
        // every instantiation also writes status 0 for the empty problems, so
        // any one launched spares the workgroup kernel's launch for them
        if (wave_max > 64 && overlaps(65, 128)) {
            lsap_wave_kernel<CT, 2><<<wgrid, wblock, 0, s>>>(a, n_problems);
            empty_done = true;
        }
        if (wave_max > 128 && overlaps(129, 256)) {
            lsap_wave_kernel<CT, 4><<<wgrid, wblock, 0, s>>>(a, n_problems);
            empty_done = true;
        }
        if (wave_max > 256 && overlaps(257, 512)) {
            lsap_wave_kernel<CT, 8><<<wgrid, wblock, 0, s>>>(a, n_problems);
            empty_done = true;
        }
        // 12 columns per lane for long sides of 513-768 (576 x 24 at 24
        // detections per view): a quarter fewer slots per Dijkstra step than 16
        if (wave_max > 512 && overlaps(513, 768)) {
            lsap_wave_kernel<CT, 12, 512><<<wgrid, wblock, 0, s>>>(a, n_problems);
            empty_done = true;
        }
        if (wave_max > 768 && overlaps(769, 1024)) {
            lsap_wave_kernel<CT, 16, 768><<<wgrid, wblock, 0, s>>>(a, n_problems);
            empty_done = true;
        }
    }
    const bool big = long_max > wave_max && !sparse_all;   // anything left for the workgroup kernels
    int reg_max = o.lsap_reg_max_cols == 0 ? kRegMaxCols : o.lsap_reg_max_cols;
    reg_max = reg_max < 0 ? 0 : (reg_max > kRegMaxCols ? kRegMaxCols : reg_max);
    a.reg_max_cols = reg_max > wave_max ? reg_max : 0;
    // long sides in (max(wave_max, reg_max), lsap_mreg_max_cols] with short
    // sides <= 1024: G = ceil(long / 4096) workgroups per problem with the
    // column state in registers, persistent slots of G co-resident workgroups
    int mreg_max = o.lsap_mreg_max_cols == 0 ? kMregMaxCols : o.lsap_mreg_max_cols;
    mreg_max = mreg_max < 0 ? 0 : (mreg_max > kMregMaxCols ? kMregMaxCols : mreg_max);
    a.mreg_lo = wave_max > a.reg_max_cols ? wave_max : a.reg_max_cols;
    if (big && mreg_max > a.mreg_lo && overlaps((int64_t)a.mreg_lo + 1, mreg_max)) {
        const int64_t hi = long_max < mreg_max ? long_max : mreg_max;
        const int mg = (int)((hi + kMregCols - 1) / kMregCols);
        const int cap = (int)(long_max < kRegMaxShort ? long_max : kRegMaxShort);
        const size_t lds = mreg_lds_bytes(cap);
        const void *kern = reinterpret_cast<const void *>(&lsap_mreg_kernel<CT>);
        int occ = 0, cus = 0, dev = 0;
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kMregNT, lds) == hipSuccess) {
            // slots in whole groups of 8 (one per XCD): the grid never exceeds co-residency
            const int64_t per_xcd = (int64_t)cus * occ / (8 * mg);
            const int64_t slots = per_xcd * 8 < n_problems ? per_xcd * 8 : n_problems;
            if (slots >= 1) {
                a.mreg_g = mg;
                a.mreg_slots = (int32_t)slots;
                a.mreg_max_cols = mreg_max;
                a.mreg_nr_cap = cap;
                if (hipMemsetAsync(a.sync, 0, sync_bytes, s) != hipSuccess)
                    return mvm_fail(MVM_ERR_HIP, "hipMemsetAsync(lsap sync) failed");
                int32_t n_arg = n_problems;
                void *params[] = {&a, &n_arg};
                const dim3 grid((unsigned)(8 * mg * ((slots + 7) / 8))), block(kMregNT);
                if (hipLaunchCooperativeKernel(kern, grid, block, params, (unsigned)lds, s) != hipSuccess) {
                    (void)hipGetLastError();
                    a.mreg_g = 0;                  // the other classes take these problems
                }
            }
        }
    }
    // Few large problems: G co-resident workgroups per problem (cooperative
    // launch guarantees co-residency).  Default: as many workgroups per
    // problem as the chip holds, up to 16, when that is at least 2; -1 off.
    int G = o.lsap_multi_g == 0 ? -1 : (o.lsap_multi_g < 0 ? 0 : o.lsap_multi_g);
    const int64_t groups8 = ((int64_t)n_problems + 7) / 8;     // problems per XCD slot
    int occ = 0, cus = 0, dev = 0;
    if (G != 0 && G != 1 && big && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(&lsap_multi_kernel<CT>),
                                                     kLsapThreads, 0) == hipSuccess) {
        const int64_t capacity = (int64_t)cus * occ;
        const int64_t fit = capacity / (8 * groups8);
        if (G < 0) G = (int)(fit > kMultiMaxG ? kMultiMaxG : fit);
        if (G > kMultiMaxG) G = kMultiMaxG;
        if ((int64_t)G > fit) G = (int)fit;   // never exceed co-residency
    } else {
        G = 0;
    }
    if (G >= 2 && big) {
        a.multi_g = G;
        if (hipMemsetAsync(a.sync, 0, sync_bytes, s) != hipSuccess)
            return mvm_fail(MVM_ERR_HIP, "hipMemsetAsync(lsap sync) failed");
        int32_t n_arg = n_problems;
        void *params[] = {&a, &n_arg};
        const dim3 grid((unsigned)(8 * G * groups8)), block(kLsapThreads);
        if (hipLaunchCooperativeKernel(reinterpret_cast<const void *>(&lsap_multi_kernel<CT>), grid, block,
                                       params, 0, s) != hipSuccess) {
            (void)hipGetLastError();
            a.multi_g = 0;                     // fall back to one workgroup per problem
        }
    }
    // long sides in (wave_max, lsap_reg_max_cols] with short sides <= 1024:
    // one workgroup per problem with the column state in registers
    if (a.multi_g <= 1 && big && a.reg_max_cols > 0 && overlaps((int64_t)wave_max + 1, a.reg_max_cols)) {
        a.reg_nc_cap = (int32_t)(long_max < a.reg_max_cols ? long_max : a.reg_max_cols);
        a.reg_nr_cap = (int32_t)(long_max < kRegMaxShort ? long_max : kRegMaxShort);
        const size_t lds = (size_t)a.reg_nc_cap * 8 + (size_t)a.reg_nr_cap * 12;
        // 512 threads x 8 columns: ~100 VGPRs, two workgroups per CU
        const bool wide = o.lsap_reg_threads == 1024;
        if (o.lsap_reg_threads != 0 && o.lsap_reg_threads != 512 && !wide)
            return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "lsap_reg_threads %d not 512 or 1024",
                            (int)o.lsap_reg_threads);
        const void *kern = wide ? reinterpret_cast<const void *>(&lsap_reg_kernel<CT, 1024, 4>)
                                : reinterpret_cast<const void *>(&lsap_reg_kernel<CT, 512, 8>);
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
        if (wide)
            lsap_reg_kernel<CT, 1024, 4><<<dim3((unsigned)n_problems), dim3(1024), lds, s>>>(a);
        else
            lsap_reg_kernel<CT, 512, 8><<<dim3((unsigned)n_problems), dim3(512), lds, s>>>(a);
    }
    // one workgroup per problem: 256 threads (8 batched columns per thread) up to
    // lsap_mid_max_cols long-side columns, 1024 threads (4 per thread) above.
    // MI355X: 4096 x 64 problems 4.00 vs 4.36 ms per 1000 with 256 threads;
    // 65536 x 256: 52 vs 80 ms per 200 with 1024 (tools/tune_lsap.py)
    a.mid_max_cols = o.lsap_mid_max_cols ? o.lsap_mid_max_cols : 8192;
    // long sides in (wave_max, lsap_lds_max_cols]: column state in LDS
    int lds_max = o.lsap_lds_max_cols == 0 ? kLdsMaxCols : o.lsap_lds_max_cols;
    lds_max = lds_max < 0 ? 0 : (lds_max > kLdsMaxCols ? kLdsMaxCols : lds_max);
    a.lds_max_cols = lds_max > wave_max ? lds_max : 0;
    a.lds_small_cols = o.lsap_lds_small_cols ? o.lsap_lds_small_cols : 2048;
    if (a.multi_g <= 1 && big && a.lds_max_cols > 0) {
        // dynamic LDS sized for the class's longest side (the batch's when bounded)
        auto lds_for = [&](int64_t hi) {
            return (size_t)(long_max < hi ? long_max : hi) * kLdsStateBytes;
        };
        const int64_t small_hi = a.lds_small_cols < a.lds_max_cols ? a.lds_small_cols : a.lds_max_cols;
        if (small_hi > wave_max && overlaps((int64_t)wave_max + 1, small_hi)) {
            const size_t lds = lds_for(small_hi);
            if (lds > 64 * 1024 &&
                hipFuncSetAttribute(reinterpret_cast<const void *>(&lsap_kernel<CT, 256, true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
            lsap_kernel<CT, 256, true><<<dim3((unsigned)n_problems), dim3(256), lds, s>>>(a);
        }
        const int64_t big_lo = (small_hi > wave_max ? small_hi : wave_max) + 1;
        if (a.lds_max_cols >= big_lo && overlaps(big_lo, a.lds_max_cols)) {
            const size_t lds = lds_for(a.lds_max_cols);
            if (lds > 64 * 1024 &&
                hipFuncSetAttribute(reinterpret_cast<const void *>(&lsap_kernel<CT, kLsapThreads, true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
            lsap_kernel<CT, kLsapThreads, true><<<dim3((unsigned)n_problems), dim3(kLsapThreads), lds, s>>>(a);
        }
    }
    const int64_t lo256 = (int64_t)(a.lds_max_cols > wave_max ? a.lds_max_cols : wave_max) + 1;
    const int64_t hi256 = a.mid_max_cols;
    if (!empty_done || (a.multi_g <= 1 && big && overlaps(lo256, hi256)))
        lsap_kernel<CT, 256><<<dim3((unsigned)n_problems), dim3(256), 0, s>>>(a);
    if (a.multi_g <= 1 && big && long_max > (hi256 > lo256 - 1 ? hi256 : lo256 - 1))
        lsap_kernel<CT, kLsapThreads><<<dim3((unsigned)n_problems), dim3(kLsapThreads), 0, s>>>(a);
    return mvm_check_launch("lsap_kernel");
}

}  // namespace

extern "C" {

int64_t mvm_lsap_plan_ex(int32_t n_problems, const int64_t *rows, const int64_t *cols,
                         int32_t cost_dtype, int64_t *ws_offs, int64_t *out_offs) {
    if (n_problems < 0 || (n_problems > 0 && (!rows || !cols || !ws_offs || !out_offs))) {
        mvm_set_error("mvm_lsap_plan: invalid arguments");
        return -1;
    }
    if (cost_dtype != MVM_F32 && cost_dtype != MVM_F64) {
        mvm_set_error("mvm_lsap_plan: cost_dtype must be MVM_F32 or MVM_F64");
        return -1;
    }
    const size_t elem = cost_dtype == MVM_F64 ? sizeof(double) : sizeof(float);
    int64_t w = 0, o = 0;
    for (int32_t p = 0; p < n_problems; ++p) {
        if (rows[p] < 0 || cols[p] < 0 || rows[p] > 0x7FFFFFFF || cols[p] > 0x7FFFFFFF) {
            mvm_set_error("mvm_lsap_plan: problem dimensions out of range");
            return -1;
        }
        ws_offs[p] = w;
        out_offs[p] = o;
        const bool tr = cols[p] < rows[p];
        const int64_t nr = tr ? cols[p] : rows[p], nc = tr ? rows[p] : cols[p];
        // room for whichever class solves it: the dense layout, or the
        // candidate lists of the wide class (mvm_lsap_sparse.h)
        int64_t need = (rows[p] && cols[p]) ? (int64_t)lsap_layout(nr, nc, tr, elem).total : 0;
        if (rows[p] && cols[p] && nc <= kSpMaxCols && nr <= kSpMaxShort) {
            const int64_t sp = (int64_t)lsap_sparse_layout(nr, nc, elem, tr).total;
            need = sp > need ? sp : need;
        }
        w += need;
        o += rows[p] < cols[p] ? rows[p] : cols[p];
    }
    ws_offs[n_problems] = w;
    out_offs[n_problems] = o;
    // barrier + reduction slots of lsap_multi_kernel, at the END of the workspace
    return w + (int64_t)n_problems * (int64_t)kSyncBytes;
}

int64_t mvm_lsap_plan(int32_t n_problems, const int64_t *rows, const int64_t *cols,
                      int64_t *ws_offs, int64_t *out_offs) {
    return mvm_lsap_plan_ex(n_problems, rows, cols, MVM_F32, ws_offs, out_offs);
}

int mvm_lsap_solve_ex(const void *cost_dev, int32_t cost_dtype, const int64_t *cost_offs_dev,
                      const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                      const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                      int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                      int64_t long_min, int64_t long_max, const mvm_options *opts,
                      mvm_stream_t stream) {
    return mvm_lsap_solve_ex2(cost_dev, cost_dtype, cost_offs_dev, dims_dev, n_problems, ws_offs_dev,
                              out_offs_dev, workspace_dev, workspace_bytes, row_ind_dev, col_ind_dev,
                              status_dev, long_min, long_max, long_max, opts, stream);
}

int mvm_lsap_solve_ex2(const void *cost_dev, int32_t cost_dtype, const int64_t *cost_offs_dev,
                       const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                       const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                       int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                       int64_t long_min, int64_t long_max, int64_t short_max,
                       const mvm_options *opts, mvm_stream_t stream) {
    return mvm_lsap_solve_ex3(cost_dev, cost_dtype, cost_offs_dev, dims_dev, n_problems, ws_offs_dev,
                              out_offs_dev, workspace_dev, workspace_bytes, row_ind_dev, col_ind_dev,
                              status_dev, long_min, long_max, short_max, nullptr, nullptr, nullptr,
                              opts, stream);
}

int mvm_lsap_solve_ex3(const void *cost_dev, int32_t cost_dtype, const int64_t *cost_offs_dev,
                       const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                       const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                       int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                       int64_t long_min, int64_t long_max, int64_t short_max,
                       const uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev,
                       const int64_t *segs_dev, const mvm_options *opts, mvm_stream_t stream) {
    mvm_clear_error();
    mvm_options o;
    int st = mvm_resolve_options(opts, o);
    if (st) return st;
    if (cost_dtype != MVM_F32 && cost_dtype != MVM_F64)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "cost_dtype %d", (int)cost_dtype);
    if (o.lsap_multi_g > kMultiMaxG)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "lsap_multi_g %d > %d", (int)o.lsap_multi_g, kMultiMaxG);
    if (o.lsap_sparse_blocks < 0 || o.lsap_sparse_blocks > 64)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "lsap_sparse_blocks %d not in 0..64",
                        (int)o.lsap_sparse_blocks);
    if (n_problems < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative n_problems");
    if (n_problems == 0) return MVM_OK;
    // one workgroup of up to 1024 threads per problem: the dispatch packet's
    // 32-bit work-item count bounds the batch
    if ((int64_t)n_problems * kLsapThreads > 0xFFFFFFFFLL)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "%d problems in one batch: split it (at most %lld)",
                        (int)n_problems, 0xFFFFFFFFLL / kLsapThreads);
    // cost / row_ind / col_ind may be NULL when every problem is empty
    if (!cost_offs_dev || !dims_dev || !ws_offs_dev || !out_offs_dev || !status_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (!workspace_dev && workspace_bytes)
        return mvm_fail(MVM_ERR_WORKSPACE, "null workspace");
    const size_t sync_bytes = (size_t)n_problems * kSyncBytes;
    if (workspace_bytes < sync_bytes) return mvm_fail(MVM_ERR_WORKSPACE, "workspace smaller than the plan");
    LsapArgs a{cost_dev, cost_offs_dev, dims_dev, ws_offs_dev,
               reinterpret_cast<unsigned char *>(workspace_dev), out_offs_dev, row_ind_dev,
               col_ind_dev, status_dev, 0, 0, 0,
               reinterpret_cast<unsigned char *>(
                   (reinterpret_cast<uintptr_t>(workspace_dev) + workspace_bytes - sync_bytes) &
                   ~(uintptr_t)255),   // at or after the per-problem regions (all 256-aligned)
               0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bmin8_dev, bmin8_offs_dev, segs_dev};
    if (bmin8_dev && (!bmin8_offs_dev || !segs_dev))
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "bmin8 needs its offsets and segment lengths");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (cost_dtype == MVM_F64)
        return lsap_launch<double>(a, n_problems, sync_bytes, long_min, long_max, short_max, o, s);
    return lsap_launch<float>(a, n_problems, sync_bytes, long_min, long_max, short_max, o, s);
}

int mvm_lsap_solve_bounded(const float *cost_dev, const int64_t *cost_offs_dev,
                           const int64_t *dims_dev, int32_t n_problems,
                           const int64_t *ws_offs_dev, const int64_t *out_offs_dev,
                           void *workspace_dev, size_t workspace_bytes, int64_t *row_ind_dev,
                           int64_t *col_ind_dev, int32_t *status_dev, int64_t long_min,
                           int64_t long_max, mvm_stream_t stream) {
    return mvm_lsap_solve_ex(cost_dev, MVM_F32, cost_offs_dev, dims_dev, n_problems, ws_offs_dev,
                             out_offs_dev, workspace_dev, workspace_bytes, row_ind_dev, col_ind_dev,
                             status_dev, long_min, long_max, nullptr, stream);
}

int mvm_lsap_solve(const float *cost_dev, const int64_t *cost_offs_dev, const int64_t *dims_dev,
                   int32_t n_problems, const int64_t *ws_offs_dev, const int64_t *out_offs_dev,
                   void *workspace_dev, size_t workspace_bytes, int64_t *row_ind_dev,
                   int64_t *col_ind_dev, int32_t *status_dev, mvm_stream_t stream) {
    return mvm_lsap_solve_bounded(cost_dev, cost_offs_dev, dims_dev, n_problems, ws_offs_dev,
                                  out_offs_dev, workspace_dev, workspace_bytes, row_ind_dev,
                                  col_ind_dev, status_dev, 1, INT64_MAX, stream);
}

}  // extern "C"
