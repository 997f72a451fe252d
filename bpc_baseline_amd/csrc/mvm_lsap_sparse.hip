// mvm_lsap_sparse.hip — scipy's assignment for wide problems through candidate lists.
//
// Same result as mvm_lsap.hip's kernels (scipy 1.14's shortest augmenting
// path, oracle/lsap.py), different decomposition, for problems whose long
// side L (<= 65,536) is much longer than the short side S (<= 1,024): the
// flattened (N*M, P) cubes of match_objects (epipolar_matching.py:100-116) at
// tens to hundreds of detections per view.  The dense kernels scan all L
// columns at every Dijkstra step (65,536 per step at 256 per view, split over
// 16 workgroups that meet once per step).  Here one workgroup solves a
// problem alone and a step touches only the assigned columns (at most S) and
// one short candidate list, because a column no search has assigned yet has
// v == 0 and an r that is a monotone function of its cost alone (the
// argument and its model: oracle/lsap_sparse.py, checked against scipy's
// restatement in tests/test_lsap_sparse_model.py).  Three launches:
//
//   sp_blockmin_kernel   every cost entry read once (HBM-bound): the minimum
//                        of each 32-column block of each short-side row, as
//                        ordered integer keys; NaN / -inf flag the problem;
//   sp_lists_kernel      one wave per short-side row: theta = the 16th
//                        smallest of the lanes' block minima; the list = every column with
//                        cost <= theta (>= 16 entries, <= 128, else the row
//                        is scanned densely when it is needed);
//   sp_solve_kernel      one 256-thread workgroup per problem: per step the
//                        assigned columns' costs of the visited row (one
//                        gather) and the row's list (one load), one block
//                        reduction, scipy's decision rule.
#include "mvm_lsap_sparse.h"

#include <math.h>
#include <stdint.h>

#include "mvm_device.h"
#include "mvm_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int kSpNT = 256;
constexpr int kSpRowGroups = 16;   // sp_lists_kernel workgroups per problem (4 rows each at a time)

template <typename CT>
struct SpKey;
template <>
struct SpKey<float> {
    using T = uint32_t;
    static constexpr T kMax = 0xFFFFFFFFu;
    // order-preserving integer image of a non-NaN float, with -0 taken as +0
    __device__ static T of(float x) {
        const uint32_t b = __float_as_uint(x + 0.0f);
        return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    }
    __device__ static float val(T k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k); }
    __device__ static float next_up(float x) { return nextafterf(x, INFINITY); }
};
template <>
struct SpKey<double> {
    using T = uint64_t;
    static constexpr T kMax = ~0ull;
    __device__ static T of(double x) {
        const uint64_t b = (uint64_t)__double_as_longlong(x + 0.0);
        return (b >> 63) ? ~b : (b | (1ull << 63));
    }
    __device__ static double val(T k) {
        return __longlong_as_double((long long)((k >> 63) ? (k & ~(1ull << 63)) : ~k));
    }
    __device__ static double next_up(double x) { return nextafter(x, (double)INFINITY); }
};

template <typename CT>
__device__ __forceinline__ bool sp_invalid(CT v) {
    return (v != v) || (v == -(CT)INFINITY);
}

// ---- wave / workgroup reductions (DPP row steps, then the four rows) -------

template <int CTRL>
__device__ __forceinline__ double sp_dpp_f64(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)b, (int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(b >> 32), (int)(uint32_t)(b >> 32), CTRL,
                                               0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

__device__ __forceinline__ double sp_readlane_f64(double x, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// minimum over the wave (values are never NaN), uniform
__device__ __forceinline__ double sp_wave_min(double x) {
    x = fmin(x, sp_dpp_f64<0xB1>(x));
    x = fmin(x, sp_dpp_f64<0x4E>(x));
    x = fmin(x, sp_dpp_f64<0x141>(x));
    x = fmin(x, sp_dpp_f64<0x140>(x));
    return fmin(fmin(sp_readlane_f64(x, 0), sp_readlane_f64(x, 16)),
                fmin(sp_readlane_f64(x, 32), sp_readlane_f64(x, 48)));
}

template <int CTRL>
__device__ __forceinline__ int sp_dpp_i32(int x) {
    return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ int sp_wave_min_i32(int x) {
    x = min(x, sp_dpp_i32<0xB1>(x));
    x = min(x, sp_dpp_i32<0x4E>(x));
    x = min(x, sp_dpp_i32<0x141>(x));
    x = min(x, sp_dpp_i32<0x140>(x));
    return min(min(__builtin_amdgcn_readlane(x, 0), __builtin_amdgcn_readlane(x, 16)),
               min(__builtin_amdgcn_readlane(x, 32), __builtin_amdgcn_readlane(x, 48)));
}

__device__ __forceinline__ float sp_first_lane(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ double sp_first_lane(double x) {
    const long long b = __double_as_longlong(x);
    return __longlong_as_double(((long long)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)b));
}

__device__ __forceinline__ uint32_t sp_wave_max_u32(uint32_t x) {
    x = max(x, (uint32_t)sp_dpp_i32<0xB1>((int)x));
    x = max(x, (uint32_t)sp_dpp_i32<0x4E>((int)x));
    x = max(x, (uint32_t)sp_dpp_i32<0x141>((int)x));
    x = max(x, (uint32_t)sp_dpp_i32<0x140>((int)x));
    return max(max((uint32_t)__builtin_amdgcn_readlane((int)x, 0), (uint32_t)__builtin_amdgcn_readlane((int)x, 16)),
               max((uint32_t)__builtin_amdgcn_readlane((int)x, 32), (uint32_t)__builtin_amdgcn_readlane((int)x, 48)));
}

__device__ __forceinline__ long long sp_wave_max_i64(long long x) {
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_xor(x, o);
        x = y > x ? y : x;
    }
    return x;
}

__device__ __forceinline__ int sp_mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// n / d and n % d for 0 <= n, d < 2^22 from a float reciprocal rd = 1/d: the
// estimate is within one of the quotient, one correction step makes it exact
__device__ __forceinline__ int sp_div(int n, int d, float rd, int &r) {
    int q = (int)((float)n * rd);
    r = n - q * d;
    if (r < 0) {
        --q;
        r += d;
    } else if (r >= d) {
        ++q;
        r -= d;
    }
    return q;
}

// ---- 1. block minima ---------------------------------------------------------

// W[s][j] (short-side row s, long-side column j) of a problem
template <typename CT>
__device__ __forceinline__ CT sp_w(const CT *C0, bool tr, int S, int L, int s, int j) {
    return tr ? C0[(int64_t)j * S + s] : C0[(int64_t)s * L + j];
}

// W[s][j] of problem p, from its cost, or -- a cube-free problem
// (mvm_lsap_solve_resid) -- recomputed from its scene's fp64 pair residuals
// with the cube's own arithmetic (cube_f32, mvm_device.h): column j = i * M +
// jj of the flattened (N*M, P) cube, short-side row s = k, so
// W[k][i M + jj] = float32(((e12[i][jj] + e13T[k][i]) + e23T[k][jj]) / 3),
// the bits mvm_triplet_cost_argmin would have stored at cube[i][jj][k]
template <typename CT>
struct SpSrc {
    const CT *C0;
    const double *e12, *e13t, *e23t;   // e12 != nullptr: the residual form
    int S, L, M, ld;
    float rM;
    bool tr;
    __device__ __forceinline__ CT at(int s, int j) const {
        if (e12) {
            int jj;
            const int i = sp_div(j, M, rM, jj);
            return (CT)cube_f32(e12[i * ld + jj], e13t[s * ld + i], e23t[s * ld + jj]);
        }
        return sp_w(C0, tr, S, L, s, j);
    }
};

// problem p's source; seg = lsap_sparse_seg (the residual form needs it: a
// cube's M), else the residual form is invalid (ok = false)
template <typename CT>
__device__ __forceinline__ SpSrc<CT> sp_src(const LsapSparseArgs &a, int p, bool tr, int S, int L, int seg,
                                            bool &ok) {
    SpSrc<CT> c{};
    c.C0 = reinterpret_cast<const CT *>(a.cost) + (a.cost ? a.cost_offs[p] : 0);
    c.S = S;
    c.L = L;
    c.tr = tr;
    ok = true;
    if (a.resid) {
        ok = seg > 0;
        c.M = seg > 0 ? seg : 1;
        c.rM = 1.0f / (float)c.M;
        c.ld = a.resid_ld;
        c.e12 = a.resid + (int64_t)p * a.resid_stride;
        c.e13t = c.e12 + (int64_t)a.resid_rows * a.resid_ld;
        c.e23t = c.e13t + (int64_t)a.resid_rows * a.resid_ld;
    }
    return c;
}

template <typename CT>
__global__ __launch_bounds__(kSpNT) void sp_blockmin_kernel(LsapSparseArgs a, int32_t n, int32_t tpp) {
    using K = SpKey<CT>;
    using KT = typename K::T;
    constexpr int kKeys = 32768 / (int)sizeof(KT);         // 32 KiB of LDS keys per pass
    constexpr int VW = 16 / (int)sizeof(CT);               // elements per 16-byte load
    __shared__ KT s_key[kKeys];
    const int p = (int)(blockIdx.x / (unsigned)tpp), w = (int)(blockIdx.x % (unsigned)tpp);
    if (p >= n) return;
    const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
    if (!lsap_sparse_class(a.lo, a.wave_max, R, Kd)) return;
    const bool tr = Kd < R;
    const int S = (int)(tr ? Kd : R), L = (int)(tr ? R : Kd);
    if (lsap_sparse_seg(a, p, tr, L)) return;              // sp_bmin8_reduce_kernel's
    const int j0 = w * kSpTileCols;
    if (j0 >= L) return;
    const int j1 = min(j0 + kSpTileCols, L);
    const SpLayout y = lsap_sparse_layout(S, L, sizeof(CT), tr, a.bm32 != nullptr);
    unsigned char *ws = a.ws + a.ws_offs[p];
    KT *bm = reinterpret_cast<KT *>(ws + y.bm);
    const CT *C0 = reinterpret_cast<const CT *>(a.cost) + a.cost_offs[p];
    const int nb = (L + kSpBlock - 1) / kSpBlock;
    int bp = 64;                                           // blocks per LDS pass
    while (bp > 1 && S * bp > kKeys) bp >>= 1;
    const int t = threadIdx.x;
    const int G = S / VW;                                  // 16-byte groups per tall row
    // tall input, whole 16-byte groups, 16-byte aligned, and a group count that
    // divides the workgroup: every thread keeps one group's running minima
    const bool fast = tr && S % VW == 0 && kSpNT % G == 0 &&
                      ((reinterpret_cast<uintptr_t>(C0)) & 15) == 0;
    int bad = 0;
    for (int pj0 = j0; pj0 < j1; pj0 += bp * kSpBlock) {
        const int pj1 = min(pj0 + bp * kSpBlock, j1), nbk = (pj1 - pj0 + kSpBlock - 1) / kSpBlock;
        for (int x = t; x < S * bp; x += kSpNT) s_key[x] = K::kMax;
        __syncthreads();
        if (fast) {
            const int q = kSpNT / G, g = t % G, r0 = t / G, nr = pj1 - pj0;
            KT run[VW];
#pragma unroll
            for (int v = 0; v < VW; ++v) run[v] = K::kMax;
            int cur = r0 >> 5;
            // eight 16-byte loads in flight per thread, then their minima
            for (int rb = r0; rb < nr; rb += 8 * q) {
                uint4 raw[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int r = rb + u * q;
                    raw[u] = r < nr ? *reinterpret_cast<const uint4 *>(C0 + (int64_t)(pj0 + r) * S + g * VW)
                                    : make_uint4(0u, 0u, 0u, 0u);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int r = rb + u * q;
                    if (r >= nr) continue;
                    const int blk = r >> 5;
                    if (blk != cur) {
#pragma unroll
                        for (int v = 0; v < VW; ++v) {
                            atomicMin(&s_key[(g * VW + v) * bp + cur], run[v]);
                            run[v] = K::kMax;
                        }
                        cur = blk;
                    }
                    CT val[VW];
                    *reinterpret_cast<uint4 *>(val) = raw[u];
#pragma unroll
                    for (int v = 0; v < VW; ++v) {
                        bad |= sp_invalid(val[v]);
                        const KT kk = K::of(val[v]);
                        run[v] = kk < run[v] ? kk : run[v];
                    }
                }
            }
            if (r0 < nr) {
#pragma unroll
                for (int v = 0; v < VW; ++v) atomicMin(&s_key[(g * VW + v) * bp + cur], run[v]);
            }
        } else {
            // any layout: one element per thread and step, (row, column) stepped
            // incrementally (no division in the loop)
            const int W = pj1 - pj0;
            const int64_t total = (int64_t)S * W;
            if (tr) {                                      // element e: tall row e / S, s = e % S
                int r = t / S, s = t % S;
                const int dq = kSpNT / S, dr = kSpNT % S;
                for (int64_t e = t; e < total; e += kSpNT) {
                    const CT v = C0[(int64_t)(pj0 + r) * S + s];
                    bad |= sp_invalid(v);
                    atomicMin(&s_key[s * bp + (r >> 5)], K::of(v));
                    r += dq;
                    s += dr;
                    if (s >= S) {
                        s -= S;
                        ++r;
                    }
                }
            } else {                                       // element e: s = e / W, column e % W
                int s = t / W, jj = t % W;
                const int dq = kSpNT / W, dr = kSpNT % W;
                for (int64_t e = t; e < total; e += kSpNT) {
                    const CT v = C0[(int64_t)s * L + pj0 + jj];
                    bad |= sp_invalid(v);
                    atomicMin(&s_key[s * bp + (jj >> 5)], K::of(v));
                    s += dq;
                    jj += dr;
                    if (jj >= W) {
                        jj -= W;
                        ++s;
                    }
                }
            }
        }
        __syncthreads();
        for (int x = t; x < S * nbk; x += kSpNT) {
            const int s = x / nbk, bb = x - s * nbk;
            bm[(int64_t)s * nb + (pj0 / kSpBlock) + bb] = s_key[s * bp + bb];
        }
        __syncthreads();
    }
    bad = __syncthreads_or(bad);
    if (t == 0) reinterpret_cast<int32_t *>(ws + y.flags)[w] = bad;
}

// ---- 1'. block minima from a cube's 8-row minima ------------------------------
// Problem p with lsap_sparse_seg(p) = seg (a cube's M): block (g, jt) is the
// columns g*seg + [32 jt, min(32 jt + 32, seg)), i.e. the 8-row groups 4 jt ..
// 4 jt + 3 of segment g, whose minima mvm_triplet_cost_argmin_bmin8 wrote as
// 16-bit keys (the upper half of the 32-bit key: a lower bound h << 16 of the
// minimum, which is at most (h << 16) | 0xFFFF): 2 B per 8 cost entries are
// read instead of the whole cost.  bm receives that UPPER bound (+inf's key
// at most), so theta = the tb-th smallest over the lanes is still a cost that
// >= tb blocks reach; sp_lists_kernel tests candidates with the lower bound.
// One workgroup per 64 blocks; NaN keys (0) flag the problem.
__device__ __forceinline__ uint32_t sp_b8_upper(uint32_t h) {
    return min((h << 16) | 0xFFFFu, 0xFF800000u);
}

__global__ __launch_bounds__(kSpNT) void sp_bmin8_reduce_kernel(LsapSparseArgs a, int32_t n) {
    constexpr int kKeys = 8448;                            // 33 KiB of LDS keys per pass
    constexpr int kTiles = kSpMaxBlocks / 64;
    __shared__ uint32_t s_key[kKeys];
    const int p = (int)(blockIdx.x / kTiles), w = (int)(blockIdx.x % kTiles);
    if (p >= n) return;
    const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
    if (!lsap_sparse_class(a.lo, a.wave_max, R, Kd)) return;
    const bool tr = Kd < R;
    const int S = (int)(tr ? Kd : R), L = (int)(tr ? R : Kd);
    const int seg = lsap_sparse_seg(a, p, tr, L);
    if (!seg) return;
    const int bps = (seg + 31) / 32, bps8 = (seg + 7) / 8, nb = (L / seg) * bps;
    const int b0 = w * 64;
    if (b0 >= nb) return;
    const int b1 = min(b0 + 64, nb);
    const SpLayout y = lsap_sparse_layout(S, L, sizeof(float), tr);
    unsigned char *ws = a.ws + a.ws_offs[p];
    uint32_t *bm = reinterpret_cast<uint32_t *>(ws + y.bm);
    const uint16_t *B8 = a.bmin8 + a.bmin8_offs[p];
    // LDS keys [column][block], rows of bp + 1 words (the per-(key, block)
    // stores below walk the keys: stride 1 word mod 32 banks)
    int bp = 64;
    while (bp > 1 && S * (bp + 1) > kKeys) bp >>= 1;
    const int RB = bp + 1;
    const int t = threadIdx.x;
    const int G = S / 8;                                   // threads per group row (8 keys each)
    const bool fast = S % 8 == 0 && kSpNT % G == 0 && ((reinterpret_cast<uintptr_t>(B8)) & 15) == 0;
    auto invalid = [](uint32_t h) { return h < 0x8000u; };   // NaN (0); a cube holds no -inf
    int bad = 0;
    for (int pb0 = b0; pb0 < b1; pb0 += bp) {
        const int pb1 = min(pb0 + bp, b1);              // every (key, block < pb1 - pb0) is written below
        // local row x -> its 8-row group, or -1 past the segment's end
        auto group = [&](int x) {
            const int b = pb0 + (x >> 2), u = x & 3;
            const int g = b / bps, jt = b - g * bps;
            return 4 * jt + u < bps8 ? g * bps8 + 4 * jt + u : -1;
        };
        if (fast) {
            // thread: keys 8 g8 .. 8 g8 + 7 of blocks lb = t / G + q m, each
            // block's (up to) four 8-row groups loaded together, two blocks at
            // a time (eight 16-byte loads in flight); one thread per (key, block):
            // plain LDS stores
            const int q = kSpNT / G, g8 = t % G, nbk = pb1 - pb0;
            for (int lb0 = t / G; lb0 < nbk; lb0 += 2 * q) {
                uint4 v[2][4];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int lb = lb0 + h * q;
                        const int r = lb < nbk ? group(4 * lb + u) : -1;
                        v[h][u] = r >= 0 ? *reinterpret_cast<const uint4 *>(B8 + (int64_t)r * S + 8 * g8)
                                         : make_uint4(~0u, ~0u, ~0u, ~0u);
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int lb = lb0 + h * q;
                    if (lb >= nbk) continue;
                    // the four groups' minima per 16-bit lane of each dword
                    uint32_t m[4];
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        uint32_t lo = 0xFFFFu, hi = 0xFFFFu;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const uint32_t x = d == 0 ? v[h][u].x : d == 1 ? v[h][u].y : d == 2 ? v[h][u].z : v[h][u].w;
                            lo = min(lo, x & 0xFFFFu);
                            hi = min(hi, x >> 16);
                        }
                        bad |= invalid(lo) | invalid(hi);
                        m[d] = lo | (hi << 16);
                    }
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        s_key[(8 * g8 + 2 * d) * RB + lb] = m[d] & 0xFFFFu;
                        s_key[(8 * g8 + 2 * d + 1) * RB + lb] = m[d] >> 16;
                    }
                }
            }
        } else {
            // any short side: one thread per (key, block), the block's (up
            // to) four 8-row groups loaded together, consecutive threads on
            // consecutive keys (the round-4 form: one LDS atomic per key read)
            const int nbk = pb1 - pb0;
            for (int e = t; e < S * nbk; e += kSpNT) {
                const int lb = e / S, sc = e - lb * S;
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = group(4 * lb + u);
                    v[u] = r >= 0 ? (uint32_t)B8[(int64_t)r * S + sc] : 0xFFFFu;
                }
                const uint32_t m = min(min(v[0], v[1]), min(v[2], v[3]));
                bad |= invalid(m);
                s_key[sc * RB + lb] = m;
            }
        }
        __syncthreads();
        const int nbk = pb1 - pb0;
        for (int x = t; x < S * nbk; x += kSpNT) {
            const int sc = x / nbk, bb = x - sc * nbk;
            bm[(int64_t)sc * nb + pb0 + bb] = sp_b8_upper(s_key[sc * RB + bb]);
        }
        __syncthreads();
    }
    bad = __syncthreads_or(bad);
    if (t == 0) reinterpret_cast<int32_t *>(ws + y.flags)[w] = bad;
}

// ---- 2. candidate lists --------------------------------------------------------

template <typename CT, bool EXT>
__global__ __launch_bounds__(kSpNT) void sp_lists_kernel(LsapSparseArgs a, int32_t n) {
    using K = SpKey<CT>;
    using KT = typename K::T;
    constexpr int kQ = kSpMaxCols / kSpBlock / 64;         // block keys per lane (32)
    __shared__ int32_t s_cand[kSpNT / 64][kSpLCap];
    __shared__ int32_t s_grp[kSpNT / 64][kSpLCap];
    constexpr int kWaveLanes = 64;
    const int p = (int)(blockIdx.x / kSpRowGroups), grp = (int)(blockIdx.x % kSpRowGroups);
    if (p >= n) return;
    const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
    if (!lsap_sparse_class(a.lo, a.wave_max, R, Kd)) return;
    const bool tr = Kd < R;
    const int S = (int)(tr ? Kd : R), L = (int)(tr ? R : Kd);
    const SpLayout y = lsap_sparse_layout(S, L, sizeof(CT), tr, a.bm32 != nullptr);
    unsigned char *ws = a.ws + a.ws_offs[p];
    constexpr bool ext = EXT;                              // block minima from mvm_triplet_minima (a.bm32)
    int32_t *lcol = reinterpret_cast<int32_t *>(ws + y.lcol);
    CT *lval = reinterpret_cast<CT *>(ws + y.lval);
    int32_t *ln = reinterpret_cast<int32_t *>(ws + y.ln);
    CT *theta_out = reinterpret_cast<CT *>(ws + y.theta);
    // blocks: 32 columns over the whole long side, or (a cube's) segments of
    // seg columns cut in blocks of 32 (block b = segment b / bps, part b % bps)
    const int seg0 = lsap_sparse_seg(a, p, tr, L), seg = seg0 ? seg0 : L;
    bool src_ok;
    const SpSrc<CT> src = sp_src<CT>(a, p, tr, S, L, seg0, src_ok);
    if (!src_ok || (ext && !seg0)) return;                 // sp_solve_kernel reports it
    // block b = g * bps + jt (segment g, part jt); lane l holds b = l, l + 64,
    // ... -- one part of 32 segments, so each lane minimum ranges over 32
    // different long-side rows (theta is taken over the lane minima).  ext:
    // the blocks sit in mvm_triplet_minima's order, part-major -- b at
    // jt * npad + g of a row of bps * npad keys (segments padded to a multiple
    // of 16 with kMax) -- and lane l holds the 32 keys at 32 l .. 32 l + 31
    // (one part, or two, of 32 consecutive segments: the same spread, four
    // 16-byte loads of 16-bit keys)
    const int bps = (seg + kSpBlock - 1) / kSpBlock, nseg = L / seg;
    const int nb = nseg * bps;
    const int npad = ext ? (nseg + 15) & ~15 : nseg;
    const int rowk = npad * bps;                           // keys per row in memory
    const float rbps = 1.0f / (float)bps, rnpad = 1.0f / (float)npad;
    auto decode = [&](int b, int &jt) { return sp_div(b, bps, rbps, jt); };   // -> g, jt
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    // the block (g * bps + jt) lane `lane` holds in its q-th key
    // ext: lane l holds the kpl keys at kpl l .. kpl l + kpl - 1 (kpl = 32 when
    // a row has 2,048 keys, fewer for smaller problems, so that every lane
    // still holds keys and theta is taken over 64 lane minima)
    const int kpl = ext ? (rowk + 63) >> 6 : 0;
    auto block_of = [&](int q) {
        if (!ext) return lane + 64 * q;
        int g;
        const int jt = sp_div(kpl * lane + q, npad, rnpad, g);
        return g * bps + jt;
    };
    const KT *bm = reinterpret_cast<const KT *>(ws + y.bm);
    const uint16_t *bm16 = ext ? a.bm32 + a.bm32_offs[p] : nullptr;   // ext: 16-bit keys
    int bad = 0;                                           // ext: a NaN entry (key 0) in these rows
    for (int s = grp * (kSpNT / 64) + wave; s < S; s += kSpRowGroups * (kSpNT / 64)) {
        KT k[kQ];
        // the row base wave-uniform (a scalar base + 32-bit lane offsets)
        const int64_t s_u = __builtin_amdgcn_readfirstlane(s);
        if constexpr (!ext) {
            const KT *row = bm + s_u * rowk;
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int idx = lane + 64 * q;
                k[q] = idx < nb ? row[idx] : K::kMax;
            }
        } else {
            // 16-bit keys h: the block's upper bound (h << 16) | 0xFFFF, +inf's
            // key for h = 0xFF80 (every entry +inf), 0xFFFF padding -> kMax
            static_assert(kQ == 32 && sizeof(KT) == 4, "ext: at most 32 keys per lane");
            auto up = [](uint32_t h) -> KT {
                return h == 0xFFFFu ? K::kMax : h >= 0xFF80u ? (KT)0xFF800000u : (KT)((h << 16) | 0xFFFFu);
            };
            const uint16_t *row16 = bm16 + s_u * rowk;
            // kpl == 32 means rowk == 2,048 exactly (npad a multiple of 16, bps <= 8):
            // four 16-byte loads per lane, all inside the row
            if (kpl == 32) {
                const uint4 *r4 = reinterpret_cast<const uint4 *>(row16) + 4 * lane;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const uint4 w = r4[v];
                    const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        k[8 * v + 2 * e] = up(d[e] & 0xFFFFu);
                        k[8 * v + 2 * e + 1] = up(d[e] >> 16);
                    }
                }
            } else {
                const uint16_t *lp = row16 + kpl * lane;    // immediate offsets per key
                const int nk = min(kpl, rowk - kpl * lane);  // this lane's keys (may be <= 0)
#pragma unroll
                for (int q = 0; q < kQ; ++q) k[q] = q < nk ? up(lp[q]) : K::kMax;
            }
        }
        KT lm = k[0];                                      // this lane's smallest block key
#pragma unroll
        for (int q = 1; q < kQ; ++q) lm = k[q] < lm ? k[q] : lm;
        if (ext) bad |= !(lm >> (8 * sizeof(KT) - 1));     // a NaN's key: below every value's
        KT thr = K::kMax;
        CT theta = (CT)INFINITY;
        if (nb > a.tb) {
            // theta: the tb-th smallest of the 64 lanes' minima (lane l holds
            // blocks l, l + 64, ...), so >= tb blocks hold a cost <= theta;
            // a search over one value per lane (32 steps of one compare), where
            // the tb-th smallest block minimum itself took 32 compares per step
            if constexpr (ext) {
                // ext keys are (h << 16) | 0xFFFF (or kMax): search h, 16 steps
                uint32_t lo = 0, hi = 0xFFFFu;
                const uint32_t lh = (uint32_t)(lm >> 16);
                while (lo < hi) {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    if (__popcll(__ballot(lh <= mid)) >= a.tb) hi = mid;
                    else lo = mid + 1;
                }
                thr = (KT)((lo << 16) | 0xFFFFu);
            } else {
                KT lo = 0, hi = K::kMax;
                while (lo < hi) {
                    const KT mid = lo + (hi - lo) / 2;
                    if (__popcll(__ballot(lm <= mid)) >= a.tb) hi = mid;
                    else lo = mid + 1;
                }
                thr = lo;
            }
            theta = K::val(thr);
        }
        // candidate blocks (uniform count): every block holding a cost <= theta
        // (from the cube's 16-bit minima, bm holds upper bounds: a block may
        // hold a cost <= theta when its lower bound, the upper half, is <= thr)
        const bool groups8 = seg0 && a.bmin8;              // refine them to 8-column groups
        // 16-bit-derived keys (the 8-row minima, or ext's block upper bounds)
        // compare by their lower bound, the upper half
        const KT lowmask = groups8 || ext ? (KT)0xFFFF0000u : ~(KT)0;
        int ncand = 0;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            // (ext: padding holds kMax, above every key of a block)
            const bool c = (k[q] & lowmask) <= thr && (ext ? k[q] != K::kMax : lane + 64 * q < nb);
            const uint64_t m = __ballot(c);
            if (c) {
                const int pos = ncand + sp_mbcnt(m);
                if (pos < kSpLCap) {
                    if (groups8) {                          // the block index
                        s_cand[wave][pos] = block_of(q);
                    } else {                                // its first column | its width << 16
                        int jt;
                        const int g = decode(block_of(q), jt);
                        s_cand[wave][pos] = (g * seg + jt * kSpBlock) | (min(kSpBlock, seg - jt * kSpBlock) << 16);
                    }
                }
            }
            ncand += __popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        // the cube's 8-row minima tell which of a candidate block's four
        // 8-column groups hold a cost <= theta (one key read per group): the
        // gather below then reads those groups only, ~a quarter of the columns
        int nent = ncand, eshift = 5;                      // entries, and log2 of lanes per entry
        int32_t *ent = s_cand[wave];
        if (groups8 && ncand <= kSpLCap) {
            const int bps8 = (seg + 7) / 8;
            const uint16_t *B8 = a.bmin8 + a.bmin8_offs[p];
            int ng = 0;
            for (int m0 = 0; m0 < ncand; m0 += 16) {      // 16 blocks x 4 groups per pass
                const int idx = m0 + (lane >> 2), u = lane & 3;
                bool c = false;
                int e = 0;
                if (idx < ncand) {
                    int jt;
                    const int g = decode(s_cand[wave][idx], jt);
                    const int g8 = 4 * jt + u;
                    if (g8 < bps8) {
                        c = ((KT)B8[(int64_t)(g * bps8 + g8) * S + s] << 16) <= thr;
                        e = (g * seg + 8 * g8) | (min(8, seg - 8 * g8) << 16);
                    }
                }
                const uint64_t m = __ballot(c);
                if (c) {
                    const int pos = ng + sp_mbcnt(m);
                    if (pos < kSpLCap) s_grp[wave][pos] = e;
                }
                ng += __popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
            nent = ng;                                     // every group listed holds an entry
            eshift = 3;
            ent = s_grp[wave];
        }
        int cnt = kSpLCap + 1;
        if (nent <= kSpLCap) {
            cnt = 0;
            const int per = kWaveLanes >> eshift, emask = (1 << eshift) - 1;   // entries per wave load
            for (int m0 = 0; m0 < nent; m0 += 8 * per) {   // 8 loads in flight
                CT val[8];
                int col[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int idx = m0 + u * per + (lane >> eshift);
                    const int cb = idx < nent ? ent[idx] : 0;
                    const int j = (cb & 0xFFFF) + (lane & emask);
                    col[u] = (lane & emask) < (cb >> 16) ? j : -1;
                    val[u] = col[u] >= 0 ? src.at(s, j) : (CT)0;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const bool keep = col[u] >= 0 && val[u] <= theta;
                    const uint64_t m = __ballot(keep);
                    if (keep) {
                        const int pos = cnt + sp_mbcnt(m);
                        if (pos < kSpLCap) {
                            lcol[(int64_t)s * kSpLCap + pos] = col[u];
                            lval[(int64_t)s * kSpLCap + pos] = val[u];
                        }
                    }
                    cnt += __popcll(m);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            ln[s] = cnt <= kSpLCap ? cnt : -1;
            theta_out[s] = theta;
        }
    }
    if (ext) {                                             // this row group's NaN flag
        bad = __syncthreads_or(bad);
        if (threadIdx.x == 0) reinterpret_cast<int32_t *>(ws + y.flags)[grp] = bad;
    }
}

// ---- 3. the solver ------------------------------------------------------------

struct SpRec {
    double a;          // smallest shortest-path cost over the wave's assigned columns
    double f;          // smallest r over the wave's free list entries
    int32_t a_pos;     // scan position of the first assigned column holding a
    int32_t a_q;       // its slot (-1: none)
    int32_t a_ps;      // its path step
    int32_t f_any;     // some list entry of the wave is free
    int32_t tail_q;    // the slot at scan position n_rem - 1 (-1: none in this wave)
    uint32_t f_key;    // first step: the latest-in-scan-order key among the wave's free
                       // list entries at f ((L-1-c) << 16 | c; 0: none)
};

// dynamic LDS of sp_solve_kernel: bitmaps of lw words, row and step arrays of cap
__host__ __device__ inline size_t sp_solve_lds_bytes(int lw, int cap) {
    return (size_t)2 * lw * 4 + (size_t)8 * (cap + 4 * (cap + 1)) + (size_t)4 * (3 * cap + 5 * (cap + 1));
}

template <typename CT>
__device__ __forceinline__ double sp_block_min(double x, double *s_red, int wave) {
    x = sp_wave_min(x);
    if ((threadIdx.x & 63) == 0) s_red[wave] = x;
    __syncthreads();
    const double r = fmin(fmin(s_red[0], s_red[1]), fmin(s_red[2], s_red[3]));
    __syncthreads();
    return r;
}

__device__ __forceinline__ long long sp_block_max_i64(long long x, long long *s_red, int wave) {
    x = sp_wave_max_i64(x);
    if ((threadIdx.x & 63) == 0) s_red[wave] = x;
    __syncthreads();
    long long r = s_red[0];
    for (int w = 1; w < kSpNT / 64; ++w) r = s_red[w] > r ? s_red[w] : r;
    __syncthreads();
    return r;
}

template <typename CT, int KS>
__global__ __launch_bounds__(kSpNT) __attribute__((amdgpu_waves_per_eu(KS == 1 ? 4 : 1))) void sp_solve_kernel(LsapSparseArgs a, int32_t n, int32_t lw) {
    __shared__ SpRec s_rec[2][kSpNT / 64];
    __shared__ double s_redd[kSpNT / 64];
    __shared__ long long s_redl[kSpNT / 64];
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    const int p = blockIdx.x;
    if (p >= n) return;
    const int64_t R = a.dims[2 * p], Kd = a.dims[2 * p + 1];
    if (R == 0 || Kd == 0) {                                 // scipy: an empty assignment
        if (threadIdx.x == 0) a.status[p] = 0;
        return;
    }
    if (!lsap_sparse_class(a.lo, a.wave_max, R, Kd)) {
        // cube-free: nothing else can solve it (there is no cost to read)
        if (a.resid && threadIdx.x == 0) a.status[p] = kSpStatusBounds;
        return;
    }
    const bool tr = Kd < R;
    const int S = (int)(tr ? Kd : R), L = (int)(tr ? R : Kd);
    const int cap = a.s_cap;
    // the LDS was sized by the launch's bounds (short_max -> cap and the slots
    // per thread, long_max -> the bitmaps' lw words): a problem past them
    // would write out of range or drop slots; refuse it
    bool src_ok;
    const SpSrc<CT> src = sp_src<CT>(a, p, tr, S, L, lsap_sparse_seg(a, p, tr, L), src_ok);
    if (S > cap || L > 32 * lw || (KS == 1 && S > kSpNT) || !src_ok) {
        if (threadIdx.x == 0) a.status[p] = kSpStatusBounds;
        return;
    }
    const SpLayout y = lsap_sparse_layout(S, L, sizeof(CT), tr, a.bm32 != nullptr);
    const unsigned char *ws = a.ws + a.ws_offs[p];
    const int32_t *lcol = reinterpret_cast<const int32_t *>(ws + y.lcol);
    const CT *lval = reinterpret_cast<const CT *>(ws + y.lval);
    const int32_t *ln = reinterpret_cast<const int32_t *>(ws + y.ln);
    const CT *theta = reinterpret_cast<const CT *>(ws + y.theta);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

    uint32_t *s_asg = reinterpret_cast<uint32_t *>(s_dyn);   // [lw] assigned columns
    uint32_t *s_mvb = s_asg + lw;                             // [lw] free columns moved this search
    double *s_u = reinterpret_cast<double *>(s_mvb + lw);     // [cap] row duals
    double *s_m = s_u + cap;                                  // [cap+1] step minimum
    double *s_mp = s_m + cap + 1;                             // [cap+1] minVal of the step's scan
    double *s_f = s_mp + cap + 1;                             // [cap+1] free minimum of the step's row
    double *s_rb = s_f + cap + 1;                             // [cap+1] r at beta (NaN: scan densely)
    int32_t *s_c4r = reinterpret_cast<int32_t *>(s_rb + cap + 1);   // [cap] row -> slot
    int32_t *s_r4c = s_c4r + cap;                             // [cap] slot -> row
    int32_t *s_col = s_r4c + cap;                             // [cap] slot -> column
    int32_t *s_i = s_col + cap;                               // [cap+1] step row
    int32_t *s_sl = s_i + cap + 1;                            // [cap+1] step's chosen slot
    int32_t *s_ps = s_sl + cap + 1;                           // [cap+1] its path step
    int32_t *s_mvc = s_ps + cap + 1;                          // [cap+1] moved free column
    int32_t *s_mvp = s_mvc + cap + 1;                         // [cap+1] ... its scan position

    // NaN / -inf anywhere (sp_blockmin_kernel's tile flags): scipy's ValueError
    {
        const int seg = lsap_sparse_seg(a, p, tr, L);      // whose tiles wrote the flags
        const int nt = a.bm32 ? kSpRowGroups                // sp_lists_kernel's row groups
                       : seg  ? ((L / seg) * ((seg + kSpBlock - 1) / kSpBlock) + 63) / 64
                              : (L + kSpTileCols - 1) / kSpTileCols;
        const int32_t *fl = reinterpret_cast<const int32_t *>(ws + y.flags);
        int bad = 0;
        for (int x = t; x < nt; x += kSpNT) bad |= fl[x];
        if (__syncthreads_or(bad)) {
            if (t == 0) a.status[p] = 1;
            return;
        }
    }
    // statistics (kSpStats): rows whose list overflowed, then per search
    __shared__ int s_novf;
    if (t == 0) s_novf = 0;
    int n_dense_min = 0, n_dense_tie = 0, n_steps = 0;   // thread 0's (uniform) counts
    for (int x = t; x < lw; x += kSpNT) {
        s_asg[x] = 0u;
        s_mvb[x] = 0u;
    }
    __syncthreads();
    {
        int ovf = 0;
        for (int x = t; x < S; x += kSpNT) {
            s_u[x] = 0.0;
            s_c4r[x] = -1;
            ovf += ln[x] < 0;
        }
        if (ovf) atomicAdd(&s_novf, ovf);
    }
    // slot state: slot q = t + 256 m lives in thread t's registers
    double v[KS], spc[KS];
    int32_t col[KS], pos[KS], ps[KS];
    // cube-free: the slot's column as cube (i, j) and its e12, set when the
    // column is assigned (a slot keeps its column), so a step gathers only the
    // visited row's e13T / e23T entries
    int32_t sic[KS], sjc[KS];
    double se12[KS];
    uint32_t rem = 0;                                         // bit m: slot removed this search
#pragma unroll
    for (int m = 0; m < KS; ++m) {
        v[m] = 0.0;
        col[m] = -1;
        sic[m] = sjc[m] = 0;
        se12[m] = 0.0;
    }
    __syncthreads();
    auto asg = [&](int j) { return (s_asg[j >> 5] >> (j & 31)) & 1u; };
    auto mvd = [&](int j) { return (s_mvb[j >> 5] >> (j & 31)) & 1u; };
    auto rfree = [](double mp, CT c, double ui) { return ((mp + (double)c) - ui) - 0.0; };

    // a step's row data: its list, theta, and the raw entries at the slots'
    // columns (resid: the e13T / e23T values; else the cost).  The first step
    // of search cur + 1 visits row cur + 1, so its loads are issued during
    // search cur and stay in flight across its barriers (which wait for LDS
    // only); a slot assigned at the end of search cur loads its own then
    struct RowData {
        int nl;                                               // (lane 0 of each wave: the row's
        CT th;                                                //  values, broadcast where used)
        int lc;
        CT lv;
        double x[KS], y[KS];                                  // resid: e13T, e23T; else x = the cost
    };
    auto load_row = [&](int i_any, int n_slots) {
        const int i = __builtin_amdgcn_readfirstlane(i_any);   // uniform
        RowData d;
        // one lane loads them, so nothing converts them to scalars (a wait
        // for the load) before the step that uses them
        d.nl = lane == 0 ? ln[i] : 0;
        d.th = lane == 0 ? theta[i] : (CT)0;
        d.lc = 0;
        d.lv = (CT)0;
        if (t < kSpLCap) {
            d.lc = lcol[(int64_t)i * kSpLCap + t];
            d.lv = lval[(int64_t)i * kSpLCap + t];
        }
#pragma unroll
        for (int m = 0; m < KS; ++m) {
            const bool has = t + kSpNT * m < n_slots;
            d.x[m] = d.y[m] = 0.0;
            if (src.e12) {
                if (has) {
                    d.x[m] = src.e13t[i * src.ld + sic[m]];
                    d.y[m] = src.e23t[i * src.ld + sjc[m]];
                }
            } else if (has) {
                d.x[m] = (double)src.at(i, col[m]);
            }
        }
        return d;
    };
    RowData pf = load_row(0, 0);                              // search 0's first step

    int par = 0;
    for (int cur = 0; cur < S; ++cur) {
        const int na = cur;                                   // slots 0 .. na-1 are assigned columns
        RowData rd = pf;
#pragma unroll
        for (int m = 0; m < KS; ++m) {
            spc[m] = INFINITY;
            ps[m] = -1;
            pos[m] = L - 1 - col[m];
        }
        rem = 0;
        int i = cur, k = 0, n_rem = L, n_mv = 0;
        double m_prev = 0.0, F = INFINITY, lowest = INFINITY;
        int sink = -1, sink_ps = -1;
        while (true) {
            // ---- one Dijkstra step: every load of the step in flight at once
            // (the first step's were issued during the previous search)
            if (k > 0) rd = load_row(i, na);
            const double ui = s_u[i];
            const int nl = __builtin_amdgcn_readfirstlane(rd.nl);
            const CT th = sp_first_lane(rd.th);
            CT cv[KS];
#pragma unroll
            for (int m = 0; m < KS; ++m) {
                const int q = t + kSpNT * m;
                const bool live = q < na && !((rem >> m) & 1u);
                if (src.e12)
                    cv[m] = live ? (CT)cube_f32(se12[m], rd.x[m], rd.y[m]) : (CT)0;
                else
                    cv[m] = live ? (CT)rd.x[m] : (CT)0;
            }
            const int lc = rd.lc;
            const CT lv = rd.lv;
            double ba = INFINITY;
            int bpos = 0x7FFFFFFF, bq = -1, bps = -1, tq = -1;
#pragma unroll
            for (int m = 0; m < KS; ++m) {
                const int q = t + kSpNT * m;
                if (q < na && !((rem >> m) & 1u)) {
                    const double r = ((m_prev + (double)cv[m]) - ui) - v[m];
                    if (r < spc[m]) {
                        spc[m] = r;
                        ps[m] = k;
                    }
                    if (spc[m] < ba || (spc[m] == ba && pos[m] < bpos)) {
                        ba = spc[m];
                        bpos = pos[m];
                        bq = q;
                        bps = ps[m];
                    }
                    if (pos[m] == n_rem - 1) tq = q;
                }
            }
            double fr = INFINITY;
            int fany = 0;
            if (t < kSpLCap && t < nl && !asg(lc)) {
                fr = rfree(m_prev, lv, ui);
                fany = 1;
            }
            // wave records
            {
                const double wa = sp_wave_min(ba);
                const bool el = bq >= 0 && ba == wa;
                const int wpos = sp_wave_min_i32(el ? bpos : 0x7FFFFFFF);
                const uint64_t win = __ballot(el && bpos == wpos);
                const int wl = win ? (int)__builtin_ctzll(win) : 0;
                const int wq = win ? __builtin_amdgcn_readlane(bq, wl) : -1;
                const int wps = win ? __builtin_amdgcn_readlane(bps, wl) : -1;
                const double wf = sp_wave_min(fr);
                const uint64_t fa = __ballot(fany);
                const uint64_t tm = __ballot(tq >= 0);
                const int wt = tm ? __builtin_amdgcn_readlane(tq, (int)__builtin_ctzll(tm)) : -1;
                // the first step's free ties, for the sink without the tie scan
                // (no column is moved yet in a search's first step)
                uint32_t wk = 0;
                if (k == 0)
                    wk = sp_wave_max_u32(fany && fr == wf ? ((uint32_t)(L - 1 - lc) << 16) | (uint32_t)lc : 0u);
                if (lane == 0) s_rec[par][wave] = SpRec{wa, wf, wpos, wq, wps, fa != 0, wt, wk};
            }
            __syncthreads();
            double A = INFINITY, fk = INFINITY;
            int apos = 0x7FFFFFFF, aq = -1, aps = -1, f_any = 0, tail_q = -1;
            uint32_t fkey = 0;
#pragma unroll
            for (int w = 0; w < kSpNT / 64; ++w) {
                const SpRec r = s_rec[par][w];
                if (r.a_q >= 0 && (r.a < A || (r.a == A && r.a_pos < apos))) {
                    A = r.a;
                    apos = r.a_pos;
                    aq = r.a_q;
                    aps = r.a_ps;
                }
                if (r.f < fk) fkey = r.f_key;
                else if (r.f == fk) fkey = max(fkey, r.f_key);
                fk = fmin(fk, r.f);
                f_any |= r.f_any;
                tail_q = r.tail_q >= 0 ? r.tail_q : tail_q;
            }
            par ^= 1;
            double rb;
            if (nl < 0 || !f_any) {
                // no free list entry (or no list): the row's free minimum densely
                ++n_dense_min;
                double d = INFINITY;
                for (int j0 = t; j0 < L; j0 += kSpNT * 8) {
                    CT c[8];
                    bool ok[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int j = j0 + kSpNT * u;
                        ok[u] = j < L && !asg(j);
                        c[u] = ok[u] ? src.at(i, j) : (CT)0;
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (ok[u]) d = fmin(d, rfree(m_prev, c[u], ui));
                }
                fk = sp_block_min<CT>(d, s_redd, wave);
                rb = NAN;                                     // ties need the dense scan too
            } else {
                rb = isinf(th) ? (double)INFINITY : rfree(m_prev, SpKey<CT>::next_up(th), ui);
            }
            if (t == 0) {
                s_i[k] = i;
                s_mp[k] = m_prev;
                s_f[k] = fk;
                s_rb[k] = rb;
            }
            // the next search's first row, once this step's row data is used
            // (issued earlier, a wait for this step's loads would cover them)
            if (k == 0 && cur + 1 < S) pf = load_row(cur + 1, na);
            F = fmin(F, fk);
            lowest = fmin(A, F);
            if (!(lowest < INFINITY)) break;                  // infeasible
            if (!(A < F) && k == 0 && fkey != 0 && fk == lowest && nl >= 0 && rb == rb && rb != lowest) {
                // the search's first row holds the minimum in its list, and no
                // entry off the list can tie: its latest tie is the sink
                sink = (int)(fkey & 0xFFFFu);
                sink_ps = 0;
                if (t == 0) {
                    s_m[k] = lowest;
                    s_sl[k] = -1;
                    s_ps[k] = 0;
                }
                break;
            }
            if (!(A < F)) {
                // a free column reaches the minimum: the one latest in scan
                // order among every visited row's free ties is the sink
                __syncthreads();                              // s_f / s_rb / moved list of this search
                long long best = -1;
                for (int s = 0; s <= k; ++s) {
                    if (s_f[s] != lowest) continue;
                    const int is = s_i[s];
                    const double mp = s_mp[s], us = s_u[is], rbs = s_rb[s];
                    const int nls = ln[is];
                    const bool dense = nls < 0 || rbs != rbs || rbs == lowest;
                    n_dense_tie += dense;
                    long long key = -1;
                    if (!dense) {
                        if (t < nls) {
                            const int c = lcol[(int64_t)is * kSpLCap + t];
                            if (!asg(c) && !mvd(c) && rfree(mp, lval[(int64_t)is * kSpLCap + t], us) == lowest)
                                key = ((long long)(L - 1 - c) << 16) | c;
                        }
                    } else {
                        for (int j0 = t; j0 < L; j0 += kSpNT * 8) {
                            CT c[8];
                            bool ok[8];
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int j = j0 + kSpNT * u;
                                ok[u] = j < L && !asg(j) && !mvd(j);
                                c[u] = ok[u] ? src.at(is, j) : (CT)0;
                            }
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int j = j0 + kSpNT * u;
                                if (ok[u] && rfree(mp, c[u], us) == lowest) {
                                    const long long kk = ((long long)(L - 1 - j) << 16) | j;
                                    key = kk > key ? kk : key;
                                }
                            }
                        }
                    }
                    for (int mm = t; mm < n_mv; mm += kSpNT) {   // free columns off their default place
                        const int c = s_mvc[mm];
                        if (rfree(mp, src.at(is, c), us) == lowest) {
                            const long long kk = ((long long)s_mvp[mm] << 16) | c;
                            key = kk > key ? kk : key;
                        }
                    }
                    key = sp_block_max_i64(key, s_redl, wave);
                    if (key > best) {                         // the first row reaching it is its path
                        best = key;
                        sink_ps = s;
                    }
                }
                sink = (int)(best & 0xFFFF);
                if (t == 0) {
                    s_m[k] = lowest;
                    s_sl[k] = -1;
                    s_ps[k] = sink_ps;
                }
                break;
            }
            // an assigned column is the minimum: remove it (swap-with-last) and
            // continue from its row
            const int last = n_rem - 1;
            if (apos != last) {
                if (tail_q >= 0) {                            // an assigned column sits at the tail
#pragma unroll
                    for (int m = 0; m < KS; ++m)
                        if (t + kSpNT * m == tail_q) pos[m] = apos;
                } else {
                    int hit = -1;                             // a moved free column at the tail?
                    for (int mm = lane; mm < n_mv; mm += 64) {
                        const uint64_t b = __ballot(s_mvp[mm] == last);
                        if (b) hit = mm - lane + (int)__builtin_ctzll(b);
                    }
                    hit = __builtin_amdgcn_readfirstlane(hit);
                    if (t == 0) {
                        if (hit >= 0) {
                            s_mvp[hit] = apos;
                        } else {                              // the column at its default place
                            const int c = L - 1 - last;
                            s_mvc[n_mv] = c;
                            s_mvp[n_mv] = apos;
                            s_mvb[c >> 5] |= 1u << (c & 31);
                        }
                    }
                    if (hit < 0) ++n_mv;
                }
            }
#pragma unroll
            for (int m = 0; m < KS; ++m)
                if (t + kSpNT * m == aq) rem |= 1u << m;
            if (t == 0) {
                s_m[k] = lowest;
                s_sl[k] = aq;
                s_ps[k] = aps;
            }
            --n_rem;
            m_prev = lowest;
            i = s_r4c[aq];
            if (++k > S) {                                    // cannot happen: each step removes a slot
                if (t == 0) a.status[p] = 3;
                return;
            }
        }
        n_steps += k + 1;
        if (sink < 0) {                                       // infeasible: scipy's ValueError
            if (t == 0) a.status[p] = 2;
            return;
        }
        // ---- duals, the new assigned column, the augmenting path
        if (t == 0) s_u[cur] += lowest;
        for (int tt = 1 + t; tt <= k; tt += kSpNT) s_u[s_i[tt]] += lowest - s_m[tt - 1];
#pragma unroll
        for (int m = 0; m < KS; ++m) {
            if ((rem >> m) & 1u) v[m] -= lowest - spc[m];
            if (t + kSpNT * m == na) {                       // slot na: the sink, v stays 0
                col[m] = sink;
                v[m] = 0.0;
                if (src.e12) {
                    int jj;
                    sic[m] = sp_div(sink, src.M, src.rM, jj);
                    sjc[m] = jj;
                    se12[m] = src.e12[sic[m] * src.ld + jj];
                }
                if (cur + 1 < S) {                            // its entry of the next search's first row
                    if (src.e12) {
                        pf.x[m] = src.e13t[(cur + 1) * src.ld + sic[m]];
                        pf.y[m] = src.e23t[(cur + 1) * src.ld + sjc[m]];
                    } else {
                        pf.x[m] = (double)src.at(cur + 1, sink);
                    }
                }
            }
        }
        for (int mm = t; mm < n_mv; mm += kSpNT) {
            const int c = s_mvc[mm];
            atomicAnd(&s_mvb[c >> 5], ~(1u << (c & 31)));
        }
        if (t == 0) {
            s_col[na] = sink;
            s_asg[sink >> 5] |= 1u << (sink & 31);
            int kk = k;
            while (true) {                                    // path[j_kk] = i_(its path step)
                const int s = s_ps[kk], i2 = s_i[s];
                const int q = kk == k ? na : s_sl[kk];
                s_c4r[i2] = q;
                s_r4c[q] = i2;
                if (s == 0) break;
                kk = s - 1;
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        int32_t *stt = reinterpret_cast<int32_t *>(a.ws + a.ws_offs[p] + y.stats);
        stt[0] = n_dense_min;
        stt[1] = n_dense_tie;
        stt[2] = s_novf;
        stt[3] = n_steps;
    }
    // ---- output in scipy's order
    const int64_t o = a.out_offs[p];
    if (tr) {
        for (int kk = t; kk < S; kk += kSpNT) {
            const int rk = s_col[s_c4r[kk]];
            int rank = 0;
            for (int k2 = 0; k2 < S; ++k2) rank += s_col[s_c4r[k2]] < rk;
            a.row_ind[o + rank] = rk;
            a.col_ind[o + rank] = kk;
        }
    } else {
        for (int kk = t; kk < S; kk += kSpNT) {
            a.row_ind[o + kk] = kk;
            a.col_ind[o + kk] = s_col[s_c4r[kk]];
        }
    }
    if (t == 0) a.status[p] = 0;
}

template <typename CT>
int sp_launch(const LsapSparseArgs &a0, int32_t n, int64_t long_max, hipStream_t s) {
    LsapSparseArgs a = a0;
    const int64_t lmax = long_max < kSpMaxCols ? long_max : kSpMaxCols;
    const int tpp = (int)((lmax + kSpTileCols - 1) / kSpTileCols);
    if ((int64_t)n * tpp * kSpNT > 0xFFFFFFFFLL || (int64_t)n * kSpRowGroups * kSpNT > 0xFFFFFFFFLL ||
        (int64_t)n * (kSpMaxBlocks / 64) * kSpNT > 0xFFFFFFFFLL)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "%d problems in one batch: split it", (int)n);
    if (sizeof(CT) != sizeof(float)) {                      // the cube's minima are float keys
        a.bmin8 = nullptr;
        a.bmin8_offs = nullptr;
        a.segs = nullptr;
        a.resid = nullptr;
        a.bm32 = nullptr;
        a.bm32_offs = nullptr;
    }
    // cube-free: every problem of the class takes its block minima from the
    // 8-row minima (a problem that cannot is refused by sp_solve_kernel)
    if (!a.resid) sp_blockmin_kernel<CT><<<dim3((unsigned)(n * tpp)), dim3(kSpNT), 0, s>>>(a, n, tpp);
    if (a.bmin8 && !a.bm32)
        sp_bmin8_reduce_kernel<<<dim3((unsigned)(n * (kSpMaxBlocks / 64))), dim3(kSpNT), 0, s>>>(a, n);
    if (sizeof(CT) == 4 && a.bm32)                           // (a double problem has no bm32)
        sp_lists_kernel<CT, sizeof(CT) == 4><<<dim3((unsigned)(n * kSpRowGroups)), dim3(kSpNT), 0, s>>>(a, n);
    else
        sp_lists_kernel<CT, false><<<dim3((unsigned)(n * kSpRowGroups)), dim3(kSpNT), 0, s>>>(a, n);
    const int cap = a.s_cap;
    const int lw = (int)(((lmax + 63) / 64) * 2);            // even: the f64 arrays stay 8-aligned
    const size_t lds = sp_solve_lds_bytes(lw, cap);
    const void *kern = cap <= kSpNT ? reinterpret_cast<const void *>(&sp_solve_kernel<CT, 1>)
                                    : reinterpret_cast<const void *>(&sp_solve_kernel<CT, 4>);
    if (lds > 64 * 1024 && hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) != hipSuccess)
        return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
    if (cap <= kSpNT)
        sp_solve_kernel<CT, 1><<<dim3((unsigned)n), dim3(kSpNT), lds, s>>>(a, n, lw);
    else
        sp_solve_kernel<CT, 4><<<dim3((unsigned)n), dim3(kSpNT), lds, s>>>(a, n, lw);
    return mvm_check_launch("lsap_sparse");
}

}  // namespace

int lsap_sparse_launch_f32(const LsapSparseArgs &a, int32_t n, int64_t long_max, hipStream_t s) {
    return sp_launch<float>(a, n, long_max, s);
}

int lsap_sparse_launch_f64(const LsapSparseArgs &a, int32_t n, int64_t long_max, hipStream_t s) {
    return sp_launch<double>(a, n, long_max, s);
}

// ================================================================ C ABI ====
extern "C" {

int64_t mvm_lsap_sparse_stats_offset(int64_t rows, int64_t cols) {
    const bool tr = cols < rows;
    return (int64_t)lsap_sparse_layout(tr ? cols : rows, tr ? rows : cols, sizeof(float), tr).stats;
}

void mvm_lsap_sparse_bounds(int32_t *min_cols, int32_t *max_cols, int32_t *max_short) {
    if (min_cols) *min_cols = kSparseMinCols;
    if (max_cols) *max_cols = kSpMaxCols;
    if (max_short) *max_short = kSpMaxShort;
}

int64_t mvm_lsap_plan_resid(int32_t n_problems, const int64_t *rows, const int64_t *cols,
                            int64_t *ws_offs, int64_t *out_offs) {
    if (n_problems < 0 || (n_problems > 0 && (!rows || !cols || !ws_offs || !out_offs))) {
        mvm_set_error("mvm_lsap_plan_resid: invalid arguments");
        return -1;
    }
    int64_t w = 0, o = 0;
    for (int32_t p = 0; p < n_problems; ++p) {
        if (rows[p] < 0 || cols[p] < 0 || rows[p] > 0x7FFFFFFF || cols[p] > 0x7FFFFFFF) {
            mvm_set_error("mvm_lsap_plan_resid: problem dimensions out of range");
            return -1;
        }
        ws_offs[p] = w;
        out_offs[p] = o;
        const bool tr = cols[p] < rows[p];
        const int64_t nr = tr ? cols[p] : rows[p], nc = tr ? rows[p] : cols[p];
        // only the candidate-list class's lists (no transposed cost: there is none)
        if (rows[p] && cols[p] && nc <= kSpMaxCols && nr <= kSpMaxShort)
            w += (int64_t)lsap_sparse_layout(nr, nc, sizeof(float), tr, true).total;
        o += rows[p] < cols[p] ? rows[p] : cols[p];
    }
    ws_offs[n_problems] = w;
    out_offs[n_problems] = o;
    return w;
}

int mvm_lsap_solve_resid(const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                         const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                         int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                         int64_t long_min, int64_t long_max, int64_t short_max,
                         const uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev,
                         const uint16_t *bm32_dev, const int64_t *bm32_offs_dev,
                         const int64_t *segs_dev, const double *resid_dev, int32_t max_n,
                         const mvm_options *opts, mvm_stream_t stream) {
    mvm_clear_error();
    mvm_options o;
    int st = mvm_resolve_options(opts, o);
    if (st) return st;
    if (o.lsap_sparse_blocks < 0 || o.lsap_sparse_blocks > 64)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "lsap_sparse_blocks %d not in 0..64",
                        (int)o.lsap_sparse_blocks);
    if (n_problems < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative n_problems");
    if (n_problems == 0) return MVM_OK;
    if (!dims_dev || !ws_offs_dev || !out_offs_dev || !status_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (max_n < 0 || max_n > kChunk)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "mvm_lsap_solve_resid: views of at most %d detections "
                        "(max_n %d)", kChunk, (int)max_n);
    const int sp_lo = o.lsap_sparse_min_cols == 0 ? kSparseMinCols
                                                  : (o.lsap_sparse_min_cols < 0 ? 0 : o.lsap_sparse_min_cols);
    int wave_max = o.lsap_wave_max_cols == 0 ? 1024 : o.lsap_wave_max_cols;
    wave_max = wave_max < 0 ? 0 : (wave_max > 1024 ? 1024 : wave_max);
    if (long_max >= 1) {
        // there is no cost for any other class to read: every non-empty
        // problem must be the candidate-list class's (tall: P <= 256 < its long side)
        if (sp_lo <= 0 || long_min < sp_lo || long_min <= wave_max || long_max > kSpMaxCols ||
            short_max < 1 || short_max > kSpMaxShort)
            return mvm_fail(MVM_ERR_INVALID_ARGUMENT,
                            "mvm_lsap_solve_resid: long sides [%lld, %lld] / short sides <= %lld are not "
                            "all of the candidate-list class (long sides >= %d, > %d, <= %d; short sides "
                            "<= %d)", (long long)long_min, (long long)long_max, (long long)short_max, sp_lo,
                            wave_max, kSpMaxCols, kSpMaxShort);
        if ((bmin8_dev && !bmin8_offs_dev) || !bm32_dev || !bm32_offs_dev || !segs_dev || !resid_dev ||
            !workspace_dev || !row_ind_dev || !col_ind_dev)   // (the 8-row minima are optional)
            return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    }
    (void)workspace_bytes;   // the per-problem regions come from mvm_lsap_plan_resid's offsets
    LsapSparseArgs sa{nullptr, nullptr, dims_dev, ws_offs_dev,
                      reinterpret_cast<unsigned char *>(workspace_dev), out_offs_dev, row_ind_dev,
                      col_ind_dev, status_dev, sp_lo > 0 ? sp_lo : 1, wave_max,
                      (int32_t)(short_max < 1 ? 1 : short_max), bmin8_dev,
                      bmin8_dev ? bmin8_offs_dev : nullptr, segs_dev,
                      o.lsap_sparse_blocks ? o.lsap_sparse_blocks : kSpTB};
    const int ld = (max_n + 3) / 4 * 4;
    sa.resid = resid_dev;
    sa.resid_ld = ld;
    sa.resid_rows = max_n;
    sa.resid_stride = (int64_t)3 * max_n * ld;
    sa.bm32 = bm32_dev;
    sa.bm32_offs = bm32_offs_dev;
    return sp_launch<float>(sa, n_problems, long_max < 1 ? 1 : long_max,
                            reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
