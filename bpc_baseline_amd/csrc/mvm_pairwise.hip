// mvm_pairwise.hip — the pairwise residual kernel (C2/C3 hot path) and its C ABI.
//
// Hot path of the reference: bpc/inference/epipolar_matching.py
//   epipolar_error (:5-28)  ->  pair residual, factorised into per-detection
//                              normalised epipolar lines (O(n)) + an 8-flop
//                              fp64 point-line evaluation per pair (O(n^2))
//   (new) per-row argmin over the stored float32 values
//
// Workload shape: HBM-write bound (4 bytes of float32 output per pair, inputs
// O(n)).  Layout per workgroup (256 threads = 4 waves of 64):
//   * the workgroup owns 4*RPW*RG rows of one (scene, pair); wave w owns RPW
//     rows of each of the RG row groups;
//   * the normalised lines of the view's columns are computed once per
//     workgroup into LDS; per 256-column chunk every lane of every wave holds
//     4 consecutive columns in registers and sweeps its RPW rows, so each row
//     store is one 16-byte-per-lane, 1 KiB-per-wave coalesced store;
//   * the per-row argmin is tracked per lane in registers across chunks and
//     reduced across the wave once per row group at the end.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <type_traits>

#include "mvmatch.h"
#include "mvm_device.h"
#include "mvm_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int kMaxColTile = 1024;   // column lines resident in LDS per workgroup

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
    int64_t ld;                 // row stride of each matrix; 0 -> n_b rounded up to row_align
    int32_t row_align;          // >= 1: rows start every roundup(n_b, row_align) floats
    int32_t n_cams, n_pairs, row_blocks;
    int32_t rows_per_wg;        // kWaves * RPW * row groups
    int32_t col_tile;           // columns whose lines are resident in LDS (multiple of kChunk)
    int32_t lazy;               // 1: association by pairwise_lazy_kernel when the view fits
                                // one column tile; 0: eager argmin (mvm_options)
    int32_t row_slots;          // lazy kernel: row-line slots per wave in LDS
    int32_t row_stride;         // lazy kernel: row stride within a wave's row group
                                // (1 contiguous, kWaves interleaved over the waves)
    int32_t row_interleave;     // mvm_options.pairwise_row_interleave (host side)
    int32_t xcd_fronts;         // contiguous ranges each XCD writes at once (>= 1)
    int32_t pair_a[MVM_MAX_PAIRS];
    int32_t pair_b[MVM_MAX_PAIRS];
};

struct ColRegs {
    double l0[kColsPerLane], l1[kColsPerLane], l2[kColsPerLane];
    double x[kColsPerLane], y[kColsPerLane];
    uint32_t state[kColsPerLane];   // kOk / kDeg / kNone / kWild
};
// One row x 4 columns of one lane, clean case: 7 fp64 ops + 1 int op + 1 cvt
// per pair, one 16-byte store, 3 int ops of argmin per pair.
// MASK: the tail chunk of an aligned matrix: a lane's 4 columns are all in the
// row's pitch or all past it (jbase >= lim), and only the former store
// (padding columns between n_b and the pitch hold +inf: their lines are the
// pad lines of load_tile, and +inf never wins the argmin).
template <bool ARGMIN, bool STORE, typename OutT, int NT = 1, bool MASK = false>
__device__ __forceinline__ void row_fast(const ColRegs &c, double rl0, double rl1, double rl2,
                                         double rx, double ry, OutT *drow, int jbase, Best &best,
                                         int lim = 0) {
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
        if (MASK && jbase >= lim) return;
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
                                                 int jbase, Best &best, int lim) {
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        const double d1 = __builtin_fma(c.l1[q], ry, c.l0[q] * rx) + c.l2[q];
        const double d2 = __builtin_fma(rl1, c.y[q], rl0 * c.x[q]) + rl2;
        const float v = (float)half_for_f32(__builtin_fabs(d1) + __builtin_fabs(d2));
        const int j = jbase + kWave * q;
        if (drow && j < lim) drow[j] = v;    // a pitched row's padding: +inf (pad lines)
        if (ARGMIN && c.state[q] != kNone) best_update_fast(best, v, j);
    }
}

// Generic row: degenerate lines (9999 sentinel), non-finite or huge values,
// tails, unaligned rows, no output buffer.  Column of slot q: jbase + q*jstep.
// Columns past the view but inside the row's pitch (j < lim) are stored too,
// as +inf, which is what the other paths write there.
template <bool ARGMIN, typename OutT>
__device__ __forceinline__ void row_safe(const ColRegs &c, double rl0, double rl1, double rl2,
                                         double rx, double ry, bool rdeg, OutT *drow, int jbase,
                                         int jstep, Best &best, int lim) {
#pragma unroll
    for (int q = 0; q < kColsPerLane; ++q) {
        double d1 = line_dist(c.l0[q], c.l1[q], c.l2[q], rx, ry);
        d1 = (c.state[q] == kDeg) ? kSentinel : d1;
        const double d2 = rdeg ? kSentinel : line_dist(rl0, rl1, rl2, c.x[q], c.y[q]);
        const bool valid = c.state[q] != kNone;
        // :28; a pitched row's padding is +inf whatever the row holds (a NaN
        // row point would otherwise make the pad line's value NaN)
        const double e = valid ? 0.5 * (d1 + d2) : __builtin_inf();
        const int j = jbase + q * jstep;
        // j < lim: the view's columns and a pitched row's padding (lim = ld >= n_b)
        if (drow && j < lim) drow[j] = (OutT)e;   // default policy: L2 merges partial lines
        if (ARGMIN && valid) best_update_safe(best, (float)e, j);
    }
}

// ---- lazy argmin (clean row groups) ----
// In a row group whose rows and columns are all clean (finite, non-degenerate,
// one column tile), a lane keeps per row only the float32 bits of its minimum
// (non-negative finite floats order like their bits): two v_min3_u32 per 4
// pairs instead of a compare and two selects per pair.  The winning column is
// recovered once per group (the row slot's lanes recompute the winning lane's
// values in every chunk and keep the first equal to the minimum), so the
// result is exactly np.argmin's lowest-index rule; rows whose minimum sits in
// several lanes over several chunks take the tie path.

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

// Lazy argmin: per row a lane keeps only the float32 bits of its minimum over
// the chunks it has seen -- two v_min3_u32 per 4 pairs; the column is
// recovered at the end of the row group (lazy_reduce_bits + recovery below)
// MASKED: the last chunk of a ragged view, where lanes past the row's pitch
// (st false) compute pad-line values (+inf, never a minimum) but store nothing.
template <bool STORE, int NT, bool MASKED = false>
__device__ __forceinline__ void row_fast_lazy(const ColRegs &c, double rl0, double rl1, double rl2,
                                              double rx, double ry, float *drow, int jbase,
                                              uint32_t &bbits, bool st = true) {
    float v[kColsPerLane];
    pair_bits4(c, rl0, rl1, rl2, rx, ry, v);
    if (STORE && (!MASKED || st)) store4_nt_row<NT>(reinterpret_cast<uint64_t>(drow), (uint32_t)jbase * 4u, v);
    bbits = min3_u32(min3_u32(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2])),
                     __float_as_uint(v[3]), bbits);
}

// float32 bits of the stored value of column jj (tile-local) against row slot
// line `rl` = {l0, l1, l2, x, y}: row_fast's arithmetic for one pair
__device__ __forceinline__ uint32_t pair_bits1(const double *s_l0, const double *s_l1,
                                               const double *s_l2, const double *s_x,
                                               const double *s_y, int jj, const double *rl) {
    const double d1 = __builtin_fma(s_l1[jj], rl[4], s_l0[jj] * rl[3]) + s_l2[jj];
    const double d2 = __builtin_fma(rl[1], s_y[jj], rl[0] * s_x[jj]) + rl[2];
    return __float_as_uint((float)half_for_f32(__builtin_fabs(d1) + __builtin_fabs(d2)));
}

// ---- transposed lazy reduction (the default) ----
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

// End of a clean (lazy) row group.  Lane L holds, per row slot r, the
// float32 bits of its minimum bbits[r].  One transpose through LDS: lane L
// takes row slot rs = L / LPR and the RPW lanes [seg*RPW, seg*RPW + RPW) of
// that row (seg = L % LPR), reduces them in registers, and finishes over its
// LPR lanes with DPP.  Returns the row minimum k,
// the lowest lane w holding it, and whether another lane holds it too (`tie`:
// with several chunks the lowest lane is then not necessarily the lowest
// column).  Uniform over the LPR lanes of a row slot.
template <int RPW>
__device__ __forceinline__ void lazy_reduce_bits(uint32_t *red, const uint32_t (&bbits)[RPW],
                                                 int lane, uint32_t &k, int &w, bool &tie) {
    constexpr int LPR = kWave / RPW;
    static_assert(RPW <= 32, "lane mask is 32 bits");
    const int rs = lane / LPR, seg = lane % LPR;
#pragma unroll
    for (int r = 0; r < RPW; ++r) red[r * kWave + lane] = bbits[r];
    uint32_t v[RPW];
    read_segment<RPW>(red, rs, seg, v);
    uint32_t m = v[0];
#pragma unroll
    for (int i = 1; i < RPW; ++i) m = v[i] < m ? v[i] : m;
    k = group_min_u32<RPW>(m);
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < RPW; ++i) mask |= (v[i] == k) ? (1u << i) : 0u;
    const uint32_t base = (uint32_t)(seg * RPW);
    // first and (complemented) last lane holding k: equal iff exactly one lane
    const uint32_t lo = mask ? base + (uint32_t)__builtin_ctz(mask) : 0xFFFFFFFFu;
    const uint32_t hi = mask ? ~(base + 31u - (uint32_t)__builtin_clz(mask)) : 0xFFFFFFFFu;
    const uint32_t first = group_min_u32<RPW>(lo);
    const uint32_t last = ~group_min_u32<RPW>(hi);
    w = (int)first;
    tie = first != last;
}


// ---- workgroup set-up shared by both kernels ----
// The workgroup's (scene, pair, row block) and the geometry of its matrix.
struct BlockGeom {
    int sp, na, nb, row0;
    int64_t oa, ob;
    int64_t doff;       // first float of the matrix in `dist`
    int64_t row_off0;   // first association row of the matrix
    int64_t ld;         // row stride (pitch)
    int lim;            // columns a row stores: its padding too when pitched
};

// Dispatch places workgroup b on XCD b % 8; the remap gives each XCD a
// contiguous eighth of the (scene, pair, row block)s, so a (scene, pair)'s row
// blocks share one L2 for the column points and its output region stays
// contiguous per XCD.  With xcd_fronts F > 1 the XCD's eighth is cut into F
// contiguous ranges walked side by side (its i-th workgroup takes range i % F),
// so the chip writes 8F fronts at once: the 25 GB C3 launch runs 1-2% faster
// with F = 4 on the bench line; the XCDs walking the grid together instead
// (one front) is 7-10% slower.  Every global load here comes
// before the first store (on CDNA vmcnt orders loads behind earlier stores).
// Returns false when the block lies past its matrix's rows (uniform over the
// workgroup).
__device__ __forceinline__ bool block_geometry(const PairArgs &args, double (&f)[9], BlockGeom &g) {
    uint32_t blk = blockIdx.x;
    {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8, i = blk / 8;
        const uint32_t F = (uint32_t)args.xcd_fronts, cnt = q + (x < r ? 1u : 0u);
        const uint32_t s = cnt / F, fr = i % F;
        blk = x * q + min(x, r) + fr * s + min(fr, cnt % F) + i / F;
    }
    const int rb = (int)(blk % (uint32_t)args.row_blocks);
    g.sp = (int)(blk / (uint32_t)args.row_blocks);
    const int s = g.sp / args.n_pairs;
    const int p = g.sp - s * args.n_pairs;
    const int cam_a = args.pair_a[p], cam_b = args.pair_b[p];
    const int64_t *co = args.cam_offs + (int64_t)s * args.n_cams;
    g.oa = co[cam_a];
    g.na = (int)(co[cam_a + 1] - g.oa);
    g.ob = co[cam_b];
    g.nb = (int)(co[cam_b + 1] - g.ob);
    g.row0 = rb * args.rows_per_wg;
    if (g.row0 >= g.na) return false;
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = args.F[(int64_t)g.sp * 9 + k];
    g.doff = args.dist_offs ? args.dist_offs[g.sp] : (int64_t)g.sp * args.mat_stride;
    g.row_off0 = args.row_offs ? args.row_offs[g.sp] : 0;
    const int ra = args.row_align > 1 ? args.row_align : 1;
    g.ld = args.ld ? args.ld : (int64_t)((g.nb + ra - 1) / ra) * ra;
    g.lim = (int)min(g.ld, (int64_t)0x7FFFFFFF);
    return true;
}

// Column lines of columns [c0, c0 + T) of the view -> LDS (threads stride the
// tile).  Past the view: a pad line, whose pair values are +inf (l1.p1 =
// +inf, l2.p2 = rl2 finite) -- never a row minimum, and what a pitched row's
// padding holds.
__device__ __forceinline__ void load_col_lines(const double *pts, const double (&f)[9], int64_t ob,
                                               int nb, int c0, int T, double *s_l0, double *s_l1,
                                               double *s_l2, double *s_x, double *s_y,
                                               uint32_t *s_cst) {
    for (int jj = threadIdx.x; jj < T; jj += kThreads) {
        const int j = c0 + jj;
        uint32_t st = kNone;
        double l0 = 0, l1 = 0, l2 = __builtin_inf(), x = 0, y = 0;
        if (j < nb) {
            x = pts[2 * (ob + j)];
            y = pts[2 * (ob + j) + 1];
            st = col_line(f, x, y, l0, l1, l2) ? kDeg : (tame(l2, x, y) ? kOk : kWild);
        }
        s_l0[jj] = l0;
        s_l1[jj] = l1;
        s_l2[jj] = l2;
        s_x[jj] = x;
        s_y[jj] = y;
        s_cst[jj] = st;
    }
}

// Row centroids of the workgroup's rows [row0, row0 + rows) -> LDS.
__device__ __forceinline__ void load_row_points(const double *pts, int64_t oa, int na, int row0,
                                                int rows, double *s_rpt) {
    for (int x = threadIdx.x; x < rows; x += kThreads) {
        const int i = row0 + x;
        const f64x2 v = (i < na) ? *reinterpret_cast<const f64x2 *>(pts + 2 * (oa + i))
                                 : f64x2{0.0, 0.0};
        *reinterpret_cast<f64x2 *>(s_rpt + 2 * x) = v;
    }
}

// Line {l0, l1, l2, x, y, state} of the workgroup's local row `lrow` into
// `slot` (6 doubles); rows past the view (!valid) get a degenerate record.
__device__ __forceinline__ void put_row_line(double *slot, const double *s_rpt,
                                             const double (&f)[9], int lrow, bool valid) {
    double l0 = 0, l1 = 0, l2 = 0, x = 0, y = 0;
    bool deg = true;
    if (valid) {
        x = s_rpt[2 * lrow];
        y = s_rpt[2 * lrow + 1];
        deg = row_line(f, x, y, l0, l1, l2);
    }
    slot[0] = l0;
    slot[1] = l1;
    slot[2] = l2;
    slot[3] = x;
    slot[4] = y;
    slot[5] = (double)(deg ? kDeg : (tame(l2, x, y) ? kOk : kWild));
}

// ---- the default association kernel (lazy argmin) ----
// Workgroup = 4 waves owning rows_per_wg rows of one (scene, pair) whose view
// fits one column tile (<= kMaxColTile columns).  The column lines are
// computed ONCE per workgroup into LDS; each wave sweeps groups of RPW rows:
// per 256-column chunk every lane holds 4 consecutive columns in registers
// and walks the RPW rows, one coalesced 16-byte store per lane per row, and
// keeps per row only the float32 bits of its minimum (lazy argmin, resolved
// at the group end).  A row group with a degenerate or non-finite line, or a
// matrix whose rows are not 16-byte aligned, runs the generic arithmetic one
// row at a time instead (rare; correctness only).  The eager, strided and
// multi-tile forms live in pairwise_kernel: kept out of this kernel, they
// cannot raise its register allocation or hoist their uniforms into
// SGPR spills around the lazy loop.
// Occupancy OCC: 3 waves/SIMD at RPW 16, 4 below; 2 when the workgroup's LDS
// allows no more anyway (the host picks it).
template <int RPW, int NT, int OCC = (RPW >= 16 ? 3 : 4)>
__global__ __launch_bounds__(kThreads, OCC) void pairwise_lazy_kernel(PairArgs args) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    const int T = args.col_tile;
    const int RS = args.row_slots;   // row-line slots per wave
    double *s_l0 = reinterpret_cast<double *>(s_dyn);
    double *s_l1 = s_l0 + T;
    double *s_l2 = s_l1 + T;
    double *s_x = s_l2 + T;
    double *s_y = s_x + T;
    double *s_rows = s_y + T;                          // [kWaves][RS][6]
    double *s_rpt = s_rows + kWaves * RS * 6;          // row centroids of the workgroup
    uint32_t *s_cst = reinterpret_cast<uint32_t *>(s_rpt + 2 * args.rows_per_wg);
    uint32_t *s_red = s_cst + T;                       // per wave an [RPW][64] u32 scratch

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);   // uniform by construction
    const int lane = t % kWave;
    double f[9];
    BlockGeom g;
    if (!block_geometry(args, f, g)) return;
    const int na = g.na, nb = g.nb, row0 = g.row0;
    float *const dbase = args.dist ? reinterpret_cast<float *>(args.dist) + g.doff : nullptr;
    const bool vec_ok = dbase && ((g.doff & 3) == 0) && ((g.ld & 3) == 0);
    constexpr int U = kWaves * RPW;
    // a wave's row group: local rows group_base(gi) + r * RST, r < RPW --
    // contiguous (RST 1), or interleaved over the waves (RST kWaves: at each
    // row step the four waves store four adjacent rows)
    const int RST = args.row_stride;
    auto group_base = [&](int gi) { return RST == 1 ? (gi * kWaves + wave) * RPW : gi * U + wave; };

    load_row_points(args.pts, g.oa, na, row0, args.rows_per_wg, s_rpt);
    load_col_lines(args.pts, f, g.ob, nb, 0, T, s_l0, s_l1, s_l2, s_x, s_y, s_cst);
    // the lazy argmin needs every column of the tile clean (pad lines count as clean)
    bool my_clean = nb > 0;
    for (int jj = t; jj < T; jj += kThreads) my_clean &= (s_cst[jj] != kDeg && s_cst[jj] != kWild);
    const bool tile_clean = __syncthreads_and(my_clean) != 0;

    const int n_groups = (min(args.rows_per_wg, na - row0) + U - 1) / U;   // uniform over the WG
    double *const s_roww = s_rows + wave * RS * 6;
    // all of the wave's groups fit its row slots: one lane per row computes
    // every row line up front (one pass instead of one 16-lane pass per group)
    const bool pre = RPW * n_groups <= RS;   // uniform
    if (pre && lane < RPW * n_groups) {
        const int lrow = group_base(lane / RPW) + (lane % RPW) * RST;
        put_row_line(s_roww + 6 * lane, s_rpt, f, lrow, row0 + lrow < na);
    }
    for (int gi = 0; gi < n_groups; ++gi) {
        const int xw = group_base(gi);
        const int grow0 = row0 + xw;                            // row r: grow0 + r * RST
        const int nrows = min(RPW, (na - grow0 + RST - 1) / RST);   // may be <= 0
        double(*rowp)[6] = reinterpret_cast<double(*)[6]>(s_roww + (pre ? gi * RPW * 6 : 0));
        if (!pre && lane < RPW) {   // row lines of this wave's group (wave-private LDS slots)
            int lz = lane;          // fresh per group: its LDS address is not hoisted and spilled
            __asm__ volatile("" : "+v"(lz));
            put_row_line(s_roww + 6 * lz, s_rpt, f, xw + lz * RST, lz < nrows);
        }
        if (nrows <= 0) continue;
        // the same wave reads them back (LDS executes one wave's ops in order)
        const bool rows_fast =
            (nrows == RPW) && __all(lane >= RPW || rowp[lane % RPW][5] == 0.0);
        // uniform: the whole group takes the lazy argmin (clean rows and tile)
        if (tile_clean && rows_fast && (vec_ok || !dbase)) {
            uint32_t bbits[RPW];
#pragma unroll
            for (int r = 0; r < RPW; ++r) bbits[r] = 0x7F800000u;
            // one 256-column chunk: every lane's 4 columns x the group's rows
            auto sweep_chunk = [&](int c0, auto masked) __attribute__((always_inline)) {
                constexpr bool M = decltype(masked)::value;
                const int jbase = c0 + kColsPerLane * lane;
                const bool st = jbase < g.lim;
                ColRegs c;
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) {
                    const int jj = jbase + q;
                    c.l0[q] = s_l0[jj];
                    c.l1[q] = s_l1[jj];
                    c.l2[q] = s_l2[jj];
                    c.x[q] = s_x[jj];
                    c.y[q] = s_y[jj];
                }
                if (dbase && M) {
                    // the last chunk of a ragged view: lanes past the row's
                    // pitch store nothing (per-lane predicated stores)
#pragma unroll
                    for (int r = 0; r < RPW; ++r)
                        row_fast_lazy<true, NT, true>(
                            c, rowp[r][0], rowp[r][1], rowp[r][2], rowp[r][3], rowp[r][4],
                            dbase + (int64_t)(grow0 + r * RST) * g.ld, jbase, bbits[r], st);
                } else if (dbase) {
                    const uint64_t rstep = (uint64_t)g.ld * RST * sizeof(float);
                    uint64_t rp = reinterpret_cast<uint64_t>(dbase + (int64_t)grow0 * g.ld);
                    // row r + 1's line is read from LDS before row r is
                    // computed (the scheduling barrier keeps the reads there),
                    // so its LDS latency hides behind row r's arithmetic; the
                    // row address stays a running scalar (the empty asm stops
                    // LICM hoisting all RPW row bases out of the chunk loop,
                    // where they would be spilled to VGPR lanes)
                    double cur[5], nxt[5];
#pragma unroll
                    for (int e = 0; e < 5; ++e) cur[e] = rowp[0][e];
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        if (r + 1 < RPW) {
#pragma unroll
                            for (int e = 0; e < 5; ++e) nxt[e] = rowp[r + 1][e];
                        }
                        __builtin_amdgcn_sched_barrier(0);
                        row_fast_lazy<true, NT>(c, cur[0], cur[1], cur[2], cur[3], cur[4],
                                                reinterpret_cast<float *>(rp), jbase, bbits[r]);
                        rp += rstep;
                        __asm__ volatile("" : "+s"(rp));
#pragma unroll
                        for (int e = 0; e < 5; ++e) cur[e] = nxt[e];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < RPW; ++r)
                        row_fast_lazy<false, NT>(c, rowp[r][0], rowp[r][1], rowp[r][2],
                                                 rowp[r][3], rowp[r][4], nullptr, jbase,
                                                 bbits[r]);
                }
            };
            // chunks inside the row pitch run without a per-lane test; in the
            // last chunk of a ragged view the lanes past the pitch store nothing
            // (their columns hold pad lines: +inf, never a minimum)
            const int n_full = g.lim / kChunk;
            int c0 = 0;
            for (; c0 < nb && c0 < n_full * kChunk; c0 += kChunk) sweep_chunk(c0, std::false_type{});
            if (c0 < nb) sweep_chunk(c0, std::true_type{});
            constexpr int LPR = kWave / RPW;
            constexpr int VPL = kColsPerLane * (kMaxColTile / kChunk) / LPR;
            static_assert(VPL >= 1 && LPR * VPL == kColsPerLane * (kMaxColTile / kChunk),
                          "recovery slots");
            // the lane id as a fresh value per group: everything derived
            // from it here (row slot, LDS and output addresses) is then
            // recomputed per group instead of hoisted out of the group loop
            // and spilled -- at 3 waves/SIMD (C2) those spills were reloaded
            // after the group's stores, and the in-order vmcnt wait for the
            // reload drained all of them
            int lz = lane;
            __asm__ volatile("" : "+v"(lz));
            uint32_t k;
            int w;
            bool tie;
            lazy_reduce_bits<RPW>(s_red + wave * (RPW * kWave), bbits, lz, k, w, tie);
            // the LPR lanes of row slot rs recompute lane w's values in
            // every chunk (slot idx = chunk * 4 + q) and keep the first equal to k
            const int rs = lz / LPR, seg = lz % LPR;
            const int n_ch = (nb + kChunk - 1) / kChunk;
            const double *rl = rowp[rs];
            uint32_t first = 0xFFFFFFFFu;
#pragma unroll
            for (int v = VPL - 1; v >= 0; --v) {
                const int idx = seg + LPR * v;
                const int c = idx / kColsPerLane, q = idx % kColsPerLane;
                if (c < n_ch) {
                    const uint32_t b = pair_bits1(s_l0, s_l1, s_l2, s_x, s_y,
                                                  c * kChunk + kColsPerLane * w + q, rl);
                    first = (b == k) ? (uint32_t)idx : first;
                }
            }
            first = group_min_u32<RPW>(first);
            int jwin = (int)(first / kColsPerLane) * kChunk + kColsPerLane * w +
                       (int)(first % kColsPerLane);
            // rare: several lanes hold the minimum over several chunks ->
            // the row slot's lanes scan every column for the first equal to k
            tie = tie && n_ch > 1;
            if (__builtin_expect(__any(tie), 0)) {
                if (tie) {
                    uint32_t jt = 0xFFFFFFFFu;
                    for (int jj = nb - LPR + seg; jj >= 0; jj -= LPR)
                        jt = (pair_bits1(s_l0, s_l1, s_l2, s_x, s_y, jj, rl) == k)
                                 ? (uint32_t)jj : jt;
                    jwin = (int)group_min_u32<RPW>(jt);
                }
            }
            if (seg == 0) {
                const int64_t row = g.row_off0 + grow0 + rs * RST;
                if (args.argmin) args.argmin[row] = jwin;
                if (args.minval) args.minval[row] = __uint_as_float(k);
            }
            continue;
        }
        // generic rows, one at a time: degenerate lines (9999 sentinel),
        // non-finite or huge values, rows off 16-byte alignment (lanes then
        // take strided columns: each dword store instruction writes 256
        // contiguous bytes)
        const bool str = dbase && !vec_ok;
        for (int r = 0; r < nrows; ++r) {
            const double *rl = rowp[r];
            const bool rdeg = __builtin_amdgcn_readfirstlane((int)rl[5]) == (int)kDeg;
            float *drow = dbase ? dbase + (int64_t)(grow0 + r * RST) * g.ld : nullptr;
            Best b{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
            for (int c0 = 0; c0 < nb; c0 += kChunk) {
                ColRegs c;
#pragma unroll
                for (int q = 0; q < kColsPerLane; ++q) {
                    const int jj = str ? c0 + lane + kWave * q : c0 + kColsPerLane * lane + q;
                    c.l0[q] = s_l0[jj];
                    c.l1[q] = s_l1[jj];
                    c.l2[q] = s_l2[jj];
                    c.x[q] = s_x[jj];
                    c.y[q] = s_y[jj];
                    c.state[q] = s_cst[jj];
                }
                row_safe<true, float>(c, rl[0], rl[1], rl[2], rl[3], rl[4], rdeg, drow,
                                      c0 + (str ? lane : kColsPerLane * lane), str ? kWave : 1, b,
                                      g.lim);
            }
            uint32_t kmin;
            int32_t imin;
            wave_argmin(best_key(b), b.j, kmin, imin);
            if (lane == 0) {
                const int64_t row = g.row_off0 + grow0 + r * RST;
                if (args.argmin) args.argmin[row] = (kmin == kKeyInvalid) ? -1 : imin;
                if (args.minval) args.minval[row] = value_of_key(kmin);
            }
        }
    }
}

// ---- the general kernel ----
// Everything the lazy kernel does not take: matrices without association
// (ARGMIN false), float64 output (the cube's workspace, epipolar_error),
// the eager argmin (MVM_PAIRWISE_ARGMIN_EAGER) and views of more than
// kMaxColTile columns (column lines streamed tile by tile).  Same workgroup
// layout; per row group an eager argmin (float best + index per row in
// registers) reduced across the wave at the group end.
// occupancy OCC: 3 waves/SIMD (<= 168 VGPRs) at RPW 16, 4 (<= 128) below; 2
// when the workgroup's LDS allows no more anyway (the host picks it)
template <int RPW, bool ARGMIN, typename OutT, int NT = 1, int OCC = (RPW >= 16 ? 3 : 4)>
__global__ __launch_bounds__(kThreads, OCC) void pairwise_kernel(PairArgs args) {
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

    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t / kWave);   // uniform by construction
    const int lane = t % kWave;
    double f[9];
    BlockGeom g;
    if (!block_geometry(args, f, g)) return;
    const int na = g.na, nb = g.nb, row0 = g.row0;
    const int64_t ld = g.ld;
    const int lim = g.lim;
    constexpr int U = kWaves * RPW;
    OutT *const dbase = args.dist ? reinterpret_cast<OutT *>(args.dist) + g.doff : nullptr;
    const bool vec_ok = dbase && ((g.doff & 3) == 0) && ((ld & 3) == 0);
    // unaligned float32 rows: lanes take strided columns (coalesced dword stores)
    const bool strided = dbase && !vec_ok && sizeof(OutT) == 4;

    load_row_points(args.pts, g.oa, na, row0, args.rows_per_wg, s_rpt);
    const int n_tiles = (nb + T - 1) / T;
    if (n_tiles == 1) load_col_lines(args.pts, f, g.ob, nb, 0, T, s_l0, s_l1, s_l2, s_x, s_y, s_cst);
    __syncthreads();

    const int n_groups = (min(args.rows_per_wg, na - row0) + U - 1) / U;   // uniform over the WG
    // all of the wave's groups fit in 64 rows: one lane per row computes every
    // row line up front (one pass instead of one 16-lane pass per group)
    const bool pre = RPW * n_groups <= kWave;   // uniform
    if (pre && lane < RPW * n_groups) {
        const int gi = lane / RPW, slot = lane % RPW;
        const int xw = (gi * kWaves + wave) * RPW;
        put_row_line(s_row[wave][lane], s_rpt, f, xw + slot, slot < na - (row0 + xw));
    }
    for (int gi = 0; gi < n_groups; ++gi) {
        const int xw = (gi * kWaves + wave) * RPW;
        const int grow0 = row0 + xw;
        const int nrows = min(RPW, na - grow0);                 // may be <= 0
        double(*rowp)[6] = s_row[wave] + (pre ? gi * RPW : 0);   // this group's slots
        if (!pre && lane < RPW) {   // row lines of this wave's group (wave-private LDS slots)
            int lz = lane;          // fresh per group: its LDS address is not hoisted and spilled
            __asm__ volatile("" : "+v"(lz));
            put_row_line(s_row[wave][lz], s_rpt, f, xw + lz, lz < nrows);
        }
        // the same wave reads them back (LDS executes one wave's ops in order)
        const bool rows_fast =
            (nrows == RPW) && __all(lane >= RPW || rowp[lane % RPW][5] == 0.0);

        Best best[RPW];
#pragma unroll
        for (int r = 0; r < RPW; ++r) best[r] = Best{__uint_as_float(0x7F800000u), 0x7FFFFFFF};
        for (int tile = 0; tile < n_tiles; ++tile) {
            if (n_tiles > 1) {   // large views: stream the column lines tile by tile
                __syncthreads();
                load_col_lines(args.pts, f, g.ob, nb, tile * T, T, s_l0, s_l1, s_l2, s_x, s_y,
                               s_cst);
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
                        row_fast_strided<ARGMIN>(c, rowp[r][0], rowp[r][1],
                                                 rowp[r][2], rowp[r][3],
                                                 rowp[r][4],
                                                 dbase ? reinterpret_cast<float *>(dbase + (int64_t)(grow0 + r) * ld)
                                                       : nullptr,
                                                 jbase, best[r], lim);
                    }
                } else if (tail && vec_ok && rows_fast && __all(clean_m)) {   // aligned tail chunk
                    const uint64_t rstep = (uint64_t)ld * sizeof(OutT);
                    const uint64_t rbase = reinterpret_cast<uint64_t>(dbase + (int64_t)grow0 * ld);
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        row_fast<ARGMIN, true, OutT, NT, true>(
                            c, rowp[r][0], rowp[r][1], rowp[r][2],
                            rowp[r][3], rowp[r][4],
                            reinterpret_cast<OutT *>(rbase + (uint64_t)r * rstep), jbase, best[r],
                            lim);
                    }
                } else if (fast && vec_ok) {   // the common case: clean rows, aligned output
                    const uint64_t rstep = (uint64_t)ld * sizeof(OutT);
                    uint64_t rp = reinterpret_cast<uint64_t>(dbase + (int64_t)grow0 * ld);
#pragma unroll
                    for (int r = 0; r < RPW; ++r) {
                        row_fast<ARGMIN, true, OutT, NT>(c, rowp[r][0], rowp[r][1],
                                               rowp[r][2], rowp[r][3],
                                               rowp[r][4], reinterpret_cast<OutT *>(rp),
                                               jbase, best[r]);
                        rp += rstep;
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
                            OutT *drow = dbase ? dbase + (int64_t)(grow0 + r) * ld : nullptr;
                            const bool rdeg = __builtin_amdgcn_readfirstlane(
                                                  (int)rowp[r][5]) == (int)kDeg;
                            row_safe<ARGMIN>(c, rowp[r][0], rowp[r][1],
                                             rowp[r][2], rowp[r][3],
                                             rowp[r][4], rdeg, drow, jbase, jstep, best[r], lim);
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
            int lz = lane;   // fresh per group: no hoisted, spilled row addresses
            __asm__ volatile("" : "+v"(lz));
            store_row_results<RPW>(kmin, imin, nrows, lz, args.argmin, args.minval,
                                   g.row_off0 + grow0);
        }
    }
}

// ------------------------------------------------------------ host side ----
constexpr int kRowsPerWave = 16;       // default: 64 rows per row group
constexpr int64_t kMinBlocks = 4096;   // ~8 rounds of two resident workgroups on 256 CUs
constexpr size_t kLds3PerCU = (160u << 10) / 3;   // most LDS a workgroup may take for 3 per CU

int fill_pairs(PairArgs &a, const int32_t *pair_a, const int32_t *pair_b, int n_pairs,
               int n_cams) {
    if (n_cams < 2 || n_cams > MVM_MAX_CAMS)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "n_cams=%d outside [2, %d]", n_cams, MVM_MAX_CAMS);
    if (n_pairs < 1 || n_pairs > MVM_MAX_PAIRS)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "n_pairs=%d outside [1, %d]", n_pairs, MVM_MAX_PAIRS);
    if (!pair_a || !pair_b) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pair list");
    for (int p = 0; p < n_pairs; ++p) {
        if (pair_a[p] < 0 || pair_a[p] >= n_cams || pair_b[p] < 0 || pair_b[p] >= n_cams ||
            pair_a[p] == pair_b[p])
            return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "pair %d = (%d, %d) invalid for %d cameras",
                            p, pair_a[p], pair_b[p], n_cams);
        a.pair_a[p] = pair_a[p];
        a.pair_b[p] = pair_b[p];
    }
    a.n_cams = n_cams;
    a.n_pairs = n_pairs;
    return MVM_OK;
}

// LDS of a workgroup: column lines (5 doubles + a state word per column),
// `row_slots` row lines per wave (6 doubles each), the row centroids, and for
// the lazy kernel its per-wave [RPW][64] reduction scratch.
template <int RPW>
size_t pairwise_lds_bytes(int col_tile, int rows_per_wg, int row_slots, bool lazy) {
    return (size_t)col_tile * (5 * sizeof(double) + sizeof(uint32_t)) +
           (size_t)kWaves * row_slots * 6 * sizeof(double) +
           (size_t)rows_per_wg * 2 * sizeof(double) +
           (lazy ? (size_t)kWaves * RPW * kWave * sizeof(uint32_t) : 0);
}

// Launch with `lds` bytes of dynamic LDS (above 64 KiB the kernel must opt in).
template <typename Kernel>
int launch_lds(Kernel kern, dim3 grid, dim3 block, size_t lds, hipStream_t stream,
               const PairArgs &a) {
    if (lds > 65536 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return mvm_fail(MVM_ERR_HIP, "cannot raise the dynamic LDS limit to %zu bytes", lds);
    kern<<<grid, block, lds, stream>>>(a);
    return MVM_OK;
}

template <int RPW>
int launch_pairwise_rpw(PairArgs &a, int64_t sp_count, int max_rows, int max_cols,
                        int row_groups, bool argmin, bool f64, hipStream_t stream) {
    a.col_tile = min(kMaxColTile, max(kChunk, (max_cols + kChunk - 1) / kChunk * kChunk));
    a.rows_per_wg = kWaves * RPW * row_groups;
    a.row_blocks = (max_rows + a.rows_per_wg - 1) / a.rows_per_wg;
    const dim3 grid((unsigned)(sp_count * a.row_blocks)), block(kThreads);
    // nontemporal stores for whole-line rows (views of a multiple of 32, or
    // rows pitched to 128-byte lines); rows that end mid-line share that line
    // with the next row, and L2 must merge it (default policy)
    const bool nt = max_cols % 32 == 0 || a.row_align % 32 == 0;
    // The default association path: the lazy kernel, for views of one column
    // tile.  Row slots: all of a wave's row groups when they fit in 64 (one
    // up-front row-line pass), else one group's.
    if (argmin && !f64 && a.lazy && max_cols <= kMaxColTile) {
        a.row_slots = RPW * row_groups <= kWave ? RPW * row_groups : RPW;
        // rows interleaved over the waves for views of several chunks (C3:
        // 4.065 -> 4.034 ms mean over eight output buffers, the gain on the
        // slow HBM regions); one-chunk views keep contiguous rows (C2: 0.136
        // vs 0.147 ms interleaved) -- profiles/r03/ab/c*_interleave.log
        a.row_stride = (a.row_interleave > 0 || (a.row_interleave == 0 && max_cols > kChunk))
                           ? kWaves : 1;
        const size_t lds = pairwise_lds_bytes<RPW>(a.col_tile, a.rows_per_wg, a.row_slots, true);
        // LDS for at most two workgroups per CU (C3's 1,024 column lines): the
        // register cap of three waves per SIMD buys nothing there
        const bool occ2 = lds > kLds3PerCU;
        if (nt)
            return occ2 ? launch_lds(pairwise_lazy_kernel<RPW, 1, 2>, grid, block, lds, stream, a)
                        : launch_lds(pairwise_lazy_kernel<RPW, 1>, grid, block, lds, stream, a);
        return occ2 ? launch_lds(pairwise_lazy_kernel<RPW, 0, 2>, grid, block, lds, stream, a)
                    : launch_lds(pairwise_lazy_kernel<RPW, 0>, grid, block, lds, stream, a);
    }
    a.row_slots = kWave;
    a.row_stride = 1;
    const size_t lds = pairwise_lds_bytes<RPW>(a.col_tile, a.rows_per_wg, kWave, false);
    if (f64) return launch_lds(pairwise_kernel<RPW, false, double>, grid, block, lds, stream, a);
    if (nt) {
        // two workgroups per CU by LDS: at 168 VGPRs (the three-waves cap) the
        // kernel spilled, and a scratch reload ahead of a chunk loop drains
        // every outstanding store (s_waitcnt vmcnt(0)); at two waves per SIMD
        // it has the registers (profiles/r02/alloc/c3_occ2_same_buffers.log)
        if (argmin && lds > kLds3PerCU)
            return launch_lds(pairwise_kernel<RPW, true, float, 1, 2>, grid, block, lds, stream, a);
        if (argmin) return launch_lds(pairwise_kernel<RPW, true, float, 1>, grid, block, lds, stream, a);
        return launch_lds(pairwise_kernel<RPW, false, float, 1>, grid, block, lds, stream, a);
    }
    if (argmin) return launch_lds(pairwise_kernel<RPW, true, float, 0>, grid, block, lds, stream, a);
    return launch_lds(pairwise_kernel<RPW, false, float, 0>, grid, block, lds, stream, a);
}

int launch_pairwise_common(PairArgs &a, int32_t n_scenes, int32_t max_rows, int32_t max_cols,
                           bool argmin, bool f64, const mvm_options &o, hipStream_t stream) {
    if (n_scenes < 0 || max_rows < 0 || max_cols < 0)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative n_scenes/max_rows/max_cols");
    if (n_scenes == 0 || max_rows == 0) return MVM_OK;
    switch (o.pairwise_argmin) {
    case MVM_PAIRWISE_ARGMIN_DEFAULT:
    case MVM_PAIRWISE_ARGMIN_LAZY_TRANSPOSED:
    case MVM_PAIRWISE_ARGMIN_LAZY_ROWS: a.lazy = 1; break;   // LAZY_ROWS: an alias since ABI 3
    case MVM_PAIRWISE_ARGMIN_EAGER: a.lazy = 0; break;
    default: return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "pairwise_argmin %d", (int)o.pairwise_argmin);
    }
    const int rpw = o.pairwise_rows_per_wave ? o.pairwise_rows_per_wave : kRowsPerWave;
    if (rpw != 4 && rpw != 8 && rpw != 16)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "pairwise_rows_per_wave %d not 4, 8 or 16", rpw);
    if (o.pairwise_row_interleave < -1 || o.pairwise_row_interleave > 1)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "pairwise_row_interleave %d not -1, 0 or 1",
                        (int)o.pairwise_row_interleave);
    a.row_interleave = o.pairwise_row_interleave;
    if (o.pairwise_xcd_fronts < 0 || o.pairwise_xcd_fronts > 16)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "pairwise_xcd_fronts %d outside [0, 16]",
                        (int)o.pairwise_xcd_fronts);
    if (o.pairwise_row_groups < 0 || o.pairwise_row_groups > 16)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "pairwise_row_groups %d outside [0, 16]",
                        (int)o.pairwise_row_groups);
    // default: enough row groups to amortise the column lines over ~256 rows
    // for views of more than 512 columns, ~128 rows for narrower views, never
    // more than the rows a view has -- halved to ~128 rows while the grid has
    // fewer than kMinBlocks workgroups: the last round of long-lived
    // workgroups is a tail with idle CUs (C2, 3,000 matrices of 256 rows:
    // 0.156 -> 0.143 ms per launch).  C3 keeps 256: 128-row blocks make the
    // launch far less sensitive to where its output lies (slowest/fastest
    // allocation 1.12-1.16 -> 1.05-1.09 over four boxes), but the bench line
    // itself, on one box, alternating, ran 3.5% slower with them (1.547e12 vs
    // 1.599-1.605e12, profiles/r04/slots/bench_rowblocks/).  256-column views
    // take 128 at any grid size (2,000 scenes x 3 cams: 0.298 vs 0.267 ms,
    // profiles/r03/ab/c2_2000_rowgroups.log).
    const int groups_needed = (max_rows + kWaves * rpw - 1) / (kWaves * rpw);
    const int64_t sp_count = (int64_t)n_scenes * a.n_pairs;
    int rg = o.pairwise_row_groups;
    if (!rg) {
        const int rows_cap = max_cols > 2 * kChunk ? 256 : 128;
        rg = max(1, min(groups_needed, rows_cap / (kWaves * rpw)));
        const int rg_floor = min(rg, max(1, 128 / (kWaves * rpw)));
        while (rg > rg_floor &&
               sp_count * ((max_rows + kWaves * rpw * rg - 1) / (kWaves * rpw * rg)) < kMinBlocks)
            rg /= 2;
    }
    // 4 write fronts per XCD for launches of >= 8 GB of matrices (C3, 25 GB:
    // 1.542-1.581e12 -> 1.570-1.600e12 pairs/s on two boxes); the 0.8 GB C2
    // launch gains nothing (profiles/r04/bench_ab/xcd/)
    a.xcd_fronts = o.pairwise_xcd_fronts
                       ? o.pairwise_xcd_fronts
                       : (double)sp_count * max_rows * max_cols * sizeof(float) >= 8e9 ? 4 : 1;
    const int64_t rows_per_wg = (int64_t)kWaves * rpw * rg;
    const int64_t blocks = sp_count * ((max_rows + rows_per_wg - 1) / rows_per_wg);
    if (blocks > kMaxGridBlocks)
        return mvm_fail(MVM_ERR_UNSUPPORTED, "grid of %lld workgroups too large: split the scenes",
                        (long long)blocks);
    int st;
    switch (rpw) {
    case 4: st = launch_pairwise_rpw<4>(a, sp_count, max_rows, max_cols, rg, argmin, f64, stream); break;
    case 8: st = launch_pairwise_rpw<8>(a, sp_count, max_rows, max_cols, rg, argmin, f64, stream); break;
    default: st = launch_pairwise_rpw<16>(a, sp_count, max_rows, max_cols, rg, argmin, f64, stream); break;
    }
    return st ? st : mvm_check_launch("pairwise kernel");
}

}  // namespace

// ================================================================ C ABI ====
extern "C" {

int mvm_pairwise_residual_argmin_pitched(const double *pts_dev, const int64_t *cam_offs_dev,
                                         const double *F_dev, const int32_t *pair_a,
                                         const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                         int32_t n_pairs, int32_t max_n, int32_t row_align,
                                         const int64_t *dist_offs_dev, const int64_t *row_offs_dev,
                                         float *dist_dev, int32_t *argmin_dev, float *minval_dev,
                                         const mvm_options *opts, mvm_stream_t stream) {
    mvm_clear_error();
    mvm_options o;
    int st = mvm_resolve_options(opts, o);
    if (st) return st;
    if (row_align < 1 || row_align > 256 || (row_align & (row_align - 1)))
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "row_align %d not a power of two in [1, 256]",
                        (int)row_align);
    PairArgs a{};
    st = fill_pairs(a, pair_a, pair_b, n_pairs, n_cams);
    if (st) return st;
    if (n_scenes > 0 && max_n > 0 && (!pts_dev || !cam_offs_dev || !F_dev))
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null input pointer");
    if (dist_dev && !dist_offs_dev) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "dist without dist_offs");
    if ((argmin_dev || minval_dev) && !row_offs_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "argmin/minval without row_offs");
    a.pts = pts_dev;
    a.cam_offs = cam_offs_dev;
    a.F = F_dev;
    a.dist_offs = dist_offs_dev;
    a.row_offs = row_offs_dev;
    a.dist = dist_dev;
    a.argmin = argmin_dev;
    a.minval = minval_dev;
    a.ld = 0;
    a.row_align = row_align;
    const bool want_argmin = argmin_dev || minval_dev;
    return launch_pairwise_common(a, n_scenes, max_n, max_n, want_argmin, false, o,
                                  reinterpret_cast<hipStream_t>(stream));
}

int mvm_pairwise_residual_argmin_ex(const double *pts_dev, const int64_t *cam_offs_dev,
                                    const double *F_dev, const int32_t *pair_a,
                                    const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                    int32_t n_pairs, int32_t max_n, const int64_t *dist_offs_dev,
                                    const int64_t *row_offs_dev, float *dist_dev,
                                    int32_t *argmin_dev, float *minval_dev,
                                    const mvm_options *opts, mvm_stream_t stream) {
    return mvm_pairwise_residual_argmin_pitched(pts_dev, cam_offs_dev, F_dev, pair_a, pair_b,
                                                n_scenes, n_cams, n_pairs, max_n, 1, dist_offs_dev,
                                                row_offs_dev, dist_dev, argmin_dev, minval_dev,
                                                opts, stream);
}

int mvm_pairwise_residual_argmin(const double *pts_dev, const int64_t *cam_offs_dev,
                                 const double *F_dev, const int32_t *pair_a,
                                 const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                 int32_t n_pairs, int32_t max_n, const int64_t *dist_offs_dev,
                                 const int64_t *row_offs_dev, float *dist_dev,
                                 int32_t *argmin_dev, float *minval_dev, mvm_stream_t stream) {
    return mvm_pairwise_residual_argmin_ex(pts_dev, cam_offs_dev, F_dev, pair_a, pair_b, n_scenes,
                                           n_cams, n_pairs, max_n, dist_offs_dev, row_offs_dev,
                                           dist_dev, argmin_dev, minval_dev, nullptr, stream);
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
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    if (ld <= 0 || mat_stride < 0)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "ld must be > 0 and mat_stride >= 0");
    a.pts = pts_dev;
    a.cam_offs = cam_offs_dev;
    a.F = F_dev;
    a.dist = e_dev;
    a.mat_stride = mat_stride;
    a.ld = ld;
    a.row_align = 1;
    mvm_options o;
    mvm_options_init(&o);
    return launch_pairwise_common(a, n_scenes, max_n, max_n, false, true, o,
                                  reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
