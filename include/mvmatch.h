/*
 * mvmatch.h — C ABI of the MI355X multi-view epipolar matcher.
 *
 * This is the drop-in boundary for the hot path of the reference's
 * bpc/inference/epipolar_matching.py.  The reference's boundary is a Python
 * function-call boundary (process_pose.py:24 binds compute_cost_matrix /
 * match_objects by name; camera_utils.compute_fundamental_matrix is bound at
 * process_pose.py:26); the entry points below are what that module's compute
 * reduces to once the O(n^2)/O(n^3) loops move to the GPU.  Python binds them
 * with ctypes (bpc_baseline_amd/_native.py) and registers them as PyTorch
 * custom ops (bpc_baseline_amd/ops.py); INTEGRATION.md shows the bindings.
 *
 * Conventions
 *   - every pointer argument named *_dev is a caller-allocated DEVICE pointer;
 *     pointers without the suffix are host pointers;
 *   - work is enqueued on `stream` (a hipStream_t; NULL = default stream) and
 *     nothing is synchronised: results are ready when the stream reaches them;
 *   - no allocation, no host<->device copy and no global mutable state in any
 *     launch function (safe to capture in a hipGraph, re-entrant per stream);
 *     the library reads no environment variables: kernel-path choices come
 *     only from an explicit mvm_options argument (the *_ex entry points);
 *   - return value: MVM_OK or an MVM_ERR_* code; mvm_last_error_string()
 *     gives a per-thread message for the last failing call.
 *
 * Detections use a CSR layout: pts_dev holds (x, y) float64 centroids of all
 * detections, scene-major then camera-minor; cam_offs_dev[s*C + c] ..
 * cam_offs_dev[s*C + c + 1] is the detection range of camera c in scene s.
 * Fundamental matrices are float64, row-major, one per (scene, pair):
 * F_dev[(s*P + p)*9 + 3*r + c] = F[r][c] with F mapping camera pair_a[p]
 * points to camera pair_b[p] epipolar lines (camera_utils.py:23-46).
 */
#ifndef MVMATCH_H
#define MVMATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MVM_ABI_VERSION 7
#define MVM_MAX_CAMS 8
#define MVM_MAX_PAIRS 28 /* MVM_MAX_CAMS choose 2 */

typedef struct ihipStream_t *mvm_stream_t; /* == hipStream_t */

enum {
    MVM_OK = 0,
    MVM_ERR_INVALID_ARGUMENT = 1, /* null pointer, negative size, bad pair index */
    MVM_ERR_UNSUPPORTED = 2,      /* more cameras/pairs than MVM_MAX_* */
    MVM_ERR_WORKSPACE = 3,        /* workspace smaller than required */
    MVM_ERR_HIP = 4               /* a HIP runtime call or kernel launch failed */
};

/* Element types of mvm_lsap_*_ex cost matrices. */
enum { MVM_F32 = 0, MVM_F64 = 1 };

/* Library version string ("mvmatch <semver> gfx950"). */
const char *mvm_version(void);
/* Message of the last failing call on this thread ("" if none). */
const char *mvm_last_error_string(void);
/* Static description of a status code. */
const char *mvm_status_string(int status);

/*
 * Kernel-path selection.  Every choice below selects among kernels that
 * compute the SAME outputs bit for bit (the parity tests run each path); none
 * changes what is computed, only how.  The plain entry points use the
 * compiled-in defaults, which are what mvm_options_init writes (every field
 * 0 = "default"); the *_ex entry points take a const mvm_options * (NULL =
 * defaults).  `size` must be sizeof(mvm_options) as the caller compiled it
 * (mvm_options_init sets it), so the struct can grow without breaking callers.
 */
enum {
    MVM_PAIRWISE_ARGMIN_DEFAULT = 0,     /* = LAZY_TRANSPOSED */
    MVM_PAIRWISE_ARGMIN_LAZY_TRANSPOSED, /* clean row groups: per-chunk minimum bits,
                                            one LDS transpose per row group */
    MVM_PAIRWISE_ARGMIN_LAZY_ROWS,       /* since ABI 3 an alias of LAZY_TRANSPOSED (the
                                            per-row DPP form was removed) */
    MVM_PAIRWISE_ARGMIN_EAGER            /* best value + index per pair */
};
enum {
    MVM_CUBE_DEFAULT = 0,   /* by the batch's largest view: SMALL <= 16, FUSED above */
    MVM_CUBE_SMALL,         /* one workgroup per scene (views < 64; FUSED otherwise) */
    MVM_CUBE_FUSED,         /* 16 i x 32 j tiles, pair residuals in the prologue
                               (views <= 256; k-chunked above) */
    MVM_CUBE_WORKSPACE,     /* fp64 pair matrices to the workspace, then tiles
                               (views <= 256; GENERIC above) */
    MVM_CUBE_GENERIC        /* fp64 workspace + one (i, j) row per wave */
};
typedef struct mvm_options {
    int32_t size;                   /* sizeof(mvm_options) */
    int32_t pairwise_argmin;        /* MVM_PAIRWISE_ARGMIN_* */
    int32_t pairwise_rows_per_wave; /* 0 default (16); 4, 8 or 16 */
    int32_t pairwise_row_groups;    /* 0 default (~256 rows per workgroup, ~128 for small grids); 1..16 */
    int32_t cube_kernel;            /* MVM_CUBE_* */
    int32_t cube_rows_per_instr;    /* FUSED: 0 default (by view size: 8 up to 32,
                                       then 4 / 2 / 1); 1, 2, 4 or 8 (i, j) rows per
                                       wave instruction, capped by the view size
                                       (2: <= 128, 4: <= 64, 8: <= 32) */
    int32_t lsap_wave_max_cols;     /* 0 default (1024); -1 never the one-wave
                                       kernel; else a long-side limit <= 1024 */
    int32_t lsap_multi_g;           /* 0 default (auto: as many co-resident
                                       workgroups per problem as fit, <= 16);
                                       -1 off; 2..16 forced */
    int32_t lsap_lds_max_cols;      /* 0 default (4096); -1 off: column state in LDS
                                       for long sides up to this */
    int32_t lsap_lds_small_cols;    /* 0 default (2048): ... of which up to this
                                       with 256 threads (1024 above) */
    int32_t lsap_mid_max_cols;      /* 0 default (8192): workspace-state long sides
                                       up to this with 256 threads (1024 above) */
    int32_t lsap_reg_max_cols;      /* 0 default (4096); -1 off: long sides up to this
                                       (short sides <= 1024) in one workgroup with the
                                       column state in registers (ABI 3) */
    int32_t lsap_reg_threads;       /* 0 default (512 threads, 8 columns each); 1024
                                       (4 each) */
    int32_t lsap_mreg_max_cols;     /* 0 default (65536); -1 off: long sides above
                                       lsap_reg_max_cols up to this (short sides <= 1024)
                                       over ceil(long / 4096) co-resident workgroups with
                                       the column state in registers (ABI 3) */
    int32_t pairwise_row_interleave; /* 0 default (by view size: on for views of more
                                       than 256); 1 a row group's rows interleave over
                                       the workgroup's 4 waves (at each row step they
                                       store 4 adjacent rows); -1 each wave's rows
                                       contiguous (ABI 3) */
    int32_t cube_cols_per_lane;     /* FUSED (views <= 256): 0 default (3 where the view
                                       fits 3 k per lane: <= 48 / 96 / 192 at four / two /
                                       one rows per instruction, else 4; then 5-8 k per
                                       lane at four or two rows per instruction where
                                       that keeps >= 8% more lanes busy, ABI 6); 3..8.
                                       3 lowers the rows per instruction until the view
                                       fits; 5-8 take the most rows per instruction
                                       (4 or 2) that hold the view; an error where no
                                       shape holds it (3: > 192; 5-8: > 32 k) or with a
                                       forced cube_rows_per_instr it does not fit, and
                                       for views > 256 (the k-chunked kernel) */
    int32_t pairwise_xcd_fronts;    /* 0 default (4 when the launch may write >= 8 GB of
                                       matrices -- judged from the padded bound
                                       n_scenes * n_pairs * max_n^2 * 4 B; the Python
                                       plan passes the real size's choice -- else 1);
                                       1..16: each XCD writes its eighth of the grid as
                                       this many concurrent contiguous ranges (ABI 5;
                                       +0.8-1.9% on C3, a margin of one box) */
    int32_t lsap_sparse_min_cols;   /* 0 default (4096); -1 off: problems with a long
                                       side >= this (and > the one-wave limit, <= 65536)
                                       and a short side <= 1024 are solved one workgroup
                                       each through per-row candidate lists (ABI 6) */
    int32_t lsap_sparse_blocks;     /* 0 default (16): candidate blocks (of 32 columns)
                                       per row of that class, 1..64 (ABI 6) */
    int32_t cube_tile_rows;         /* FUSED at two, four or eight rows per
                                       instruction: i rows per tile, 0 default (32 at
                                       eight rows per instruction, else 16), 16 or 32
                                       (the tile's prologue over twice the rows; ABI 6) */
} mvm_options;

/* Fill *opts with the defaults (all 0) and opts->size. */
void mvm_options_init(mvm_options *opts);

/*
 * Pairwise symmetric epipolar residuals + per-row argmin, batched over
 * (scene, camera pair).  Replaces the per-pair epipolar_error calls
 * (bpc/inference/epipolar_matching.py:5-28) with one launch; the per-row
 * argmin is SURVEY §8a row a5 (oracle: np.argmin(e_ab, axis=1)).
 *
 * For scene s and pair p = (a, b), with n_a, n_b detections in cameras a, b:
 *   e[i][j] = float32(epipolar_error(p_a[i], p_b[j], F[s, p]))       (fp64 math)
 *   dist_dev[dist_offs_dev[s*P + p] + i*n_b + j] = e[i][j]
 *   argmin_dev[row_offs_dev[s*P + p] + i] = lowest j minimising e[i][:]
 *                                             (NaN counts as smallest; -1 if n_b == 0)
 *   minval_dev[...]                         = e[i][argmin] (NaN if n_b == 0)
 * dist_dev, argmin_dev and minval_dev may each be NULL (not produced).
 * pair_a / pair_b are HOST arrays of n_pairs camera indices (a != b).
 * max_n is a host-known upper bound on every view's detection count (n_a and
 * n_b over all (scene, pair)): it sizes the grid and the LDS column tile;
 * rows/columns beyond the real counts are skipped on the device.
 */
int mvm_pairwise_residual_argmin(const double *pts_dev, const int64_t *cam_offs_dev,
                                 const double *F_dev, const int32_t *pair_a,
                                 const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                 int32_t n_pairs, int32_t max_n, const int64_t *dist_offs_dev,
                                 const int64_t *row_offs_dev, float *dist_dev,
                                 int32_t *argmin_dev, float *minval_dev, mvm_stream_t stream);
/* ... with explicit kernel-path options (NULL = defaults). */
int mvm_pairwise_residual_argmin_ex(const double *pts_dev, const int64_t *cam_offs_dev,
                                    const double *F_dev, const int32_t *pair_a,
                                    const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                    int32_t n_pairs, int32_t max_n, const int64_t *dist_offs_dev,
                                    const int64_t *row_offs_dev, float *dist_dev,
                                    int32_t *argmin_dev, float *minval_dev,
                                    const mvm_options *opts, mvm_stream_t stream);

/*
 * The same with pitched rows (ABI 3): row i of matrix (s, p) starts at
 *   dist_dev[dist_offs_dev[s*P + p] + i*ld],  ld = roundup(n_b, row_align),
 * so with row_align 32 (and matrix offsets that are multiples of 32) every
 * row starts on a 128-byte line and every store of a ragged view writes whole
 * lines.  Columns n_b .. ld-1 of a row are padding and hold +inf.  row_align
 * is a power of two in
 * [1, 256]; 1 is the unpitched layout of mvm_pairwise_residual_argmin_ex.
 * The caller sizes dist_dev and dist_offs_dev with the pitched sizes n_a*ld.
 */
int mvm_pairwise_residual_argmin_pitched(const double *pts_dev, const int64_t *cam_offs_dev,
                                         const double *F_dev, const int32_t *pair_a,
                                         const int32_t *pair_b, int32_t n_scenes, int32_t n_cams,
                                         int32_t n_pairs, int32_t max_n, int32_t row_align,
                                         const int64_t *dist_offs_dev, const int64_t *row_offs_dev,
                                         float *dist_dev, int32_t *argmin_dev, float *minval_dev,
                                         const mvm_options *opts, mvm_stream_t stream);

/*
 * Same residuals kept in float64 (no cast), written with a uniform layout:
 * matrix (s, p) starts at e_dev + (s*P + p) * mat_stride and has row stride
 * ld (>= every n_b; use a multiple of 4 for vectorised stores).  This is the
 * exact fp64 value of epipolar_error (epipolar_matching.py:28) and the input
 * of the three-camera cube.
 */
int mvm_pairwise_residual_f64(const double *pts_dev, const int64_t *cam_offs_dev,
                              const double *F_dev, const int32_t *pair_a, const int32_t *pair_b,
                              int32_t n_scenes, int32_t n_cams, int32_t n_pairs,
                              int32_t max_n, int64_t mat_stride, int64_t ld, double *e_dev,
                              mvm_stream_t stream);

/*
 * Three-camera cost cube + per-(i,j) argmin over k, batched over scenes.
 * Replaces compute_cost_matrix (epipolar_matching.py:83-98):
 *   cube[i][j][k] = float32(((e12[i][j] + e13[i][k]) + e23[j][k]) / 3)
 * with e_ab the fp64 residuals of pairs (0,1), (0,2), (1,2); F_dev holds
 * F12, F13, F23 for every scene ([S*3, 9]); cam_offs_dev has S*3+1 entries.
 *   cube_dev[cube_offs_dev[s] + (i*M + j)*P + k]
 *   argmin_dev[row_offs_dev[s] + i*M + j]   (argmin over k of the flattened
 *                                            (N*M, P) cube row; -1 if P == 0)
 * max_n bounds every view's detection count.  workspace_dev must hold
 * mvm_triplet_workspace_bytes(n_scenes, max_n) bytes (16-byte aligned).
 */
size_t mvm_triplet_workspace_bytes(int32_t n_scenes, int32_t max_n);
int mvm_triplet_cost_argmin(const double *pts_dev, const int64_t *cam_offs_dev,
                            const double *F_dev, int32_t n_scenes, int32_t max_n,
                            const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                            float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                            void *workspace_dev, size_t workspace_bytes, mvm_stream_t stream);
/* ... with explicit kernel-path options (NULL = defaults). */
int mvm_triplet_cost_argmin_ex(const double *pts_dev, const int64_t *cam_offs_dev,
                               const double *F_dev, int32_t n_scenes, int32_t max_n,
                               const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                               float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                               void *workspace_dev, size_t workspace_bytes,
                               const mvm_options *opts, mvm_stream_t stream);
/*
 * ... also writing, for the assignment that follows (mvm_lsap_solve_ex3), the
 * minimum over every group of 8 consecutive j of every (i, k) (ABI 6): for
 * scene s with view sizes N, M, P, row i * ceil(M/8) + g of P uint16 keys at
 * bmin8_dev + bmin8_offs_dev[s] holds, per k, the upper 16 bits of the
 * order-preserving key (float bits | 0x80000000) of min over j in [8g, 8g+8)
 * of cube[i][j][k] -- a lower bound of that minimum to 1/128 -- or 0 when any
 * of the eight is NaN.  The fused kernel (views of 17-256 detections, its
 * default shapes; with them requested, views of 33-48 take 32-j instead of
 * 48-j tiles) writes them itself; every other path reads them back from the
 * cube (cube_dev required).  Offsets that are multiples of 4 keys let the
 * kernel store 8 bytes per lane.
 */
int mvm_triplet_cost_argmin_bmin8(const double *pts_dev, const int64_t *cam_offs_dev,
                                  const double *F_dev, int32_t n_scenes, int32_t max_n,
                                  const int64_t *cube_offs_dev, const int64_t *row_offs_dev,
                                  float *cube_dev, int32_t *argmin_dev, float *minval_dev,
                                  uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev,
                                  void *workspace_dev, size_t workspace_bytes,
                                  const mvm_options *opts, mvm_stream_t stream);

/*
 * Cube-free association input (ABI 7): for an assignment of every scene's
 * flattened (N*M, P) cube that never reads the cube itself
 * (mvm_lsap_solve_resid, mvm_select_triangulate_resid), write only what
 * those need:
 *   bmin8_dev  optional (NULL: not written): the same 16-bit 8-row minima
 *              mvm_triplet_cost_argmin_bmin8 writes (bit for bit, same layout
 *              and offsets);
 *   bm32_dev   the candidate-list kernels' 32-column block minima as 16-bit
 *              keys: for short-side column k of scene s, nb = ceil(M/32) *
 *              npad keys at bm32_dev + bm32_offs_dev[s] + k * nb (npad =
 *              roundup(N, 16)), block (jt, i) at jt * npad + i holding h, the
 *              smallest 8-row key (upper half of the order-preserving float32
 *              key, NaN 0) of columns i * M + 32 jt .. + 31; rows i >= N
 *              0xFFFF; offsets multiples of 16 (32-byte runs), bm32_dev
 *              16-byte aligned;
 *   resid_dev  every scene's float64 pair residuals, from which the
 *              assignment recomputes the entries it reads as
 *              float32(((e12 + e13) + e23) / 3), the cube's own arithmetic:
 *                resid_dev + s * stride             e12  [N][ld]  (i, j)
 *                resid_dev + s * stride + max_n*ld  e13T [P][ld]  (k, i)
 *                resid_dev + s * stride + 2*max_n*ld e23T [P][ld] (k, j)
 *              with ld = roundup(max_n, 4), stride = 3 * max_n * ld;
 *              resid_bytes >= mvm_triplet_workspace_bytes(n_scenes, max_n)
 *              (16-byte aligned).
 * Views of at most 256 detections.  Replaces the cube's 4 B per triple of HBM
 * writes with 2 B per 32 triples (+ 2 B per 8 with bmin8_dev)
 * (epipolar_matching.py:83-98 feeding :100-116).  The group and block
 * minima are taken in float32 and every one within 8 units of a 16-bit carry
 * is recomputed exactly in fp64, so the keys are those of the cube's own
 * values bit for bit.
 */
int mvm_triplet_minima(const double *pts_dev, const int64_t *cam_offs_dev, const double *F_dev,
                       int32_t n_scenes, int32_t max_n, uint16_t *bmin8_dev,
                       const int64_t *bmin8_offs_dev, uint16_t *bm32_dev, const int64_t *bm32_offs_dev,
                       double *resid_dev, size_t resid_bytes, const mvm_options *opts,
                       mvm_stream_t stream);

/*
 * Batched rectangular linear-sum assignment, identical to
 * scipy.optimize.linear_sum_assignment (the association step of
 * match_objects, bpc/inference/epipolar_matching.py:100-116, scipy 1.14's
 * shortest-augmenting-path algorithm, same tie-breaking and output order).
 * Problem p is the row-major float32 matrix at cost_dev + cost_offs_dev[p]
 * with dims_dev[2p] rows and dims_dev[2p+1] columns (e.g. the flattened
 * (N*M, P) cube of mvm_triplet_cost_argmin).  Its min(rows, cols) assigned
 * (row, col) pairs go to row_ind_dev/col_ind_dev at out_offs_dev[p], sorted
 * by row; status_dev[p] = 0 ok, 1 NaN/-inf entries, 2 infeasible.
 * mvm_lsap_plan (HOST arrays, n+1 entries each) fills the per-problem
 * workspace byte offsets and output offsets and returns the workspace size
 * (or -1); copy both offset arrays to the device for mvm_lsap_solve.
 */
int64_t mvm_lsap_plan(int32_t n_problems, const int64_t *rows, const int64_t *cols,
                      int64_t *ws_offs, int64_t *out_offs);
int mvm_lsap_solve(const float *cost_dev, const int64_t *cost_offs_dev, const int64_t *dims_dev,
                   int32_t n_problems, const int64_t *ws_offs_dev, const int64_t *out_offs_dev,
                   void *workspace_dev, size_t workspace_bytes, int64_t *row_ind_dev,
                   int64_t *col_ind_dev, int32_t *status_dev, mvm_stream_t stream);
/*
 * mvm_lsap_solve with host-known bounds on max(rows, cols) over the non-empty
 * problems (long_max < 1: every problem is empty): kernel classes that cannot
 * have work are not launched, which matters for small batches of small
 * problems.  The bounds must hold; mvm_lsap_solve passes (1, INT64_MAX).
 */
int mvm_lsap_solve_bounded(const float *cost_dev, const int64_t *cost_offs_dev,
                           const int64_t *dims_dev, int32_t n_problems,
                           const int64_t *ws_offs_dev, const int64_t *out_offs_dev,
                           void *workspace_dev, size_t workspace_bytes, int64_t *row_ind_dev,
                           int64_t *col_ind_dev, int32_t *status_dev, int64_t long_min,
                           int64_t long_max, mvm_stream_t stream);
/*
 * Cost matrices of element type cost_dtype (MVM_F32 or MVM_F64: scipy
 * assigns a float64 matrix in float64, so a float64 caller must not be
 * narrowed), with explicit kernel-path options (NULL = defaults).  The
 * workspace must come from mvm_lsap_plan_ex with the same cost_dtype.
 */
int64_t mvm_lsap_plan_ex(int32_t n_problems, const int64_t *rows, const int64_t *cols,
                         int32_t cost_dtype, int64_t *ws_offs, int64_t *out_offs);
int mvm_lsap_solve_ex(const void *cost_dev, int32_t cost_dtype, const int64_t *cost_offs_dev,
                      const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                      const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                      int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                      int64_t long_min, int64_t long_max, const mvm_options *opts,
                      mvm_stream_t stream);
/*
 * ... with a host-known bound on min(rows, cols) as well (ABI 6): it sizes the
 * candidate-list kernels' LDS (a workgroup per problem holds state for every
 * short-side row).  mvm_lsap_solve_ex passes short_max = long_max.
 */
int mvm_lsap_solve_ex2(const void *cost_dev, int32_t cost_dtype, const int64_t *cost_offs_dev,
                       const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                       const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                       int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                       int64_t long_min, int64_t long_max, int64_t short_max,
                       const mvm_options *opts, mvm_stream_t stream);
/*
 * ... taking the block minima of cubes from mvm_triplet_cost_argmin_bmin8
 * (ABI 6): problem p's cost is a flattened (N*M, P) cube (segs_dev[p] = M)
 * whose 8-row minima are at bmin8_dev + bmin8_offs_dev[p].  The candidate-list
 * kernels then read those (N * ceil(M/8) * P keys) instead of the whole cost
 * once more; results are the same.  Ignored for float64 costs and for
 * problems outside the class; all three pointers NULL = mvm_lsap_solve_ex2.
 */
int mvm_lsap_solve_ex3(const void *cost_dev, int32_t cost_dtype, const int64_t *cost_offs_dev,
                       const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                       const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                       int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                       int64_t long_min, int64_t long_max, int64_t short_max,
                       const uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev,
                       const int64_t *segs_dev, const mvm_options *opts, mvm_stream_t stream);

/*
 * Cube-free assignment (ABI 7): mvm_lsap_solve_ex3 for the flattened (N*M, P)
 * cubes of a mvm_triplet_minima batch, without the cubes.  Problem p is
 * scene p: dims (N*M, P), segs_dev[p] = M, its pair residuals at resid_dev
 * (max_n as given to mvm_triplet_minima); the kernels recompute every entry
 * they read with the cube's arithmetic, so the result is that of
 * mvm_lsap_solve_ex3 on the cubes (and scipy's).  The candidate lists start
 * from bm32_dev (mvm_triplet_minima's 16-bit block minima, no reduction pass)
 * and, when bmin8_dev is not NULL, refine each candidate block to its 8-column
 * groups by the 8-row minima at bmin8_dev + bmin8_offs_dev[p] (without them
 * they gather whole blocks).  There is no cost for the dense classes to read, so every
 * non-empty problem must be of the candidate-list class (long sides >=
 * mvm_options.lsap_sparse_min_cols (default 4096) and > lsap_wave_max_cols
 * (1024), <= 65536; short sides <= 1024): the host bounds are checked
 * (MVM_ERR_INVALID_ARGUMENT), and a problem outside them on the device gets
 * status 4.  The workspace comes from mvm_lsap_plan_resid (the class's
 * candidate lists only: ~0.3 MB per 256^3 scene).
 * Statuses of every mvm_lsap_solve* entry point: 0 ok, 1 NaN / -inf entries
 * (scipy's ValueError), 2 infeasible, 3 internal (a co-resident wait timed
 * out), 4 the problem exceeds the bounds the call was given (short_max /
 * long_max) or, here, is outside the class.
 */
int64_t mvm_lsap_plan_resid(int32_t n_problems, const int64_t *rows, const int64_t *cols,
                            int64_t *ws_offs, int64_t *out_offs);
/* The candidate-list class's limits (ABI 7): the default lower bound of its
 * long sides (mvm_options.lsap_sparse_min_cols 0), its largest long side and
 * its largest short side.  Any pointer may be NULL. */
void mvm_lsap_sparse_bounds(int32_t *min_cols, int32_t *max_cols, int32_t *max_short);
/* Byte offset, inside a (rows x cols) problem's workspace region, of the
 * candidate-list solver's counters for it (ABI 7): int32 [4] = dense scans for
 * a row's free minimum (no list, or no free entry left in it), dense scans for
 * the free ties at a search's end, rows whose candidate list overflowed,
 * Dijkstra steps.  Written by every solve of a problem of that class. */
int64_t mvm_lsap_sparse_stats_offset(int64_t rows, int64_t cols);
int mvm_lsap_solve_resid(const int64_t *dims_dev, int32_t n_problems, const int64_t *ws_offs_dev,
                         const int64_t *out_offs_dev, void *workspace_dev, size_t workspace_bytes,
                         int64_t *row_ind_dev, int64_t *col_ind_dev, int32_t *status_dev,
                         int64_t long_min, int64_t long_max, int64_t short_max,
                         const uint16_t *bmin8_dev, const int64_t *bmin8_offs_dev,
                         const uint16_t *bm32_dev, const int64_t *bm32_offs_dev,
                         const int64_t *segs_dev, const double *resid_dev, int32_t max_n,
                         const mvm_options *opts, mvm_stream_t stream);

/*
 * On-device detection packing, replacing the per-box loop of
 * PoseEstimator._detect (bpc/inference/process_pose.py:122-140).  Input:
 * the detector's boxes of n_img images in CSR form: boxes_dev f32 [n, 4]
 * (xyxy), conf_dev f32 [n], cls_dev f32 [n], image k owning rows
 * [img_offs_dev[k], img_offs_dev[k+1]).  A box is kept when cls == class_id
 * and conf >= conf_thresh (both float32 compares, :130), in input order.
 * Output, the matcher's CSR input: counts_dev int32 [n_img],
 * cam_offs_dev int64 [n_img+1] (exclusive prefix of counts), boxes_out_dev
 * int32 [kept, 4] = int(box) (truncation toward zero, :134) and pts_dev f64
 * [kept, 2] = 0.5 * (x1 + x2), 0.5 * (y1 + y2) (:135-136).  Capacity of the
 * two row outputs must be img_offs[n_img] rows.  status_dev[0] = 1 if a kept
 * box had a non-finite coordinate or one with |x| >= 2^30 (stored as 0).
 */
int mvm_pack_detections(const float *boxes_dev, const float *conf_dev, const float *cls_dev,
                        const int64_t *img_offs_dev, int32_t n_img, float conf_thresh,
                        float class_id, int32_t *counts_dev, int64_t *cam_offs_dev,
                        double *pts_dev, int32_t *boxes_out_dev, int32_t *status_dev,
                        mvm_stream_t stream);

/*
 * Batched DLT triangulation, replacing triangulate_multi_view
 * (bpc/inference/epipolar_matching.py:118-127) as called per match by
 * PosePrediction.triangulate (process_pose.py:86-94).  Point p uses the
 * n_views projection matrices (f64, row-major 3x4) of set
 * set_of_point_dev[p] (or set p when NULL) at proj_dev + set*n_views*12 and
 * its 2-D points pts2d_dev [n_points, n_views, 2]; X_dev [n_points, 3] =
 * X[:3] / X[3] of the right singular vector of the smallest singular value
 * of the 2V x 4 system.  fp64; agrees with LAPACK to rounding (the vector is
 * unique up to sign, which the division cancels).  2 <= n_views <= 8.
 */
int mvm_triangulate_dlt(const double *proj_dev, const int32_t *set_of_point_dev,
                        const double *pts2d_dev, int32_t n_points, int32_t n_views, double *X_dev,
                        mvm_stream_t stream);

/*
 * The tail of PoseEstimator._match (process_pose.py:182-187) for a batch of
 * 3-camera scenes, after mvm_triplet_cost_argmin and mvm_lsap_solve: scene
 * s's assignment (row_ind/col_ind at lsap_out_offs_dev[s], the flattened
 * (N*M, P) cube at cube_offs_dev[s]) is filtered by cube value < threshold
 * (match_objects :111; compared in float64, as numpy 1.26 compares a float32
 * scalar with a Python number), decoded i = r / M, j = r % M, k = c
 * (:112-114), stably sorted by cost (:183) and triangulated from the
 * centroids pts_dev (CSR cam_offs_dev, 3 views per scene) with the scene's
 * projection matrices proj_dev [S, 3, 3, 4] (K @ RT[:3], :86-94).  Match w
 * of scene s (w < count_dev[s]) is written at lsap_out_offs_dev[s] + w:
 * match_dev int32 [.., 3] = (i, j, k), cost_dev f32, X_dev f64 [.., 3].
 */
int mvm_select_triangulate(const float *cube_dev, const int64_t *cube_offs_dev,
                           const int64_t *cam_offs_dev, const int64_t *lsap_out_offs_dev,
                           const int64_t *row_ind_dev, const int64_t *col_ind_dev,
                           const double *pts_dev, const double *proj_dev, int32_t n_scenes,
                           double threshold, int32_t *match_dev, float *cost_dev, double *X_dev,
                           int32_t *count_dev, mvm_stream_t stream);
/* ... cube-free (ABI 7): each assigned entry recomputed from the pair
 * residuals of mvm_triplet_minima (resid_dev, max_n as given there) with the
 * cube's arithmetic -- the same costs, matches and order as from the cube. */
int mvm_select_triangulate_resid(const double *resid_dev, int32_t max_n, const int64_t *cam_offs_dev,
                                 const int64_t *lsap_out_offs_dev, const int64_t *row_ind_dev,
                                 const int64_t *col_ind_dev, const double *pts_dev,
                                 const double *proj_dev, int32_t n_scenes, double threshold,
                                 int32_t *match_dev, float *cost_dev, double *X_dev, int32_t *count_dev,
                                 mvm_stream_t stream);

/*
 * Diagnostic: fill `bytes` (multiple of 16, 16-byte aligned) of device memory
 * with the fastest 16-byte nontemporal store stream measured on MI355X: 8 KiB
 * per workgroup, workgroups remapped so each XCD writes its own contiguous
 * eighth in order.  bench.py times it to report the achievable HBM write
 * bandwidth next to the kernels' roofline fraction (the other store patterns
 * studied in DESIGN.md §3.5 live in tools/probes/write_probes.hip).
 */
int mvm_hbm_write_probe(void *dst_dev, size_t bytes, mvm_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* MVMATCH_H */
