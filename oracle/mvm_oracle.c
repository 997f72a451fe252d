/*
 * mvm_oracle.c — CPU restatement of the reference multi-view epipolar matching
 * hot path.  TEST INFRASTRUCTURE ONLY: this file is the parity checker for the
 * HIP kernels and the CPU baseline leg of bench.py.  The product path
 * (bpc_baseline_amd) never links, loads or calls it.
 *
 * Parity pinning: the npz fixtures under tests/golden were generated in the build container by
 * importing the reference (/root/reference, stub cv2) with oracle/gen_golden.py;
 * tests/test_oracle_golden.py checks this file against them bit-for-bit
 * (fp64 bits for the scalar residuals, f32 bits for the cubes).
 *
 * Arithmetic follows bpc/inference/epipolar_matching.py as executed by numpy
 * 2.2.6 + OpenBLAS 0.3.29 in the build container (op order measured):
 *   l2 = F  @ p1  (epipolar_matching.py:13)  l2[r] = fma(F[r,0], x1, F[r,1]*y1) + F[r,2]
 *   l1 = F.T@ p2  (epipolar_matching.py:14)  l1[c] = fma(F[1,c], y2, F[0,c]*x2) + F[2,c]
 *   n  = ||l[:2]|| (:17-18)                  n = sqrt(fma(l[1], l[1], l[0]*l[0]))
 *   l /= n if n > 1e-8 (:20-23)              three correctly rounded divisions
 *   d  = |l . p| or 9999 (:25-26)            d = |fma(l[1], y, l[0]*x) + l[2]|
 *   e  = 0.5*(d1+d2) (:28)
 *   cube = f32(((e12+e13)+e23)/3) (:78-81, :96)
 *
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off, so fma() is the only
 * fused operation, exactly where written).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MVM_DEGENERATE_NORM 1e-8 /* epipolar_matching.py:20-23 */
#define MVM_SENTINEL 9999.0      /* epipolar_matching.py:25-26 (int 9999) */

/* Normalised epipolar line; deg=1 when the line norm is not > 1e-8 (NaN too). */
typedef struct {
    double l[3];
    int deg;
} line_t;

/* l2 = F @ (x, y, 1): line in the second camera induced by a first-camera point
 * (epipolar_matching.py:13, normalisation :17-23). */
static line_t line_from_row_point(const double *F, double x, double y) {
    line_t L;
    for (int r = 0; r < 3; ++r) L.l[r] = fma(F[3 * r + 0], x, F[3 * r + 1] * y) + F[3 * r + 2];
    double n = sqrt(fma(L.l[1], L.l[1], L.l[0] * L.l[0]));
    L.deg = !(n > MVM_DEGENERATE_NORM);
    if (!L.deg)
        for (int r = 0; r < 3; ++r) L.l[r] = L.l[r] / n;
    return L;
}

/* l1 = F.T @ (x, y, 1): line in the first camera induced by a second-camera
 * point (epipolar_matching.py:14, normalisation :17-23). */
static line_t line_from_col_point(const double *F, double x, double y) {
    line_t L;
    for (int c = 0; c < 3; ++c) L.l[c] = fma(F[3 + c], y, F[c] * x) + F[6 + c];
    double n = sqrt(fma(L.l[1], L.l[1], L.l[0] * L.l[0]));
    L.deg = !(n > MVM_DEGENERATE_NORM);
    if (!L.deg)
        for (int c = 0; c < 3; ++c) L.l[c] = L.l[c] / n;
    return L;
}

/* |l . (x, y, 1)| or the 9999 sentinel (epipolar_matching.py:25-26). */
static double point_line_distance(const line_t *L, double x, double y) {
    if (L->deg) return MVM_SENTINEL;
    return fabs(fma(L->l[1], y, L->l[0] * x) + L->l[2]);
}

/* epipolar_error(pt1, pt2, F) — epipolar_matching.py:5-28. */
double mvm_oracle_epipolar_error(const double *F, double x1, double y1, double x2, double y2) {
    line_t l2 = line_from_row_point(F, x1, y1);
    line_t l1 = line_from_col_point(F, x2, y2);
    double d1 = point_line_distance(&l1, x1, y1);
    double d2 = point_line_distance(&l2, x2, y2);
    return 0.5 * (d1 + d2);
}

/* epipolar_error_full — epipolar_matching.py:73-81. */
double mvm_oracle_epipolar_error_full(const double *p1, const double *p2, const double *p3,
                                      const double *F12, const double *F13, const double *F23) {
    double e12 = mvm_oracle_epipolar_error(F12, p1[0], p1[1], p2[0], p2[1]);
    double e13 = mvm_oracle_epipolar_error(F13, p1[0], p1[1], p3[0], p3[1]);
    double e23 = mvm_oracle_epipolar_error(F23, p2[0], p2[1], p3[0], p3[1]);
    return ((e12 + e13) + e23) / 3;
}

/* np.argmin ordering key on a stored float32: NaN is the minimum (first NaN
 * wins), otherwise IEEE order; ties resolve to the lowest index by scanning
 * in ascending order with a strict comparison. */
static inline int f32_less(float a, float b) {
    if (isnan(b)) return 0;
    if (isnan(a)) return 1;
    return a < b;
}

/* Column lines of one (scene, pair): the line depends on one detection only,
 * so precomputing it is bit-identical to recomputing it per pair. */
static void col_lines(const double *F, const double *pts, int64_t o, int64_t n, line_t *out) {
    for (int64_t j = 0; j < n; ++j) out[j] = line_from_col_point(F, pts[2 * (o + j)], pts[2 * (o + j) + 1]);
}

/* fp64 residual matrix e[i, j] = epipolar_error(p_a[i], p_b[j], F) (epipolar_matching.py:5-28). */
static void residual_matrix_f64(const double *F, const double *pts, int64_t oa, int64_t na,
                                int64_t ob, int64_t nb, line_t *lc, double *e) {
    col_lines(F, pts, ob, nb, lc);
    for (int64_t i = 0; i < na; ++i) {
        double xi = pts[2 * (oa + i)], yi = pts[2 * (oa + i) + 1];
        line_t lr = line_from_row_point(F, xi, yi);
        for (int64_t j = 0; j < nb; ++j) {
            double d1 = point_line_distance(&lc[j], xi, yi);
            double d2 = point_line_distance(&lr, pts[2 * (ob + j)], pts[2 * (ob + j) + 1]);
            e[i * nb + j] = 0.5 * (d1 + d2);
        }
    }
}

/* Pairwise residual matrices for every (scene, camera pair) plus the per-row
 * argmin over columns (oracle = np.argmin(e_ab, 1)).
 *   pts      f64 [sum n, 2]   detections, scene-major, camera-minor (CSR)
 *   cam_offs i64 [S*C+1]      detection offsets of (scene, camera)
 *   F        f64 [S*P, 9]     fundamental matrix of (scene, pair), row-major
 *   pairs    i32 [P, 2]       camera indices (a, b) of each pair
 *   dist_offs i64 [S*P+1]     f32 offsets of each n_a x n_b matrix in dist
 *   row_offs  i64 [S*P+1]     offsets of each pair's n_a rows in argmin/minv
 * dist / argmin / minv may each be NULL.  Rows with n_b == 0 get argmin -1
 * and minv NaN. */
void mvm_oracle_pairwise(const double *pts, const int64_t *cam_offs, const double *F,
                         const int32_t *pairs, int S, int C, int P, const int64_t *dist_offs,
                         const int64_t *row_offs, float *dist, int32_t *argmin, float *minv,
                         int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int64_t SP = (int64_t)S * P;
#pragma omp parallel
    {
        line_t *lc = NULL;
        int64_t cap = 0;
#pragma omp for schedule(dynamic, 1)
        for (int64_t sp = 0; sp < SP; ++sp) {
            int64_t s = sp / P;
            int p = (int)(sp % P);
            int a = pairs[2 * p], b = pairs[2 * p + 1];
            int64_t oa = cam_offs[s * C + a], na = cam_offs[s * C + a + 1] - oa;
            int64_t ob = cam_offs[s * C + b], nb = cam_offs[s * C + b + 1] - ob;
            const double *Fp = F + sp * 9;
            if (nb > cap) {
                free(lc);
                cap = nb;
                lc = (line_t *)malloc(sizeof(line_t) * (size_t)cap);
            }
            col_lines(Fp, pts, ob, nb, lc);
            for (int64_t i = 0; i < na; ++i) {
                double xi = pts[2 * (oa + i)], yi = pts[2 * (oa + i) + 1];
                line_t lr = line_from_row_point(Fp, xi, yi);
                float best = 0.f;
                int32_t bi = -1;
                for (int64_t j = 0; j < nb; ++j) {
                    double d1 = point_line_distance(&lc[j], xi, yi);
                    double d2 = point_line_distance(&lr, pts[2 * (ob + j)], pts[2 * (ob + j) + 1]);
                    float v = (float)(0.5 * (d1 + d2));
                    if (dist) dist[dist_offs[sp] + i * nb + j] = v;
                    if (bi < 0 || f32_less(v, best)) {
                        best = v;
                        bi = (int32_t)j;
                    }
                }
                if (argmin) argmin[row_offs[sp] + i] = bi;
                if (minv) minv[row_offs[sp] + i] = bi < 0 ? NAN : best;
            }
        }
        free(lc);
    }
}

/* Three-camera cost cube (compute_cost_matrix, epipolar_matching.py:83-98)
 * plus the per-(i,j) argmin over k of the flattened (N*M, P) cube.
 *   cam_offs i64 [S*3+1], F f64 [S*3, 9] ordered F12, F13, F23 per scene
 *   cube_offs i64 [S+1] f32 offsets of each N x M x P cube
 *   row_offs  i64 [S+1] offsets of each scene's N*M rows in argmin/minv
 * The three fp64 pair matrices are built once per scene, then every cube
 * entry is f32(((e12 + e13) + e23) / 3) exactly as epipolar_error_full. */
void mvm_oracle_cube(const double *pts, const int64_t *cam_offs, const double *F, int S,
                     const int64_t *cube_offs, const int64_t *row_offs, float *cube,
                     int32_t *argmin, float *minv, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int s = 0; s < S; ++s) {
        int64_t o1 = cam_offs[3 * s], N = cam_offs[3 * s + 1] - o1;
        int64_t o2 = cam_offs[3 * s + 1], M = cam_offs[3 * s + 2] - o2;
        int64_t o3 = cam_offs[3 * s + 2], Pn = cam_offs[3 * s + 3] - o3;
        const double *F12 = F + (int64_t)s * 27, *F13 = F12 + 9, *F23 = F12 + 18;
        int64_t mx = M > Pn ? M : Pn;
        line_t *lc = (line_t *)malloc(sizeof(line_t) * (size_t)(mx > 0 ? mx : 1));
        double *e12 = (double *)malloc(sizeof(double) * (size_t)(N * M + 1));
        double *e13 = (double *)malloc(sizeof(double) * (size_t)(N * Pn + 1));
        double *e23 = (double *)malloc(sizeof(double) * (size_t)(M * Pn + 1));
        residual_matrix_f64(F12, pts, o1, N, o2, M, lc, e12);
        residual_matrix_f64(F13, pts, o1, N, o3, Pn, lc, e13);
        residual_matrix_f64(F23, pts, o2, M, o3, Pn, lc, e23);
        for (int64_t ij = 0; ij < N * M; ++ij) {
            int64_t i = ij / M, j = ij % M;
            float best = 0.f;
            int32_t bk = -1;
            for (int64_t k = 0; k < Pn; ++k) {
                float v = (float)(((e12[ij] + e13[i * Pn + k]) + e23[j * Pn + k]) / 3);
                if (cube) cube[cube_offs[s] + ij * Pn + k] = v;
                if (bk < 0 || f32_less(v, best)) {
                    best = v;
                    bk = (int32_t)k;
                }
            }
            if (argmin) argmin[row_offs[s] + ij] = bk;
            if (minv) minv[row_offs[s] + ij] = bk < 0 ? NAN : best;
        }
        free(lc);
        free(e12);
        free(e13);
        free(e23);
    }
}

/* OpenMP thread count the baseline will use. */
/* The fp64 pair residuals of every 3-camera scene (pairs (0,1), (0,2), (1,2):
 * epipolar_matching.py:78-80) in the layout of the GPU's cube-free path
 * (include/mvmatch.h, mvm_triplet_minima): e12 [N][ld], then e13 and e23
 * TRANSPOSED, [P][ld] each, at out + s * 3 * max_n * ld.  Entries outside the
 * views are left untouched. */
void mvm_oracle_residuals(const double *pts, const int64_t *cam_offs, const double *F, int S,
                          int max_n, int64_t ld, double *out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int s = 0; s < S; ++s) {
        int64_t o1 = cam_offs[3 * s], N = cam_offs[3 * s + 1] - o1;
        int64_t o2 = cam_offs[3 * s + 1], M = cam_offs[3 * s + 2] - o2;
        int64_t o3 = cam_offs[3 * s + 2], Pn = cam_offs[3 * s + 3] - o3;
        const double *F12 = F + (int64_t)s * 27, *F13 = F12 + 9, *F23 = F12 + 18;
        int64_t mx = M > Pn ? M : Pn;
        line_t *lc = (line_t *)malloc(sizeof(line_t) * (size_t)(mx > 0 ? mx : 1));
        double *e13 = (double *)malloc(sizeof(double) * (size_t)(N * Pn + 1));
        double *e23 = (double *)malloc(sizeof(double) * (size_t)(M * Pn + 1));
        double *E12 = out + (int64_t)s * 3 * max_n * ld, *E13T = E12 + (int64_t)max_n * ld,
               *E23T = E13T + (int64_t)max_n * ld;
        double *e12 = (double *)malloc(sizeof(double) * (size_t)(N * M + 1));
        residual_matrix_f64(F12, pts, o1, N, o2, M, lc, e12);
        residual_matrix_f64(F13, pts, o1, N, o3, Pn, lc, e13);
        residual_matrix_f64(F23, pts, o2, M, o3, Pn, lc, e23);
        for (int64_t i = 0; i < N; ++i)
            for (int64_t j = 0; j < M; ++j) E12[i * ld + j] = e12[i * M + j];
        for (int64_t k = 0; k < Pn; ++k) {
            for (int64_t i = 0; i < N; ++i) E13T[k * ld + i] = e13[i * Pn + k];
            for (int64_t j = 0; j < M; ++j) E23T[k * ld + j] = e23[j * Pn + k];
        }
        free(lc);
        free(e12);
        free(e13);
        free(e23);
    }
}

int mvm_oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
