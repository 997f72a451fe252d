// mvm_pipeline.hip — the device steps on either side of the matcher
// (SURVEY §8f #3 and #4), so a batch can go detector -> matcher -> 3-D
// centres without a host round trip.
//
//  * mvm_pack_detections: the box packing of PoseEstimator._detect
//    (bpc/inference/process_pose.py:122-140): keep boxes whose class equals
//    class_id and whose float32 confidence >= the float32 threshold (:130), in
//    input order; truncate xyxy to int (:134, Python int() of a float32 =
//    truncation toward zero); centre = 0.5 * (x1 + x2) (:135-136) in float64,
//    exact.  Output is the matcher's CSR input (pts f64 [n, 2] + offsets).
//  * mvm_triangulate_dlt: triangulate_multi_view (epipolar_matching.py:118-127)
//    as called by PosePrediction.triangulate (process_pose.py:86-94): A is
//    the 2V x 4 DLT system, X the right singular vector of its smallest
//    singular value, returned as X[:3] / X[3].  One-sided Jacobi SVD in fp64,
//    one thread per point (tolerance parity with LAPACK's gesdd: the vector
//    is unique up to sign, which X[:3]/X[3] cancels).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "mvmatch.h"
#include "mvm_device.h"
#include "mvm_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int kPackThreads = 256;

// ---------------------------------------------------------- packing ----
__device__ __forceinline__ bool keep_box(const float *conf, const float *cls, int64_t k,
                                         float thresh, float class_id) {
    return (cls[k] == class_id) && (conf[k] >= thresh);
}

// per image: number of kept boxes
__global__ __launch_bounds__(kPackThreads) void pack_count_kernel(
    const float *conf, const float *cls, const int64_t *img_offs, float thresh, float class_id,
    int32_t *counts) {
    __shared__ int s_cnt;
    const int img = blockIdx.x;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const int64_t b = img_offs[img], e = img_offs[img + 1];
    int c = 0;
    for (int64_t k = b + threadIdx.x; k < e; k += kPackThreads) c += keep_box(conf, cls, k, thresh, class_id);
    atomicAdd(&s_cnt, c);
    __syncthreads();
    if (threadIdx.x == 0) counts[img] = s_cnt;
}

// exclusive prefix of the counts -> CSR offsets (one workgroup; chunked scan)
__global__ __launch_bounds__(1024) void pack_scan_kernel(const int32_t *counts, int32_t n,
                                                         int64_t *offs) {
    // each thread sums a contiguous range; the 1024 partial sums are scanned
    // with wave shuffles (64 lanes) and once more over the 16 wave totals
    __shared__ int64_t s_wave[16];
    const int t = threadIdx.x, lane = t % 64, wave = t / 64;
    const int64_t per = (n + 1023) / 1024;
    const int64_t b = (int64_t)t * per, e = min<int64_t>(n, b + per);
    int64_t sum = 0;
    for (int64_t k = b; k < e; ++k) sum += counts[k];
    int64_t x = sum;                                  // inclusive scan in the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    if (wave == 0) {                                  // inclusive scan of the wave totals
        int64_t w = lane < 16 ? s_wave[lane] : 0;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const int64_t y = __shfl_up(w, d, 64);
            if (lane >= d) w += y;
        }
        if (lane < 16) s_wave[lane] = w;
    }
    __syncthreads();
    int64_t run = x - sum + (wave > 0 ? s_wave[wave - 1] : 0);   // exclusive prefix
    if (t == 1023) offs[n] = run + sum;
    for (int64_t k = b; k < e; ++k) {
        offs[k] = run;
        run += counts[k];
    }
}

// per image: order-preserving compaction of the kept boxes
__global__ __launch_bounds__(kPackThreads) void pack_write_kernel(
    const float *boxes, const float *conf, const float *cls, const int64_t *img_offs,
    float thresh, float class_id, const int64_t *out_offs, double *pts, int32_t *boxes_out,
    int32_t *status) {
    __shared__ int s_wave[kPackThreads / 64];
    __shared__ int s_base;
    const int img = blockIdx.x;
    const int t = threadIdx.x, lane = t % 64, wave = t / 64;
    const int64_t b = img_offs[img], e = img_offs[img + 1];
    if (t == 0) s_base = 0;
    __syncthreads();
    for (int64_t k0 = b; k0 < e; k0 += kPackThreads) {
        const int64_t k = k0 + t;
        const bool keep = k < e && keep_box(conf, cls, k, thresh, class_id);
        const uint64_t m = __ballot(keep);
        const int in_wave = __builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (lane == 0) s_wave[wave] = __builtin_popcountll(m);
        __syncthreads();
        int before = s_base;
        for (int w = 0; w < wave; ++w) before += s_wave[w];
        if (keep) {
            const int64_t o = out_offs[img] + before + in_wave;
            int32_t q[4];
            bool ok = true;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float f = boxes[4 * k + c];
                ok &= isfinite(f) && fabsf(f) < 1073741824.0f;   // |x| < 2^30
                q[c] = ok ? (int32_t)f : 0;                        // int(): toward zero
            }
            if (!ok) atomicOr(status, 1);
#pragma unroll
            for (int c = 0; c < 4; ++c) boxes_out[4 * o + c] = q[c];
            pts[2 * o] = 0.5 * (double)(q[0] + q[2]);
            pts[2 * o + 1] = 0.5 * (double)(q[1] + q[3]);
        }
        __syncthreads();
        if (t == 0) {
            int tot = 0;
            for (int w = 0; w < kPackThreads / 64; ++w) tot += s_wave[w];
            s_base += tot;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------- DLT ----
constexpr int kMaxViews = MVM_MAX_CAMS;

// One-sided (Hestenes) Jacobi SVD of the 2V x 4 DLT system, fp64, fully
// unrolled for a compile-time V so A and the rotations stay in registers:
// rotate column pairs until every pair is orthogonal to one ulp; V
// accumulates the rotations.  The right singular vector of the smallest
// singular value is the column of V whose rotated A-column has the smallest
// norm.  P: V row-major 3x4 matrices; xy: V points.
template <int NV>
__device__ __forceinline__ void dlt_point(const double *P, const double *xy, double X[3]) {
    constexpr int m = 2 * NV;
    double A[m][4];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const double x = xy[2 * v], y = xy[2 * v + 1];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double p2 = P[12 * v + 8 + c];
            A[2 * v][c] = x * p2 - P[12 * v + c];          // x * P[2] - P[0]   (:122)
            A[2 * v + 1][c] = y * p2 - P[12 * v + 4 + c];  // y * P[2] - P[1]   (:123)
        }
    }
    double W[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
            for (int b = a + 1; b < 4; ++b) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int r = 0; r < m; ++r) {
                    alpha += A[r][a] * A[r][a];
                    beta += A[r][b] * A[r][b];
                    gamma += A[r][a] * A[r][b];
                }
                if (fabs(gamma) > 2.220446049250313e-16 * sqrt(alpha * beta)) {
                    rotated = true;
                    const double zeta = (beta - alpha) / (2.0 * gamma);
                    const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
                    for (int r = 0; r < m; ++r) {
                        const double ra = A[r][a], rb = A[r][b];
                        A[r][a] = c * ra - s * rb;
                        A[r][b] = s * ra + c * rb;
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double va = W[r][a], vb = W[r][b];
                        W[r][a] = c * va - s * vb;
                        W[r][b] = s * va + c * vb;
                    }
                }
            }
        }
        if (!rotated) break;
    }
    double n2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        n2[c] = 0;
#pragma unroll
        for (int r = 0; r < m; ++r) n2[c] += A[r][c] * A[r][c];
    }
    double x0 = W[0][0], x1 = W[1][0], x2 = W[2][0], w = W[3][0], bn = n2[0];
#pragma unroll
    for (int c = 1; c < 4; ++c) {
        if (n2[c] < bn) {
            bn = n2[c];
            x0 = W[0][c], x1 = W[1][c], x2 = W[2][c], w = W[3][c];
        }
    }
    X[0] = x0 / w;
    X[1] = x1 / w;
    X[2] = x2 / w;
}

template <int NV>
__global__ __launch_bounds__(256) void dlt_kernel(const double *proj, const int32_t *set_of_point,
                                                  const double *pts2d, int32_t n_points,
                                                  double *X) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_points) return;
    const int64_t set = set_of_point ? (int64_t)set_of_point[p] : p;
    double xy[2 * NV], out[3];
#pragma unroll
    for (int k = 0; k < 2 * NV; ++k) xy[k] = pts2d[p * 2 * NV + k];
    dlt_point<NV>(proj + set * NV * 12, xy, out);
    X[3 * p + 0] = out[0];
    X[3 * p + 1] = out[1];
    X[3 * p + 2] = out[2];
}

template <int NV>
void launch_dlt(const double *proj, const int32_t *sop, const double *pts2d, int32_t n, double *X,
                hipStream_t s) {
    dlt_kernel<NV><<<(n + 255) / 256, 256, 0, s>>>(proj, sop, pts2d, n, X);
}

// ------------------------------------------- select + triangulate ----
// The tail of PoseEstimator._match for a batch of 3-camera captures
// (process_pose.py:182-187 with match_objects :100-116): for scene s, the
// assignment (row_ind, col_ind) of its flattened (N*M, P) cube is filtered by
// cost < threshold, decoded i = r / M, j = r % M, k = c, stably sorted by
// cost (Python's sorted on the float32 cube values; ties keep the
// assignment's ascending-row order), and each match's centroids are
// triangulated.  One workgroup per scene; ranks by counting through an LDS
// tile of costs (non-kept entries are +inf and never precede a kept one).
constexpr int kSelThreads = 256;
constexpr int kSelTile = 1024;

// the cube entry (r, k) of scene s: read from the cube, or -- cube-free
// (mvm_select_triangulate_resid) -- recomputed from the scene's fp64 pair
// residuals (mvm_triplet_minima's layout) with the cube's own arithmetic
struct SelSrc {
    const float *cb;
    const double *e12, *e13t, *e23t;   // e12 != nullptr: the residual form
    int64_t M, P;
    int ld;
    __device__ __forceinline__ float at(int64_t r, int64_t k) const {
        if (e12) {
            const int64_t i = r / M, j = r - i * M;
            return cube_f32(e12[i * ld + j], e13t[k * ld + i], e23t[k * ld + j]);
        }
        return cb[r * P + k];
    }
};

__global__ __launch_bounds__(kSelThreads) void select_triangulate_kernel(
    const float *cube, const int64_t *cube_offs, const int64_t *cam_offs,
    const int64_t *lsap_offs, const int64_t *row_ind, const int64_t *col_ind, const double *pts,
    const double *proj, double threshold, int32_t *match, float *cost_out, double *X,
    int32_t *count, const double *resid, int64_t rstride, int32_t rld, int32_t rrows) {
    __shared__ float s_cost[kSelTile];
    __shared__ int s_kept;
    const int s = blockIdx.x, t = threadIdx.x;
    const int64_t o = lsap_offs[s], n = lsap_offs[s + 1] - o;
    const int64_t c0 = cam_offs[3 * s], c1 = cam_offs[3 * s + 1], c2 = cam_offs[3 * s + 2];
    const int64_t M = c2 - c1, P = cam_offs[3 * s + 3] - c2;
    SelSrc cb{};
    cb.M = M;
    cb.P = P;
    if (resid) {
        cb.ld = rld;
        cb.e12 = resid + (int64_t)s * rstride;
        cb.e13t = cb.e12 + (int64_t)rrows * rld;
        cb.e23t = cb.e13t + (int64_t)rrows * rld;
    } else {
        cb.cb = cube + cube_offs[s];
    }
    if (t == 0) s_kept = 0;
    for (int64_t m0 = 0; m0 < n; m0 += kSelThreads) {
        const int64_t m = m0 + t;
        float mine = INFINITY;
        if (m < n) {
            const float v = cb.at(row_ind[o + m], col_ind[o + m]);
            if ((double)v < threshold) mine = v;
        }
        int64_t rank = 0;
        for (int64_t q0 = 0; q0 < n; q0 += kSelTile) {
            __syncthreads();
            for (int q = t; q < kSelTile && q0 + q < n; q += kSelThreads) {
                const float v = cb.at(row_ind[o + q0 + q], col_ind[o + q0 + q]);
                s_cost[q] = (double)v < threshold ? v : INFINITY;
            }
            __syncthreads();
            if (mine < INFINITY) {
                const int lim = (int)min<int64_t>(kSelTile, n - q0);
                for (int q = 0; q < lim; ++q) {
                    const float v = s_cost[q];
                    rank += (v < mine) || (v == mine && q0 + q < m);
                }
            }
        }
        if (mine < INFINITY) {
            atomicAdd(&s_kept, 1);
            const int64_t r = row_ind[o + m], k = col_ind[o + m];
            const int64_t i = r / M, j = r % M, w = o + rank;
            match[3 * w + 0] = (int32_t)i;
            match[3 * w + 1] = (int32_t)j;
            match[3 * w + 2] = (int32_t)k;
            cost_out[w] = mine;
            double xy[6], out[3];
            xy[0] = pts[2 * (c0 + i)], xy[1] = pts[2 * (c0 + i) + 1];
            xy[2] = pts[2 * (c1 + j)], xy[3] = pts[2 * (c1 + j) + 1];
            xy[4] = pts[2 * (c2 + k)], xy[5] = pts[2 * (c2 + k) + 1];
            dlt_point<3>(proj + (int64_t)s * 36, xy, out);
            X[3 * w + 0] = out[0];
            X[3 * w + 1] = out[1];
            X[3 * w + 2] = out[2];
        }
    }
    __syncthreads();
    if (t == 0) count[s] = s_kept;
}

}  // namespace

extern "C" {

int mvm_pack_detections(const float *boxes_dev, const float *conf_dev, const float *cls_dev,
                        const int64_t *img_offs_dev, int32_t n_img, float conf_thresh,
                        float class_id, int32_t *counts_dev, int64_t *cam_offs_dev,
                        double *pts_dev, int32_t *boxes_out_dev, int32_t *status_dev,
                        mvm_stream_t stream) {
    mvm_clear_error();
    if (n_img < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative n_img");
    if (n_img == 0) return MVM_OK;
    // the row arrays may be NULL when every image is empty
    if (!img_offs_dev || !counts_dev || !cam_offs_dev || !status_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (hipMemsetAsync(status_dev, 0, sizeof(int32_t), s) != hipSuccess)
        return mvm_fail(MVM_ERR_HIP, "hipMemsetAsync(status) failed");
    pack_count_kernel<<<n_img, kPackThreads, 0, s>>>(conf_dev, cls_dev, img_offs_dev, conf_thresh,
                                                     class_id, counts_dev);
    pack_scan_kernel<<<1, 1024, 0, s>>>(counts_dev, n_img, cam_offs_dev);
    pack_write_kernel<<<n_img, kPackThreads, 0, s>>>(boxes_dev, conf_dev, cls_dev, img_offs_dev,
                                                     conf_thresh, class_id, cam_offs_dev, pts_dev,
                                                     boxes_out_dev, status_dev);
    return mvm_check_launch("pack_detections");
}

int mvm_triangulate_dlt(const double *proj_dev, const int32_t *set_of_point_dev,
                        const double *pts2d_dev, int32_t n_points, int32_t n_views, double *X_dev,
                        mvm_stream_t stream) {
    mvm_clear_error();
    if (n_points < 0 || n_views < 2 || n_views > kMaxViews)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "n_points >= 0 and 2 <= n_views <= %d required",
                        kMaxViews);
    if (n_points == 0) return MVM_OK;
    if (!proj_dev || !pts2d_dev || !X_dev) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    switch (n_views) {
        case 2: launch_dlt<2>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
        case 3: launch_dlt<3>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
        case 4: launch_dlt<4>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
        case 5: launch_dlt<5>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
        case 6: launch_dlt<6>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
        case 7: launch_dlt<7>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
        default: launch_dlt<8>(proj_dev, set_of_point_dev, pts2d_dev, n_points, X_dev, s); break;
    }
    return mvm_check_launch("dlt_kernel");
}

int mvm_select_triangulate(const float *cube_dev, const int64_t *cube_offs_dev,
                           const int64_t *cam_offs_dev, const int64_t *lsap_out_offs_dev,
                           const int64_t *row_ind_dev, const int64_t *col_ind_dev,
                           const double *pts_dev, const double *proj_dev, int32_t n_scenes,
                           double threshold, int32_t *match_dev, float *cost_dev, double *X_dev,
                           int32_t *count_dev, mvm_stream_t stream) {
    mvm_clear_error();
    if (n_scenes < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative n_scenes");
    if (n_scenes == 0) return MVM_OK;
    if (!cube_offs_dev || !cam_offs_dev || !lsap_out_offs_dev || !proj_dev || !count_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    select_triangulate_kernel<<<n_scenes, kSelThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        cube_dev, cube_offs_dev, cam_offs_dev, lsap_out_offs_dev, row_ind_dev, col_ind_dev, pts_dev,
        proj_dev, threshold, match_dev, cost_dev, X_dev, count_dev, nullptr, 0, 0, 0);
    return mvm_check_launch("select_triangulate_kernel");
}

int mvm_select_triangulate_resid(const double *resid_dev, int32_t max_n, const int64_t *cam_offs_dev,
                                 const int64_t *lsap_out_offs_dev, const int64_t *row_ind_dev,
                                 const int64_t *col_ind_dev, const double *pts_dev,
                                 const double *proj_dev, int32_t n_scenes, double threshold,
                                 int32_t *match_dev, float *cost_dev, double *X_dev, int32_t *count_dev,
                                 mvm_stream_t stream) {
    mvm_clear_error();
    if (n_scenes < 0 || max_n < 0) return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "negative sizes");
    if (n_scenes == 0) return MVM_OK;
    if (!resid_dev || !cam_offs_dev || !lsap_out_offs_dev || !proj_dev || !count_dev)
        return mvm_fail(MVM_ERR_INVALID_ARGUMENT, "null pointer");
    const int32_t ld = (max_n + 3) / 4 * 4;
    select_triangulate_kernel<<<n_scenes, kSelThreads, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        nullptr, nullptr, cam_offs_dev, lsap_out_offs_dev, row_ind_dev, col_ind_dev, pts_dev, proj_dev,
        threshold, match_dev, cost_dev, X_dev, count_dev, resid_dev, (int64_t)3 * max_n * ld, ld, max_n);
    return mvm_check_launch("select_triangulate_kernel");
}

}  // extern "C"
