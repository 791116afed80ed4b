// triangulate.hip — batched two-view DLT triangulation.
//
// Reference: Estimator::TriangulateSinglePoint (src/processing/Estimator.cpp:1082-1137), called per
// matched feature by TriangulateNewMapPoints (:1139-1318) and, with the same algebra, by
// Initializer::TriangulateSinglePoint (src/processing/Initializer.cpp:728-800).
//   A.row(0) = b1(0)·T1w.row(2) − b1(2)·T1w.row(0)      (f32, as the reference builds it)
//   A.row(1) = b1(1)·T1w.row(2) − b1(2)·T1w.row(1)
//   A.row(2) = b2(0)·T2w.row(2) − b2(2)·T2w.row(0)
//   A.row(3) = b2(1)·T2w.row(2) − b2(2)·T2w.row(1)
//   v = right singular vector of A for the smallest singular value (JacobiSVD .matrixV().col(3));
//   invalid if |v(3)| < 1e-10; X = v.head<3>() / v(3); invalid unless finite.
// The reference runs Eigen's f32 two-sided JacobiSVD; here the 4x4 SVD is a one-sided (Hestenes)
// Jacobi in f64 on the f32-built A (the null vector is unique up to sign, which the division
// cancels), rounded to f32 at the end.  Also returns the reprojection angle errors in pixels that
// TriangulateNewMapPoints computes for each new point (:1233-1248; the reference logs them only).
//
// Layout: one lane per candidate, everything in registers (A: 16 f64, V: 16 f64).  Per candidate
// 24 B of bearings + 8 B of pose indices in, 12 + 8 + 1 B out; the poses (64 B each) are L2
// resident.  The Jacobi sweeps are ≈1.5 kFLOP f64 per candidate: at 1 M candidates the kernel sits
// between the HBM bound (45 MB) and the FP64 bound.
#include <hip/hip_runtime.h>

#include <cmath>

#include "ctx.h"

namespace vio360 {

constexpr int kMaxSweeps = 12;

struct TriArgs {
    const float* T;        // n_poses x 16, row-major world-to-camera
    int n_poses;
    const int32_t* pair;   // n x 2
    const float* bear;     // n x 6 (b1, b2)
    int n;
    float width;           // pixel error scale (GetWidth)
    float* X;              // n x 3
    uint8_t* valid;        // n
    float* pix_err;        // n x 2 or null
};

// angle error in pixels of X against bearing b in camera T (Estimator.cpp:1233-1248, f32)
__device__ __forceinline__ float reproj_px(const float* T, const float* b, const float* X, float width) {
    float pc[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) pc[r] = ((T[4 * r] * X[0] + T[4 * r + 1] * X[1]) + T[4 * r + 2] * X[2]) + T[4 * r + 3];
    const float nrm = sqrtf((pc[0] * pc[0] + pc[1] * pc[1]) + pc[2] * pc[2]);
    float dot = 0.f;
    if (nrm > 0.f) dot = (b[0] * (pc[0] / nrm) + b[1] * (pc[1] / nrm)) + b[2] * (pc[2] / nrm);
    const float ang = acosf(fminf(1.0f, fabsf(dot)));
    return (float)((double)(ang * width) / (2.0 * M_PI));  // float·int, then / (2.0f·M_PI) in double
}

__global__ __launch_bounds__(256) void triangulate_kernel(TriArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int p1 = a.pair[2 * i], p2 = a.pair[2 * i + 1];
    float b[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) b[k] = a.bear[6 * i + k];
    float T1[16], T2[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        T1[k] = a.T[16 * p1 + k];
        T2[k] = a.T[16 * p2 + k];
    }
    // A in f32 exactly as the reference builds it; columns of A held as f64 for the sweeps
    double col[4][4], V[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        col[c][0] = (double)(b[0] * T1[8 + c] - b[2] * T1[c]);
        col[c][1] = (double)(b[1] * T1[8 + c] - b[2] * T1[4 + c]);
        col[c][2] = (double)(b[3] * T2[8 + c] - b[5] * T2[c]);
        col[c][3] = (double)(b[4] * T2[8 + c] - b[5] * T2[4 + c]);
#pragma unroll
        for (int r = 0; r < 4; ++r) V[c][r] = (r == c) ? 1.0 : 0.0;
    }
    // one-sided Jacobi: rotate column pairs until every pair is orthogonal to working precision
    for (int sweep = 0; sweep < kMaxSweeps; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    al += col[p][r] * col[p][r];
                    be += col[q][r] * col[q][r];
                    ga += col[p][r] * col[q][r];
                }
                if (fabs(ga) > 1e-15 * sqrt(al * be) && ga != 0.0) {
                    rotated = true;
                    const double zeta = (be - al) / (2.0 * ga);
                    const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const double xp = col[p][r], xq = col[q][r];
                        col[p][r] = c * xp - s * xq;
                        col[q][r] = s * xp + c * xq;
                        const double vp = V[p][r], vq = V[q][r];
                        V[p][r] = c * vp - s * vq;
                        V[q][r] = s * vp + c * vq;
                    }
                }
            }
        if (!rotated) break;
    }
    // smallest singular value = shortest column; its V column is the null vector
    int kmin = 0;
    double nmin = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double nk = ((col[k][0] * col[k][0] + col[k][1] * col[k][1]) + col[k][2] * col[k][2]) + col[k][3] * col[k][3];
        if (k == 0 || nk < nmin) {
            nmin = nk;
            kmin = k;
        }
    }
    double v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = kmin == 0 ? V[0][r] : (kmin == 1 ? V[1][r] : (kmin == 2 ? V[2][r] : V[3][r]));
    bool ok = fabs(v[3]) >= 1e-10;
    float X[3] = {0.f, 0.f, 0.f};
    if (ok) {
#pragma unroll
        for (int r = 0; r < 3; ++r) X[r] = (float)(v[r] / v[3]);
        ok = isfinite(X[0]) && isfinite(X[1]) && isfinite(X[2]);
    }
    if (!ok) X[0] = X[1] = X[2] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r) a.X[3 * i + r] = X[r];
    a.valid[i] = ok ? 1 : 0;
    if (a.pix_err) {
        a.pix_err[2 * i] = ok ? reproj_px(T1, b, X, a.width) : 0.f;
        a.pix_err[2 * i + 1] = ok ? reproj_px(T2, b + 3, X, a.width) : 0.f;
    }
}

}  // namespace vio360

using namespace vio360;

extern "C" int vio_triangulate_device(vio_ctx* ctx, const float* T_cw, int n_poses, const int32_t* pose_pair,
                                      const float* bearings, int n, int width, float* points, uint8_t* valid,
                                      float* pixel_err) {
    if (!ctx || n < 0 || n_poses < 0 || (n > 0 && (!T_cw || !pose_pair || !bearings || !points || !valid)))
        return VIO_EINVAL;
    if (n == 0) return VIO_OK;
    TriArgs a{T_cw, n_poses, pose_pair, bearings, n, (float)width, points, valid, pixel_err};
    VIO_DEVICE(ctx);
    for (hipEvent_t& ev : ctx->tri_ev)
        if (!ev) VIO_HIP(ctx, hipEventCreate(&ev));
    VIO_HIP(ctx, hipEventRecord(ctx->tri_ev[0], ctx->stream));
    hipLaunchKernelGGL(triangulate_kernel, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, a);
    VIO_HIP(ctx, hipGetLastError());
    VIO_HIP(ctx, hipEventRecord(ctx->tri_ev[1], ctx->stream));
    return VIO_OK;
}

extern "C" int vio_triangulate(vio_ctx* ctx, const float* T_cw, int n_poses, const int32_t* pose_pair,
                               const float* bearings, int n, int width, float* points, uint8_t* valid,
                               float* pixel_err) {
    if (!ctx || n < 0 || n_poses < 0 || (n > 0 && (!T_cw || !pose_pair || !bearings || !points || !valid)))
        return VIO_EINVAL;
    for (int k = 0; k < 2 * n; ++k)
        if (pose_pair[k] < 0 || pose_pair[k] >= n_poses) {
            set_error(ctx, "vio_triangulate: pose index out of range");
            return VIO_EINVAL;
        }
    if (n == 0) return VIO_OK;
    const size_t bT = sizeof(float) * 16 * (size_t)n_poses, bP = sizeof(int32_t) * 2 * (size_t)n,
                 bB = sizeof(float) * 6 * (size_t)n;
    const size_t bX = sizeof(float) * 3 * (size_t)n, bE = sizeof(float) * 2 * (size_t)n, bV = (size_t)n;
    auto al = [](size_t v) { return (v + 255) / 256 * 256; };
    char* d_in = static_cast<char*>(ctx_buffer(ctx, kSlotTriIn, al(bT) + al(bP) + al(bB)));
    char* d_out = static_cast<char*>(ctx_buffer(ctx, kSlotTriOut, al(bX) + al(bE) + al(bV)));
    if (!d_in || !d_out) {
        set_error(ctx, "vio_triangulate: device allocation failed");
        return VIO_ENOMEM;
    }
    float* dT = reinterpret_cast<float*>(d_in);
    int32_t* dP = reinterpret_cast<int32_t*>(d_in + al(bT));
    float* dB = reinterpret_cast<float*>(d_in + al(bT) + al(bP));
    float* dX = reinterpret_cast<float*>(d_out);
    float* dE = reinterpret_cast<float*>(d_out + al(bX));
    uint8_t* dV = reinterpret_cast<uint8_t*>(d_out + al(bX) + al(bE));
    hipStream_t st = ctx->stream;
    VIO_DEVICE(ctx);
    VIO_HIP(ctx, hipMemcpyAsync(dT, T_cw, bT, hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipMemcpyAsync(dP, pose_pair, bP, hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipMemcpyAsync(dB, bearings, bB, hipMemcpyHostToDevice, st));
    int rc = vio_triangulate_device(ctx, dT, n_poses, dP, dB, n, width, dX, dV, pixel_err ? dE : nullptr);
    if (rc) return rc;
    VIO_HIP(ctx, hipMemcpyAsync(points, dX, bX, hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipMemcpyAsync(valid, dV, bV, hipMemcpyDeviceToHost, st));
    if (pixel_err) VIO_HIP(ctx, hipMemcpyAsync(pixel_err, dE, bE, hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipStreamSynchronize(st));
    return VIO_OK;
}

extern "C" int vio_triangulate_kernel_ms(vio_ctx* ctx, double* ms) {
    if (!ctx || !ms || !ctx->tri_ev[1]) return VIO_EINVAL;
    float f = 0.f;
    VIO_HIP(ctx, hipEventSynchronize(ctx->tri_ev[1]));
    VIO_HIP(ctx, hipEventElapsedTime(&f, ctx->tri_ev[0], ctx->tri_ev[1]));
    *ms = f;
    return VIO_OK;
}
