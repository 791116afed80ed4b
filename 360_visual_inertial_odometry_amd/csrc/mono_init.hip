// mono_init.hip — monocular two-view initialisation on device.
//
// Reference: Initializer::TryMonocularInitialization (src/processing/Initializer.cpp:47-291):
//   ComputeEssentialMatrix (:458-621)  RANSAC over 8-point hypotheses, |b2^T E b1| < thr inliers,
//                                      refit on the best hypothesis' inliers;
//   RecoverPose (:623-697)             four (R, t) candidates from the SVD of E, cheirality by
//                                      reprojection (TestPoseCandidate :785-835, 5 px);
//   TriangulatePoints (:699-783)       mid-point of the two rays for every pair;
//   ValidateInitialization (:889-995)  reprojection error in both frames <= max_reprojection_error;
//   NormalizeScale (:997-1048)         median distance -> 1.
//
// Kernels (one initialisation = three launches on the context stream):
//   mono_hyp_kernel    one lane per RANSAC hypothesis: the 8x9 system A (f32 products, as the
//                      reference builds it), G = A^T A in f64 (products of f32 are exact in f64),
//                      cyclic Jacobi of G in LDS ([entry][lane] layout, conflict-free), null vector
//                      = eigenvector of the smallest eigenvalue, projection onto singular values
//                      (s, s, 0) through the 3x3 eigen-decomposition of E^T E;
//   mono_count_kernel  one 256-thread workgroup per hypothesis: inlier count (integer LDS atomics,
//                      exact);
//   mono_finish_kernel one workgroup: best hypothesis, refit (fixed-order f64 partial sums: lane l
//                      of 64 sums rows i = l mod 64 in increasing i, partials summed in lane order),
//                      pose candidates, triangulation, validation (sequential f32 error sum, as the
//                      reference accumulates it), bitonic sort of the distances for the median.
// The reference's Eigen f32 JacobiSVD is replaced by f64 Jacobi on the f32-built systems; the null
// vector's sign is fixed (largest |component| positive) — E and -E give the same inliers, and the
// four pose candidates are the same set.  All per-point arithmetic is the reference's f32 (this file
// is built with -ffp-contract=off).  oracle/init_oracle.c restates the same steps on the CPU.
#include <hip/hip_runtime.h>

#include <cmath>

#include "ctx.h"
#include "mono_init_dev.h"

namespace vio360 {

constexpr int kHypLanes = 32;      // hypotheses per workgroup of mono_hyp_kernel (2 x 81 f64 per lane in LDS)
constexpr int kFinThreads = 256;

struct MonoArgs {
    const float* b1;        // n x 3
    const float* b2;        // n x 3
    int n;
    const int32_t* samples; // iters x 8
    int iters;
    vio_mono_init_params p;
    float* E_hyp;           // iters x 9
    int32_t* count;         // iters
    vio_mono_init_result* res;
    uint8_t* mask;          // n
    float* points;          // 3n
    float* err;             // n (validation scratch)
};

__global__ __launch_bounds__(kHypLanes) void mono_hyp_kernel(MonoArgs a) {
    __shared__ double G[81 * kHypLanes];
    __shared__ double V[81 * kHypLanes];
    const int lane = threadIdx.x;
    const int h = blockIdx.x * kHypLanes + lane;
    if (h >= a.iters) return;
    float rows[8][9];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int i = a.samples[8 * h + r];
        float b1[3], b2[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            b1[k] = a.b1[3 * i + k];
            b2[k] = a.b2[3 * i + k];
        }
        mi_epipolar_row(b1, b2, rows[r]);
    }
    double* g = G + lane;
    double* v = V + lane;
    for (int p = 0; p < 9; ++p)
        for (int q = p; q < 9; ++q) {
            double s = 0.0;
#pragma unroll
            for (int r = 0; r < 8; ++r) s += (double)rows[r][p] * (double)rows[r][q];
            g[(p * 9 + q) * kHypLanes] = s;
            g[(q * 9 + p) * kHypLanes] = s;
        }
    double e[9];
    mi_null_vector<9>(g, v, kHypLanes, e);
    float E[9];
    mi_project_essential(e, E);
#pragma unroll
    for (int k = 0; k < 9; ++k) a.E_hyp[9 * h + k] = E[k];
}

__global__ __launch_bounds__(256) void mono_count_kernel(MonoArgs a) {
    __shared__ int cnt;
    const int h = blockIdx.x;
    if (threadIdx.x == 0) cnt = 0;
    float E[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) E[k] = a.E_hyp[9 * h + k];
    __syncthreads();
    int mine = 0;
    for (int i = threadIdx.x; i < a.n; i += 256) {
        const float b1[3] = {a.b1[3 * i], a.b1[3 * i + 1], a.b1[3 * i + 2]};
        const float b2[3] = {a.b2[3 * i], a.b2[3 * i + 1], a.b2[3 * i + 2]};
        mine += mi_epipolar_error(E, b1, b2) < a.p.ransac_threshold ? 1 : 0;
    }
    if (mine) atomicAdd(&cnt, mine);
    __syncthreads();
    if (threadIdx.x == 0) a.count[h] = cnt;
}

struct FinShared {
    double part[45][64];
    double Gf[81], Vf[81];
    float keys[kMaxInitPoints];
    uint8_t mask[kMaxInitPoints];
    float E[9];
    float Rc[4][9], tc[4][3];
    int good[4];
    int best, best_count, status, ntri, ndepth, cand;
    float scale;
};

__device__ __forceinline__ void load_pair(const MonoArgs& a, int i, float* b1, float* b2) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        b1[k] = a.b1[3 * i + k];
        b2[k] = a.b2[3 * i + k];
    }
}

__global__ __launch_bounds__(kFinThreads) void mono_finish_kernel(MonoArgs a) {
    __shared__ FinShared sh;
    const int tid = threadIdx.x;
    const int n = a.n;
    vio_mono_init_result* res = a.res;
    if (tid == 0) {
        // first strictly-best hypothesis (:567-572); best_inliers starts at 0
        int best = -1, bc = 0;
        for (int h = 0; h < a.iters; ++h)
            if (a.count[h] > bc) {
                bc = a.count[h];
                best = h;
            }
        sh.best = best;
        sh.best_count = bc;
        sh.status = bc < a.p.min_features ? VIO_INIT_ESSENTIAL_FAILED : VIO_INIT_OK;
        sh.ntri = 0;
        sh.ndepth = 0;
        for (int c = 0; c < 4; ++c) sh.good[c] = 0;
        res->best_hypothesis = best;
        res->num_inliers = bc;
        res->pose_candidate = -1;
        for (int c = 0; c < 4; ++c) res->candidate_good[c] = 0;
        res->num_triangulated = 0;
        res->num_valid = 0;
        res->mean_reproj_error = 0.f;
        res->scale_factor = 1.f;
        for (int k = 0; k < 9; ++k) res->E[k] = res->R[k] = 0.f;
        for (int k = 0; k < 3; ++k) res->t[k] = 0.f;
    }
    __syncthreads();
    // inlier mask of the best hypothesis (same float expression as mono_count_kernel)
    {
        const int best = sh.best;
        float E[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) E[k] = best >= 0 ? a.E_hyp[9 * best + k] : 0.f;
        for (int i = tid; i < n; i += kFinThreads) {
            float b1[3], b2[3];
            load_pair(a, i, b1, b2);
            const uint8_t m = (best >= 0 && mi_epipolar_error(E, b1, b2) < a.p.ransac_threshold) ? 1 : 0;
            sh.mask[i] = m;
            if (a.mask) a.mask[i] = m;
            if (a.points) {
                a.points[3 * i] = a.points[3 * i + 1] = a.points[3 * i + 2] = 0.f;
            }
        }
    }
    __syncthreads();
    if (sh.status != VIO_INIT_OK) {
        if (tid == 0) res->status = sh.status;
        return;
    }
    // refit on all inliers (:583-616): G = A^T A, fixed-order partial sums
    for (int j = tid; j < 45 * 64; j += kFinThreads) {
        const int pq = j >> 6, l = j & 63;
        const int p = mi_pq_row(pq), q = mi_pq_col(pq);
        double s = 0.0;
        for (int i = l; i < n; i += 64) {
            if (!sh.mask[i]) continue;
            float b1[3], b2[3], row[9];
            load_pair(a, i, b1, b2);
            mi_epipolar_row(b1, b2, row);
            s += (double)row[p] * (double)row[q];
        }
        sh.part[pq][l] = s;
    }
    __syncthreads();
    if (tid < 45) {
        double s = 0.0;
        for (int l = 0; l < 64; ++l) s += sh.part[tid][l];
        const int p = mi_pq_row(tid), q = mi_pq_col(tid);
        sh.Gf[p * 9 + q] = s;
        sh.Gf[q * 9 + p] = s;
    }
    __syncthreads();
    if (tid == 0) {
        double e[9];
        mi_null_vector<9>(sh.Gf, sh.Vf, 1, e);
        mi_project_essential(e, sh.E);
        // RecoverPose candidates (:631-663)
        mi_pose_candidates(sh.E, sh.Rc, sh.tc);
    }
    __syncthreads();
    // TestPoseCandidate for the four candidates over the inliers (:785-835)
    for (int j = tid; j < 4 * n; j += kFinThreads) {
        const int c = j / n, i = j - c * n;
        if (!sh.mask[i]) continue;
        float b1[3], b2[3], X[3];
        load_pair(a, i, b1, b2);
        if (!mi_triangulate(b1, b2, sh.Rc[c], sh.tc[c], X)) continue;
        const float er = mi_reproj_error(X, b1, a.p.width, a.p.height);
        float X2[3];
        mi_transform(sh.Rc[c], sh.tc[c], X, X2);
        const float ec = mi_reproj_error(X2, b2, a.p.width, a.p.height);
        if (er < 5.0f && ec < 5.0f) atomicAdd(&sh.good[c], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int bc = 0, bi = -1;
        for (int c = 0; c < 4; ++c) {
            res->candidate_good[c] = sh.good[c];
            if (sh.good[c] > bc) {
                bc = sh.good[c];
                bi = c;
            }
        }
        sh.cand = bi;
        res->pose_candidate = bi;
        for (int k = 0; k < 9; ++k) res->E[k] = sh.E[k];
        if (bi < 0 || bc < a.p.min_features) sh.status = VIO_INIT_POSE_FAILED;
    }
    __syncthreads();
    if (sh.status != VIO_INIT_OK) {
        if (tid == 0) res->status = sh.status;
        return;
    }
    const float* R = sh.Rc[sh.cand];
    const float* t = sh.tc[sh.cand];
    // TriangulatePoints over every pair (:699-726) + the per-point validation terms (:911-957)
    int ntri = 0;
    for (int i = tid; i < n; i += kFinThreads) {
        float b1[3], b2[3], X[3] = {0.f, 0.f, 0.f};
        load_pair(a, i, b1, b2);
        const bool ok = mi_triangulate(b1, b2, R, t, X);
        if (!ok) X[0] = X[1] = X[2] = 0.f;
        ntri += ok ? 1 : 0;
        float e = -1.f;  // < 0: not counted
        if (sh.mask[i] && !((double)mi_norm3(X) < 1e-6)) {
            const float er = mi_reproj_error(X, b1, a.p.width, a.p.height);
            if (!(er > a.p.max_reprojection_error)) {
                float X2[3];
                mi_transform(R, t, X, X2);
                const float ec = mi_reproj_error(X2, b2, a.p.width, a.p.height);
                if (!(ec > a.p.max_reprojection_error)) e = fmaxf(er, ec);
            }
        }
        a.err[i] = e;
        if (a.points) {
            a.points[3 * i] = X[0];
            a.points[3 * i + 1] = X[1];
            a.points[3 * i + 2] = X[2];
        }
        // NormalizeScale depths (:1010-1019); +inf sorts past the valid ones
        const float nrm = mi_norm3(X);
        const bool dv = !(nrm < 1e-6f) && nrm > 0.01f;
        sh.keys[i] = dv ? nrm : INFINITY;
        if (dv) atomicAdd(&sh.ndepth, 1);
    }
    if (ntri) atomicAdd(&sh.ntri, ntri);
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = n + tid; i < np2; i += kFinThreads) sh.keys[i] = INFINITY;
    __threadfence_block();
    __syncthreads();
    if (tid == 0) {
        res->num_triangulated = sh.ntri;
        if (sh.ntri < a.p.min_features) {
            sh.status = VIO_INIT_TRIANGULATION;
        } else {
            // sequential f32 error sum in index order, as the reference accumulates it
            float sum = 0.f;
            int cnt = 0;
            for (int i = 0; i < n; ++i) {
                const float e = a.err[i];
                if (e >= 0.f) {
                    sum += e;
                    ++cnt;
                }
            }
            res->num_valid = cnt;
            res->mean_reproj_error = cnt ? sum / (float)cnt : 0.f;
            if (cnt == 0 || cnt < a.p.min_features) sh.status = VIO_INIT_VALIDATION;
        }
    }
    __syncthreads();
    if (sh.status != VIO_INIT_OK) {
        if (tid == 0) res->status = sh.status;
        return;
    }
    // bitonic sort of the distances (ascending) for the median
    for (int k = 2; k <= np2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < np2; i += kFinThreads) {
                const int ij = i ^ j;
                if (ij > i) {
                    const float x = sh.keys[i], y = sh.keys[ij];
                    const bool up = (i & k) == 0;
                    if (up ? (x > y) : (x < y)) {
                        sh.keys[i] = y;
                        sh.keys[ij] = x;
                    }
                }
            }
            __syncthreads();
        }
    if (tid == 0) {
        const int nd = sh.ndepth;
        float scale = 1.0f;
        if (nd > 0) {
            const int mid = nd / 2;
            const float med = (nd % 2 == 0) ? (sh.keys[mid - 1] + sh.keys[mid]) / 2.0f : sh.keys[mid];
            scale = 1.0f / med;
        }
        sh.scale = scale;
        res->scale_factor = scale;
        for (int k = 0; k < 9; ++k) res->R[k] = R[k];
        for (int k = 0; k < 3; ++k) res->t[k] = t[k] * scale;
        res->status = VIO_INIT_OK;
    }
    __syncthreads();
    if (a.points) {
        const float s = sh.scale;
        for (int i = tid; i < 3 * n; i += kFinThreads) a.points[i] = a.points[i] * s;
    }
}

}  // namespace vio360

using namespace vio360;

extern "C" int vio_mono_init_solve(vio_ctx* ctx, const float* bearings1, const float* bearings2, int n,
                                   const int32_t* samples, const vio_mono_init_params* params,
                                   vio_mono_init_result* res, uint8_t* inlier_mask, float* points) {
    if (!ctx || !params || !res || n < 0 || n > kMaxInitPoints || params->ransac_iterations < 0 ||
        params->ransac_iterations > (1 << 20) || (n > 0 && (!bearings1 || !bearings2)))
        return VIO_EINVAL;
    const int iters = params->ransac_iterations;
    *res = vio_mono_init_result{};
    res->best_hypothesis = -1;
    res->pose_candidate = -1;
    res->scale_factor = 1.f;
    if (n < 5) {  // :117-120 (and ComputeEssentialMatrix's own guard, :464-466)
        res->status = VIO_INIT_TOO_FEW_BEARINGS;
        if (inlier_mask)
            for (int i = 0; i < n; ++i) inlier_mask[i] = 0;
        if (points)
            for (int i = 0; i < 3 * n; ++i) points[i] = 0.f;
        return VIO_OK;
    }
    if (iters > 0) {
        // 8 distinct indices per hypothesis: the reference's sampler never terminates for n < 8
        if (!samples || n < 8) {
            set_error(ctx, "vio_mono_init_solve: need n >= 8 and a samples array");
            return VIO_EINVAL;
        }
        for (int k = 0; k < 8 * iters; ++k)
            if (samples[k] < 0 || samples[k] >= n) {
                set_error(ctx, "vio_mono_init_solve: sample index out of range");
                return VIO_EINVAL;
            }
    }
    auto al = [](size_t v) { return (v + 255) / 256 * 256; };
    const size_t bB = sizeof(float) * 3 * (size_t)n, bS = sizeof(int32_t) * 8 * (size_t)iters,
                 bE = sizeof(float) * 9 * (size_t)iters, bC = sizeof(int32_t) * (size_t)iters,
                 bR = sizeof(vio_mono_init_result), bM = (size_t)n, bP = sizeof(float) * 3 * (size_t)n,
                 bErr = sizeof(float) * (size_t)n;
    const size_t total = 2 * al(bB) + al(bS) + al(bE) + al(bC) + al(bR) + al(bM) + al(bP) + al(bErr);
    VIO_DEVICE(ctx);
    char* d = static_cast<char*>(ctx_buffer(ctx, kSlotMonoInit, total));
    if (!d) {
        set_error(ctx, "vio_mono_init_solve: device allocation failed");
        return VIO_ENOMEM;
    }
    MonoArgs a{};
    size_t off = 0;
    auto take = [&](size_t b) { char* p = d + off; off += al(b); return p; };
    float* dB1 = reinterpret_cast<float*>(take(bB));
    float* dB2 = reinterpret_cast<float*>(take(bB));
    int32_t* dS = reinterpret_cast<int32_t*>(take(bS));
    a.E_hyp = reinterpret_cast<float*>(take(bE));
    a.count = reinterpret_cast<int32_t*>(take(bC));
    a.res = reinterpret_cast<vio_mono_init_result*>(take(bR));
    a.mask = reinterpret_cast<uint8_t*>(take(bM));
    a.points = reinterpret_cast<float*>(take(bP));
    a.err = reinterpret_cast<float*>(take(bErr));
    a.b1 = dB1;
    a.b2 = dB2;
    a.n = n;
    a.samples = dS;
    a.iters = iters;
    a.p = *params;
    hipStream_t st = ctx->stream;
    for (hipEvent_t& ev : ctx->init_ev)
        if (!ev) VIO_HIP(ctx, hipEventCreate(&ev));
    VIO_HIP(ctx, hipMemcpyAsync(dB1, bearings1, bB, hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipMemcpyAsync(dB2, bearings2, bB, hipMemcpyHostToDevice, st));
    if (iters) VIO_HIP(ctx, hipMemcpyAsync(dS, samples, bS, hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipEventRecord(ctx->init_ev[0], st));
    if (iters) {
        hipLaunchKernelGGL(mono_hyp_kernel, dim3((iters + kHypLanes - 1) / kHypLanes), dim3(kHypLanes), 0, st, a);
        VIO_HIP(ctx, hipGetLastError());
        hipLaunchKernelGGL(mono_count_kernel, dim3(iters), dim3(256), 0, st, a);
        VIO_HIP(ctx, hipGetLastError());
    }
    hipLaunchKernelGGL(mono_finish_kernel, dim3(1), dim3(kFinThreads), 0, st, a);
    VIO_HIP(ctx, hipGetLastError());
    VIO_HIP(ctx, hipEventRecord(ctx->init_ev[1], st));
    VIO_HIP(ctx, hipMemcpyAsync(res, a.res, bR, hipMemcpyDeviceToHost, st));
    if (inlier_mask) VIO_HIP(ctx, hipMemcpyAsync(inlier_mask, a.mask, bM, hipMemcpyDeviceToHost, st));
    if (points) VIO_HIP(ctx, hipMemcpyAsync(points, a.points, bP, hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipStreamSynchronize(st));
    return VIO_OK;
}

extern "C" int vio_mono_init_kernel_ms(vio_ctx* ctx, double* ms) {
    if (!ctx || !ms || !ctx->init_ev[1]) return VIO_EINVAL;
    float f = 0.f;
    VIO_HIP(ctx, hipEventSynchronize(ctx->init_ev[1]));
    VIO_HIP(ctx, hipEventElapsedTime(&f, ctx->init_ev[0], ctx->init_ev[1]));
    *ms = f;
    return VIO_OK;
}
