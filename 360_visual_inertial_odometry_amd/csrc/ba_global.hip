// ba_global.hip — global bundle adjustment (config 5: 1000 KF x 50k landmarks) on MI355X.
//
// Same maths and Ceres-2.0 LM semantics as the windowed solver (ba_kernel.hip), for problems whose
// reduced camera system no longer fits one workgroup (RunBA / RunFullBA over hundreds of keyframes,
// src/optimization/Optimizer.cpp:304-491).  The LM control stays on the host (ba_global_host.cpp,
// scalars only); every O(N_obs) / O(L) / O(n^2..n^3) step is a kernel here:
//   gba_eval_kernel        BAFactor::Evaluate + Huber/Corrector, one lane per observation
//   gba_lin_lm_kernel      per-landmark V = Jl^T Jl, g_l, Jacobi scale (schur_eliminator_impl.h)
//   gba_lin_pose_kernel    per-pose U = Jp^T Jp, g_p (one wavefront per pose, shuffle reductions)
//   gba_step_lm_kernel     V~ = sVs + D^2 and its inverse (3x3 LLT), per landmark
//   gba_step_obs_kernel    W = (s Jp)^T (s Jl), Y = W V~^-1 per observation
//   gba_schur_kernel       S = diag(sUs + D^2) - sum Y W^T, one wavefront per 6x6 destination block,
//                          contributions pre-sorted by destination (deterministic, no atomics)
//   chol_* kernels         blocked right-looking Cholesky of S (64x64 tiles): diagonal POTRF + inverse
//                          in LDS, TRSM and the trailing SYRK/GEMM on v_mfma_f64_16x16x4_f64
//   trsv kernels           blocked forward / backward substitution with the diagonal inverses
//   gba_backsub_kernel     y_l = V~^-1 (g~_l - W^T y_p)
//   gba_model_kernel       model cost change, step / parameter norms, candidate = x + s*(-y)
// Reductions write per-block partials reduced in a fixed order: results are run-to-run bitwise stable.
#include <float.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>

#include "ba_factor_dev.h"
#include "ba_global.h"
#include "chol_dev.h"
#include "lie_dev.h"

namespace vio360 {

uint64_t gba_layout_sig_ba_global() { return gba_layout_sig(); }

constexpr int GT = 256;  // threads per block of the element-wise kernels

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
    return v;
}
// block reduction (GT threads) of up to 4 values: lane 0 of the block returns them
template <int NV>
__device__ __forceinline__ void block_reduce_store(double* v, double* out, bool is_max) {
    __shared__ double red[GT / 64][NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = is_max ? wave_max_d(v[q]) : wave_sum_d(v[q]);
    if ((threadIdx.x & 63) == 0)
        for (int q = 0; q < NV; ++q) red[threadIdx.x >> 6][q] = v[q];
    __syncthreads();
    if (threadIdx.x == 0)
        for (int q = 0; q < NV; ++q) {
            double r = red[0][q];
            for (int w = 1; w < GT / 64; ++w) r = is_max ? fmax(r, red[w][q]) : r + red[w][q];
            out[q] = r;
        }
}

// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(GT) gba_setup_kernel(GbaArgs A) {
    int k = blockIdx.x * GT + threadIdx.x;
    if (k >= A.K) return;
    const double* pr = A.pose_raw + 24 * k;
    double* pi = A.pinit + 24 * k;
    polar3(pr, pi);
    for (int i = 0; i < 3; ++i) pi[9 + i] = pr[9 + i];
    polar3(pr + 12, pi + 12);
    for (int i = 0; i < 3; ++i) pi[21 + i] = pr[21 + i];
}

__global__ void __launch_bounds__(GT) gba_pose_cache_kernel(GbaArgs A, const double* xp) {
    int k = blockIdx.x * GT + threadIdx.x;
    if (k >= A.K) return;
    pose_cache_one(A.pinit + 24 * k, xp + 6 * k, A.pc + 36 * k);
}

// cost (and Jacobians) at (pose cache, xl).  mode: 0 = active blocks, cost only; 1 = active blocks
// with Jacobians; 2 = the fixed (all-constant) blocks, cost only.  partial[blockIdx] = sum.
__global__ void __launch_bounds__(GT) gba_eval_kernel(GbaArgs A, const double* xl, int mode, double* partial) {
    const int N = A.N;
    int o = blockIdx.x * GT + threadIdx.x;
    double cost = 0.0;
    if (o < N) {
        int k = A.obs_kf[o], l = A.obs_lm[o];
        bool active = A.pose_f[k] >= 0 || A.lm_var[l];
        if ((mode == 2) != active) {
            const double* pc = A.pc + 36 * k;
            double Pw[3] = {xl[3 * l], xl[3 * l + 1], xl[3 * l + 2]};
            double r[2], Jp[12], Jl[6];
            bool jz;
            factor_eval(pc, A.pose_raw + 24 * k + 12, Pw, (double)A.obs_uv[2 * o], (double)A.obs_uv[2 * o + 1], A.cols,
                        A.rows, A.Lw, false, false, mode == 1, r, Jp, Jl, jz);
            double cst, sc;
            huber(A.huber, r[0] * r[0] + r[1] * r[1], cst, sc);
            cost = cst;
            if (mode == 1) {
                A.r[o] = r[0] * sc;
                A.r[N + o] = r[1] * sc;
#pragma unroll
                for (int i = 0; i < 12; ++i) A.jp[(size_t)i * N + o] = jz ? 0.0 : Jp[i] * sc;
#pragma unroll
                for (int i = 0; i < 6; ++i) A.jl[(size_t)i * N + o] = jz ? 0.0 : Jl[i] * sc;
            }
        }
    }
    double v[1] = {cost};
    block_reduce_store<1>(v, partial + blockIdx.x, false);
}

// fixed-order sum (or max) of n partials into out[0] — one block
__global__ void __launch_bounds__(GT) gba_reduce_kernel(const double* partial, int n, double* out, int is_max) {
    double acc = is_max ? 0.0 : 0.0;
    for (int i = threadIdx.x; i < n; i += GT) acc = is_max ? fmax(acc, partial[i]) : acc + partial[i];
    double v[1] = {acc};
    block_reduce_store<1>(v, out, is_max != 0);
}

// per landmark: V (6 packed), g_l (3), s_l at the first linearisation; partial = max |g_l|
__global__ void __launch_bounds__(GT) gba_lin_lm_kernel(GbaArgs A, int first, double* partial) {
    const int N = A.N, L = A.L;
    int l = blockIdx.x * GT + threadIdx.x;
    double gm = 0.0;
    if (l < L && A.lm_var[l]) {
        double v[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
        for (int o = A.lm_ptr[l]; o < A.lm_ptr[l + 1]; ++o) {
            double a0 = A.jl[o], a1 = A.jl[(size_t)N + o], a2 = A.jl[2 * (size_t)N + o];
            double b0 = A.jl[3 * (size_t)N + o], b1 = A.jl[4 * (size_t)N + o], b2 = A.jl[5 * (size_t)N + o];
            double ra = A.r[o], rb = A.r[N + o];
            v[0] += a0 * a0 + b0 * b0; v[1] += a0 * a1 + b0 * b1; v[2] += a0 * a2 + b0 * b2;
            v[3] += a1 * a1 + b1 * b1; v[4] += a1 * a2 + b1 * b2; v[5] += a2 * a2 + b2 * b2;
            g[0] += a0 * ra + b0 * rb; g[1] += a1 * ra + b1 * rb; g[2] += a2 * ra + b2 * rb;
        }
        for (int i = 0; i < 6; ++i) A.V[(size_t)i * L + l] = v[i];
        for (int i = 0; i < 3; ++i) A.gl[(size_t)i * L + l] = g[i];
        // Ceres' |x - Plus(x, -g)| term (trust_region_minimizer.cc:288-299)
        const double* xl = A.x_lm + 3 * (size_t)l;
        gm = fmax(fabs(xl[0] - (xl[0] + (-g[0]))), fmax(fabs(xl[1] - (xl[1] + (-g[1]))), fabs(xl[2] - (xl[2] + (-g[2])))));
        if (first) {
            A.sl[l] = 1.0 / (1.0 + sqrt(v[0]));
            A.sl[(size_t)L + l] = 1.0 / (1.0 + sqrt(v[3]));
            A.sl[2 * (size_t)L + l] = 1.0 / (1.0 + sqrt(v[5]));
        }
    }
    double vv[1] = {gm};
    block_reduce_store<1>(vv, partial + blockIdx.x, true);
}

// per pose (one wavefront): U (21 packed upper) and g_p (6) into A.U[27k]; f-space gradient,
// column norms, Jacobi scale; partial[blockIdx] = max |g_p|
__global__ void __launch_bounds__(GT) gba_lin_pose_kernel(GbaArgs A, int first, double* partial) {
    const int N = A.N;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k = blockIdx.x * (GT / 64) + wid;
    double gm = 0.0;
    if (k < A.K && A.pose_f[k] >= 0) {
        double acc[27];
#pragma unroll
        for (int i = 0; i < 27; ++i) acc[i] = 0.0;
        for (int q = A.kf_ptr[k] + lane; q < A.kf_ptr[k + 1]; q += 64) {
            int o = A.kf_obs[q];
            double a[6], b[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) { a[i] = A.jp[(size_t)i * N + o]; b[i] = A.jp[(size_t)(6 + i) * N + o]; }
            double ra = A.r[o], rb = A.r[N + o];
            int idx = 0;
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = i; j < 6; ++j) acc[idx++] += a[i] * a[j] + b[i] * b[j];
#pragma unroll
            for (int i = 0; i < 6; ++i) acc[21 + i] += a[i] * ra + b[i] * rb;
        }
#pragma unroll
        for (int i = 0; i < 27; ++i) acc[i] = wave_sum_d(acc[i]);
        if (lane < 27) {
            double mine = 0.0;
#pragma unroll
            for (int i = 0; i < 27; ++i) mine = lane == i ? acc[i] : mine;
            A.U[27 * k + lane] = mine;
        }
        const int pf = A.pose_f[k];
        if (lane < 6) {
            double g = 0.0, cs = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                g = lane == i ? acc[21 + i] : g;
                int di = i * 6 - (i * (i - 1)) / 2;
                cs = lane == i ? acc[di] : cs;
            }
            A.gf[pf + lane] = g;
            A.colsq_f[pf + lane] = cs;
            if (first) A.sf[pf + lane] = 1.0 / (1.0 + sqrt(cs));
        }
        for (int i = 0; i < 6; ++i) {
            const double xv = A.x_pose[6 * (size_t)k + i];
            gm = fmax(gm, fabs(xv - (xv + (-acc[21 + i]))));
        }
    }
    __shared__ double red[GT / 64];
    if (lane == 0) red[wid] = gm;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = red[0];
        for (int w = 1; w < GT / 64; ++w) r = fmax(r, red[w]);
        partial[blockIdx.x] = r;
    }
}

// V~ = s V s + D^2 (D^2 = clamp(diag(s V s))/radius), inverse by LLT; bad -> partial = 1
__global__ void __launch_bounds__(GT) gba_step_lm_kernel(GbaArgs A, double radius, double* partial) {
    const int L = A.L;
    const double dmin = 1e-6, dmax = 1e32;
    int l = blockIdx.x * GT + threadIdx.x;
    double bad = 0.0;
    if (l < L && A.lm_var[l]) {
        double s0 = A.sl[l], s1 = A.sl[(size_t)L + l], s2 = A.sl[2 * (size_t)L + l];
        double v[6];
        for (int i = 0; i < 6; ++i) v[i] = A.V[(size_t)i * L + l];
        double a00 = v[0] * s0 * s0, a01 = v[1] * s0 * s1, a02 = v[2] * s0 * s2;
        double a11 = v[3] * s1 * s1, a12 = v[4] * s1 * s2, a22 = v[5] * s2 * s2;
        a00 += fmin(fmax(a00, dmin), dmax) / radius;
        a11 += fmin(fmax(a11, dmin), dmax) / radius;
        a22 += fmin(fmax(a22, dmin), dmax) / radius;
        if (!(a00 > 0.0)) bad = 1.0;
        double l00 = sqrt(a00), l10 = a01 / l00, l20 = a02 / l00;
        double t11 = a11 - l10 * l10;
        if (!(t11 > 0.0)) bad = 1.0;
        double l11 = sqrt(t11), l21 = (a12 - l20 * l10) / l11;
        double t22 = a22 - l20 * l20 - l21 * l21;
        if (!(t22 > 0.0)) bad = 1.0;
        double l22 = sqrt(t22);
        double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
        double i10 = -l10 * i00 * i11, i21 = -l21 * i11 * i22;
        double i20 = -(l20 * i00 + l21 * i10) * i22;
        A.Vi[l] = i00 * i00 + i10 * i10 + i20 * i20;
        A.Vi[(size_t)L + l] = i10 * i11 + i20 * i21;
        A.Vi[2 * (size_t)L + l] = i20 * i22;
        A.Vi[3 * (size_t)L + l] = i11 * i11 + i21 * i21;
        A.Vi[4 * (size_t)L + l] = i21 * i22;
        A.Vi[5 * (size_t)L + l] = i22 * i22;
    }
    double v1[1] = {bad};
    block_reduce_store<1>(v1, partial + blockIdx.x, true);
}

// f-space LM diagonal and rhs, padding rows of the reduced system
__global__ void __launch_bounds__(GT) gba_step_f_kernel(GbaArgs A, double radius) {
    int f = blockIdx.x * GT + threadIdx.x;
    if (f >= A.nfp) return;
    if (f < A.nf) {
        double d = A.colsq_f[f] * A.sf[f] * A.sf[f];
        d = fmin(fmax(d, 1e-6), 1e32);
        A.Df[f] = sqrt(d / radius);
        A.bf[f] = A.sf[f] * A.gf[f];
    } else {
        A.Df[f] = 0.0;
        A.bf[f] = 0.0;
    }
}

// per observation: W = (s_p Jp)^T (s_l Jl) (6x3, row-major) and Y = W V~^-1
__global__ void __launch_bounds__(GT) gba_step_obs_kernel(GbaArgs A) {
    const int N = A.N, L = A.L;
    int o = blockIdx.x * GT + threadIdx.x;
    if (o >= N) return;
    int k = A.obs_kf[o], l = A.obs_lm[o];
    int pf = A.pose_f[k];
    if (pf < 0 || !A.lm_var[l]) return;
    double s0 = A.sl[l], s1 = A.sl[(size_t)L + l], s2 = A.sl[2 * (size_t)L + l];
    double vi[6];
    for (int i = 0; i < 6; ++i) vi[i] = A.Vi[(size_t)i * L + l];
    double b0 = A.jl[o] * s0, b1 = A.jl[(size_t)N + o] * s1, b2 = A.jl[2 * (size_t)N + o] * s2;
    double d0 = A.jl[3 * (size_t)N + o] * s0, d1 = A.jl[4 * (size_t)N + o] * s1, d2 = A.jl[5 * (size_t)N + o] * s2;
    double* W = A.Wo + 18 * (size_t)o;
    double* Y = A.Yo + 18 * (size_t)o;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double sp = A.sf[pf + i];
        double a = A.jp[(size_t)i * N + o] * sp, e = A.jp[(size_t)(6 + i) * N + o] * sp;
        double W0 = a * b0 + e * d0, W1 = a * b1 + e * d1, W2 = a * b2 + e * d2;
        W[3 * i] = W0; W[3 * i + 1] = W1; W[3 * i + 2] = W2;
        Y[3 * i] = W0 * vi[0] + W1 * vi[1] + W2 * vi[2];
        Y[3 * i + 1] = W0 * vi[1] + W1 * vi[3] + W2 * vi[4];
        Y[3 * i + 2] = W0 * vi[2] + W1 * vi[4] + W2 * vi[5];
    }
}

// S lower triangle, one wavefront per 6x6 destination block (pa >= pb pose blocks):
//   S[pa,pb] = [pa == pb] (s U s + D^2) - sum over co-observations Y_oa W_ob^T
// lane (i, j) < 36 sums entry (i, j) over the block's contributions in list (landmark) order, four at a
// time with their loads in flight.  Measured and not kept (round 5, profiles/r5_gba_schur_ab.log): 8-deep
// batches (1.0 ms per launch against 0.55: the deeper batch's registers halve the waves in flight), 4-deep
// batches with the tail predicated instead of serial (0.69-0.81 ms), a lane per block (36 sums per lane,
// 16-B row loads: 1.2 ms, every load instruction touching 64 lines).
__global__ void __launch_bounds__(GT) gba_schur_kernel(GbaArgs A) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long d = (long long)blockIdx.x * (GT / 64) + wid;
    if (d >= A.n_dest) return;
    const int pa = A.dest_a[d], pb = A.dest_b[d];
    if (lane >= 36) return;
    const int i = lane / 6, j = lane % 6;
    double acc = 0.0;
    const int cbeg = A.dest_ptr[d], cend = A.dest_ptr[d + 1];
    int c = cbeg;
    for (; c + 4 <= cend; c += 4) {
        double y[4][3], w[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double* Y = A.Yo + 18 * (size_t)A.contrib_a[c + u] + 3 * i;
            const double* W = A.Wo + 18 * (size_t)A.contrib_b[c + u] + 3 * j;
#pragma unroll
            for (int e = 0; e < 3; ++e) { y[u][e] = Y[e]; w[u][e] = W[e]; }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += y[u][0] * w[u][0] + y[u][1] * w[u][1] + y[u][2] * w[u][2];
    }
    for (; c < cend; ++c) {
        const double* Y = A.Yo + 18 * (size_t)A.contrib_a[c] + 3 * i;
        const double* W = A.Wo + 18 * (size_t)A.contrib_b[c] + 3 * j;
        acc += Y[0] * W[0] + Y[1] * W[1] + Y[2] * W[2];
    }
    const int fa = 6 * pa + i, fb = 6 * pb + j;
    double v = -acc;
    if (pa == pb) {
        const int k = A.pose_of_block[pa];
        int a = min(i, j), b = max(i, j);
        int idx = a * 6 - (a * (a - 1)) / 2 + (b - a);
        v += A.U[27 * k + idx] * A.sf[fa] * A.sf[fb];
        if (i == j) v += A.Df[fa] * A.Df[fa];
    }
    A.S[(size_t)fa * A.nfp + fb] = v;
}

// padding rows/cols [nf, nfp) of S: identity
__global__ void __launch_bounds__(GT) gba_pad_kernel(GbaArgs A) {
    const int pad = A.nfp - A.nf;
    int e = blockIdx.x * GT + threadIdx.x;
    if (e >= pad * A.nfp) return;
    int r = A.nf + e / A.nfp, c = e % A.nfp;
    A.S[(size_t)r * A.nfp + c] = (r == c) ? 1.0 : 0.0;
}

// rhs: b_p -= sum_{o in obs(p)} Y_o g~_l(o)   (one wavefront per pose)
__global__ void __launch_bounds__(GT) gba_rhs_kernel(GbaArgs A) {
    const int L = A.L;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k = blockIdx.x * (GT / 64) + wid;
    if (k >= A.K || A.pose_f[k] < 0) return;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int q = A.kf_ptr[k] + lane; q < A.kf_ptr[k + 1]; q += 64) {
        int o = A.kf_obs[q], l = A.obs_lm[o];
        if (!A.lm_var[l]) continue;
        double g0 = A.gl[l] * A.sl[l], g1 = A.gl[(size_t)L + l] * A.sl[(size_t)L + l];
        double g2 = A.gl[2 * (size_t)L + l] * A.sl[2 * (size_t)L + l];
        const double* Y = A.Yo + 18 * (size_t)o;
#pragma unroll
        for (int i = 0; i < 6; ++i) acc[i] += Y[3 * i] * g0 + Y[3 * i + 1] * g1 + Y[3 * i + 2] * g2;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) acc[i] = wave_sum_d(acc[i]);
    if (lane < 6) {
        double mine = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) mine = lane == i ? acc[i] : mine;
        A.bf[A.pose_f[k] + lane] -= mine;
    }
}

// ------------------------------------------------------------------------------------------
// Blocked Cholesky, NB = 64.  Lower triangle of S (row-major, leading dimension n).
constexpr int NB = 64;
using d4 = __attribute__((ext_vector_type(4))) double;

// diagonal block: in-LDS right-looking Cholesky + lower-triangular inverse (for TRSM / TRSV).
// One barrier per column: the trailing update reads the unscaled column j (T[i][c] -= T[i][j] T[c][j] / d)
// and the column is scaled after the barrier, which the next column's update never touches.
// Diagonal block k (64x64): L_kk and L_kk^-1, blocked over 16x16 tiles in LDS.  For each tile
// column J: one wave factors the diagonal tile (chol16_wave), the panel tiles below become
// L_IJ = S_IJ Linv_J^T and the trailing lower tiles S_IK -= L_IJ L_KJ^T, both on
// v_mfma_f64_16x16x4_f64, one tile per wave.  The inverse is then built block row by block row,
// X_IJ = -Linv_II sum_{J<=K<I} L_IK X_KJ, again on MFMA.  Dynamic LDS: CHOL_DIAG_LDS bytes.
constexpr int TLD = NB + 1;  // odd row stride: the column reads of the MFMA operands spread over banks
constexpr size_t CHOL_DIAG_LDS = sizeof(double) * (2 * NB * TLD + 4 * 256 + 256 + 4 * 16 * 17);
// factor the 64x64 block held in T (lower part, row stride TLD) in place into L and build X = L^-1
// (X zeroed by the caller); LB / LT / P: scratch as laid out by diag_lds_layout.  Returns nonzero
// (the same in every thread) when a pivot is not positive.
// (a call: inlined into chol_diag_kernel / chol_chain_kernel it removes their 12-B stack but costs the chained
// Cholesky ≈ 5 % per LM iteration, profiles/r5s_gba_inline_ab.log -- those launches are one workgroup wide)
__device__ int diag_block_lds(double* T, double* X, double* LB, double* LT, double* P, int& bad_s) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    constexpr int NT = NB / 16;
    // trailing update of the lower tile (I, K) by tile column J
    auto trail = [&](int I, int Kt, int J) {
        const int c0 = 16 * J;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        const double* Ai = T + 16 * I * TLD + c0;
        const double* Bk = T + 16 * Kt * TLD + c0;
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const double a = Ai[r16 * TLD + 4 * st + kk];
            const double bb = Bk[r16 * TLD + 4 * st + kk];
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
        }
        double* C = T + 16 * I * TLD + 16 * Kt;
#pragma unroll
        for (int r = 0; r < 4; ++r) C[(kk + 4 * r) * TLD + r16] -= acc[r];
    };
    // one-step look-ahead (as the window solver's cholesky_solve_rhs): after the panel of column J,
    // wave 0 updates and factors the next diagonal tile while the other waves finish column J's
    // trailing update; each tile still receives its updates in column order
    if (wid == 0) {
        const int bad = chol16_wave<true>(T, TLD, LB, LT, lane);
        if (lane == 0) bad_s = bad;
    }
    __syncthreads();
    for (int J = 0; J < NT; ++J) {
        const int c0 = 16 * J;
        if (bad_s) return 1;
        const double* lb = LB + 256 * J;
        for (int I = J + 1 + wid; I < NT; I += 4) {  // panel
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            double* A = T + 16 * I * TLD + c0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const double a = A[r16 * TLD + 4 * st + kk];
                const double bb = lb[(4 * st + kk) * 16 + r16];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(kk + 4 * r) * TLD + r16] = acc[r];
        }
        __syncthreads();
        if (J + 1 == NT) break;
        if (wid == 0) {
            trail(J + 1, J + 1, J);
            wave_lds_sync();
            const int bad = chol16_wave<true>(T + (c0 + 16) * TLD + c0 + 16, TLD, LB + 256 * (J + 1), LT, lane);
            if (lane == 0) bad_s = bad;
        } else {
            const int m = NT - J - 1, nt = m * (m + 1) / 2;
            for (int t = wid; t < nt; t += 3) {  // trailing lower tiles (I, K), J < K <= I, except (J+1, J+1)
                int I = 0, tt = t;
                while (tt > I) { tt -= I + 1; ++I; }
                trail(I + J + 1, tt + J + 1, J);
            }
        }
        __syncthreads();
    }
    if (bad_s) return 1;
    for (int e = threadIdx.x; e < NT * 256; e += 256) {  // diagonal tiles of the inverse
        const int J = e >> 8, q = (e >> 4) & 15, i = e & 15;
        X[(16 * J + q) * TLD + 16 * J + i] = LB[256 * J + 16 * i + q];
    }
    __syncthreads();
    for (int I = 1; I < NT; ++I) {
        if (wid < I) {
            const int J = wid;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            for (int K = J; K < I; ++K)
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    const double a = T[(16 * I + r16) * TLD + 16 * K + 4 * st + kk];
                    const double bb = X[(16 * K + 4 * st + kk) * TLD + 16 * J + r16];
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
                }
            double* Pw = P + wid * 16 * 17;
#pragma unroll
            for (int r = 0; r < 4; ++r) Pw[(kk + 4 * r) * 17 + r16] = acc[r];
            wave_lds_sync();
            d4 acc2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const double a = LB[256 * I + (4 * st + kk) * 16 + r16];  // Linv_II[r16][4 st + kk]
                const double bb = Pw[(4 * st + kk) * 17 + r16];
                acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc2, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) X[(16 * I + kk + 4 * r) * TLD + 16 * J + r16] = -acc2[r];
        }
        __syncthreads();
    }
    return 0;
}

__global__ void __launch_bounds__(256) chol_diag_kernel(double* S, int n, int k, double* Linv, int* fail) {
    extern __shared__ double dyn[];
    double* T = dyn;             // [NB][TLD] S_kk, then L_kk
    double* X = T + NB * TLD;    // [NB][TLD] L_kk^-1
    double* LB = X + NB * TLD;   // [4][16 m][16 c] = Linv_J[c][m] of the diagonal tiles
    double* LT = LB + 4 * 256;   // scratch of chol16_wave
    double* P = LT + 256;        // [4 waves][16][17] product scratch of the inverse
    __shared__ int bad_s;
    double* blk = S + (size_t)k * NB * n + (size_t)k * NB;
    {
        constexpr int PER = NB * NB / 256;  // loads first, then the LDS stores
        double v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int e = threadIdx.x + 256 * u, r = e >> 6, c = e & 63;
            v[u] = c <= r ? blk[(size_t)r * n + c] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int e = threadIdx.x + 256 * u, r = e >> 6, c = e & 63;
            T[r * TLD + c] = v[u];
            X[r * TLD + c] = 0.0;
        }
    }
    __syncthreads();
    if (diag_block_lds(T, X, LB, LT, P, bad_s)) {
        if (threadIdx.x == 0) *fail = 1;
        return;
    }
    double* Li = Linv + (size_t)k * NB * NB;
    for (int e = threadIdx.x; e < NB * NB; e += 256) {
        const int r = e >> 6, c = e & 63;
        if (c <= r) blk[(size_t)r * n + c] = T[r * TLD + c];
        Li[e] = X[r * TLD + c];
    }
}

// two 64x64 tiles into LDS: all 32 global loads of a lane are issued before the first LDS store
// (one memory round trip instead of sixteen)
__device__ __forceinline__ void stage_tiles(double (*As)[NB + 1], double (*Bs)[NB + 1], const double* A, size_t lda,
                                            const double* B, size_t ldb) {
    constexpr int PER = NB * NB / 256;
    double va[PER], vb[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int e = threadIdx.x + 256 * u, r = e / NB, c = e % NB;
        va[u] = A[(size_t)r * lda + c];
        vb[u] = B[(size_t)r * ldb + c];
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int e = threadIdx.x + 256 * u, r = e / NB, c = e % NB;
        As[r][c] = va[u];
        Bs[r][c] = vb[u];
    }
}

// 64x64x64 tile product on MFMA f64: acc(wave's 32x32) += A(64xK) * B(64xK)^T from LDS
// wave w: rows 32*(w>>1) .. +32, cols 32*(w&1) .. +32 ; 2x2 MFMA 16x16 tiles
__device__ __forceinline__ void mfma_tile_ABt(const double (*As)[NB + 1], const double (*Bs)[NB + 1], d4 acc[2][2],
                                              int wid, int lane) {
    const int r0 = 32 * (wid >> 1), c0 = 32 * (wid & 1);
    const int li = lane & 15, lk = lane >> 4;
    for (int kk = 0; kk < NB; kk += 4) {
        double a[2], b[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            a[t] = As[r0 + 16 * t + li][kk + lk];   // A[i][k]
            b[t] = Bs[c0 + 16 * t + li][kk + lk];   // B^T[k][j] = B[j][k]
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj) acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
    }
}

// panel: A_ik <- A_ik * Linv_kk^T for every block row i > k
__global__ void __launch_bounds__(256) chol_trsm_kernel(double* S, int n, int k, const double* Linv) {
    __shared__ double As[NB][NB + 1];
    __shared__ double Bs[NB][NB + 1];
    const int i = k + 1 + blockIdx.x;
    double* blk = S + (size_t)i * NB * n + (size_t)k * NB;
    const double* Li = Linv + (size_t)k * NB * NB;
    stage_tiles(As, Bs, blk, (size_t)n, Li, NB);
    __syncthreads();
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    d4 acc[2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0, 0, 0, 0};
    mfma_tile_ABt(As, Bs, acc, wid, lane);
    const int r0 = 32 * (wid >> 1), c0 = 32 * (wid & 1);
    for (int ti = 0; ti < 2; ++ti)
        for (int tj = 0; tj < 2; ++tj)
            for (int q = 0; q < 4; ++q) {
                int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                blk[(size_t)r * n + c] = acc[ti][tj][q];
            }
}

// trailing update: A_ij -= A_ik A_jk^T for k < j <= i (lower block triangle), one tile per block.
// part 0: every tile; part 1: the first trailing column only (j = k+1, the next step's diagonal
// block and panel); part 2: the rest (j >= k+2) — the look-ahead split of gba_launch_cholesky; part 3:
// part 2 without its first tile, the diagonal block (k+2, k+2) (the chained schedule's diagonal
// workgroup applies that one itself, chol_chain_kernel).
// tile t of the update (one workgroup); As / Bs: NB x (NB + 1) doubles of LDS each
__device__ __forceinline__ void syrk_tile(double* S, int n, int k, int part, long long t, double (*As)[NB + 1],
                                          double (*Bs)[NB + 1]) {
    if (part == 3) {
        part = 2;
        ++t;
    }
    // t -> (i, j) with 0 <= jj <= ii < m, i = k+1+ii, j = k+1+jj
    int ii = 0, jj = 0;
    if (part == 1) {
        ii = (int)t;
    } else {
        ii = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
        while ((long long)(ii + 1) * (ii + 2) / 2 <= t) ++ii;
        while ((long long)ii * (ii + 1) / 2 > t) --ii;
        jj = (int)(t - (long long)ii * (ii + 1) / 2);
        if (part == 2) { ++ii; ++jj; }  // the triangle below-right of the first trailing column
    }
    const int i = k + 1 + ii, j = k + 1 + jj;
    const double* Aik = S + (size_t)i * NB * n + (size_t)k * NB;
    const double* Ajk = S + (size_t)j * NB * n + (size_t)k * NB;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r0 = 32 * (wid >> 1), c0 = 32 * (wid & 1);
    double* C = S + (size_t)i * NB * n + (size_t)j * NB;
    // the lane's 16 destination values are fetched first: their latency overlaps the staging and
    // the MFMAs instead of following them
    double cv[2][2][4];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                cv[ti][tj][q] = C[(size_t)r * n + c];
            }
    stage_tiles(As, Bs, Aik, (size_t)n, Ajk, (size_t)n);
    __syncthreads();
    d4 acc[2][2];
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0, 0, 0, 0};
    mfma_tile_ABt(As, Bs, acc, wid, lane);
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                if (i != j || c <= r) C[(size_t)r * n + c] = cv[ti][tj][q] - acc[ti][tj][q];
            }
}
__global__ void __launch_bounds__(256) chol_syrk_kernel(double* S, int n, int k, int part) {
    __shared__ double As[NB][NB + 1];
    __shared__ double Bs[NB][NB + 1];
    syrk_tile(S, n, k, part, blockIdx.x, As, Bs);
}

// forward substitution step k: y_k = Linv_kk b_k (every block recomputes it from the final b_k;
// block 0 publishes it), then b_r -= L_rk y_k for the 32 rows of the block below: 8 lanes per row,
// each lane two-term products over 4 double2 column pairs, reduced over its 8 lanes — the row dot of
// trsv_fwd_persistent_kernel in the same order, so both paths give the same bits
__global__ void __launch_bounds__(256) trsv_fwd_kernel(const double* S, int n, int k, const double* Linv, double* b,
                                                       double* y) {
    __shared__ double yk[NB];
    __shared__ double pt[4][64];
    const double* Li = Linv + (size_t)k * NB * NB;
    {   // y_k[r] = Linv_kk[r][:] b_k as the four 16-column group sums ((p0 + p1) + (p2 + p3))
        const int r = threadIdx.x & 63, g = threadIdx.x >> 6;
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int q = 16 * g + u;
            if (q <= r) s += Li[r * NB + q] * b[k * NB + q];
        }
        pt[g][r] = s;
    }
    __syncthreads();
    if (threadIdx.x < NB) yk[threadIdx.x] = (pt[0][threadIdx.x] + pt[1][threadIdx.x]) + (pt[2][threadIdx.x] + pt[3][threadIdx.x]);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < NB) y[k * NB + threadIdx.x] = yk[threadIdx.x];
    const int lane = threadIdx.x & 63, c8 = lane & 7;
    const int r = (k + 1) * NB + blockIdx.x * 32 + (threadIdx.x >> 3);
    double2 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = r < n ? *reinterpret_cast<const double2*>(S + (size_t)r * n + (size_t)k * NB + 16 * j + 2 * c8)
                     : make_double2(0.0, 0.0);
    double yv[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        yv[j][0] = yk[16 * j + 2 * c8];
        yv[j][1] = yk[16 * j + 2 * c8 + 1];
    }
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) t += v[j].x * yv[j][0] + v[j].y * yv[j][1];
#pragma unroll
    for (int off = 4; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
    if (c8 == 0 && r < n) b[r] -= t;
}

// backward substitution step k (k = nblk-1 .. 0): x_k = Linv_kk^T y_k, y_c -= sum_q L[kNB+q][c] x_k[q]
// for c < kNB: 64 columns per block, the q-sum split over 4 thread groups and combined in LDS
__global__ void __launch_bounds__(256) trsv_bwd_kernel(const double* S, int n, int k, const double* Linv, double* y,
                                                       double* x) {
    __shared__ double xk[NB];
    __shared__ double part[4][64];
    const double* Li = Linv + (size_t)k * NB * NB;
    {   // x_k[c] = Linv_kk[:][c] . y_k as the four 16-row group sums ((p0 + p1) + (p2 + p3))
        const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int q = 16 * g + u;
            if (q >= c) s += Li[q * NB + c] * y[k * NB + q];
        }
        part[g][c] = s;
    }
    __syncthreads();
    if (threadIdx.x < NB) xk[threadIdx.x] = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < NB) x[k * NB + threadIdx.x] = xk[threadIdx.x];
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    double s = 0.0;
    if (c < k * NB) {
        double v[16];  // loads first, then the ordered sum
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = S[(size_t)(k * NB + g * 16 + u) * n + c];
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u] * xk[g * 16 + u];
    }
    part[g][cl] = s;
    __syncthreads();
    if (g == 0 && c < k * NB) y[c] -= (part[0][cl] + part[1][cl]) + (part[2][cl] + part[3][cl]);
}

// ------------------------------------------------------------------------------------------
// Persistent triangular solves: one workgroup per 64-row block, all blocks resident at once
// (nblk <= 256 workgroups of 256 threads, no LDS to speak of), each block publishing its solution
// slice through a flag.  Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, sc1 form): the
// slice is stored with agent-scope relaxed (sc1, write-through) stores, every storing wave waits
// vmcnt(0), a workgroup barrier, then one lane stores the flag sc1; the consumer polls the flag with
// sc1 loads from one lane, joins a barrier and loads the slice with sc1 global loads.  Flags sit
// one per 128-B line.  The arithmetic is the per-step kernels' above, in the same order (each row /
// column dot reduced the same way, the updates applied in the same k order), so the results are
// bitwise theirs; what goes is 2 x nblk launches and the idle tail of every step.
constexpr int FLAG_STRIDE = 32;  // ints: one flag per 128-B line
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) int gint;
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load((gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// bounded spins (chol_dev.h wait_expired: 2 s of wall clock, orders of magnitude above any legitimate
// wait -- a whole LM iteration is ~5 ms); a timed-out wait sets the solve's timeout word, which the host
// reports as a device error
__device__ __forceinline__ bool flag_wait(int* f) {
    // bounded spin: a producer that never arrives ends the wait instead of hanging the GPU
    const unsigned long long t0 = wait_clock();
    for (;;) {
        if (__hip_atomic_load((gint*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return true;
        if (wait_expired(t0)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}
// triangular-solve hand-off without a flag: the consumer polls the 64 values themselves (set to this
// NaN pattern before the solve; each 8-B value is stored whole), one round trip instead of flag +
// data.  Called by the 64 lanes of one wave; false on a timed-out wait.
constexpr unsigned long long kUnsetBits = ~0ull;
__device__ __forceinline__ bool poll_block(const double* p, double& v) {
    bool pend = true;
    const unsigned long long t0 = wait_clock();
    for (;;) {
        if (pend) {
            v = ld_sc1(p);
            pend = (unsigned long long)__double_as_longlong(v) == kUnsetBits;
        }
        if (__ballot(pend) == 0ull) return true;
        if (wait_expired(t0)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ void flag_publish(int* f) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((gint*)f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Chained Cholesky launch k (the critical chain of the look-ahead schedule, one launch per block
// column, no waits inside): workgroup b < m = nblk - k - 1 forms the panel block L_{k+1+b, k}: column
// k-1's update of S_{k+1+b, k}, then the product with L_kk^-T (L_kk^-1 is final: the previous launch
// wrote it).  Workgroup 0 then goes on to the next diagonal block d = k+1: column k-1's update of S_dd
// (the first tile of chol_syrk_kernel part 2 of step k-1, which the trailing update therefore leaves
// out: part 3), column k's update with the panel block L_{d,k} it has just formed (still in LDS, no
// hand-off), the factor and L_dd^-1 (diag_block_lds).  Launch k = -1: workgroup 0 factors block 0.
// The arithmetic is chol_syrk_kernel's, chol_diag_kernel's and chol_trsm_kernel's in the same order:
// bitwise the three-launch schedule.  Workgroups past m (trail > 0: `trail` of them) apply step k-1's
// trailing update right of block column k+1 (part 3 of step k-1, its tiles in order): disjoint from
// block columns k and k+1 and from S_dd, after panel k-1 (the previous launch) and before launch k+1,
// so the look-ahead needs no second stream for it.  Workgroup 1 (the owner of L_{k+2,k}) also forms column k's
// product L_{k+2,k} L_{k+2,k}^T for the next launch's diagonal block into a scratch block (Linv past its nblk
// inverses, two blocks by parity): the next workgroup 0 subtracts it where it formed it itself before, so its
// chain holds three 64^3 products instead of four -- same operands, same code, same bits.  Dynamic LDS:
// CHOL_DIAG_LDS bytes.  fail: set by a non-positive pivot; later launches then do nothing (the host rejects
// the step).  Linv: nblk + 2 blocks.
__global__ void __launch_bounds__(256) chol_chain_kernel(double* S, int n, int k, double* Linv, int* fail, int trail) {
    extern __shared__ double dyn[];
    double (*As)[NB + 1] = reinterpret_cast<double (*)[NB + 1]>(dyn);
    double (*Bs)[NB + 1] = reinterpret_cast<double (*)[NB + 1]>(dyn + NB * TLD);
    const int nblk = n / NB, own = k >= 0 ? nblk - k - 1 : 1;  // the launch's own workgroups
    if ((int)blockIdx.x >= own) {
        if ((int)blockIdx.x - own < trail) syrk_tile(S, n, k - 1, 3, (long long)blockIdx.x - own, As, Bs);
        return;
    }
    if (*fail) return;
    __shared__ int bad_s;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r0 = 32 * (wid >> 1), c0 = 32 * (wid & 1);
    const bool lead = blockIdx.x == 0;
    const int d = k + 1;  // workgroup 0: the next diagonal block
    constexpr int PER = NB * NB / 256;
    // every global load of the workgroup first: the panel block, the diagonal block (workgroup 0),
    // column k-1's operand blocks, L_kk^-1
    double cv[2][2][4], dv[2][2][4], pv[2][2][4], va[PER], vb[PER], vl[PER];
    const int i = k + 1 + (int)blockIdx.x;
    double* C = S + (size_t)i * NB * n + (size_t)k * NB;
    double* D = S + (size_t)d * NB * n + (size_t)d * NB;
    // column k-1's product for S_dd, L_{d,k-1} L_{d,k-1}^T: formed by workgroup 1 of the previous launch (the
    // owner of L_{d,k-1}) into the scratch block of d's parity -- off this workgroup's chain
    double* const P2 = Linv + (size_t)nblk * NB * NB;  // two 64x64 scratch blocks past the inverses
    const double* P2d = P2 + (size_t)(d & 1) * NB * NB;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                cv[ti][tj][q] = k >= 0 ? C[(size_t)r * n + c] : 0.0;
                dv[ti][tj][q] = lead && c <= r ? D[(size_t)r * n + c] : 0.0;
                pv[ti][tj][q] = lead && k > 0 && c <= r ? P2d[r * NB + c] : 0.0;
            }
    if (k > 0) {
        const double* Aik = S + (size_t)i * NB * n + (size_t)(k - 1) * NB;
        const double* Ajk = S + (size_t)k * NB * n + (size_t)(k - 1) * NB;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int e = threadIdx.x + 256 * u, r = e / NB, c = e % NB;
            va[u] = Aik[(size_t)r * n + c];
            vb[u] = Ajk[(size_t)r * n + c];
        }
    }
    if (k >= 0) {
        const double* Li = Linv + (size_t)k * NB * NB;
#pragma unroll
        for (int u = 0; u < PER; ++u) vl[u] = Li[threadIdx.x + 256 * u];
    }
    auto to_lds = [&](double (*X)[NB + 1], const double* v) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int e = threadIdx.x + 256 * u;
            X[e / NB][e % NB] = v[u];
        }
    };
    auto tile_product = [&](d4 acc[2][2]) {  // acc = As Bs^T
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = d4{0, 0, 0, 0};
        mfma_tile_ABt(As, Bs, acc, wid, lane);
    };
    auto sub = [&](double (&x)[2][2][4], d4 acc[2][2], bool lower) {  // x -= acc (lower: c <= r only)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                    if (!lower || c <= r) x[ti][tj][q] = x[ti][tj][q] - acc[ti][tj][q];
                }
    };
    d4 acc[2][2];
    if (k > 0) {  // column k-1: S_ik -= A_{i,k-1} A_{k,k-1}^T, and (workgroup 0, i = d) S_dd -= A_{d,k-1} A_{d,k-1}^T
        to_lds(As, va);
        to_lds(Bs, vb);
        __syncthreads();
        tile_product(acc);
        sub(cv, acc, false);
        if (lead) {  // S_dd -= L_{d,k-1} L_{d,k-1}^T (the previous launch's product, same operands and code)
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                        if (c <= r) dv[ti][tj][q] = dv[ti][tj][q] - pv[ti][tj][q];
                    }
        }
        __syncthreads();  // every wave is done with As / Bs
    }
    if (k >= 0) {  // L_ik = S_ik L_kk^-T
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                    As[r][c] = cv[ti][tj][q];
                }
        to_lds(Bs, vl);
        __syncthreads();
        tile_product(acc);
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                    C[(size_t)r * n + c] = acc[ti][tj][q];
                }
        if (blockIdx.x == 1) {
            // the next launch's column-k product for its diagonal block d + 1 = k + 2: L_{k+2,k} L_{k+2,k}^T from
            // the panel block just formed, exactly as workgroup 0 would form it (the same LDS operands)
            __syncthreads();
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                        As[r][c] = acc[ti][tj][q];
                        Bs[r][c] = acc[ti][tj][q];
                    }
            __syncthreads();
            d4 acc2[2][2];
            tile_product(acc2);
            double* P2n = P2 + (size_t)((k + 2) & 1) * NB * NB;
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                        P2n[r * NB + c] = acc2[ti][tj][q];
                    }
            return;
        }
        if (!lead) return;
        __syncthreads();
        // column k: S_dd -= L_dk L_dk^T with the panel block just formed (the stored values)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                    As[r][c] = acc[ti][tj][q];
                    Bs[r][c] = acc[ti][tj][q];
                }
        __syncthreads();
        d4 acc2[2][2];
        tile_product(acc2);
        sub(dv, acc2, true);
        __syncthreads();
    }
    // the diagonal block d: into the T area (As, upper part 0), factor, L_dd and L_dd^-1 out
    double* T = dyn;
    double* X = T + NB * TLD;
    double* LB = X + NB * TLD;
    double* LT = LB + 4 * 256;
    double* P = LT + 256;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + 16 * ti + (lane >> 4) + 4 * q, c = c0 + 16 * tj + (lane & 15);
                As[r][c] = dv[ti][tj][q];
            }
    for (int e = threadIdx.x; e < NB * NB; e += 256) X[(e >> 6) * TLD + (e & 63)] = 0.0;
    __syncthreads();
    if (diag_block_lds(T, X, LB, LT, P, bad_s)) {
        if (threadIdx.x == 0) *fail = 1;
        return;
    }
    double* Li = Linv + (size_t)d * NB * NB;
    for (int e = threadIdx.x; e < NB * NB; e += 256) {
        const int r = e >> 6, c = e & 63;
        if (c <= r) D[(size_t)r * n + c] = T[r * TLD + c];
        Li[e] = X[r * TLD + c];
    }
}

// Two 64-row blocks per workgroup (TG): a hand-off per pair instead of per block; the second
// block's dependency on the first is resolved inside the workgroup.  The diagonal inverses are
// staged in LDS before the first wait (they are final), the off-diagonal rows of every step are
// loaded before its wait.
constexpr int TG = 2;
constexpr int LIS = NB + 1;  // odd LDS row stride

// forward: workgroup j owns row blocks r = TG j + rl: b_r -= L_rk y_k for k = 0 .. r-1 (k order,
// each row dot reduced over 8 lanes, see below), y_r = Linv_rr b_r.  y_k is final once none of its 64 values is the unset pattern (poll_block);
// flags[FLAG_STRIDE 2 nblk]: set on a timed-out wait.
__global__ void __launch_bounds__(256) trsv_fwd_persistent_kernel(const double* S, int n, const double* Linv,
                                                                  double* b, double* y, double* x, int* flags) {
    __shared__ double bs[TG * NB];
    __shared__ double yk[NB];
    __shared__ double part[TG][4][64];
    __shared__ double LiS[TG][NB * LIS];
    __shared__ int ok_s;
    const int nblk = n / NB, r0 = TG * blockIdx.x, nl = min(TG, nblk - r0);
    const int rw = threadIdx.x & 63, g = threadIdx.x >> 6;  // row in the block, 16-column group
    for (int e = threadIdx.x; e < nl * NB; e += 256) {
        bs[e] = b[r0 * NB + e];
        x[r0 * NB + e] = __longlong_as_double((long long)kUnsetBits);  // polled by the backward solve
    }
    for (int rl = 0; rl < nl; ++rl) {
        const double* Li = Linv + (size_t)(r0 + rl) * NB * NB;
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = Li[threadIdx.x + 256 * u];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = threadIdx.x + 256 * u;
            LiS[rl][(e >> 6) * LIS + (e & 63)] = v[u];
        }
    }
    if (threadIdx.x == 0) ok_s = 1;
    __syncthreads();
    // the off-diagonal rows stream as 128-B row segments, 8 lanes per row: a row dot is 8 two-term
    // products per lane reduced over its 8 lanes (3 exchange levels: a 32-lane butterfly per row was
    // a serial chain of LDS permutes, 4.4 us per step against 2.4 us)
    const int lane = threadIdx.x & 63;
    // L_(r0+1),r0 (final; needed between y_r0 and y_r0+1, on the hand-off chain): loaded up front
    static_assert(TG == 2, "one later local block");
    double2 v21[2][4];  // the main loop's 8-lanes-per-row layout, 16 rows per wave
#pragma unroll
    for (int gr = 0; gr < 2; ++gr)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 16 * g + 8 * gr + (lane >> 3);
            v21[gr][j] = nl == 2 ? *reinterpret_cast<const double2*>(S + (size_t)((r0 + 1) * NB + row) * n + (size_t)r0 * NB + 16 * j + 2 * (lane & 7))
                                 : make_double2(0.0, 0.0);
        }
    for (int k = 0; k < r0; ++k) {
        double pv = 0.0;
        if (threadIdx.x < NB) pv = ld_sc1(y + k * NB + lane);  // first poll, ahead of the row loads
        // 8 lanes per row (lane = 8 rr + c8), 4 row groups per wave; instruction j of a group reads
        // columns [16 j, 16 j + 16) of its 8 rows (128 B per row), lane c8 the pair 16 j + 2 c8
        double2 v[4][4];
#pragma unroll
        for (int gr = 0; gr < 4; ++gr)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = 32 * g + 8 * gr + (lane >> 3);  // rl NB + row in the block
                v[gr][j] = (row >> 6) < nl ? *reinterpret_cast<const double2*>(S + (size_t)(r0 * NB + row) * n + (size_t)k * NB + 16 * j + 2 * (lane & 7))
                                           : make_double2(0.0, 0.0);
            }
        if (threadIdx.x < NB) {
            if (__ballot((unsigned long long)__double_as_longlong(pv) == kUnsetBits) != 0ull &&
                !poll_block(y + k * NB + lane, pv) && lane == 0) {
                ok_s = 0;
                flags[FLAG_STRIDE * 2 * nblk] = 1;
            }
            yk[lane] = pv;
        }
        __syncthreads();
        if (!ok_s) return;
        double yv[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            yv[j][0] = yk[16 * j + 2 * (lane & 7)];
            yv[j][1] = yk[16 * j + 2 * (lane & 7) + 1];
        }
#pragma unroll
        for (int gr = 0; gr < 4; ++gr) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) t += v[gr][j].x * yv[j][0] + v[gr][j].y * yv[j][1];
#pragma unroll
            for (int off = 4; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
            const int row = 32 * g + 8 * gr + (lane >> 3);
            if ((lane & 7) == 0 && (row >> 6) < nl) bs[row] -= t;
        }
        __syncthreads();
    }
    for (int rl = 0; rl < nl; ++rl) {
        const int r = r0 + rl;
        // the later local block's rows of L_.r: L_(r0+1),r0 (v21, loaded at the start)
        {   // y_r = Linv_rr b_r as the four 16-column group sums (trsv_fwd_kernel)
            double t = 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int q = 16 * g + u;
                if (q <= rw) t += LiS[rl][rw * LIS + q] * bs[rl * NB + q];
            }
            part[0][g][rw] = t;
        }
        __syncthreads();
        if (threadIdx.x < NB) {
            const double t = (part[0][0][rw] + part[0][1][rw]) + (part[0][2][rw] + part[0][3][rw]);
            st_sc1(y + r * NB + threadIdx.x, t);
            yk[threadIdx.x] = t;
            b[r * NB + threadIdx.x] = bs[rl * NB + threadIdx.x];
        }
        __syncthreads();  // yk
        if (rl + 1 < nl) {
#pragma unroll
            for (int gr = 0; gr < 2; ++gr) {
                double t = 0.0;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    t += v21[gr][j].x * yk[16 * j + 2 * (lane & 7)] + v21[gr][j].y * yk[16 * j + 2 * (lane & 7) + 1];
#pragma unroll
                for (int off = 4; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
                if ((lane & 7) == 0) bs[NB + 16 * g + 8 * gr + (lane >> 3)] -= t;
            }
        }
        __syncthreads();
    }
}

// backward: workgroup j owns column blocks c = nblk - 1 - (TG j + cl) (the last ones first):
// y_c -= L_kc^T x_k for k = nblk-1 .. c+1 (k order, each as the four 16-row group sums
// ((p0 + p1) + (p2 + p3))), x_c = Linv_cc^T y_c.  x_k is final once none of its values is the unset pattern.
__global__ void __launch_bounds__(256) trsv_bwd_persistent_kernel(const double* S, int n, const double* Linv,
                                                                  double* y, double* x, int* flags) {
    __shared__ double ys[TG * NB];  // ys[cl NB + i]: column block c_hi - cl
    __shared__ double xk[NB];
    __shared__ double part[TG][4][64];
    __shared__ double LiS[TG][NB * LIS];
    __shared__ int ok_s;
    const int nblk = n / NB, c_hi = nblk - 1 - TG * blockIdx.x, nl = min(TG, c_hi + 1);
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
    // L_c_hi,(c_hi-1) (needed between x_c_hi and x_c_hi-1, on the hand-off chain): loaded up front
    double v12[16];
#pragma unroll
    for (int u = 0; u < 16; ++u)
        v12[u] = nl == 2 ? S[(size_t)(c_hi * NB + g * 16 + u) * n + (size_t)(c_hi - 1) * NB + cl] : 0.0;
    for (int e = threadIdx.x; e < nl * NB; e += 256) ys[e] = y[(c_hi - e / NB) * NB + (e % NB)];
    for (int bl = 0; bl < nl; ++bl) {
        const double* Li = Linv + (size_t)(c_hi - bl) * NB * NB;
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = Li[threadIdx.x + 256 * u];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = threadIdx.x + 256 * u;
            LiS[bl][(e >> 6) * LIS + (e & 63)] = v[u];
        }
    }
    if (threadIdx.x == 0) ok_s = 1;
    __syncthreads();
    for (int k = nblk - 1; k > c_hi; --k) {
        double pv = 0.0;
        if (threadIdx.x < NB) pv = ld_sc1(x + k * NB + cl);  // first poll, ahead of the column loads
        double v[TG][16];
#pragma unroll
        for (int bl = 0; bl < TG; ++bl)
#pragma unroll
            for (int u = 0; u < 16; ++u)
                v[bl][u] = bl < nl ? S[(size_t)(k * NB + g * 16 + u) * n + (size_t)(c_hi - bl) * NB + cl] : 0.0;
        if (threadIdx.x < NB) {
            if (__ballot((unsigned long long)__double_as_longlong(pv) == kUnsetBits) != 0ull &&
                !poll_block(x + k * NB + cl, pv) && cl == 0) {
                ok_s = 0;
                flags[FLAG_STRIDE * 2 * nblk] = 1;
            }
            xk[cl] = pv;
        }
        __syncthreads();
        if (!ok_s) return;
#pragma unroll
        for (int bl = 0; bl < TG; ++bl) {
            double t = 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u) t += v[bl][u] * xk[g * 16 + u];
            part[bl][g][cl] = t;
        }
        __syncthreads();
        if (g < nl) ys[g * NB + cl] -= (part[g][0][cl] + part[g][1][cl]) + (part[g][2][cl] + part[g][3][cl]);
        __syncthreads();
    }
    for (int bl = 0; bl < nl; ++bl) {
        const int c = c_hi - bl;
        // the rows of block c_hi against column block c_hi - 1: v12, loaded at the start
        {   // x_c = Linv_cc^T y_c as the four 16-row group sums (trsv_bwd_kernel)
            double t = 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int q = 16 * g + u;
                if (q >= cl) t += LiS[bl][q * LIS + cl] * ys[bl * NB + q];
            }
            part[0][g][cl] = t;
        }
        __syncthreads();
        if (threadIdx.x < NB) {
            const double t = (part[0][0][cl] + part[0][1][cl]) + (part[0][2][cl] + part[0][3][cl]);
            st_sc1(x + c * NB + threadIdx.x, t);
            xk[threadIdx.x] = t;
            y[c * NB + threadIdx.x] = ys[bl * NB + threadIdx.x];
        }
        __syncthreads();  // xk
        if (bl + 1 < nl) {
            double t = 0.0;
#pragma unroll
            for (int u = 0; u < 16; ++u) t += v12[u] * xk[g * 16 + u];
            part[0][g][cl] = t;
            __syncthreads();
            if (g == 0) ys[NB + cl] -= (part[0][0][cl] + part[0][1][cl]) + (part[0][2][cl] + part[0][3][cl]);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// landmark back-substitution y_l = V~^-1 (g~_l - sum W^T y_p); partial = non-finite flag
__global__ void __launch_bounds__(GT) gba_backsub_kernel(GbaArgs A, double* partial) {
    const int L = A.L;
    int l = blockIdx.x * GT + threadIdx.x;
    double fin = 0.0;
    if (l < L && A.lm_var[l]) {
        double s[3] = {A.sl[l], A.sl[(size_t)L + l], A.sl[2 * (size_t)L + l]};
        double rhs[3];
        for (int c = 0; c < 3; ++c) rhs[c] = A.gl[(size_t)c * L + l] * s[c];
        for (int o = A.lm_ptr[l]; o < A.lm_ptr[l + 1]; ++o) {
            int pf = A.pose_f[A.obs_kf[o]];
            if (pf < 0) continue;
            const double* W = A.Wo + 18 * (size_t)o;
            for (int c = 0; c < 3; ++c) {
                double w = 0.0;
                for (int i = 0; i < 6; ++i) w += W[3 * i + c] * A.xf[pf + i];
                rhs[c] -= w;
            }
        }
        double vi[6];
        for (int i = 0; i < 6; ++i) vi[i] = A.Vi[(size_t)i * L + l];
        double y0 = vi[0] * rhs[0] + vi[1] * rhs[1] + vi[2] * rhs[2];
        double y1 = vi[1] * rhs[0] + vi[3] * rhs[1] + vi[4] * rhs[2];
        double y2 = vi[2] * rhs[0] + vi[4] * rhs[1] + vi[5] * rhs[2];
        A.yl[l] = y0; A.yl[(size_t)L + l] = y1; A.yl[2 * (size_t)L + l] = y2;
        if (!isfinite(y0) || !isfinite(y1) || !isfinite(y2)) fin = 1.0;
    }
    int f = blockIdx.x * GT + threadIdx.x;
    if (f < A.nf && !isfinite(A.xf[f])) fin = 1.0;
    double v[1] = {fin};
    block_reduce_store<1>(v, partial + blockIdx.x, true);
}

// per observation model change; candidate poses/points and step norms.
// partial[3*block + {0,1,2}] = model change, |x - cand|^2, |cand|^2
__global__ void __launch_bounds__(GT) gba_model_kernel(GbaArgs A, double* partial) {
    const int N = A.N, L = A.L, K = A.K;
    int t = blockIdx.x * GT + threadIdx.x;
    double mc = 0.0, sn = 0.0, xn = 0.0;
    if (t < N) {
        int o = t;
        int k = A.obs_kf[o], l = A.obs_lm[o];
        int pf = A.pose_f[k];
        bool lv = A.lm_var[l];
        if (pf >= 0 || lv) {
            double m0 = 0, m1 = 0;
            if (pf >= 0)
                for (int i = 0; i < 6; ++i) {
                    double d = -A.xf[pf + i] * A.sf[pf + i];
                    m0 += A.jp[(size_t)i * N + o] * d;
                    m1 += A.jp[(size_t)(6 + i) * N + o] * d;
                }
            if (lv)
                for (int c = 0; c < 3; ++c) {
                    double d = -A.yl[(size_t)c * L + l] * A.sl[(size_t)c * L + l];
                    m0 += A.jl[(size_t)c * N + o] * d;
                    m1 += A.jl[(size_t)(3 + c) * N + o] * d;
                }
            mc -= m0 * (A.r[o] + m0 / 2.0) + m1 * (A.r[N + o] + m1 / 2.0);
        }
    }
    if (t < 6 * K) {
        int k = t / 6, i = t % 6;
        int pf = A.pose_f[k];
        double x = A.x_pose[t];
        double c = pf >= 0 ? x + (-A.xf[pf + i] * A.sf[pf + i]) : x;
        A.c_pose[t] = c;
        if (pf >= 0) { double d = x - c; sn += d * d; xn += c * c; }
    }
    if (t < 3 * L) {
        int l = t / 3, c = t % 3;
        double x = A.x_lm[t];
        double cnd = A.lm_var[l] ? x + (-A.yl[(size_t)c * L + l] * A.sl[(size_t)c * L + l]) : x;
        A.c_lm[t] = cnd;
        if (A.lm_var[l]) { double d = x - cnd; sn += d * d; xn += cnd * cnd; }
    }
    double v[3] = {mc, sn, xn};
    __shared__ double out3[3];
    block_reduce_store<3>(v, out3, false);
    if (threadIdx.x == 0) {
        partial[3 * blockIdx.x] = out3[0];
        partial[3 * blockIdx.x + 1] = out3[1];
        partial[3 * blockIdx.x + 2] = out3[2];
    }
}

// fixed-order reduction of strided partials: out[q] = sum_i partial[stride*i + q]
__global__ void __launch_bounds__(GT) gba_reduce3_kernel(const double* partial, int n, double* out) {
    double a[3] = {0, 0, 0};
    for (int i = threadIdx.x; i < n; i += GT)
        for (int q = 0; q < 3; ++q) a[q] += partial[3 * i + q];
    block_reduce_store<3>(a, out, false);
}

// chi^2 + outlier flags + bad landmarks at the final point (Optimizer.cpp:415-456, 888-928)
__global__ void __launch_bounds__(GT) gba_post_kernel(GbaArgs A, double* chi2, uint8_t* outl, uint8_t* bad,
                                                      double* partial) {
    int l = blockIdx.x * GT + threadIdx.x;
    double cin = 0, cout_ = 0, cbad = 0;
    if (l < A.L) {
        int li = 0, lo = 0;
        for (int o = A.lm_ptr[l]; o < A.lm_ptr[l + 1]; ++o) {
            int k = A.obs_kf[o];
            double Pw[3] = {A.x_lm[3 * l], A.x_lm[3 * l + 1], A.x_lm[3 * l + 2]};
            double ch = factor_chi2(A.pc + 36 * k, Pw, (double)A.obs_uv[2 * o], (double)A.obs_uv[2 * o + 1], A.cols,
                                    A.rows, A.info, false, false);
            bool is_out = ch > A.chi2_thr;
            chi2[o] = ch;
            outl[o] = is_out;
            if (is_out) lo++; else li++;
        }
        bool b = !A.lm_marg[l] && li == 0 && lo >= 2;
        bad[l] = b;
        cin = li; cout_ = lo; cbad = b;
    }
    double v[3] = {cin, cout_, cbad};
    __shared__ double out3[3];
    block_reduce_store<3>(v, out3, false);
    if (threadIdx.x == 0) {
        partial[3 * blockIdx.x] = out3[0];
        partial[3 * blockIdx.x + 1] = out3[1];
        partial[3 * blockIdx.x + 2] = out3[2];
    }
}

// ------------------------------------------------------------------------------------------
// launchers (host-callable)
static inline dim3 g1(long long n) { return dim3((unsigned)((n + GT - 1) / GT)); }

hipError_t gba_launch_setup(const GbaArgs& A, hipStream_t s) {
    hipLaunchKernelGGL(gba_setup_kernel, g1(A.K), dim3(GT), 0, s, A);
    return hipGetLastError();
}
hipError_t gba_launch_eval(const GbaArgs& A, const double* xp, const double* xl, int mode, double* partial,
                           double* out, hipStream_t s) {
    hipLaunchKernelGGL(gba_pose_cache_kernel, g1(A.K), dim3(GT), 0, s, A, xp);
    hipLaunchKernelGGL(gba_eval_kernel, g1(A.N), dim3(GT), 0, s, A, xl, mode, partial);
    hipLaunchKernelGGL(gba_reduce_kernel, dim3(1), dim3(GT), 0, s, (const double*)partial, (int)g1(A.N).x, out, 0);
    return hipGetLastError();
}
hipError_t gba_launch_linearise(const GbaArgs& A, int first, double* partial, double* out_gmax, hipStream_t s) {
    const int nbl = (int)g1(A.L).x;
    const int nbp = (A.K + GT / 64 - 1) / (GT / 64);
    hipLaunchKernelGGL(gba_lin_lm_kernel, dim3(nbl), dim3(GT), 0, s, A, first, partial);
    hipLaunchKernelGGL(gba_lin_pose_kernel, dim3(nbp), dim3(GT), 0, s, A, first, partial + nbl);
    hipLaunchKernelGGL(gba_reduce_kernel, dim3(1), dim3(GT), 0, s, (const double*)partial, nbl + nbp, out_gmax, 1);
    return hipGetLastError();
}
hipError_t gba_launch_step_prep(const GbaArgs& A, double radius, double* partial, double* out_bad, hipStream_t s) {
    const int nbl = (int)g1(A.L).x;
    hipLaunchKernelGGL(gba_step_lm_kernel, dim3(nbl), dim3(GT), 0, s, A, radius, partial);
    hipLaunchKernelGGL(gba_reduce_kernel, dim3(1), dim3(GT), 0, s, (const double*)partial, nbl, out_bad, 1);
    hipLaunchKernelGGL(gba_step_f_kernel, g1(A.nfp), dim3(GT), 0, s, A, radius);
    hipLaunchKernelGGL(gba_step_obs_kernel, g1(A.N), dim3(GT), 0, s, A);
    if (A.n_dest > 0)
        hipLaunchKernelGGL(gba_schur_kernel, dim3((unsigned)((A.n_dest + GT / 64 - 1) / (GT / 64))), dim3(GT), 0, s, A);
    if (A.nfp > A.nf)
        hipLaunchKernelGGL(gba_pad_kernel, g1((long long)(A.nfp - A.nf) * A.nfp), dim3(GT), 0, s, A);
    hipLaunchKernelGGL(gba_rhs_kernel, dim3((A.K + GT / 64 - 1) / (GT / 64)), dim3(GT), 0, s, A);
    return hipGetLastError();
}
// Blocked right-looking Cholesky with a one-step look-ahead: after the panel of step k, the first
// trailing column (the next diagonal block and panel) is updated on the main stream, which then
// factors block k+1 and its panel while the rest of step k's trailing update runs on a side stream;
// the main stream joins it before the next first-column update.  Every tile sees the same updates
// in the same k order as the plain schedule (bitwise the same factor).
// > 64 KB of LDS: opt in, on the current device, before any launch or stream capture of the Cholesky
hipError_t gba_cholesky_attributes() {
    hipError_t e = hipFuncSetAttribute((const void*)chol_diag_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)CHOL_DIAG_LDS);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)chol_chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)CHOL_DIAG_LDS);
    return e;
}
constexpr long long kGbaFuseTrail = 2500;  // trailing updates of at most this many tiles in the next step's launch
hipError_t gba_reset_timeout(const GbaArgs& A, hipStream_t s) {
    int* tmo = gba_timeout_word(A);
    if (!tmo) return hipSuccess;
    // (VIO_GBA_TEST_TIMEOUT=1: the word starts set, as after a timed-out wait -- the host's device-error
    // path, exercised by tests/test_ba_gpu.py::test_wait_timeouts_report_device_errors)
    static std::atomic<int> test_tmo{[] {
        const char* v = std::getenv("VIO_GBA_TEST_TIMEOUT");
        return v && v[0] == '1' ? 1 : 0;
    }()};  // one-shot: the first factorisation of the process only
    return hipMemsetAsync(tmo, test_tmo.exchange(0) ? 1 : 0, sizeof(int), s);
}
hipError_t gba_launch_cholesky(const GbaArgs& A, int* fail, hipStream_t s) {
    const int n = A.nfp, nblk = n / NB;
    hipStream_t r = A.side;
    hipEvent_t ev_panel = A.ev[0], ev_rest = A.ev[1];
    if (!r || !ev_panel || !ev_rest) {  // no side stream: the plain schedule
        for (int k = 0; k < nblk; ++k) {
            hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(256), CHOL_DIAG_LDS, s, A.S, n, k, A.Linv, fail);
            const int m = nblk - k - 1;
            if (m > 0) {
                hipLaunchKernelGGL(chol_trsm_kernel, dim3(m), dim3(256), 0, s, A.S, n, k, (const double*)A.Linv);
                hipLaunchKernelGGL(chol_syrk_kernel, dim3((unsigned)((long long)m * (m + 1) / 2)), dim3(256), 0, s,
                                   A.S, n, k, 0);
            }
        }
        return hipGetLastError();
    }
    hipError_t e;
    // trailing updates of at most fuse_trail tiles (the late steps, where the cross-stream round trip of
    // the look-ahead costs more than the update) ride in the next launch; larger ones overlap it on the
    // side stream
    static const long long fuse_trail = [] {
        const char* v = std::getenv("VIO_GBA_FUSE_TRAIL");
        return v ? std::atoll(v) : kGbaFuseTrail;
    }();
    // VIO_GBA_FUSE_M=0 (A/B tests): separate update / diagonal / panel launches per step instead of the
    // chained launches
    static const bool separate = [] {
        const char* v = std::getenv("VIO_GBA_FUSE_M");
        return v && std::atoi(v) == 0;
    }();
    if (!separate) {
        // chained: launch k forms the panels of block column k and factors diagonal block k+1
        // (chol_chain_kernel); column k-1's trailing update (part 3) runs inside it or beside it on the
        // side stream, and launch k+1 follows both
        hipLaunchKernelGGL(chol_chain_kernel, dim3(1), dim3(256), CHOL_DIAG_LDS, s, A.S, n, -1, A.Linv, fail, 0);
        for (int k = 0; k + 1 < nblk; ++k) {
            const int m = nblk - k - 1;  // panel block rows of column k
            const long long tiles = k > 0 ? (long long)m * (m + 1) / 2 - 1 : 0;  // part 3 of step k-1
            const bool side = tiles > fuse_trail;
            if (side) {
                if ((e = hipEventRecord(ev_panel, s)) != hipSuccess) return e;  // panel k-1 final
                if ((e = hipStreamWaitEvent(r, ev_panel, 0)) != hipSuccess) return e;
                hipLaunchKernelGGL(chol_syrk_kernel, dim3((unsigned)tiles), dim3(256), 0, r, A.S, n, k - 1, 3);
                if ((e = hipEventRecord(ev_rest, r)) != hipSuccess) return e;
            }
            const int trail = side ? 0 : (int)tiles;
            hipLaunchKernelGGL(chol_chain_kernel, dim3(m + trail), dim3(256), CHOL_DIAG_LDS, s, A.S, n, k, A.Linv,
                               fail, trail);
            if (side && (e = hipStreamWaitEvent(s, ev_rest, 0)) != hipSuccess) return e;
        }
        return hipGetLastError();
    }
    // separate launches: step k = column k-1's update of block column k (k > 0), diagonal block k, panel
    // k; trail: tiles of step k-1's trailing update (part 2) before them
    auto step = [&](int k, int trail) {
        const int m = nblk - k - 1;
        if (trail > 0)
            hipLaunchKernelGGL(chol_syrk_kernel, dim3(trail), dim3(256), 0, s, A.S, n, k - 1, 2);
        if (k > 0) hipLaunchKernelGGL(chol_syrk_kernel, dim3(m + 1), dim3(256), 0, s, A.S, n, k - 1, 1);
        hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(256), CHOL_DIAG_LDS, s, A.S, n, k, A.Linv, fail);
        if (m > 0) hipLaunchKernelGGL(chol_trsm_kernel, dim3(m), dim3(256), 0, s, A.S, n, k, (const double*)A.Linv);
    };
    step(0, 0);
    for (int k = 0; k + 1 < nblk; ++k) {
        const int m = nblk - k - 1;  // trailing block rows of step k
        const long long tiles = (long long)(m - 1) * m / 2;  // its trailing update right of block column k+1
        if (m >= 2 && tiles <= fuse_trail) {
            step(k + 1, (int)tiles);
            continue;
        }
        if ((e = hipEventRecord(ev_panel, s)) != hipSuccess) return e;  // panel k final
        if (m >= 2) {
            if ((e = hipStreamWaitEvent(r, ev_panel, 0)) != hipSuccess) return e;
            hipLaunchKernelGGL(chol_syrk_kernel, dim3((unsigned)((long long)(m - 1) * m / 2)), dim3(256), 0, r, A.S, n,
                               k, 2);
            if ((e = hipEventRecord(ev_rest, r)) != hipSuccess) return e;
        }
        step(k + 1, 0);
        if (m >= 2 && (e = hipStreamWaitEvent(s, ev_rest, 0)) != hipSuccess) return e;
    }
    return hipGetLastError();
}
static bool gba_per_step_solve() {  // VIO_GBA_PERSISTENT_SOLVE=0: the per-step kernels (A/B tests)
    static const bool per_step = [] {
        const char* v = std::getenv("VIO_GBA_PERSISTENT_SOLVE");
        return v && v[0] == '0';
    }();
    return per_step;
}
int gba_solve_persistent_wgs(const GbaArgs& A) {
    const int nblk = A.nfp / NB;
    return A.flags && nblk >= 1 && nblk <= 256 && !gba_per_step_solve() ? (nblk + TG - 1) / TG : 0;
}
hipError_t gba_launch_solve(const GbaArgs& A, hipStream_t s) {
    const int n = A.nfp, nblk = n / NB;
    if (gba_solve_persistent_wgs(A)) {  // every block resident: the persistent solves
        // y: the unset pattern (polled by the forward solve; x is reset by the forward kernel); the
        // timeout word was cleared before the Cholesky (gba_reset_timeout)
        hipError_t e = hipMemsetAsync(A.yv, 0xff, sizeof(double) * (size_t)n, s);
        if (e != hipSuccess) return e;
        const unsigned g = (unsigned)((nblk + TG - 1) / TG);
        hipLaunchKernelGGL(trsv_fwd_persistent_kernel, dim3(g), dim3(256), 0, s, (const double*)A.S, n,
                           (const double*)A.Linv, A.bf, A.yv, A.xf, A.flags);
        hipLaunchKernelGGL(trsv_bwd_persistent_kernel, dim3(g), dim3(256), 0, s, (const double*)A.S, n,
                           (const double*)A.Linv, A.yv, A.xf, A.flags);
        return hipGetLastError();
    }
    for (int k = 0; k < nblk; ++k) {
        int rows = n - (k + 1) * NB;
        int nb = rows > 0 ? (rows + 31) / 32 : 1;
        hipLaunchKernelGGL(trsv_fwd_kernel, dim3(nb), dim3(256), 0, s, (const double*)A.S, n, k,
                           (const double*)A.Linv, A.bf, A.yv);
    }
    for (int k = nblk - 1; k >= 0; --k) {
        int cols = k * NB;
        int nb = cols > 0 ? (cols + 63) / 64 : 1;
        hipLaunchKernelGGL(trsv_bwd_kernel, dim3(nb), dim3(256), 0, s, (const double*)A.S, n, k,
                           (const double*)A.Linv, A.yv, A.xf);
    }
    return hipGetLastError();
}
hipError_t gba_launch_backsub(const GbaArgs& A, double* partial, double* out_nonfinite, hipStream_t s) {
    const int nb = (int)g1(std::max(A.L, A.nf)).x;
    hipLaunchKernelGGL(gba_backsub_kernel, dim3(nb), dim3(GT), 0, s, A, partial);
    hipLaunchKernelGGL(gba_reduce_kernel, dim3(1), dim3(GT), 0, s, (const double*)partial, nb, out_nonfinite, 1);
    return hipGetLastError();
}
hipError_t gba_launch_model(const GbaArgs& A, double* partial, double* out3, hipStream_t s) {
    long long m = std::max((long long)A.N, std::max(6LL * A.K, 3LL * A.L));
    const int nb = (int)g1(m).x;
    hipLaunchKernelGGL(gba_model_kernel, dim3(nb), dim3(GT), 0, s, A, partial);
    hipLaunchKernelGGL(gba_reduce3_kernel, dim3(1), dim3(GT), 0, s, (const double*)partial, nb, out3);
    return hipGetLastError();
}
hipError_t gba_launch_post(const GbaArgs& A, double* chi2, uint8_t* outl, uint8_t* bad, double* partial, double* out3,
                           hipStream_t s) {
    hipLaunchKernelGGL(gba_pose_cache_kernel, g1(A.K), dim3(GT), 0, s, A, (const double*)A.x_pose);
    const int nb = (int)g1(A.L).x;
    hipLaunchKernelGGL(gba_post_kernel, dim3(nb), dim3(GT), 0, s, A, chi2, outl, bad, partial);
    hipLaunchKernelGGL(gba_reduce3_kernel, dim3(1), dim3(GT), 0, s, (const double*)partial, nb, out3);
    return hipGetLastError();
}

}  // namespace vio360
