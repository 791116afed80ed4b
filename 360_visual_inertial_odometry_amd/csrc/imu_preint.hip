// imu_preint.hip — IMU preintegration on device, the producer of the
// InertialFactorFixedGravity inputs (vio_preint).
//
// Reference: IMUPreintegrator::Preintegrate / IntegrateMeasurement / UpdateCovariance
// (src/processing/IMUPreintegrator.cpp:143-274), Rodrigues / RightJacobian / SkewSymmetric
// (:313-356).  All arithmetic is f32 as in the reference (Eigen::Matrix3f); dt_total is the f64
// accumulator of f32 steps.  Compiled with -ffp-contract=off so every expression rounds as written:
// 3x3 products sum k = 0, 1, 2 in order, scalar factors are applied after the product, sin / cos of
// the rotation angle are the correctly rounded f32 values (f64 evaluation rounded once), which is
// what oracle/imu_oracle.c computes — the parity test is bitwise.
//
// Layout: nine lanes per interval (a keyframe pair).  An interval is a strictly sequential chain of
// ~50 steps at 200 Hz / 4 Hz keyframes, so the parallelism is across intervals (every window of a
// batch, every keyframe pair) and, inside one, across the covariance: each lane owns one position
// of the 3x3-block structure of the 9x9 covariance (9 entries), the ΔR / ΔV / ΔP / Jacobian chain
// is evaluated by all nine; everything stays in registers.  The 9x9 sandwich A·C·Aᵀ + B·N·Bᵀ of
// UpdateCovariance is evaluated on its non-zero pattern only (A = I + dt·E₆₃, B non-zero in
// columns 3..5); the dropped terms are exact zeros, so the result equals the dense product
// summed in index order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"

namespace vio360 {

constexpr int kLanesPerInterval = 9;
constexpr int kIntervalsPerBlock = 64 / kLanesPerInterval;  // 7

struct ImuInterval {  // one interval's inputs, in registers
    double t0, t1;
    float bg[3], ba[3];
};

struct ImuArgs {
    const vio_imu_data* imu;
    int n_imu;
    const double* t0;  // n
    const double* t1;  // n
    const float* bg;   // n*3 or null (= 0)
    const float* ba;   // n*3 or null (= 0)
    int n;
    vio_imu_noise noise;
    vio_preint* out;
    float* cov_bias;   // n*6
    uint8_t* valid;    // n
};

__device__ __forceinline__ void mm3(const float* A, const float* B, float* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[3 * i + j] = (A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j]) + A[3 * i + 2] * B[6 + j];
}

// Aᵀ·B
__device__ __forceinline__ void mtm3(const float* A, const float* B, float* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[3 * i + j] = (A[i] * B[j] + A[3 + i] * B[3 + j]) + A[6 + i] * B[6 + j];
}

__device__ __forceinline__ void mv3(const float* A, const float* v, float* o) {
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = (A[3 * i] * v[0] + A[3 * i + 1] * v[1]) + A[3 * i + 2] * v[2];
}

// A·[v]× with [v]×'s zero entries dropped from the k-ordered sums: adding an exact ±0 leaves every
// non-zero sum unchanged, so this equals mm3(A, skew(v)) (up to the sign of an exactly zero entry)
__device__ __forceinline__ void mm3_skew(const float* A, const float* v, float* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        C[3 * i + 0] = A[3 * i + 1] * v[2] + A[3 * i + 2] * -v[1];
        C[3 * i + 1] = A[3 * i + 0] * -v[2] + A[3 * i + 2] * v[0];
        C[3 * i + 2] = A[3 * i + 0] * v[1] + A[3 * i + 1] * -v[0];
    }
}

__device__ __forceinline__ void skew3(const float* v, float* S) {
    S[0] = 0.f;   S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2];  S[4] = 0.f;   S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0];  S[8] = 0.f;
}

// Rodrigues (:321-336) and RightJacobian (:338-354) of the same ω·dt
__device__ __forceinline__ void rodrigues_jr(const float* w, float* R, float* Jr) {
    // sqrtf is correctly rounded here; __fsqrt_rn is not on this toolchain (tools/probe/imu_math_probe.hip:
    // 15 % of 1M arguments differ from the IEEE result)
    const float th = sqrtf((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    if (th < 1e-6f) {
        float S[9];
        skew3(w, S);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const float id = (i % 4 == 0) ? 1.f : 0.f;
            R[i] = id + S[i];
            Jr[i] = id - 0.5f * S[i];
        }
        return;
    }
    const float ax[3] = {w[0] / th, w[1] / th, w[2] / th};
    float K[9], KK[9];
    skew3(ax, K);
    mm3_skew(K, ax, KK);
    const float s = (float)sin((double)th), c = (float)cos((double)th);
    const float a = 1.f - c, b = (1.f - c) / th, d = (th - s) / th;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const float id = (i % 4 == 0) ? 1.f : 0.f;
        R[i] = (id + s * K[i]) + a * KK[i];
        Jr[i] = (id - b * K[i]) + d * KK[i];
    }
}

__global__ __launch_bounds__(64) void imu_preint_kernel(ImuArgs a) {
    // 9 lanes per interval (7 intervals per wave, lane 63 idle); lane q = 3·bi + bj owns the
    // covariance entries C(bi + 3·u, bj + 3·v), u, v = 0..2 — the closure of UpdateCovariance's
    // dependencies (row block 2 += dt·row block 1, column block 2 += dt·column block 1, B·N·Bᵀ on
    // blocks 1..2), so the lanes never exchange data.  The 3x3 chain (ΔR, ΔV, ΔP, Jacobians) is
    // evaluated redundantly by the 9 lanes; lane 0 writes it.
    const int g = threadIdx.x / kLanesPerInterval, q = threadIdx.x % kLanesPerInterval;
    const int i = blockIdx.x * kIntervalsPerBlock + g;
    if (g >= kIntervalsPerBlock || i >= a.n) return;
    const int bi = q / 3, bj = q % 3;
    ImuInterval iv;
    iv.t0 = a.t0[i];
    iv.t1 = a.t1[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        iv.bg[k] = a.bg ? a.bg[3 * i + k] : 0.f;
        iv.ba[k] = a.ba ? a.ba[3 * i + k] : 0.f;
    }
    // filtered range [lo, hi): first timestamp >= t0, first timestamp >= t1 (sorted input)
    int lo = 0, hi = a.n_imu;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (a.imu[m].timestamp < iv.t0) lo = m + 1; else hi = m;
    }
    int e = lo;
    hi = a.n_imu;
    while (e < hi) {
        const int m = (e + hi) >> 1;
        if (a.imu[m].timestamp < iv.t1) e = m + 1; else hi = m;
    }
    const int cnt = e - lo;
    vio_preint* o = a.out + i;
    if (cnt <= 0) {  // Preintegrate returns nullptr (:165-169)
        if (q == 0) {
            float* of = reinterpret_cast<float*>(o);
            for (int k = 0; k < (int)(sizeof(vio_preint) / sizeof(float)); ++k) of[k] = 0.f;
            for (int k = 0; k < 6; ++k) a.cov_bias[6 * i + k] = 0.f;
            a.valid[i] = 0;
        }
        return;
    }
    const float gn2 = a.noise.gyro_noise * a.noise.gyro_noise;   // Nga(0..2) never reaches cov9: B's
    (void)gn2;                                                    // columns 0..2 are zero (:259-263)
    const float an2 = a.noise.accel_noise * a.noise.accel_noise;
    const float gbn2 = a.noise.gyro_bias_noise * a.noise.gyro_bias_noise;
    const float abn2 = a.noise.accel_bias_noise * a.noise.accel_bias_noise;

    float dR[9] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f};
    float dV[3] = {0.f, 0.f, 0.f}, dP[3] = {0.f, 0.f, 0.f};
    float JRg[9], JVg[9], JVa[9], JPg[9], JPa[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) JRg[k] = JVg[k] = JVa[k] = JPg[k] = JPa[k] = 0.f;
    float C[9];  // C[3u + v] = cov(bi + 3u, bj + 3v)
#pragma unroll
    for (int k = 0; k < 9; ++k) C[k] = 0.f;
    float walk[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    double dt_total = 0.0;

    // samples s and s+1 in registers, s+2 loaded at the top of step s (its latency hides behind the
    // step's arithmetic instead of stalling the next step)
    double t_prev = a.imu[lo].timestamp;
    vio_imu_data m = a.imu[lo];
    vio_imu_data m_next = a.imu[lo + (cnt > 1 ? 1 : 0)];
    for (int s = 0; s < cnt; ++s) {
        const vio_imu_data m_pre = a.imu[lo + min(s + 2, cnt - 1)];
        float dt;
        if (s == 0) dt = cnt > 1 ? (float)(m_next.timestamp - m.timestamp) : 0.002f;
        else dt = (float)(m.timestamp - t_prev);
        t_prev = m.timestamp;
        dt = fmaxf(0.0005f, fminf(dt, 0.02f));

        // IntegrateMeasurement (:195-236)
        const float gyr[3] = {m.gx - iv.bg[0], m.gy - iv.bg[1], m.gz - iv.bg[2]};
        const float acc[3] = {m.ax - iv.ba[0], m.ay - iv.ba[1], m.az - iv.ba[2]};
        const float wdt[3] = {gyr[0] * dt, gyr[1] * dt, gyr[2] * dt};
        float dRi[9], Jr[9], T[9], U[9];
        rodrigues_jr(wdt, dRi, Jr);
        mtm3(dRi, Jr, T);
#pragma unroll
        for (int k = 0; k < 9; ++k) JRg[k] = -T[k] * dt;
        mm3_skew(JVa, acc, T);
        mm3(T, JRg, U);
#pragma unroll
        for (int k = 0; k < 9; ++k) JVg[k] = JVg[k] + U[k];
        mm3_skew(JPa, acc, T);
        mm3(T, JRg, U);
#pragma unroll
        for (int k = 0; k < 9; ++k) JPg[k] = (JPg[k] + U[k]) + JVg[k] * dt;
        float Racc[3];
        mv3(dR, acc, Racc);  // old ΔR
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            JVa[k] = JVa[k] + dR[k] * dt;
            JPa[k] = (JPa[k] + JVa[k] * dt) + ((0.5f * dR[k]) * dt) * dt;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float v_old = dV[k];
            dV[k] = v_old + Racc[k] * dt;
            dP[k] = dP[k] + (v_old * dt + ((0.5f * Racc[k]) * dt) * dt);
        }
        mm3(dR, dRi, T);
#pragma unroll
        for (int k = 0; k < 9; ++k) dR[k] = T[k];

        // UpdateCovariance (:238-274) with the updated ΔR.  A·C: row block 2 += dt·row block 1
#pragma unroll
        for (int v = 0; v < 3; ++v) C[6 + v] = dt * C[3 + v] + C[6 + v];
        // (A·C)·Aᵀ: column block 2 += dt·column block 1
#pragma unroll
        for (int u = 0; u < 3; ++u) C[3 * u + 2] = C[3 * u + 1] * dt + C[3 * u + 2];
        // B·N·Bᵀ on blocks 1..2: B(3+r, 3+c) = ΔR·dt, B(6+r, 3+c) = ((0.5·ΔR)·dt)·dt.  The lane needs
        // B rows bi (block 1), 3+bi (block 2) and bj, 3+bj; ΔR rows picked by selects (a per-lane
        // index into a register array would become a waterfall loop)
        float Bi[2][3], Bj[2][3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float ri = bi == 0 ? dR[k] : (bi == 1 ? dR[3 + k] : dR[6 + k]);
            const float rj = bj == 0 ? dR[k] : (bj == 1 ? dR[3 + k] : dR[6 + k]);
            Bi[0][k] = ri * dt;
            Bi[1][k] = ((0.5f * ri) * dt) * dt;
            Bj[0][k] = rj * dt;
            Bj[1][k] = ((0.5f * rj) * dt) * dt;
        }
#pragma unroll
        for (int u = 1; u < 3; ++u) {
            const float M0 = Bi[u - 1][0] * an2, M1 = Bi[u - 1][1] * an2, M2 = Bi[u - 1][2] * an2;
#pragma unroll
            for (int v = 1; v < 3; ++v) {
                const float p = (M0 * Bj[v - 1][0] + M1 * Bj[v - 1][1]) + M2 * Bj[v - 1][2];
                C[3 * u + v] = C[3 * u + v] + p;
            }
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            walk[k] = walk[k] + gbn2 * dt;
            walk[3 + k] = walk[3 + k] + abn2 * dt;
        }
        dt_total += (double)dt;
        m = m_next;
        m_next = m_pre;
    }

#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) o->cov9[9 * (bi + 3 * u) + bj + 3 * v] = C[3 * u + v];
    if (q != 0) return;
    for (int k = 0; k < 9; ++k) {
        o->delta_R[k] = dR[k];
        o->J_Rg[k] = JRg[k];
        o->J_Vg[k] = JVg[k];
        o->J_Va[k] = JVa[k];
        o->J_Pg[k] = JPg[k];
        o->J_Pa[k] = JPa[k];
    }
    for (int k = 0; k < 3; ++k) {
        o->delta_V[k] = dV[k];
        o->delta_P[k] = dP[k];
        o->gyro_bias[k] = iv.bg[k];
        o->accel_bias[k] = iv.ba[k];
    }
    o->_pad[0] = o->_pad[1] = 0.f;
    o->dt_total = dt_total;
    for (int k = 0; k < 6; ++k) a.cov_bias[6 * i + k] = walk[k];
    a.valid[i] = 1;
}

static size_t align_up(size_t v, size_t al) { return (v + al - 1) / al * al; }

}  // namespace vio360

using namespace vio360;

static int launch_preint(vio_ctx* ctx, const ImuArgs& a) {
    VIO_DEVICE(ctx);
    for (hipEvent_t& ev : ctx->imu_ev)
        if (!ev) VIO_HIP(ctx, hipEventCreate(&ev));
    VIO_HIP(ctx, hipEventRecord(ctx->imu_ev[0], ctx->stream));
    hipLaunchKernelGGL(imu_preint_kernel, dim3((a.n + kIntervalsPerBlock - 1) / kIntervalsPerBlock), dim3(64), 0,
                       ctx->stream, a);
    VIO_HIP(ctx, hipGetLastError());
    VIO_HIP(ctx, hipEventRecord(ctx->imu_ev[1], ctx->stream));
    ctx->imu_ms = 0.f;  // resolved by vio_imu_preintegrate_kernel_ms
    return VIO_OK;
}

static const vio_imu_noise kDefaultNoise = {1.0e-4f, 1.0e-3f, 1.0e-6f, 1.0e-5f};

extern "C" int vio_imu_preintegrate_device(vio_ctx* ctx, const vio_imu_data* imu, int n_imu, const double* t_start,
                                           const double* t_end, int n, const float* gyro_bias,
                                           const float* accel_bias, const vio_imu_noise* noise, vio_preint* out,
                                           uint8_t* valid, float* cov_bias_diag) {
    if (!ctx || n < 0 || n_imu < 0 || (n > 0 && (!t_start || !t_end || !out || !valid || !cov_bias_diag)) ||
        (n_imu > 0 && !imu))
        return VIO_EINVAL;
    if (n == 0) return VIO_OK;
    ImuArgs a{imu, n_imu, t_start, t_end, gyro_bias, accel_bias, n, noise ? *noise : kDefaultNoise, out,
              cov_bias_diag, valid};
    return launch_preint(ctx, a);
}

extern "C" int vio_imu_preintegrate(vio_ctx* ctx, const vio_imu_data* imu, int n_imu, const double* t_start,
                                    const double* t_end, int n, const float* gyro_bias, const float* accel_bias,
                                    const vio_imu_noise* noise, vio_preint* out, uint8_t* valid,
                                    float* cov_bias_diag) {
    if (!ctx || n < 0 || n_imu < 0 || (n > 0 && (!t_start || !t_end || !out || !valid)) || (n_imu > 0 && !imu))
        return VIO_EINVAL;
    for (int k = 1; k < n_imu; ++k)
        if (!(imu[k].timestamp >= imu[k - 1].timestamp)) {
            set_error(ctx, "vio_imu_preintegrate: IMU samples not sorted by timestamp");
            return VIO_EINVAL;
        }
    if (n == 0) return VIO_OK;
    if (n_imu == 0) {  // Preintegrate: empty measurement list → nullptr (:148-151)
        std::memset(out, 0, sizeof(vio_preint) * (size_t)n);
        std::memset(valid, 0, (size_t)n);
        if (cov_bias_diag) std::memset(cov_bias_diag, 0, sizeof(float) * 6 * (size_t)n);
        return VIO_OK;
    }
    const size_t b_t = align_up(sizeof(double) * (size_t)n, 256), b_b = align_up(sizeof(float) * 3 * (size_t)n, 256);
    const size_t b_pre = align_up(sizeof(vio_preint) * (size_t)n, 256);
    const size_t b_cov = align_up(sizeof(float) * 6 * (size_t)n, 256);
    const size_t b_val = align_up((size_t)n, 256);
    auto* d_imu = static_cast<vio_imu_data*>(ctx_buffer(ctx, kSlotImuData, sizeof(vio_imu_data) * (size_t)n_imu));
    auto* d_iv = static_cast<char*>(ctx_buffer(ctx, kSlotImuIntervals, 2 * b_t + 2 * b_b));
    auto* d_out = static_cast<char*>(ctx_buffer(ctx, kSlotImuOut, b_pre + b_cov + b_val));
    if (!d_imu || !d_iv || !d_out) {
        set_error(ctx, "vio_imu_preintegrate: device allocation failed");
        return VIO_ENOMEM;
    }
    hipStream_t st = ctx->stream;
    VIO_DEVICE(ctx);
    VIO_HIP(ctx, hipMemcpyAsync(d_imu, imu, sizeof(vio_imu_data) * (size_t)n_imu, hipMemcpyHostToDevice, st));
    ImuArgs a;
    a.imu = d_imu;
    a.n_imu = n_imu;
    a.t0 = reinterpret_cast<const double*>(d_iv);
    a.t1 = reinterpret_cast<const double*>(d_iv + b_t);
    a.bg = gyro_bias ? reinterpret_cast<const float*>(d_iv + 2 * b_t) : nullptr;
    a.ba = accel_bias ? reinterpret_cast<const float*>(d_iv + 2 * b_t + b_b) : nullptr;
    VIO_HIP(ctx, hipMemcpyAsync(d_iv, t_start, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, st));
    VIO_HIP(ctx, hipMemcpyAsync(d_iv + b_t, t_end, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, st));
    if (gyro_bias)
        VIO_HIP(ctx, hipMemcpyAsync(d_iv + 2 * b_t, gyro_bias, sizeof(float) * 3 * (size_t)n, hipMemcpyHostToDevice, st));
    if (accel_bias)
        VIO_HIP(ctx, hipMemcpyAsync(d_iv + 2 * b_t + b_b, accel_bias, sizeof(float) * 3 * (size_t)n,
                                    hipMemcpyHostToDevice, st));
    a.n = n;
    a.noise = noise ? *noise : kDefaultNoise;
    a.out = reinterpret_cast<vio_preint*>(d_out);
    a.cov_bias = reinterpret_cast<float*>(d_out + b_pre);
    a.valid = reinterpret_cast<uint8_t*>(d_out + b_pre + b_cov);
    int rc = launch_preint(ctx, a);
    if (rc) return rc;
    VIO_HIP(ctx, hipMemcpyAsync(out, a.out, sizeof(vio_preint) * (size_t)n, hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipMemcpyAsync(valid, a.valid, (size_t)n, hipMemcpyDeviceToHost, st));
    if (cov_bias_diag)
        VIO_HIP(ctx, hipMemcpyAsync(cov_bias_diag, a.cov_bias, sizeof(float) * 6 * (size_t)n, hipMemcpyDeviceToHost, st));
    VIO_HIP(ctx, hipStreamSynchronize(st));
    return VIO_OK;
}

extern "C" int vio_imu_preintegrate_kernel_ms(vio_ctx* ctx, double* ms) {
    if (!ctx || !ms) return VIO_EINVAL;
    if (ctx->imu_ms < 0.f || !ctx->imu_ev[1]) {
        set_error(ctx, "vio_imu_preintegrate_kernel_ms: no preintegration has run on this context");
        return VIO_EINVAL;
    }
    float f = 0.f;
    VIO_HIP(ctx, hipEventSynchronize(ctx->imu_ev[1]));
    VIO_HIP(ctx, hipEventElapsedTime(&f, ctx->imu_ev[0], ctx->imu_ev[1]));
    *ms = f;
    return VIO_OK;
}
