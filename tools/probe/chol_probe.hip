// Micro-probe: cycle breakdown of the window solver's blocked Cholesky + triangular solves
// (diagonal-tile factor / panel / trailing update / solves) for one workgroup, variant 0 = the
// production formulation, variant 1 = candidate rewrite.  Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
using d4 = __attribute__((ext_vector_type(4))) double;
constexpr int NFM = 96, THR = 256;
struct Sh {
    double S[NFM * (NFM + 1)];
    double stage[3392];
    double b[NFM];
    int chol_bad;
};
__host__ __device__ constexpr int s_ld(int nf) { return (16 * ((nf + 15) >> 4)) | 1; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsq_nr(double p) {
    double r = __builtin_amdgcn_rsq(p);
    double h = 0.5 * p;
    r = r * fma(-h * r, r, 1.5);
    r = r * fma(-h * r, r, 1.5);
    return r;
}
#define STAMP(slot)                                                     \
    do {                                                                \
        if (threadIdx.x == 0) {                                         \
            long long t_ = (long long)__builtin_amdgcn_s_memtime();     \
            tm[slot] += t_ - tl;                                        \
            tl = t_;                                                    \
        }                                                               \
    } while (0)

template <int V>
__device__ bool chol(Sh& sh, int nf, long long* tm) {
    long long tl = (long long)__builtin_amdgcn_s_memtime();
    double* S = sh.S;
    double* LB = sh.stage;
    double* LT = sh.stage + 256 * 6;  // variant 1: row-major L of the diagonal tile
    const int ls = s_ld(nf), nb = (nf + 15) >> 4;
    constexpr int NW = THR / 64;
    const int wid = wave_id(), lane = threadIdx.x & 63;
    const int r16 = lane & 15, kk = lane >> 4;
    for (int J = 0; J < nb; ++J) {
        const int c0 = 16 * J;
        if (wid == 0) {
            const int i = r16;
            double d[16], il[16];
            const double* row = S + (c0 + i) * ls + c0;
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = row[k];
            int bad = 0;
            double x[16];
            if (V == 3) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const double piv = readlane_d(d[j], j);
                    bad |= !(piv > 0.0);
                    const double r = rsq_nr(piv);
                    il[j] = r;
                    const double cj = i == j ? piv * r : d[j] * r;
                    if (kk == 0) LT[16 * j + i] = i >= j ? cj : 0.0;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int k = j + 1; k < 16; ++k) d[k] -= cj * LT[16 * j + k];
                    // row j of L is complete: x[j] = (delta_ij - sum_{m<j} L[j][m] x[m]) / L[j][j]
                    double s = j == i ? 1.0 : 0.0;
#pragma unroll
                    for (int m = 0; m < j; ++m) s -= LT[16 * m + j] * x[m];
                    x[j] = s * r;
                }
            } else if (V == 2) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const double piv = readlane_d(d[j], j);
                    bad |= !(piv > 0.0);
                    const double r = rsq_nr(piv);
                    il[j] = r;
                    const double cj = i == j ? piv * r : d[j] * r;
                    if (kk == 0) LT[16 * j + i] = i >= j ? cj : 0.0;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                    for (int k = j + 1; k < 16; ++k) d[k] -= cj * LT[16 * j + k];
                }
            } else
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const double piv = readlane_d(d[j], j);
                bad |= !(piv > 0.0);
                double cj;
                if (V == 0) {
                    const double lj = sqrt(piv);
                    il[j] = 1.0 / lj;
                    cj = i == j ? lj : d[j] * il[j];
                } else {
                    const double r = rsq_nr(piv);
                    il[j] = r;
                    cj = i == j ? piv * r : d[j] * r;
                }
                d[j] = cj;
#pragma unroll
                for (int k = j + 1; k < 16; ++k) d[k] -= cj * readlane_d(cj, k);
            }
            if (V == 3) {
            } else if (V == 2) {
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    double s = q == i ? 1.0 : 0.0;
#pragma unroll
                    for (int m = 0; m < q; ++m) s -= LT[16 * m + q] * x[m];
                    x[q] = s * il[q];
                }
            } else if (V == 0) {
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    double s = q == i ? 1.0 : 0.0;
#pragma unroll
                    for (int m = 0; m < q; ++m) s -= readlane_d(d[m], q) * x[m];
                    x[q] = s * il[q];
                }
            } else {
                if (kk == 0) {
#pragma unroll
                    for (int m = 0; m < 16; ++m) LT[16 * i + m] = d[m];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    double s = q == i ? 1.0 : 0.0;
#pragma unroll
                    for (int m = 0; m < q; ++m) s -= LT[16 * q + m] * x[m];
                    x[q] = s * il[q];
                }
            }
            if (kk == 0) {
                double* dst = LB + 256 * J + 16 * i;
#pragma unroll
                for (int q = 0; q < 16; ++q) dst[q] = x[q];
            }
            if (lane == 0) sh.chol_bad = bad;
        }
        __syncthreads();
        STAMP(0);
        if (sh.chol_bad) return false;
        const double* lb = LB + 256 * J;
        for (int I = J + 1 + wid; I < nb; I += NW) {
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            double* A = S + 16 * I * ls + c0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const double a = A[r16 * ls + 4 * st + kk];
                const double bb = lb[(4 * st + kk) * 16 + r16];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(kk + 4 * r) * ls + r16] = acc[r];
        }
        __syncthreads();
        STAMP(1);
        const int m = nb - J - 1, nt = m * (m + 1) / 2;
        for (int t = wid; t < nt; t += NW) {
            int I = 0, tt = t;
            while (tt > I) { tt -= I + 1; ++I; }
            const int Kt = tt + J + 1;
            I += J + 1;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            const double* Ai = S + 16 * I * ls + c0;
            const double* Bk = S + 16 * Kt * ls + c0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const double a = Ai[r16 * ls + 4 * st + kk];
                const double bb = Bk[r16 * ls + 4 * st + kk];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
            }
            double* C = S + 16 * I * ls + 16 * Kt;
#pragma unroll
            for (int r = 0; r < 4; ++r) C[(kk + 4 * r) * ls + r16] -= acc[r];
        }
        __syncthreads();
        STAMP(2);
    }
    if (V == 3) {
        if (wid == 0) {
            double* y = sh.b;
            for (int J = 0; J < nb; ++J) {
                const double* lb = LB + 256 * J;
                double v = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) v += lb[16 * (kk + 4 * q) + r16] * y[16 * J + kk + 4 * q];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (kk == 0) y[16 * J + r16] = v;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double yj[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) yj[q] = y[16 * J + kk + 4 * q];
                for (int I = J + 1; I < nb; ++I) {
                    const double* Lr = S + (16 * I + r16) * ls + 16 * J + kk;
                    double u = 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) u += Lr[4 * q] * yj[q];
                    u += __shfl_xor(u, 16, 64);
                    u += __shfl_xor(u, 32, 64);
                    if (kk == 0) y[16 * I + r16] -= u;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            for (int J = nb - 1; J >= 0; --J) {
                const double* lb = LB + 256 * J;
                double v = 0.0;
#pragma unroll
                for (int q = 0; q < 4; ++q) v += lb[16 * r16 + kk + 4 * q] * y[16 * J + kk + 4 * q];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (kk == 0) y[16 * J + r16] = v;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double xj[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) xj[q] = y[16 * J + kk + 4 * q];
                for (int I = J - 1; I >= 0; --I) {
                    // r_I[c] -= sum_r L[16J + r][16I + c] x_J[r]
                    const double* Lc = S + (16 * J + kk) * ls + 16 * I + r16;
                    double u = 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) u += Lc[4 * q * ls] * xj[q];
                    u += __shfl_xor(u, 16, 64);
                    u += __shfl_xor(u, 32, 64);
                    if (kk == 0) y[16 * I + r16] -= u;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    } else if (wid == 0) {
        double* y = sh.b;
        for (int J = 0; J < nb; ++J) {
            const double* Lr = S + (16 * J + r16) * ls;
            double p0 = 0.0, p1 = 0.0;
            int cix = kk;
            for (; cix + 4 < 16 * J; cix += 8) { p0 += Lr[cix] * y[cix]; p1 += Lr[cix + 4] * y[cix + 4]; }
            if (cix < 16 * J) p0 += Lr[cix] * y[cix];
            double t = p0 + p1;
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            t = y[16 * J + r16] - t;
            const double* lb = LB + 256 * J;
            double v = 0.0;
            if (V == 2) {
                double* TB = LT + 256;
                if (kk == 0) TB[r16] = t;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int q = 0; q < 4; ++q) v += lb[16 * (kk + 4 * q) + r16] * TB[kk + 4 * q];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
            } else
#pragma unroll
            for (int mm = 0; mm < 16; ++mm) v += lb[16 * mm + r16] * readlane_d(t, mm);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (kk == 0) y[16 * J + r16] = v;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        for (int J = nb - 1; J >= 0; --J) {
            double p0 = 0.0, p1 = 0.0;
            int cix = 16 * (J + 1) + kk;
            const int cend = 16 * nb;
            for (; cix + 4 < cend; cix += 8) {
                p0 += S[cix * ls + 16 * J + r16] * y[cix];
                p1 += S[(cix + 4) * ls + 16 * J + r16] * y[cix + 4];
            }
            if (cix < cend) p0 += S[cix * ls + 16 * J + r16] * y[cix];
            double t = p0 + p1;
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            t = y[16 * J + r16] - t;
            const double* lb = LB + 256 * J;
            double v = 0.0;
            if (V == 2) {
                double* TB = LT + 256;
                if (kk == 0) TB[r16] = t;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int q = 0; q < 4; ++q) v += lb[16 * r16 + kk + 4 * q] * TB[kk + 4 * q];
                v += __shfl_xor(v, 16, 64);
                v += __shfl_xor(v, 32, 64);
            } else
#pragma unroll
            for (int mm = 0; mm < 16; ++mm) v += lb[16 * r16 + mm] * readlane_d(t, mm);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (kk == 0) y[16 * J + r16] = v;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();
    STAMP(3);
    return true;
}

template <int V>
__global__ void __launch_bounds__(THR) kern(const double* Sin, const double* bin, double* xout, long long* tm,
                                            int nf, int reps) {
    extern __shared__ double dyn[];
    Sh& sh = *reinterpret_cast<Sh*>(dyn);
    const int ls = s_ld(nf), np = 16 * ((nf + 15) >> 4);
    __shared__ long long tms[4];
    if (threadIdx.x < 4) tms[threadIdx.x] = 0;
    for (int r = 0; r < reps; ++r) {
        for (int e = threadIdx.x; e < np * ls; e += THR) sh.S[e] = Sin[e];
        for (int e = threadIdx.x; e < np; e += THR) sh.b[e] = bin[e];
        __syncthreads();
        long long t4[4] = {0, 0, 0, 0};
        chol<V>(sh, nf, t4);
        if (threadIdx.x == 0)
            for (int k = 0; k < 4; ++k) tms[k] += t4[k];
        __syncthreads();
    }
    for (int e = threadIdx.x; e < nf; e += THR) xout[e] = sh.b[e];
    if (threadIdx.x < 4) tm[threadIdx.x] = tms[threadIdx.x] / reps;
}

int main() {
    const int nf = 90, ls = s_ld(nf), np = 96;
    std::vector<double> S(np * ls, 0.0), b(np, 0.0), M(nf * nf);
    srand(7);
    for (auto& v : M) v = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < nf; ++i)
        for (int j = 0; j < nf; ++j) {
            double s = i == j ? nf : 0.0;
            for (int k = 0; k < nf; ++k) s += M[i * nf + k] * M[j * nf + k];
            S[i * ls + j] = s;
        }
    for (int i = nf; i < np; ++i) S[i * ls + i] = 1.0;
    for (int i = 0; i < nf; ++i) b[i] = (rand() / (double)RAND_MAX) - 0.5;
    double *dS, *db, *dx;
    long long* dt;
    (void)hipMalloc(&dS, S.size() * 8);
    (void)hipMalloc(&db, np * 8);
    (void)hipMalloc(&dx, np * 8);
    (void)hipMalloc(&dt, 4 * 8);
    (void)hipMemcpy(dS, S.data(), S.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, b.data(), np * 8, hipMemcpyHostToDevice);
    const size_t lds = sizeof(Sh);
    (void)hipFuncSetAttribute((const void*)kern<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)kern<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)kern<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute((const void*)kern<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    std::vector<double> x0(np), x1(np), x2(np), x3(np);
    for (int v = 0; v < 4; ++v) {
        if (v == 0) kern<0><<<1, THR, lds>>>(dS, db, dx, dt, nf, 50);
        else if (v == 1) kern<1><<<1, THR, lds>>>(dS, db, dx, dt, nf, 50);
        else if (v == 2) kern<2><<<1, THR, lds>>>(dS, db, dx, dt, nf, 50);
        else kern<3><<<1, THR, lds>>>(dS, db, dx, dt, nf, 50);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        long long t[4];
        (void)hipMemcpy(t, dt, 32, hipMemcpyDeviceToHost);
        (void)hipMemcpy(v == 0 ? x0.data() : v == 1 ? x1.data() : v == 2 ? x2.data() : x3.data(), dx, np * 8, hipMemcpyDeviceToHost);
        printf("variant %d: diag %lld panel %lld trailing %lld solves %lld total %lld (memtime ticks)\n", v, t[0],
               t[1], t[2], t[3], t[0] + t[1] + t[2] + t[3]);
    }
    // residual of both solutions
    for (int v = 0; v < 4; ++v) {
        const std::vector<double>& x = v == 0 ? x0 : v == 1 ? x1 : v == 2 ? x2 : x3;
        double rn = 0, bn = 0;
        for (int i = 0; i < nf; ++i) {
            double s = 0;
            for (int j = 0; j < nf; ++j) s += (i >= j ? S[i * ls + j] : S[j * ls + i]) * x[j];
            rn = fmax(rn, fabs(s - b[i]));
            bn = fmax(bn, fabs(b[i]));
        }
        printf("variant %d: max |Sx-b| / max|b| = %.3e\n", v, rn / bn);
    }
    double dmax = 0;
    for (int i = 0; i < nf; ++i) dmax = fmax(dmax, fabs(x0[i] - x3[i]) / (fabs(x0[i]) + 1e-300));
    printf("max rel diff v0 vs v1 = %.3e\n", dmax);
    return 0;
}
