// Micro-probe: shader-clock cost of one wave factoring a 16x16 SPD tile (chol_dev.h chol16_wave) and of
// its pieces, repeated R times on LDS-resident tiles.  Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../360_visual_inertial_odometry_amd/csrc/chol_dev.h"

using namespace vio360;

// factor only (no inverse), pivots by readlane
__device__ __forceinline__ int chol16_factor_only(double* A, int ld, double* lt, int lane) {
    const int i = lane & 15, kk = lane >> 4;
    double d[16];
    const double* row = A + i * ld;
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = row[k];
    int bad = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const double piv = readlane_d(d[j], j);
        bad |= !(piv > 0.0);
        const double r = rsq_nr(piv);
        const double cj = i == j ? piv * r : d[j] * r;
        d[j] = cj;
#pragma unroll
        for (int k = j + 1; k < 16; ++k) d[k] -= cj * readlane_d(cj, k);
    }
    if (kk == 0) {
#pragma unroll
        for (int m = 0; m < 16; ++m) lt[16 * m + i] = d[m];
    }
    return bad;
}

// factor with the next pivot's column updated first (explicit look-ahead)
__device__ __forceinline__ int chol16_la(double* A, int ld, double* lbt, double* lt, int lane) {
    const int i = lane & 15, kk = lane >> 4;
    double d[16], il[16];
    const double* row = A + i * ld;
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = row[k];
    int bad = 0;
    // lane-uniform copies of the pivot candidates: p[k] = current d[k] of lane k
    double piv = readlane_d(d[0], 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        bad |= !(piv > 0.0);
        const double r = rsq_nr(piv);
        il[j] = r;
        const double cj = i == j ? piv * r : d[j] * r;
        d[j] = cj;
        if (j + 1 < 16) {
            const double c1 = readlane_d(cj, j + 1);
            d[j + 1] -= cj * c1;
            piv = readlane_d(d[j + 1], j + 1);
        }
#pragma unroll
        for (int k = j + 2; k < 16; ++k) d[k] -= cj * readlane_d(cj, k);
    }
    if (kk == 0) {
#pragma unroll
        for (int m = 0; m < 16; ++m) lt[16 * m + i] = d[m];
    }
    wave_lds_sync();
    double x[16], s[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) s[q] = q == i ? 1.0 : 0.0;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        x[m] = s[m] * il[m];
#pragma unroll
        for (int q = m + 1; q < 16; ++q) s[q] -= lt[16 * m + q] * x[m];
    }
    if (kk == 0) {
        double* dst = lbt + 16 * i;
#pragma unroll
        for (int q = 0; q < 16; ++q) dst[q] = x[q];
    }
    return bad;
}


// fused: inverse columns accumulated in the pivot loop (the factor's column broadcasts are the
// inverse's L entries), next pivot from lane-uniform scalars; BC = 0 readlane broadcast, 1 LDS
template <int BC>
__device__ __forceinline__ int chol16_fused(double* A, int ld, double* lbt, double* colbuf, int lane) {
    const int i = lane & 15, kk = lane >> 4;
    double d[16], s[16], x[16];
    const double* row = A + i * ld;
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = row[k];
#pragma unroll
    for (int q = 0; q < 16; ++q) s[q] = q == i ? 1.0 : 0.0;
    int bad = 0;
    double piv = readlane_d(d[0], 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        double a = 0.0, b = 0.0;
        if (j + 1 < 16) {
            a = readlane_d(d[j + 1], j + 1);
            b = readlane_d(d[j], j + 1);
        }
        bad |= !(piv > 0.0);
        const double r = rsq_nr(piv);
        const double cj = d[j] * r;
        d[j] = cj;
        x[j] = s[j] * r;
        if (j + 1 < 16) {
            const double c1 = b * r;
            piv = fma(-c1, c1, a);
        }
        if (BC == 0) {
#pragma unroll
            for (int k = j + 1; k < 16; ++k) {
                const double ck = readlane_d(cj, k);
                d[k] = fma(-ck, cj, d[k]);
                s[k] = fma(-ck, x[j], s[k]);
            }
        } else {
            double* cb = colbuf + 16 * (j & 1);
            if (kk == 0) cb[i] = cj;
            if (BC == 1) wave_lds_sync();
            else __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = j + 1; k < 16; ++k) {
                const double ck = cb[k];
                d[k] = fma(-ck, cj, d[k]);
                s[k] = fma(-ck, x[j], s[k]);
            }
        }
    }
    if (kk == 0) {
        double* dst = lbt + 16 * i;
#pragma unroll
        for (int q = 0; q < 16; ++q) dst[q] = x[q];
    }
    return bad;
}


// the scalar pivot chain alone: 16 x (rsq + 2 Newton steps, product, fma); NR = Newton steps
template <int NR>
__device__ __forceinline__ int chain16(double* A, int ld, double* lbt, int lane) {
    double piv = A[0], a = A[1], b = A[2];
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        double r = __builtin_amdgcn_rsq(piv);
        const double h = 0.5 * piv;
        if (NR >= 1) r = r * fma(-h * r, r, 1.5);
        if (NR >= 2) r = r * fma(-h * r, r, 1.5);
        acc += r;
        const double c1 = b * r;
        piv = fma(-c1, c1, a + 1.0);
    }
    if (lane == 0) lbt[0] = acc;
    return 0;
}

__global__ void __launch_bounds__(64) probe(const double* Ain, int V, int R, long long* cyc, double* out) {
    __shared__ double A[16 * 17], lbt[256], lt[256];
    const int lane = threadIdx.x;
    for (int e = lane; e < 256; e += 64) A[(e / 16) * 17 + e % 16] = Ain[e];
    __syncthreads();
    int bad = 0;
    const long long t0 = (long long)__builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
        if (V == 0) bad |= chol16_wave<false>(A, 17, lbt, lt, lane);
        else if (V == 1) bad |= chol16_factor_only(A, 17, lt, lane);
        else if (V == 2) bad |= chol16_la(A, 17, lbt, lt, lane);
        else if (V == 3) bad |= chol16_fused<0>(A, 17, lbt, lt, lane);
        else if (V == 4) bad |= chol16_fused<1>(A, 17, lbt, lt, lane);
        else if (V == 5) bad |= chol16_fused<2>(A, 17, lbt, lt, lane);
        else if (V == 6) bad |= chain16<2>(A, 17, lbt, lane);
        else if (V == 7) bad |= chain16<1>(A, 17, lbt, lane);
        else bad |= chain16<0>(A, 17, lbt, lane);
        wave_lds_sync();
    }
    const long long t1 = (long long)__builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[V] = (t1 - t0) / R;
    for (int e = lane; e < 256; e += 64) out[256 * V + e] = (V == 1 ? lt[e] : lbt[e]) + bad;
}

int main() {
    double h[256];
    srand(3);
    double M[256];
    for (int e = 0; e < 256; ++e) M[e] = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = i == j ? 16.0 : 0.0;
            for (int k = 0; k < 16; ++k) s += M[16 * i + k] * M[16 * j + k];
            h[16 * i + j] = s;
        }
    double *dA, *dout;
    long long* dc;
    hipMalloc(&dA, sizeof h);
    hipMalloc(&dout, 9 * 256 * sizeof(double));
    hipMalloc(&dc, 16 * sizeof(long long));
    hipMemcpy(dA, h, sizeof h, hipMemcpyHostToDevice);
    for (int V = 0; V < 9; ++V) {
        probe<<<1, 64>>>(dA, V, 200, dc, dout);
    }
    hipDeviceSynchronize();
    long long c[16];
    double o[2304];
    hipMemcpy(c, dc, sizeof c, hipMemcpyDeviceToHost);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    double md = 0, m3 = 0, m4 = 0, m5 = 0;
    for (int e = 0; e < 256; ++e) {
        md = fmax(md, fabs(o[e] - o[512 + e]));
        m3 = fmax(m3, fabs(o[e] - o[768 + e]));
        m4 = fmax(m4, fabs(o[e] - o[1024 + e]));
        m5 = fmax(m5, fabs(o[e] - o[1280 + e]));
    }
    printf("chol16: full %lld  factor-only %lld  look-ahead full %lld  fused-readlane %lld  fused-lds %lld fused-lds-nofence %lld cycles per tile; "
           "|dLinv| la %.3e fused-rl %.3e fused-lds %.3e nofence %.3e\n", c[0], c[1], c[2], c[3], c[4], c[5], md, m3, m4, m5);
    printf("chain16 (per tile): 2NR %lld 1NR %lld 0NR %lld\n", c[6], c[7], c[8]);
    return 0;
}
