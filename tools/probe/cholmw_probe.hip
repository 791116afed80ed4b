// Micro-probe: shader-clock cost of the window solver's reduced solve (an n x n SPD system in LDS, n = 54
// pose rows, plus the 36-row velocity / bias block) by
//   V0  chol6_solve2 (chol_dev.h, the shipped 6x6-blocked LLT over all 256 threads), 54 alone
//   V1  chol6_solve2 on both systems (54 + 36), as ph_solve calls it
//   V2  chol_mw: lane = row, the columns split over NW waves (CB columns each), one s_barrier per pivot,
//       the pivot column published through LDS, look-ahead of the owner's next column; 54 alone
//   V3  chol_mw on both: 54 over waves 0-2 (18 columns each) + 36 over wave 3 (one wave)
//   V4  chol_tile_solve2 on both (trailing matrix in MFMA tile registers, 6-column block steps)
// Diagnostic only (tools/, not shipped).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../360_visual_inertial_odometry_amd/csrc/chol_dev.h"

using namespace vio360;

constexpr int LD = 97;  // ph_solve's s_ld(90)

// Solves A x = b for SPD A (n x n, lower part at A with row stride lda; b as row n of A) with waves
// [w0, w0 + NW) of the workgroup; lane i of every participating wave holds row i (i <= n; row n = b)
// restricted to the wave's CB columns [CB (w - w0), CB (w - w0 + 1)).  Pivot j: its owner wave factors
// it (rsq + Newton), publishes L[:, j] to colbuf, applies it to its own next column first (look-ahead:
// the next pivot's chain overlaps the others' bulk updates); after a barrier of the NW waves every wave
// applies L[:, j] to its remaining columns.  The rhs row rides along (lane n ends with y = L^-1 b).  L and
// 1/L[j][j] go to Lout (row stride ldl) / dinv; then one wave solves L^T x = y column-oriented.
// bar(): the barrier of the participating waves (a workgroup barrier here).
template <int NW, int CB, int NMAXR, int NSTEP, int NPAD = 0>
__device__ __forceinline__ int chol_mw(const double* A, int lda, int n, int w0, double* colbuf, double* Lout, int ldl,
                                       double* dinv, double* x) {
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6) - w0;  // wave index within the system
    const bool part = wv >= 0 && wv < NW;
    double d[CB];
    const int cbase = CB * wv;
    if (part) {
        const double* arow = A + min(lane, n) * lda;
#pragma unroll
        for (int q = 0; q < CB; ++q) {
            const int k = cbase + q;
            const double v = k < n ? arow[k] : 0.0;
            d[q] = (lane < n) ? (k <= lane ? v : 0.0) : (lane == n ? v : 0.0);
        }
    }
    int bad = 0;
    double piv_next = 0.0;
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {  // NSTEP: the barrier count, equal for systems sharing barriers
        const bool act = j < n;
        const int o = j / CB, q = j % CB;
        double* cb = colbuf + (j & 1) * 64;
        if (act && part && wv == o) {
            double piv;
            if (q == 0) piv = readlane_d(d[0], j);  // first pivot of this owner: its column is up to date
            else piv = piv_next;
            bad |= !(piv > 0.0);
            const double r = rsq_nr(piv);
            double c = lane == j ? piv * r : d[q] * r;
            if (lane < j) c = 0.0;
            d[q] = c;
            cb[lane] = c;
            if (lane == j) dinv[j] = r;
            if (q + 1 < CB && j + 1 < n) {
                const double c1 = readlane_d(c, j + 1);
                d[q + 1] -= c * c1;
                piv_next = readlane_d(d[q + 1], j + 1);
            }
        }
        __syncthreads();
        if (act && part) {
            const double ci = cb[lane];
#pragma unroll
            for (int qq = 0; qq < CB; ++qq) {
                const int k = cbase + qq;
                const bool skip = k <= j || (wv == o && qq == q + 1);
                const double lk = cb[min(k, 63)];
                if (!skip) d[qq] -= ci * lk;
            }
        }
    }
    for (int e = 0; e < NPAD; ++e) __syncthreads();  // the barrier count of a longer system sharing them
    if (part && lane <= n) {
#pragma unroll
        for (int q = 0; q < CB; ++q) {
            const int k = cbase + q;
            if (k < n) Lout[lane * ldl + k] = (k <= lane || lane == n) ? d[q] : 0.0;
        }
    }
    __syncthreads();
    if (wv == 0) {  // L^T x = y, column-oriented, lane = column
        double e[NMAXR];
#pragma unroll
        for (int m = 0; m < NMAXR; ++m) e[m] = (m < n && lane < m) ? Lout[m * ldl + lane] : 0.0;
        double tt = lane < n ? Lout[n * ldl + lane] : 0.0;
        const double dv = lane < n ? dinv[lane] : 0.0;
#pragma unroll
        for (int m = NMAXR - 1; m >= 0; --m) {
            if (m < n) {
                const double xm = readlane_d(tt * dv, m);
                tt = lane == m ? xm : tt - e[m] * xm;
            }
        }
        if (lane < n) x[lane] = tt;
    }
    __syncthreads();
    return bad;
}

template <int V>
__global__ void __launch_bounds__(256, 1) probe(const double* gA, const double* gB, int n0, int n1, int reps,
                                                double* gx, unsigned long long* cyc) {
    __shared__ double S[100 * LD];
    __shared__ double xs[2][64];
    __shared__ double scr[4][128];
    __shared__ double Lb[2][64 * 65];
    __shared__ double dv[2][64];
    __shared__ int flag;
    __shared__ unsigned long long tsum[16];
    if (threadIdx.x < 16) tsum[threadIdx.x] = 0;
    unsigned long long tot = 0;
    for (int r = 0; r < reps; ++r) {
        // system 0 at S (rows 0..n0, rhs row n0), system 1 at S + (n0 + 1) * LD + n0 (rhs row n1)
        double* A1 = S + (n0 + 1) * LD + n0;
        for (int e = threadIdx.x; e < 100 * LD; e += 256) S[e] = 0.0;
        __syncthreads();
        for (int e = threadIdx.x; e < (n0 + 1) * 64; e += 256) S[(e / 64) * LD + e % 64] = gA[e];
        for (int e = threadIdx.x; e < (n1 + 1) * 64; e += 256)
            if (e % 64 < 40) A1[(e / 64) * LD + e % 64] = gB[e];
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        if (V == 0) {
            chol6_solve2<256>(S, n0, A1, 0, LD, xs[0], xs[1], scr[0], scr[1], &flag);
        } else if (V == 1) {
            chol6_solve2<256>(S, n0, A1, n1, LD, xs[0], xs[1], scr[0], scr[1], &flag);
        } else if (V == 2) {
            chol_mw<4, 16, 56, 54>(S, LD, n0, 0, scr[0], Lb[0], 65, dv[0], xs[0]);
        } else if (V == 3) {
            // both systems share the barriers: waves 0-2 run the 54-system, wave 3 the 36-system
            const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            if (wv < 3) chol_mw<3, 18, 56, 54>(S, LD, n0, 0, scr[0], Lb[0], 65, dv[0], xs[0]);
            else chol_mw<1, 40, 40, 36, 18>(A1, LD, n1, 3, scr[2], Lb[1], 65, dv[1], xs[1]);
        } else if (V == 4) {
            chol_tile_solve2<4, 3>(S, n0, A1, n1, LD, xs[0], xs[1], &Lb[0][0], &flag, tsum);
        } else if (V == 5) {
            chol_tile_solve2<4, 0>(S, n0, A1, 0, LD, xs[0], xs[1], &Lb[0][0], &flag, tsum);
        } else if (V == 6) {
            chol_tile_solve2<3, 0>(A1, n1, S, 0, LD, xs[1], xs[0], &Lb[0][0], &flag, tsum);
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        tot += t1 - t0;
        __syncthreads();
    }
    if (threadIdx.x < 64) {
        gx[threadIdx.x] = xs[0][threadIdx.x];
        gx[64 + threadIdx.x] = xs[1][threadIdx.x];
    }
    if (threadIdx.x == 0) *cyc = tot / reps;
    if (V == 4 && threadIdx.x == 0)
        printf("   V4 phases per solve: set-up %llu  factor %llu  -- %llu  backward %llu\n", tsum[0] / reps, tsum[1] / reps,
               tsum[2] / reps, tsum[3] / reps);
    if (V == 4 && threadIdx.x == 0)
        printf("   V4 tile wave: (a1) %llu  barrier1 %llu  (a2) %llu  inverse %llu  barrier2 %llu\n", tsum[4] / reps,
               tsum[5] / reps, tsum[6] / reps, tsum[7] / reps, tsum[8] / reps);
    if (V == 4 && threadIdx.x == 0)
        printf("   V4 diag wave: wait %llu  loads %llu  factor+panel %llu  stores %llu\n", tsum[9] / reps, tsum[10] / reps,
               tsum[11] / reps, tsum[12] / reps);
}

static void make_spd(int n, double* A /* (n+1) x 64, lower + rhs row */, unsigned seed) {
    srand(seed);
    static double M[64][64];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) M[i][j] = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < (n + 1) * 64; ++i) A[i] = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = i == j ? n : 0.0;
            for (int k = 0; k < n; ++k) s += M[i][k] * M[j][k];
            A[i * 64 + j] = s;
        }
    for (int i = 0; i < n; ++i) A[n * 64 + i] = i + 1.0;
}
static double resid(int n, const double* A, const double* x) {
    double res = 0;
    for (int i = 0; i < n; ++i) {
        double s = -A[n * 64 + i];
        for (int j = 0; j < n; ++j) s += (j <= i ? A[i * 64 + j] : A[j * 64 + i]) * x[j];
        res = fmax(res, fabs(s));
    }
    return res;
}

int main() {
    const int n0 = 54, n1 = 36, reps = 50;
    static double A[65 * 64], B[65 * 64];
    make_spd(n0, A, 3);
    make_spd(n1, B, 5);
    double *dA, *dB, *dx;
    unsigned long long* dc;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dB, sizeof(B));
    hipMalloc(&dx, 128 * 8);
    hipMalloc(&dc, 8);
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
    void (*fns[7])(const double*, const double*, int, int, int, double*, unsigned long long*) = {
        probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>};
    const char* names[7] = {"chol6_solve2 54", "chol6_solve2 54+36", "chol_mw 4x16 54", "chol_mw 3x18 54 + 1x40 36",
                            "chol_tile_solve2 54+36", "chol_tile_solve2 54", "chol_tile_solve2 36"};
    for (int v = 0; v < 7; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(fns[v], dim3(1), dim3(256), 0, 0, dA, dB, n0, n1, reps, dx, dc);
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        }
        unsigned long long cyc;
        double x[128];
        hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
        hipMemcpy(x, dx, sizeof(x), hipMemcpyDeviceToHost);
        const double r0 = v == 6 ? 0.0 : resid(n0, A, x), r1 = (v == 1 || v == 3 || v == 4 || v == 6) ? resid(n1, B, x + 64) : 0.0;
        printf("V%d %-28s cycles/solve %7llu  resid %.2e %.2e\n", v, names[v], cyc, r0, r1);
    }
    return 0;
}
