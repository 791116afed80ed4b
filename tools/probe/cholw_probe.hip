// Micro-probe: shader-clock cost of one wave solving an n x n SPD system in registers (chol_dev.h
// chol_wave_solve) against variants of its column broadcast.  Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../360_visual_inertial_odometry_amd/csrc/chol_dev.h"

using namespace vio360;

// V: 0 = LDS broadcast, compiler-scheduled (chol_wave_solve's loop); 1 = the column preloaded into
// registers before the updates; 2 = v_readlane broadcasts; 3 = LDS broadcast in chunks of 8, the
// next chunk's reads issued before the current chunk's updates
template <int NMAX, int V>
__device__ __forceinline__ int chol_var(double* A, int lda, const double* b, int n, double* x, double* col, int lane) {
    double d[NMAX];
    const double* arow = A + min(lane, NMAX - 1) * lda;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {  // unconditional loads, then selects (no divergent LDS reads)
        const double av = arow[k], bv = b[k];
        d[k] = lane < n ? (k <= lane ? av : 0.0) : (lane == n && k < n ? bv : 0.0);
    }
    int bad = 0;
    double dinv = 0.0;
#pragma unroll
    for (int j = 0; j < NMAX - 1; ++j) {
        if (j < n) {
            const double piv = readlane_d(d[j], j);
            bad |= !(piv > 0.0);
            const double r = rsq_nr(piv);
            const double c = lane == j ? piv * r : d[j] * r;
            d[j] = c;
            if (lane == j) dinv = r;
            if (V == 2) {
#pragma unroll
                for (int k = j + 1; k < NMAX; ++k) d[k] -= c * readlane_d(c, k);
            } else {
                double* cb = col + (j & 1) * NMAX;
                cb[lane] = c;
                wave_lds_sync();
                if (V == 0) {
#pragma unroll
                    for (int k = j + 1; k < NMAX; ++k) d[k] -= c * cb[k];
                } else if (V == 1) {
                    double cv[NMAX];
#pragma unroll
                    for (int k = j + 1; k < NMAX; ++k) cv[k] = cb[k];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = j + 1; k < NMAX; ++k) d[k] -= c * cv[k];
                } else {
                    constexpr int CH = 8;
                    double cv[2][CH];
#pragma unroll
                    for (int q = 0; q < CH; ++q) cv[0][q] = j + 1 + q < NMAX ? cb[j + 1 + q] : 0.0;
#pragma unroll
                    for (int k0 = j + 1; k0 < NMAX; k0 += CH) {
                        const int cur = ((k0 - j - 1) / CH) & 1;
                        if (k0 + CH < NMAX) {
#pragma unroll
                            for (int q = 0; q < CH; ++q) cv[cur ^ 1][q] = k0 + CH + q < NMAX ? cb[k0 + CH + q] : 0.0;
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int q = 0; q < CH; ++q)
                            if (k0 + q < NMAX) d[k0 + q] -= c * cv[cur][q];
                    }
                }
            }
        }
    }
    if (lane == n) {
#pragma unroll
        for (int k = 0; k < NMAX; ++k) col[k] = d[k];
    }
    if (lane < n) {
        double* w = A + lane * lda;
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (k < n) w[k] = k <= lane ? d[k] : 0.0;
    }
    wave_lds_sync();
    double e[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; ++m) e[m] = (m < n && lane < n) ? A[m * lda + lane] : 0.0;
    double t = lane < n ? col[lane] : 0.0;
#pragma unroll
    for (int m = NMAX - 2; m >= 0; --m) {
        if (m < n) {
            const double xm = readlane_d(t * dinv, m);
            t = lane == m ? xm : t - e[m] * xm;
        }
    }
    if (lane < n) x[lane] = t;
    wave_lds_sync();
    return bad;
}


// V 4 / 5: no per-pivot guard (the matrix padded to NMAX-1 rows with identity, the right-hand side in
// lane NMAX-1), so the whole factorisation is one basic block; the next column's pivot chain (column
// j+1 updated through one v_readlane) comes before the bulk update of pivot j, which the scheduler can
// overlap with it.  4: bulk by LDS broadcast, 5: bulk by v_readlane.
template <int NMAX, int V>
__device__ __forceinline__ int chol_pad(double* A, int lda, const double* b, int n, double* x, double* col, int lane) {
    constexpr int NR = NMAX - 1;  // matrix rows (padded); lane NR holds the right-hand side
    double d[NMAX];
    const double* arow = A + lane * lda;
#pragma unroll
    for (int k = 0; k < NMAX; ++k)
        d[k] = lane < n ? (k <= lane ? arow[k] : 0.0) : lane < NR ? (k == lane ? 1.0 : 0.0) : (k < n ? b[k] : 0.0);
    int bad = 0;
    double dinv = 0.0;
    double piv = readlane_d(d[0], 0);
#pragma unroll
    for (int j = 0; j < NR; ++j) {
        bad |= !(piv > 0.0);
        const double r = rsq_nr(piv);
        const double c = lane == j ? piv * r : d[j] * r;
        d[j] = c;
        if (lane == j) dinv = r;
        if (j + 1 < NR) {
            const double c1 = readlane_d(c, j + 1);
            d[j + 1] -= c * c1;
            piv = readlane_d(d[j + 1], j + 1);
        }
        if (V == 5) {
#pragma unroll
            for (int k = j + 2; k < NR; ++k) d[k] -= c * readlane_d(c, k);
        } else {
            double* cb = col + (j & 1) * NMAX;
            cb[lane] = c;
            wave_lds_sync();
#pragma unroll
            for (int k = j + 2; k < NR; ++k) d[k] -= c * cb[k];
        }
    }
    if (lane == NR) {
#pragma unroll
        for (int k = 0; k < NMAX; ++k) col[k] = d[k];
    }
    if (lane < n) {
        double* w = A + lane * lda;
#pragma unroll
        for (int k = 0; k < NMAX; ++k)
            if (k < n) w[k] = k <= lane ? d[k] : 0.0;
    }
    wave_lds_sync();
    double e[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; ++m) e[m] = (m < n && lane < n) ? A[m * lda + lane] : 0.0;
    double t = lane < n ? col[lane] : 0.0;
#pragma unroll
    for (int m = NMAX - 2; m >= 0; --m) {
        if (m < n) {
            const double xm = readlane_d(t * dinv, m);
            t = lane == m ? xm : t - e[m] * xm;
        }
    }
    if (lane < n) x[lane] = t;
    wave_lds_sync();
    return bad;
}

// V 6: rolled pivot loop (instruction-cache sized): the register array is a window over the row,
// d[k] = entry at column j + k, shifted left by one per pivot (each update writes d[k-1] from d[k],
// so the shift costs nothing); the pivot blocks of 8 are unrolled with the window width shrinking by
// 8 per block (R = NMAX - 8 blk), the pivots inside a block are a runtime loop.  The next column's
// entry d[0] is updated first (its L[j+1][j] by v_readlane) so the next pivot's rsq chain overlaps
// the bulk update.  L rows go to Lscr (ld ldl; garbage above the diagonal, masked in the solve).
template <int NMAX>
__device__ __forceinline__ int chol_roll(const double* A, int lda, const double* b, int n, double* x, double* col,
                                         double* Lscr, int ldl, int lane) {
    double d[NMAX];
    const double* arow = A + min(lane, NMAX - 1) * lda;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {  // unconditional loads, then selects (no divergent LDS reads)
        const double av = arow[k], bv = b[k];
        d[k] = lane < n ? (k <= lane ? av : 0.0) : (lane == n && k < n ? bv : 0.0);
    }
    int bad = 0;
    double dinv = 0.0;
    double piv = readlane_d(d[0], 0);
    bad |= n > 0 && !(piv > 0.0);
    double r = rsq_nr(piv);
    int j = 0;
#pragma unroll
    for (int blk = 0; blk < NMAX / 8; ++blk) {
        constexpr int dummy = 0;
        (void)dummy;
        const int R = NMAX - 8 * blk;
        const int jend = min(8 * blk + 8, n);
        for (; j < jend; ++j) {
            const double c = lane == j ? piv * r : d[0] * r;
            if (lane == j) dinv = r;
            Lscr[lane * ldl + j] = c;
            double* cb = col + (j & 1) * (NMAX + 8);
            cb[lane] = c;
            const double c1 = readlane_d(c, j + 1);
            d[0] = d[1] - c * c1;
            piv = readlane_d(d[0], j + 1);
            bad |= (j + 1 < n) && !(piv > 0.0);
            r = rsq_nr(piv);
            wave_lds_sync();
#pragma unroll
            for (int k = 1; k < NMAX - 1; ++k)
                if (k < R - 1) d[k] = d[k + 1] - c * cb[j + 1 + k];
            d[R - 1] = 0.0;
        }
    }
    wave_lds_sync();
    double e[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; ++m) {
        const double v = Lscr[m * ldl + lane];
        e[m] = (m < n && lane < m) ? v : 0.0;
    }
    const double tv = Lscr[n * ldl + lane];
    double t = lane < n ? tv : 0.0;
#pragma unroll
    for (int m = NMAX - 2; m >= 0; --m) {
        if (m < n) {
            const double xm = readlane_d(t * dinv, m);
            t = lane == m ? xm : t - e[m] * xm;
        }
    }
    if (lane < n) x[lane] = t;
    wave_lds_sync();
    return bad;
}

constexpr int LD = 65;
template <int V>
__global__ void __launch_bounds__(256, 1) probe(const double* gA, const double* gb, int n, int reps, double* gx,
                                                unsigned long long* cyc) {
    __shared__ double S[64 * LD];
    __shared__ double bb[64];
    __shared__ double col[256];
    __shared__ double Lscr[64 * 65];
    const int lane = threadIdx.x & 63;
    unsigned long long tot = 0;
    for (int r = 0; r < reps; ++r) {
        for (int e = threadIdx.x; e < 64 * LD; e += 256) S[e] = gA[e];
        if (threadIdx.x < 64) bb[threadIdx.x] = gb[threadIdx.x];
        __syncthreads();
        if (V == 7) {  // all threads: 6x6-blocked LLT (rhs as row n)
            __shared__ int flag;
            for (int f = threadIdx.x; f < n; f += 256) S[n * LD + f] = bb[f];
            __syncthreads();
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            chol6_solve2<256>(S, n, S, 0, LD, bb, bb, Lscr, Lscr + 64, &flag);
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            tot += t1 - t0;
        } else if (threadIdx.x < 64) {
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            if (V < 4) chol_var<64, V>(S, LD, bb, n, bb, col, lane);
            else if (V < 6) chol_pad<64, V>(S, LD, bb, n, bb, col, lane);
            else chol_roll<64>(S, LD, bb, n, bb, col, Lscr, 65, lane);
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            tot += t1 - t0;
        }
        __syncthreads();
    }
    if (threadIdx.x < 64) gx[threadIdx.x] = bb[threadIdx.x];
    if (threadIdx.x == 0) *cyc = tot / reps;
}

int main() {
    const int n = 54, reps = 20;
    double A[64 * LD] = {0}, b[64] = {0};
    srand(3);
    // A = M M^T + n I (SPD), lower part stored
    double M[64][64];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) M[i][j] = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = i == j ? n : 0.0;
            for (int k = 0; k < n; ++k) s += M[i][k] * M[j][k];
            A[i * LD + j] = s;
        }
    for (int i = 0; i < n; ++i) b[i] = i + 1.0;
    double *dA, *db, *dx;
    unsigned long long* dc;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&db, sizeof(b));
    hipMalloc(&dx, sizeof(b));
    hipMalloc(&dc, 8);
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    hipMemcpy(db, b, sizeof(b), hipMemcpyHostToDevice);
    void (*fns[8])(const double*, const double*, int, int, double*, unsigned long long*) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>};
    for (int v = 0; v < 8; ++v) {
        hipLaunchKernelGGL(fns[v], dim3(1), dim3(256), 0, 0, dA, db, n, reps, dx, dc);
        unsigned long long cyc;
        double x[64];
        hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
        hipMemcpy(x, dx, sizeof(x), hipMemcpyDeviceToHost);
        double res = 0;
        for (int i = 0; i < n; ++i) {
            double s = -b[i];
            for (int j = 0; j < n; ++j) s += (j <= i ? A[i * LD + j] : A[j * LD + i]) * x[j];
            res = fmax(res, fabs(s));
        }
        printf("variant %d: n=%d cycles/solve %llu  max|Ax-b| %.3e\n", v, n, cyc, res);
    }
    return 0;
}
