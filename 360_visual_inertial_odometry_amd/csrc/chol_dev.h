// chol_dev.h — wave-level pieces of the blocked LDS Cholesky shared by the window solver
// (ba_kernel.hip, reduced camera system <= 96^2) and the global solver's diagonal blocks
// (ba_global.hip, 64^2 tiles of the config-5 system).  Reduced solve of Ceres' Schur complement
// (schur_complement_solver.cc:118-356: LLT of S); fixed operation order, no atomics.
#pragma once
#include <hip/hip_runtime.h>

namespace vio360 {

__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// 1/sqrt(p) to full double precision: hardware estimate + two Newton-Raphson steps
__device__ __forceinline__ double rsq_nr(double p) {
    double r = __builtin_amdgcn_rsq(p);
    const double h = 0.5 * p;
    r = r * fma(-h * r, r, 1.5);
    r = r * fma(-h * r, r, 1.5);
    return r;
}

// LDS writes of this wave visible to its own later reads (no workgroup barrier)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave factors the 16x16 SPD tile A (LDS, row stride ld, lower part read): lane i (mod 16) holds
// row i, pivots and column entries are broadcast with v_readlane.  Outputs
//   lbt[16 m + c] = Linv[c][m]   (L^-1 transposed, the B operand of the panel MFMAs)
//   A            <- L (lower, zeros above) when WRITE_L
// using lt[256] as scratch.  Returns nonzero (the same on every lane) if a pivot is not positive.
// Pivots of rows >= nvalid are not checked (a right-hand-side row carried through the factorisation).
template <bool WRITE_L>
__device__ __forceinline__ int chol16_wave(double* A, int ld, double* lbt, double* lt, int lane, int nvalid = 16) {
    const int i = lane & 15, kk = lane >> 4;
    double d[16], il[16];
    const double* row = A + i * ld;
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = row[k];  // k > i: upper triangle, never used
    int bad = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const double piv = readlane_d(d[j], j);
        bad |= j < nvalid && !(piv > 0.0);
        const double r = rsq_nr(piv);
        il[j] = r;
        const double cj = i == j ? piv * r : d[j] * r;
        d[j] = cj;
#pragma unroll
        for (int k = j + 1; k < 16; ++k) d[k] -= cj * readlane_d(cj, k);
    }
    if (kk == 0) {
#pragma unroll
        for (int m = 0; m < 16; ++m) lt[16 * m + i] = d[m];
    }
    wave_lds_sync();
    // column i of Linv (lower): x[q] = Linv[q][i]; L[q][m] read as an LDS broadcast.  Column-oriented:
    // once x[m] is known every later s[q] takes its term at once (independent FMAs, a 16-step critical
    // path); each s[q] still subtracts its terms in ascending m, so the values are those of the
    // row-oriented substitution bit for bit.
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
        if (WRITE_L) {
            double* out = A + i * ld;
#pragma unroll
            for (int m = 0; m < 16; ++m) out[m] = m <= i ? d[m] : 0.0;
        }
    }
    return bad;
}

// One wave solves the n x n SPD system A x = b (n <= NMAX - 1) by an unblocked right-looking
// Cholesky in registers, with no workgroup barrier: lane i holds row i of A (lower part; entries
// above the diagonal are zero), lane n holds b, so the factorisation itself runs the forward
// substitution (lane n ends with y = L^-1 b).  Pivot j: the pivot is broadcast by v_readlane, the
// column c_i = L[i][j] is published to LDS (col, two buffers of NMAX doubles) and every lane updates
// its row d[k] -= c_i L[k][j] (k > j) from broadcast LDS reads; L[i][j] is the textbook
// (A[i][j] - sum_{m<j} L[i][m] L[j][m]) / L[j][j] with the sum in ascending m.  Then L is written back
// over A (full rows, zeros above the diagonal), read column-wise (odd row stride: conflict-free), and
// the backward substitution x_m = (y_m - sum_{k>m} L[k][m] x_k) / L[m][m] runs column-oriented with
// one broadcast per step.  x (LDS, n) may alias b.  Returns nonzero (the same on every lane) if a pivot
// is not positive.  Used for the diagonal blocks of the window's reduced system: with the reference's
// zero IMU pose Jacobians (Factors.cpp:1415-1419, 1471-1475) the pose block and the velocity/bias
// block of S are uncoupled and each is factored by its own wave.
template <int NMAX>
__device__ __forceinline__ int chol_wave_solve(double* A, int lda, const double* b, int n, double* x, double* col,
                                               int lane) {
    double d[NMAX];
    const double* arow = A + lane * lda;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) d[k] = lane < n ? (k <= lane ? arow[k] : 0.0) : (lane == n && k < n ? b[k] : 0.0);
    int bad = 0;
    double dinv = 0.0;  // 1 / L[lane][lane]
#pragma unroll
    for (int j = 0; j < NMAX - 1; ++j) {
        if (j < n) {
            const double piv = readlane_d(d[j], j);
            bad |= !(piv > 0.0);
            const double r = rsq_nr(piv);
            const double c = lane == j ? piv * r : d[j] * r;
            d[j] = c;
            if (lane == j) dinv = r;
            double* cb = col + (j & 1) * NMAX;
            cb[lane] = c;
            wave_lds_sync();
#pragma unroll
            for (int k = j + 1; k < NMAX; ++k) d[k] -= c * cb[k];
        }
    }
    // lane n publishes y; L (rows) over A
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
    double e[NMAX];  // column `lane` of L: e[m] = L[m][lane] (zero for m < lane)
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

}  // namespace vio360
