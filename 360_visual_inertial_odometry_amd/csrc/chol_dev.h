// chol_dev.h — wave-level pieces of the blocked LDS Cholesky shared by the window solver
// (ba_kernel.hip, reduced camera system <= 96^2) and the global solver's diagonal blocks
// (ba_global.hip, 64^2 tiles of the config-5 system).  Reduced solve of Ceres' Schur complement
// (schur_complement_solver.cc:118-356: LLT of S); fixed operation order, no atomics.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>

namespace vio360 {

__device__ __forceinline__ double readlane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// 1/sqrt(p) to full double precision: hardware estimate r0 (relative error e0 well below 2^-20) and one
// third-order correction r0 (1 + e/2 + 3 e^2 / 8), e = 1 - p r0^2 (remaining error ~ e^3 < 2^-60): four
// dependent operations after the estimate instead of two Newton steps' six -- it sits on the pivot chain
// of every Cholesky here
__device__ __forceinline__ double rsq_nr(double p) {
    const double r = __builtin_amdgcn_rsq(p);
    const double e = fma(-p * r, r, 1.0);
    return fma(r * e, fma(e, 0.375, 0.5), r);
}

// Wall-clock bound of an inter-workgroup wait: s_memrealtime counts a constant 100 MHz clock, so the
// bound does not depend on how long one poll takes (an sc1 load round trip is 0.1-2 us depending on
// placement and load).  A wait that has not completed after kWaitTicks (2 s: a whole global-BA LM
// iteration is ~5 ms, a window solve ~1 ms) gives up, and the caller reports a device error.
constexpr unsigned long long kWaitTicks = 200000000ull;
__device__ __forceinline__ unsigned long long wait_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool wait_expired(unsigned long long t0) { return wait_clock() - t0 > kWaitTicks; }

// An LDS pointer the compiler must treat as an opaque register value: accesses at constant offsets from it
// then fold into the 16-bit immediate of ds_read / ds_write.  Without it, a region placed above 64 KB of
// LDS (the window kernels' stage area follows the 75 KB reduced matrix) has its constant addresses folded
// into absolute values that do not fit the immediate: every access site gets an address register of its
// own, the unrolled loops hoist them, and the cluster kernel spilled them to scratch.
template <class T>
__device__ __forceinline__ T* lds_base(T* p) {
    auto q = (__attribute__((address_space(3))) T*)p;
    asm volatile("" : "+v"(q));
    return (T*)q;
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

// Blocked right-looking LLT with 6x6 blocks (one block per pose) of up to two independent SPD systems
// by all NT threads of the workgroup, the two systems sharing the barriers: system s is the n_s x n_s
// matrix (n_s a multiple of 6) at A_s in LDS (row stride lda, lower part read), its right-hand side
// stored as row n_s (columns < n_s), which the factorisation turns into y = L^-1 b (the forward
// substitution rides along as an extra row).  Per block column j:
//   (b) one thread per row below the diagonal block forms the panel L[i][6j+c] = (A[i][6j+c] -
//       sum_m L[i][6j+m] L[6j+c][6j+m]) / L[6j+c][6j+c] (L_jj and 1/L[c][c] held in registers);
//   (c) the trailing update A[i][k] -= L[i][6j+m] L[k][6j+m] (m ascending) as (row, 6-column strip)
//       tasks; with a one-step look-ahead: lanes 0-5 of wave s first update the next diagonal block of
//       system s (lane u = its row u) and factor it in registers (pivots and column entries by
//       v_readlane, 1/L[c][c] into inv_s), while the other waves take the remaining tasks.
// Each L[i][k] is the textbook (A[i][k] - sum_{m<k} L[i][m] L[k][m]) / L[k][k] with the sum in
// ascending m.  Then the block backward substitution x_j = L_jj^-T (y_j - sum_{i>j} L_ij^T x_i) leaves
// x in x_s.  The critical chain is n/6 six-pivot factors and panels; the O(n^3) work is spread over
// the other waves.  Returns false (uniformly) when a pivot is not positive.  flag: one LDS int.
// 6x6 diagonal factor by lanes 0..5 of one wave: d = row `lane` of the block (lower part), in place
__device__ __forceinline__ int chol6_diag(double (&d)[6], int lane, double& my_inv) {
    int bad = 0;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const double piv = readlane_d(d[c], c);
        bad |= !(piv > 0.0);
        const double r = rsq_nr(piv);
        const double v = lane == c ? piv * r : d[c] * r;
        d[c] = v;
        if (lane == c) my_inv = r;
#pragma unroll
        for (int k = c + 1; k < 6; ++k) d[k] -= v * readlane_d(v, k);
    }
    return bad;
}
// L^T x = y by one wave, column-oriented (n <= 128, lane k holds t_k and t_{k+64}): for m from the
// last row, x_m = t_m / L[m][m] (inv = 1 / diagonal), then every t_k (k < m) takes its term L[m][k] x_m
// at once -- one broadcast and one FMA per step on the chain (the block version ran a 6-long dependent
// chain per block on one thread plus two workgroup barriers per block).  y is row n of A (row stride
// lda; the forward substitution rode along as that row); x may not alias A.
__device__ __forceinline__ void chol_backward_wave(const double* A, int lda, int n, const double* inv, double* x,
                                                   int lane) {
    const double* y = A + (size_t)n * lda;
    double t0 = lane < n ? y[lane] : 0.0, t1 = lane + 64 < n ? y[lane + 64] : 0.0;
    double a0 = n > 0 && lane < n - 1 ? A[(size_t)(n - 1) * lda + lane] : 0.0;  // row m, loaded one step ahead
    double a1 = n > 0 && lane + 64 < n - 1 ? A[(size_t)(n - 1) * lda + lane + 64] : 0.0;
    for (int m = n - 1; m >= 0; --m) {
        const double r0 = a0, r1 = a1;
        if (m > 0) {  // the next row's entries, in flight during this step's chain
            a0 = lane < m - 1 ? A[(size_t)(m - 1) * lda + lane] : 0.0;
            a1 = lane + 64 < m - 1 ? A[(size_t)(m - 1) * lda + lane + 64] : 0.0;
        }
        const double tm = m < 64 ? readlane_d(t0, m) : readlane_d(t1, m - 64);
        const double xm = tm * inv[m];
        if (m < 64) t0 = lane == m ? xm : (lane < m ? t0 - r0 * xm : t0);
        else {
            t0 = t0 - r0 * xm;
            t1 = lane + 64 == m ? xm : (lane + 64 < m ? t1 - r1 * xm : t1);
        }
    }
    if (lane < n) x[lane] = t0;
    if (lane + 64 < n) x[lane + 64] = t1;
}

// The 6x6 diagonal block at B (row stride lda, lower part current) factored by one whole wave, every lane
// holding the whole block in registers (no cross-lane broadcast on the pivot chain): lane u < 6 writes
// row u of L back and 1 / L[u][u] to inv[u].  Element by element the operations of chol6_diag (L[i][k]
// -= L[i][c] L[k][c], c ascending; L[c][c] = p rsq(p)): the same bits.  Returns nonzero (every lane) on a
// non-positive pivot.
__device__ __forceinline__ int chol6_diag_wave(double* B, int lda, double* inv, int lane) {
    double b[21];  // b[i (i + 1) / 2 + k] = entry (i, k), k <= i
#pragma unroll
    for (int i = 0, q = 0; i < 6; ++i)
#pragma unroll
        for (int k = 0; k <= i; ++k, ++q) b[q] = B[i * lda + k];
    int bad = 0;
    double r[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const double piv = b[c * (c + 1) / 2 + c];
        bad |= !(piv > 0.0);
        r[c] = rsq_nr(piv);
        b[c * (c + 1) / 2 + c] = piv * r[c];
#pragma unroll
        for (int i = c + 1; i < 6; ++i) b[i * (i + 1) / 2 + c] *= r[c];
#pragma unroll
        for (int i = c + 1; i < 6; ++i)
#pragma unroll
            for (int k = c + 1; k <= i; ++k) b[i * (i + 1) / 2 + k] -= b[i * (i + 1) / 2 + c] * b[k * (k + 1) / 2 + c];
    }
    if (lane < 6) {
        double* w = B + lane * lda;
#pragma unroll
        for (int u = 0; u < 6; ++u)
            if (lane == u) {
#pragma unroll
                for (int k = 0; k <= u; ++k) w[k] = b[u * (u + 1) / 2 + k];
                inv[u] = r[u];
            }
    }
    return bad;
}

template <int NT>
__device__ __forceinline__ bool chol6_solve2(double* A0, int n0, double* A1, int n1, int lda, double* x0, double* x1, double* inv0,
                             double* inv1, int* flag) {
    const int t = (int)threadIdx.x, wid = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int nb0 = n0 / 6, nb1 = n1 / 6, nb = nb0 > nb1 ? nb0 : nb1;
    // waves not factoring a diagonal block take the trailing-update tasks
    const int wfirst = nb1 > 0 ? 2 : 1, nworker = NT - 64 * wfirst, tw = t - 64 * wfirst;
    if (t == 0) *flag = 0;
    // diagonal block 0 of each system (its wave, every lane)
    if (wid < 2 && (wid == 0 ? nb0 : nb1) > 0) {
        const int bad = chol6_diag_wave(wid == 0 ? A0 : A1, lda, wid == 0 ? inv0 : inv1, lane);
        if (bad && lane == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (*flag) return false;
    for (int j = 0; j < nb; ++j) {
        const int c0 = 6 * j, r0 = c0 + 6;
        const int np0 = j < nb0 ? n0 + 1 - r0 : 0, np1 = j < nb1 ? n1 + 1 - r0 : 0;
        // (b) panel rows (the right-hand-side row included)
        for (int e = t; e < np0 + np1; e += NT) {
            const bool s1 = e >= np0;
            double* A = s1 ? A1 : A0;
            const double* inv = s1 ? inv1 : inv0;
            const int i = r0 + (s1 ? e - np0 : e);
            double l[21], iv[6];  // L_jj (lower, row-major packed) and 1 / diagonal, loaded together
#pragma unroll
            for (int c = 0, q = 0; c < 6; ++c)
#pragma unroll
                for (int m = 0; m <= c; ++m, ++q) l[q] = A[(c0 + c) * lda + c0 + m];
#pragma unroll
            for (int c = 0; c < 6; ++c) iv[c] = inv[c0 + c];
            double* row = A + i * lda + c0;
            double a[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) a[c] = row[c];
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                double v = a[c];
#pragma unroll
                for (int m = 0; m < c; ++m) v -= a[m] * l[c * (c + 1) / 2 + m];
                a[c] = v * iv[c];
            }
#pragma unroll
            for (int c = 0; c < 6; ++c) row[c] = a[c];
        }
        __syncthreads();
        // (c) trailing update: tasks (row u, strip q) over a rows x strips grid per system
        const int R0 = np0, R1 = np1;  // rows incl. the rhs row
        if (wid < wfirst) {
            // look-ahead: this wave's system's next diagonal block, updated and factored by lanes 0..5
            const bool s1 = wid == 1;
            const int R = s1 ? R1 : R0;
            if (R >= 7) {  // a next diagonal block exists (6 matrix rows + the rhs row)
                double* A = s1 ? A1 : A0;
                double* inv = s1 ? inv1 : inv0;
                if (lane < 6) {  // lane u: row u of the block, updated by panel j
                    const double* li = A + (r0 + lane) * lda + c0;
                    double l[6];
#pragma unroll
                    for (int m = 0; m < 6; ++m) l[m] = li[m];
#pragma unroll
                    for (int kk = 0; kk < 6; ++kk) {
                        if (kk > lane) continue;
                        const double* lk = A + (r0 + kk) * lda + c0;
                        double a = A[(r0 + lane) * lda + r0 + kk];
#pragma unroll
                        for (int m = 0; m < 6; ++m) a -= l[m] * lk[m];
                        A[(r0 + lane) * lda + r0 + kk] = a;
                    }
                }
                wave_lds_sync();
                const int bad = chol6_diag_wave(A + r0 * lda + r0, lda, inv + r0, lane);
                if (bad && lane == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {
            const int S0 = R0 > 1 ? (R0 - 2) / 6 + 1 : 0, S1 = R1 > 1 ? (R1 - 2) / 6 + 1 : 0;
            const int T0 = R0 * S0, T1 = R1 * S1;
            for (int e = tw; e < T0 + T1; e += nworker) {
                const bool s1 = e >= T0;
                const int ee = s1 ? e - T0 : e, S = s1 ? S1 : S0, R = s1 ? R1 : R0;
                const int u = ee / S, q = ee - u * S;
                const int kmax = u <= R - 2 ? u : R - 2;  // last column index (local) of row u
                if (6 * q > kmax) continue;
                if (q == 0 && u < 6 && (s1 ? wfirst > 1 : true)) continue;  // the next diagonal block: look-ahead
                double* A = s1 ? A1 : A0;
                const int i = r0 + u;
                const double* li = A + i * lda + c0;
                double l[6];
#pragma unroll
                for (int m = 0; m < 6; ++m) l[m] = li[m];
#pragma unroll
                for (int kk = 0; kk < 6; ++kk) {
                    const int k = 6 * q + kk;
                    if (k > kmax) break;
                    const double* lk = A + (r0 + k) * lda + c0;
                    double a = A[i * lda + r0 + k];
#pragma unroll
                    for (int m = 0; m < 6; ++m) a -= l[m] * lk[m];
                    A[i * lda + r0 + k] = a;
                }
            }
        }
        __syncthreads();
        if (*flag) return false;
    }
    // backward substitution L^T x = y (y = row n_s): one wave per system, column-oriented (chol_backward_wave)
    if (wid == 0 && nb0 > 0) chol_backward_wave(A0, lda, n0, inv0, x0, lane);
    else if (wid == 1 && nb1 > 0) chol_backward_wave(A1, lda, n1, inv1, x1, lane);
    __syncthreads();
    return true;
}

// Right-looking LLT with 6-column block steps of up to two independent SPD systems (the window's pose
// block and velocity / bias block: the reference's IMU pose Jacobians are zero, Factors.cpp:1415-1475),
// the trailing matrices held in REGISTERS as 16x16 MFMA tiles for the whole factorisation.  Roles (one
// 256-thread workgroup): wave s < 2 factors system s; waves 2 and 3 own the lower tiles of both systems
// (rows incl. the right-hand-side row n_s, padded to 16; tile g -> wave 2 + g % 2, slot g / 2).  Per
// block column J (c0 = 6 J, the step index a compile-time constant on the tile waves):
//   (a1) the tile waves apply panel J-1 to the tiles holding columns of block J (C -= P P^T on
//        v_mfma_f64_16x16x4_f64, two k-steps, panel columns 6, 7 zero; panel rows < c0 zero, so
//        finished entries never change) and write block column J (rows >= c0) to the column buffer E;
//   (b)  after a barrier, wave s factors diagonal block J in registers (every lane the whole 6x6 block:
//        no cross-lane broadcast on the pivot chain) and solves its panel row (lane l: row c0 + 6 + l, the
//        rhs row included: the forward substitution rides along) into the panel buffer of parity J & 1,
//        L into A_s, 1 / L[c][c] into dv;  meanwhile
//   (a2) the tile waves apply panel J-1 (the other buffer) to their remaining tiles and invert the
//        previous diagonal block (L_{J-1}^-1 for the blocked backward substitution, off-diagonal entries
//        into the unused upper triangle of A_s);
// then a barrier.  LDS traffic without divergent branches: masked-off lanes load clamped rows and store
// to trash rows.  The backward substitution L^T x = y runs per 6-block with the inverted diagonal blocks.
// Each L entry is the textbook value up to the summation order of the MFMA update.  scr:
// chol_tile_scratch_doubles() of LDS (16-B aligned).  Returns false (uniformly) on a non-positive pivot.
// Requires n_s % 6 == 0, n_s + 1 <= 64 (T_s <= 4 tile rows).
using cd4 = __attribute__((ext_vector_type(4))) double;
using cd2 = __attribute__((ext_vector_type(2))) double;
constexpr int kTilePW = 8;     // panel / column-buffer row width (6 columns + 2 zero k-columns)
constexpr int kTileRows = 112; // panel rows of both systems (7 tile rows)
constexpr int kPanelStride = (kTileRows + 2) * kTilePW;  // + row kTileRows (always zero) + a trash row
__host__ __device__ constexpr int chol_tile_rows(int n) { return n > 0 ? (n + 16) / 16 : 0; }
__host__ __device__ constexpr bool chol_tile_fits(int n0, int n1) {
    return n0 % 6 == 0 && n1 % 6 == 0 && chol_tile_rows(n0) <= 4 && chol_tile_rows(n1) <= 4 &&
           chol_tile_rows(n0) + chol_tile_rows(n1) <= kTileRows / 16;
}
// panels (2 parities) | column buffer (kTileRows + a trash row) | inverse diagonals (2 x kTileRows)
__host__ __device__ constexpr int chol_tile_scratch_doubles() { return 2 * kPanelStride + (kTileRows + 1) * kTilePW + 2 * kTileRows; }

// v = vals[lane == idx ? q : ...]: the value of a per-lane index into a register array (select chain)
template <int N>
__device__ __forceinline__ double pick_d(const double (&vals)[N], int idx) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < N; ++q) v = idx == q ? vals[q] : v;
    return v;
}

// L_JJ^-1 of the 6x6 lower block at B (row stride lda) with 1 / diagonal r: off-diagonal entries Linv[i][k]
// (i > k) stored transposed at B[k lda + i] (the unused upper triangle), one store per lane (lanes < 15)
__device__ __forceinline__ void chol6_inv_upper(double* B, int lda, const double* r, int lane, double* trash) {
    double l[21], rr[6], v[21];
#pragma unroll
    for (int i = 0, q = 0; i < 6; ++i)
#pragma unroll
        for (int k = 0; k <= i; ++k, ++q) l[q] = B[i * lda + k];
#pragma unroll
    for (int c = 0; c < 6; ++c) rr[c] = r[c];
#pragma unroll
    for (int c = 0; c < 6; ++c) {  // column c of the inverse: v[i][c], i >= c
        v[c * (c + 1) / 2 + c] = rr[c];
#pragma unroll
        for (int i = c + 1; i < 6; ++i) {
            double acc = 0.0;
#pragma unroll
            for (int m = c; m < i; ++m) acc += l[i * (i + 1) / 2 + m] * v[m * (m + 1) / 2 + c];
            v[i * (i + 1) / 2 + c] = -rr[i] * acc;
        }
    }
    // lane e < 15: off-diagonal entry e in row-major order (i, k), i > k
    double off[15];
    int oi = 0, ok = 0;
#pragma unroll
    for (int i = 1, e = 0; i < 6; ++i)
#pragma unroll
        for (int k = 0; k < i; ++k, ++e) {
            off[e] = v[i * (i + 1) / 2 + k];
            if (lane == e) { oi = i; ok = k; }
        }
    const double val = pick_d(off, lane);
    *(lane < 15 ? B + ok * lda + oi : trash + (lane & 7)) = val;
}

// L^T x = y by one wave, 6-block column-oriented, n <= 63 (lane k holds t_k): y = row n of A, L below the
// diagonal of A, the diagonal blocks' inverses as chol6_inv_upper left them (1 / L[c][c] in dv); the next
// block's operands are requested before this block's chain.  x may not alias A.
__device__ __forceinline__ void chol6_backward_blk(const double* A, int lda, int n, const double* dv, double* x, int lane) {
    double t = A[(size_t)n * lda + (lane < n ? lane : 0)];
    t = lane < n ? t : 0.0;
    double li[21], lk[6];
    auto fetch = [&](int c0) {
#pragma unroll
        for (int i = 0, q = 0; i < 6; ++i)
#pragma unroll
            for (int k = 0; k <= i; ++k, ++q) li[q] = i == k ? dv[c0 + i] : A[(c0 + k) * lda + c0 + i];  // Linv[i][k]
#pragma unroll
        for (int m = 0; m < 6; ++m) lk[m] = A[(c0 + m) * lda + lane];  // L[c0 + m][lane] (used for lane < c0)
    };
    if (n >= 6) fetch(n - 6);
    for (int c0 = n - 6; c0 >= 0; c0 -= 6) {
        double tj[6], cli[21], clk[6];
#pragma unroll
        for (int q = 0; q < 21; ++q) cli[q] = li[q];
#pragma unroll
        for (int m = 0; m < 6; ++m) clk[m] = lane < c0 ? lk[m] : 0.0;
        if (c0 >= 6) fetch(c0 - 6);
#pragma unroll
        for (int m = 0; m < 6; ++m) tj[m] = readlane_d(t, c0 + m);
#pragma unroll
        for (int m = 0; m < 6; ++m) {  // x_m = sum_{i >= m} Linv[i][m] t_i
            double acc = 0.0;
#pragma unroll
            for (int i = m; i < 6; ++i) acc += cli[i * (i + 1) / 2 + m] * tj[i];
            t = lane == c0 + m ? acc : t - clk[m] * acc;
        }
    }
    if (lane < n) x[lane] = t;
}

// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N - 1>{}): indices as constants
template <class F, int... Q>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Q...>) {
    (f(std::integral_constant<int, Q>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// compile-time tile geometry of chol_tile_solve2: systems of T0 and T1 tile rows (T = (n + 16) / 16),
// tile g of the lower tiles (system 0 row-major, then system 1) -> tile wave g % 2, slot g / 2
template <int T0, int T1, int W>
struct CholTiles {
    static constexpr int NT0 = T0 * (T0 + 1) / 2, NTOT = NT0 + T1 * (T1 + 1) / 2;
    static constexpr int NS = (NTOT - W + 1) / 2;  // slots of tile wave W
    static constexpr int g(int q) { return W + 2 * q; }
    static constexpr int sys(int q) { return g(q) >= NT0 ? 1 : 0; }
    static constexpr int loc(int q) { return sys(q) ? g(q) - NT0 : g(q); }
    static constexpr int a(int q) {
        int gg = loc(q), r = 0;
        while (gg > r) { gg -= r + 1; ++r; }
        return r;
    }
    static constexpr int b(int q) { return loc(q) - a(q) * (a(q) + 1) / 2; }
    static constexpr int soff(int q) { return sys(q) ? 16 * T0 : 0; }  // first row of the system in P / E
};

// the tile wave's part of chol_tile_solve2 (wave 2 + W): its tiles stay in registers for the whole
// factorisation; two barriers per block column, matching the factoring waves' loop
template <int T0, int T1, int W>
__device__ __forceinline__ void chol_tile_wave(const double* A0, int n0, const double* A1, int n1, int lda, double* A0w,
                                               double* A1w, double* Pb, double* E, double* dv, int nb0, int nb1, int nb,
                                               int lane, unsigned long long* tm) {
    using G = CholTiles<T0, T1, W>;
    // (diagnostic, tm non-null: lane 0 of wave 2 adds shader clocks of [4] part 1 + column out, [5] barrier 1,
    // [6] part 2 + inverse, [8] barrier 2)
    unsigned long long tlast = tm ? __builtin_amdgcn_s_memtime() : 0;
    auto tmark = [&](int slot) {
        if (tm && threadIdx.x == 128) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            tm[slot] += tt - tlast;
            tlast = tt;
        }
    };
    constexpr int NS = G::NS > 0 ? G::NS : 1;
    double* const trash = E + kTileRows * kTilePW;
    cd4 acc[NS];
    static_for<NS>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        acc[q] = cd4{0.0, 0.0, 0.0, 0.0};
        if constexpr (q < G::NS) {
            constexpr int s = G::sys(q), ta = G::a(q), tb = G::b(q);
            const double* A = s ? A1 : A0;
            const int n = s ? n1 : n0;
            const int col = 16 * tb + (lane & 15);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = 16 * ta + (lane >> 4) + 4 * i;
                const bool in = row <= n && col <= row && col < n;
                const double v = A[(in ? row : 0) * lda + (in ? col : 0)];
                acc[q][i] = in ? v : 0.0;
            }
        }
    });
    __syncthreads();  // panels zeroed
    // block steps as compile-time J (at most 64 / 6 + 1 for 4 tile rows): which slots hold block column
    // J is then a constant, and panel J-1 is applied to those first (part 1), to the rest after the barrier
    // (part 2); operands of a part's slots are requested before its MFMAs
    constexpr int NBMAX = (16 * (T0 > T1 ? T0 : T1)) / 6 + 1;
    static_for<NBMAX>([&](auto JJ) {
        constexpr int J = decltype(JJ)::value, c0 = 6 * J;
        if (J >= nb) return;  // uniform: the factoring waves' loop has nb steps
        const double* P = Pb + ((J & 1) ^ 1) * kPanelStride;  // panel J-1
        auto update = [&](auto Part1) {
            constexpr bool part1 = decltype(Part1)::value;
            double av[NS][2], bv[NS][2];
            static_for<NS>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                if constexpr (q < G::NS) {
                    constexpr int c16 = 16 * G::b(q);
                    if constexpr (J > 0 && (c16 <= c0 + 5 && c16 + 15 >= c0) == part1) {
                        constexpr int pa = G::soff(q) + 16 * G::a(q), pb = G::soff(q) + 16 * G::b(q);
#pragma unroll
                        for (int kh = 0; kh < 2; ++kh) {
                            av[q][kh] = -P[(pa + (lane & 15)) * kTilePW + 4 * kh + (lane >> 4)];
                            bv[q][kh] = P[(pb + (lane & 15)) * kTilePW + 4 * kh + (lane >> 4)];
                        }
                    }
                }
            });
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
                static_for<NS>([&](auto Q) {
                    constexpr int q = decltype(Q)::value;
                    if constexpr (q < G::NS) {
                        constexpr int c16 = 16 * G::b(q);
                        if constexpr (J > 0 && (c16 <= c0 + 5 && c16 + 15 >= c0) == part1)
                            acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q][kh], bv[q][kh], acc[q], 0, 0, 0);
                    }
                });
        };
        update(std::true_type{});
        static_for<NS>([&](auto Q) {  // block column J out of the tiles holding it (others: the trash row)
            constexpr int q = decltype(Q)::value;
            if constexpr (q < G::NS) {
                constexpr int s = G::sys(q), c16 = 16 * G::b(q), r16 = 16 * G::a(q), so = G::soff(q);
                if constexpr (c16 <= c0 + 5 && c16 + 15 >= c0 && r16 + 15 >= c0) {
                    const int col = c16 + (lane & 15), n = (J < (s ? nb1 : nb0)) ? (s ? n1 : n0) : -1;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = r16 + (lane >> 4) + 4 * i;
                        const bool in = col >= c0 && col < c0 + 6 && row >= c0 && row <= n;
                        *(in ? E + (so + row) * kTilePW + col - c0 : trash + (lane & 7)) = acc[q][i];
                    }
                }
            }
        });
        tmark(4);
        __syncthreads();
        tmark(5);
        if constexpr (J > 0) {
            update(std::false_type{});
            if (J - 1 < (W ? nb1 : nb0))  // the previous diagonal block's inverse (wave 2: system 0, wave 3: system 1)
                chol6_inv_upper((W ? A1w : A0w) + (c0 - 6) * lda + c0 - 6, lda, dv + (W ? kTileRows : 0) + c0 - 6, lane, trash);
        }
        tmark(6);
        __syncthreads();
        tmark(8);
    });
}

template <int T0, int T1>
__device__ __forceinline__ bool chol_tile_solve2(double* A0, int n0, double* A1, int n1, int lda, double* x0, double* x1,
                                                 double* scr, int* flag, unsigned long long* tm = nullptr) {
    static_assert(T0 <= 4 && T1 <= 4 && T0 + T1 <= kTileRows / 16, "chol_tile_solve2: one panel row per lane");
    // tm (diagnostic, may be null): shader clocks of [set-up, factorisation, -, backward] seen by thread 0
    unsigned long long tlast = tm ? __builtin_amdgcn_s_memtime() : 0;
    auto tmark = [&](int slot) {
        if (tm && threadIdx.x == 0) {
            const unsigned long long tt = __builtin_amdgcn_s_memtime();
            tm[slot] += tt - tlast;
            tlast = tt;
        }
    };
    const int t = (int)threadIdx.x, lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);
    const int nb0 = n0 / 6, nb1 = n1 / 6, nb = nb0 > nb1 ? nb0 : nb1;
    A0 = lds_base(A0);
    A1 = lds_base(A1);
    scr = lds_base(scr);
    constexpr int soff1 = 16 * T0;                     // system 1's first row in the panel / column buffers
    double* const Pb = scr;                            // panel buffers, parity p at Pb + p * kPanelStride
    double* const E = scr + 2 * kPanelStride;          // column buffer; row kTileRows: trash
    double* const trash = E + kTileRows * kTilePW;
    double* const dv = E + (kTileRows + 1) * kTilePW;  // 1 / L[c][c]: system 0 at dv, system 1 at dv + kTileRows
    for (int e = t; e < 2 * kPanelStride; e += 256) Pb[e] = 0.0;
    if (t == 0) *flag = 0;
    tmark(0);
    if (wid >= 2) {
        if (wid == 2) chol_tile_wave<T0, T1, 0>(A0, n0, A1, n1, lda, A0, A1, Pb, E, dv, nb0, nb1, nb, lane, tm);
        else chol_tile_wave<T0, T1, 1>(A0, n0, A1, n1, lda, A0, A1, Pb, E, dv, nb0, nb1, nb, lane, nullptr);
    } else {
        __syncthreads();  // panels zeroed, the tiles loaded
        const int s = wid, n = s ? n1 : n0, nbs = s ? nb1 : nb0;
        double* const A = s ? A1 : A0;
        const double* const Es = E + (s ? soff1 : 0) * kTilePW;
        double* const inv = dv + (s ? kTileRows : 0);
        int bad = 0;
        for (int J = 0; J < nb; ++J) {
            const int c0 = 6 * J, par = J & 1;
            __syncthreads();  // block column J in E
            tmark(9);
            // (b) diagonal block J and the panel row below it, wave s for system s
            if (J < nbs) {
                double* const P = Pb + par * kPanelStride + (s ? soff1 : 0) * kTilePW;
                double* const Ptrash = Pb + par * kPanelStride + (kTileRows + 1) * kTilePW;
                const int rA = c0 + 6 + lane;
                const bool live = rA <= n;
                cd2 dr[6][3], er[3];
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int p = 0; p < 3; ++p) dr[i][p] = *reinterpret_cast<const cd2*>(Es + (c0 + i) * kTilePW + 2 * p);
                const double* erow = Es + (live ? rA : n) * kTilePW;
#pragma unroll
                for (int p = 0; p < 3; ++p) er[p] = *reinterpret_cast<const cd2*>(erow + 2 * p);
                double l[21], ea[6];
#pragma unroll
                for (int i = 0, qq = 0; i < 6; ++i)
#pragma unroll
                    for (int k = 0; k <= i; ++k, ++qq) l[qq] = dr[i][k >> 1][k & 1];
#pragma unroll
                for (int c = 0; c < 6; ++c) ea[c] = er[c >> 1][c & 1];
                tmark(10);
                double r[6];
#pragma unroll
                for (int c = 0; c < 6; ++c) {
                    const double piv = l[c * (c + 1) / 2 + c];
                    bad |= !(piv > 0.0);
                    r[c] = rsq_nr(piv);
                    l[c * (c + 1) / 2 + c] = piv * r[c];
#pragma unroll
                    for (int i = c + 1; i < 6; ++i) l[i * (i + 1) / 2 + c] *= r[c];
#pragma unroll
                    for (int i = c + 1; i < 6; ++i)
#pragma unroll
                        for (int k = c + 1; k <= i; ++k) l[i * (i + 1) / 2 + k] -= l[i * (i + 1) / 2 + c] * l[k * (k + 1) / 2 + c];
                    // the panel's column c as soon as L's column c is known
#pragma unroll
                    for (int m = 0; m < c; ++m) ea[c] -= ea[m] * l[c * (c + 1) / 2 + m];
                    ea[c] *= r[c];
                }
                tmark(11);
                // panel row (or the trash row), the previous panel's rows of this buffer zeroed (lanes < 12)
                double* prow = live ? P + rA * kTilePW : Ptrash;
#pragma unroll
                for (int p = 0; p < 3; ++p) *reinterpret_cast<cd2*>(prow + 2 * p) = cd2{ea[2 * p], ea[2 * p + 1]};
                const int zr = c0 - 6 + lane;
                double* zrow = (lane < 12 && zr >= 0) ? P + zr * kTilePW : Ptrash;
#pragma unroll
                for (int p = 0; p < 3; ++p) *reinterpret_cast<cd2*>(zrow + 2 * p) = cd2{0.0, 0.0};
                // L: the panel row; the diagonal block's strictly lower entries and 1 / L[c][c] from lane 0 (every
                // lane holds them: plain stores instead of per-lane select chains).  Nothing reads the block's
                // diagonal or upper entries: the pivots go to inv, chol6_inv_upper writes L_JJ^-1 above the diagonal
                double* arow = live ? A + rA * lda + c0 : trash;
#pragma unroll
                for (int c = 0; c < 6; ++c) arow[c] = ea[c];
                if (lane == 0) {
#pragma unroll
                    for (int i = 1; i < 6; ++i)
#pragma unroll
                        for (int k = 0; k < i; ++k) A[(c0 + i) * lda + c0 + k] = l[i * (i + 1) / 2 + k];
#pragma unroll
                    for (int c = 0; c < 6; ++c) inv[c0 + c] = r[c];
                }
            }
            tmark(12);
            __syncthreads();  // panel J in P
            tmark(13);
        }
        if (bad && lane == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    tmark(1);
    if (*flag) return false;
    // the last diagonal blocks' inverses, then the backward substitution by wave s
    if (wid >= 2) {
        const int s = wid - 2, nbs = s ? nb1 : nb0;
        if (nbs > 0)
            chol6_inv_upper((s ? A1 : A0) + 6 * (nbs - 1) * lda + 6 * (nbs - 1), lda, dv + (s ? kTileRows : 0) + 6 * (nbs - 1),
                            lane, E + kTileRows * kTilePW);
    }
    __syncthreads();
    if (wid == 0 && nb0 > 0) chol6_backward_blk(A0, lda, n0, dv, x0, lane);
    else if (wid == 1 && nb1 > 0) chol6_backward_blk(A1, lda, n1, dv + kTileRows, x1, lane);
    __syncthreads();
    tmark(3);
    return true;
}

// One system of chol_mw_solve2 on waves [w0, w0 + NW) of the workgroup: lane i holds row i (i < n;
// lane n holds the right-hand side) restricted to the wave's CB columns [CB v, CB v + CB), v = wave - w0.
// Pivot j: its owner wave (j / CB) factors it (rsq + Newton), writes L[:, j] to colbuf and updates its
// own next column first (look-ahead: the next pivot's chain overlaps the other waves' bulk updates);
// after the workgroup barrier every wave applies L[:, j] to its remaining columns (A[i][k] -= L[i][j]
// L[k][j], m ascending per element: the textbook left-to-right sum of every L[i][k]).  nsteps (>= n,
// uniform) is the barrier count both systems share.  L goes back over A (row stride lda; the rhs row
// becomes y = L^-1 b), 1 / L[j][j] to dinv.  Returns nonzero on a non-positive pivot (owner waves).
template <int NW, int CB, int NSMAX>
__device__ __forceinline__ int chol_mw_factor(double* A, int lda, int n, int nsteps, int w0, double* colbuf,
                                              double* dinv) {
    const int t = (int)threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6) - w0;
    const bool part = wv >= 0 && wv < NW;
    double d[CB];
    const int cbase = CB * wv;
    if (part) {
        const double* arow = A + (lane <= n ? lane : n) * lda;
#pragma unroll
        for (int q = 0; q < CB; ++q) {
            const int k = cbase + q;
            const double v = k < n ? arow[k] : 0.0;
            d[q] = lane < n ? (k <= lane ? v : 0.0) : (lane == n ? v : 0.0);
        }
    }
    int bad = 0;
    double piv_next = 0.0;
#pragma unroll
    for (int j = 0; j < NSMAX; ++j) {
        if (j >= nsteps) break;  // uniform: both systems stop together
        const bool act = j < n;
        const int o = j / CB, q = j % CB;
        double* cb = colbuf + (j & 1) * 64;
        if (act && part && wv == o) {
            const double piv = q == 0 ? readlane_d(d[0], j) : piv_next;
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
                const double lk = cb[k < 63 ? k : 63];
                if (k > j && !(wv == o && qq == q + 1)) d[qq] -= ci * lk;
            }
        }
    }
    if (part && lane <= n) {
        double* w = A + lane * lda;
#pragma unroll
        for (int q = 0; q < CB; ++q) {
            const int k = cbase + q;
            if (k < n) w[k] = (k <= lane || lane == n) ? d[q] : 0.0;
        }
    }
    return bad;
}
// L^T x = y by one wave (lane = column m), column-oriented from the last row: x may alias nothing in A
template <int NMAX>
__device__ __forceinline__ void chol_mw_backward(const double* A, int lda, int n, const double* dinv, double* x,
                                                 int lane) {
    double tt = lane < n ? A[n * lda + lane] : 0.0;
    const double dv = lane < n ? dinv[lane] : 0.0;
#pragma unroll
    for (int m = NMAX - 1; m >= 0; --m) {
        if (m < n) {
            const double e = lane < m ? A[m * lda + lane] : 0.0;
            const double xm = readlane_d(tt * dv, m);
            tt = lane == m ? xm : tt - e * xm;
        }
    }
    if (lane < n) x[lane] = tt;
}
// The window's block-diagonal reduced system: the pose block (n0 <= 54) over waves 0-1 and the velocity /
// bias block (n1 <= 54) over waves 2-3, 27 columns per wave, one code path (the per-wave system chosen by
// pointer), both systems sharing the per-pivot barriers (see chol_mw_factor); right-hand sides as row
// n_s of each block.  Returns false (uniformly) on a non-positive pivot.  colbuf: 256 doubles, dinv0 /
// dinv1: n_s doubles, flag: one LDS int.
__device__ __forceinline__ bool chol_mw_solve2(double* A0, int n0, double* A1, int n1, int lda, double* x0, double* x1,
                                      double* colbuf, double* dinv0, double* dinv1, int* flag) {
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nsteps = n0 > n1 ? n0 : n1;
    if (threadIdx.x == 0) *flag = 0;
    __syncthreads();
    const bool s1 = wid >= 2;
    const int bad = chol_mw_factor<2, 27, 54>(s1 ? A1 : A0, lda, s1 ? n1 : n0, nsteps, s1 ? 2 : 0,
                                             colbuf + (s1 ? 128 : 0), s1 ? dinv1 : dinv0);
    if (bad) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    if (*flag) return false;
    if (wid == 0 || (wid == 2 && n1 > 0))
        chol_mw_backward<54>(s1 ? A1 : A0, lda, s1 ? n1 : n0, s1 ? dinv1 : dinv0, s1 ? x1 : x0, lane);
    __syncthreads();
    return true;
}

}  // namespace vio360
