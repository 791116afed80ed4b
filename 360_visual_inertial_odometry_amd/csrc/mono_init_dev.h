// mono_init_dev.h — device arithmetic of the monocular initialiser (Initializer.cpp), see mono_init.hip.
// Float expressions follow the reference's Eigen f32 evaluation order; build with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "vio360.h"

namespace vio360 {

constexpr int kMaxInitPoints = 4096;

// row of the epipolar system, b2^T E b1 = 0 (:505-519): A(i, 3r + c) = b2[r] * b1[c]
__device__ __forceinline__ void mi_epipolar_row(const float* b1, const float* b2, float* row) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) row[3 * r + c] = b2[r] * b1[c];
}

// |b2^T E b1| (:551): (b2^T E) first, then the dot with b1
__device__ __forceinline__ float mi_epipolar_error(const float* E, const float* b1, const float* b2) {
    float w[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) w[c] = (b2[0] * E[c] + b2[1] * E[3 + c]) + b2[2] * E[6 + c];
    return fabsf((w[0] * b1[0] + w[1] * b1[1]) + w[2] * b1[2]);
}

// upper-triangle enumeration of a 9x9 matrix: pq -> (p, q), p <= q, row-major
__device__ __forceinline__ int mi_pq_row(int pq) {
    int p = 0;
    while (pq >= 9 - p) {
        pq -= 9 - p;
        ++p;
    }
    return p;
}
__device__ __forceinline__ int mi_pq_col(int pq) {
    int p = 0;
    while (pq >= 9 - p) {
        pq -= 9 - p;
        ++p;
    }
    return p + pq;
}

// cyclic Jacobi eigen-decomposition of a symmetric N x N matrix A (element (p,q) at A[(pN+q)*st]);
// V (same layout) receives the eigenvectors as columns, A's diagonal the eigenvalues.
template <int N>
__device__ inline void mi_jacobi(double* A, double* V, int st) {
    for (int p = 0; p < N; ++p)
        for (int q = 0; q < N; ++q) V[(p * N + q) * st] = p == q ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0, dg = 0.0;
        for (int p = 0; p < N; ++p) {
            dg += A[(p * N + p) * st] * A[(p * N + p) * st];
            for (int q = p + 1; q < N; ++q) off += A[(p * N + q) * st] * A[(p * N + q) * st];
        }
        if (!(off > 1e-32 * dg)) break;
        for (int p = 0; p < N - 1; ++p)
            for (int q = p + 1; q < N; ++q) {
                const double apq = A[(p * N + q) * st];
                if (apq == 0.0) continue;
                const double app = A[(p * N + p) * st], aqq = A[(q * N + q) * st];
                const double theta = (aqq - app) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < N; ++k) {
                    if (k == p || k == q) continue;
                    const double akp = A[(k * N + p) * st], akq = A[(k * N + q) * st];
                    const double np = c * akp - s * akq, nq = s * akp + c * akq;
                    A[(k * N + p) * st] = np;
                    A[(p * N + k) * st] = np;
                    A[(k * N + q) * st] = nq;
                    A[(q * N + k) * st] = nq;
                }
                A[(p * N + p) * st] = app - t * apq;
                A[(q * N + q) * st] = aqq + t * apq;
                A[(p * N + q) * st] = 0.0;
                A[(q * N + p) * st] = 0.0;
                for (int k = 0; k < N; ++k) {
                    const double vkp = V[(k * N + p) * st], vkq = V[(k * N + q) * st];
                    V[(k * N + p) * st] = c * vkp - s * vkq;
                    V[(k * N + q) * st] = s * vkp + c * vkq;
                }
            }
    }
}

// eigenvector of the smallest eigenvalue (first on ties), largest |component| made positive
template <int N>
__device__ inline void mi_null_vector(double* A, double* V, int st, double* e) {
    mi_jacobi<N>(A, V, st);
    int kmin = 0;
    for (int k = 1; k < N; ++k)
        if (A[(k * N + k) * st] < A[(kmin * N + kmin) * st]) kmin = k;
    int imax = 0;
    for (int i = 0; i < N; ++i) {
        e[i] = V[(i * N + kmin) * st];
        if (fabs(e[i]) > fabs(e[imax])) imax = i;
    }
    if (e[imax] < 0.0)
        for (int i = 0; i < N; ++i) e[i] = -e[i];
}

// SVD of a 3x3 f32 matrix through the eigen-decomposition of M^T M in f64: singular values
// s[0] >= s[1] >= s[2], right vectors v[k] (columns), left vectors u[k] = M v[k] / s[k] for k < 2,
// third columns u2 = u0 x u1, v2 = v0 x v1 (proper rotations).
__device__ inline void mi_svd3(const float* M, double (*u)[3], double* s, double (*v)[3]) {
    double A[9], V[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            A[3 * i + j] = ((double)M[i] * (double)M[j] + (double)M[3 + i] * (double)M[3 + j]) +
                           (double)M[6 + i] * (double)M[6 + j];
    mi_jacobi<3>(A, V, 1);
    int o[3] = {0, 1, 2};
    // descending eigenvalues, stable on ties
    for (int i = 1; i < 3; ++i)
        for (int j = i; j > 0 && A[4 * o[j]] > A[4 * o[j - 1]]; --j) {
            const int tmp = o[j];
            o[j] = o[j - 1];
            o[j - 1] = tmp;
        }
    for (int k = 0; k < 3; ++k) {
        const double l = A[4 * o[k]];
        s[k] = l > 0.0 ? sqrt(l) : 0.0;
        for (int i = 0; i < 3; ++i) v[k][i] = V[3 * i + o[k]];
    }
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < 3; ++i) {
            const double mv = ((double)M[3 * i] * v[k][0] + (double)M[3 * i + 1] * v[k][1]) + (double)M[3 * i + 2] * v[k][2];
            u[k][i] = s[k] > 0.0 ? mv / s[k] : 0.0;
        }
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    v[2][0] = v[0][1] * v[1][2] - v[0][2] * v[1][1];
    v[2][1] = v[0][2] * v[1][0] - v[0][0] * v[1][2];
    v[2][2] = v[0][0] * v[1][1] - v[0][1] * v[1][0];
}

// E from the null vector, projected to singular values (s, s, 0) with s = (s0 + s1) / 2 (:525-538)
__device__ inline void mi_project_essential(const double* e, float* E) {
    float Ec[9];
    for (int k = 0; k < 9; ++k) Ec[k] = (float)e[k];
    double u[3][3], s[3], v[3][3];
    mi_svd3(Ec, u, s, v);
    const double sigma = (s[0] + s[1]) * 0.5;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) E[3 * i + j] = (float)(sigma * (u[0][i] * v[0][j] + u[1][i] * v[1][j]));
}

__device__ __forceinline__ float mi_det3(const float* m) {  // cofactor expansion along the first row
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) + m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// RecoverPose's four candidates (:636-663): R1 = U W V^T, R2 = U W^T V^T, t1 = U.col(2) normalised
__device__ inline void mi_pose_candidates(const float* E, float (*Rc)[9], float (*tc)[3]) {
    double u[3][3], s[3], v[3][3];
    mi_svd3(E, u, s, v);
    // U W: columns (u1, -u0, u2); U W^T: columns (-u1, u0, u2)
    float R1[9], R2[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            R1[3 * i + j] = (float)((u[1][i] * v[0][j] - u[0][i] * v[1][j]) + u[2][i] * v[2][j]);
            R2[3 * i + j] = (float)((u[0][i] * v[1][j] - u[1][i] * v[0][j]) + u[2][i] * v[2][j]);
        }
    float t1[3] = {(float)u[2][0], (float)u[2][1], (float)u[2][2]};
    if (mi_det3(R1) < 0.f) {
        for (int k = 0; k < 9; ++k) R1[k] = -R1[k];
        for (int k = 0; k < 3; ++k) t1[k] = -t1[k];
    }
    if (mi_det3(R2) < 0.f)
        for (int k = 0; k < 9; ++k) R2[k] = -R2[k];
    const float nrm = sqrtf((t1[0] * t1[0] + t1[1] * t1[1]) + t1[2] * t1[2]);
    for (int k = 0; k < 3; ++k) t1[k] = t1[k] / nrm;
    for (int k = 0; k < 9; ++k) {
        Rc[0][k] = R1[k];
        Rc[1][k] = R1[k];
        Rc[2][k] = R2[k];
        Rc[3][k] = R2[k];
    }
    for (int k = 0; k < 3; ++k) {
        tc[0][k] = t1[k];
        tc[1][k] = -t1[k];
        tc[2][k] = t1[k];
        tc[3][k] = -t1[k];
    }
}

__device__ __forceinline__ float mi_dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
__device__ __forceinline__ float mi_norm3(const float* a) { return sqrtf(mi_dot3(a, a)); }

// R x + t (f32 matrix-vector, then + t)
__device__ __forceinline__ void mi_transform(const float* R, const float* t, const float* x, float* y) {
#pragma unroll
    for (int r = 0; r < 3; ++r) y[r] = ((R[3 * r] * x[0] + R[3 * r + 1] * x[1]) + R[3 * r + 2] * x[2]) + t[r];
}

// TriangulateSinglePoint (:728-783): mid-point of the rays, in frame-1 coordinates
__device__ inline bool mi_triangulate(const float* b1, const float* b2, const float* R, const float* t, float* X) {
    float tr[3], b2f1[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        tr[c] = -((R[c] * t[0] + R[3 + c] * t[1]) + R[6 + c] * t[2]);
        b2f1[c] = (R[c] * b2[0] + R[3 + c] * b2[1]) + R[6 + c] * b2[2];
    }
    const float a00 = mi_dot3(b1, b1);
    const float a10 = mi_dot3(b1, b2f1);
    const float a01 = -a10;
    const float a11 = -mi_dot3(b2f1, b2f1);
    const float r0 = mi_dot3(b1, tr), r1 = mi_dot3(b2f1, tr);
    const float det = a00 * a11 - a01 * a10;
    if (fabsf(det) < 1e-10f) return false;
    // Eigen 2x2 inverse: its own determinant, 1/det, cofactors
    const float invdet = 1.0f / (a00 * a11 - a10 * a01);
    const float i00 = a11 * invdet, i01 = -a01 * invdet, i10 = -a10 * invdet, i11 = a00 * invdet;
    const float l0 = i00 * r0 + i01 * r1, l1 = i10 * r0 + i11 * r1;
    if (!isfinite(l0) || !isfinite(l1)) return false;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float p1 = l0 * b1[c];
        const float p2 = l1 * b2f1[c] + tr[c];
        X[c] = (p1 + p2) / 2.0f;
    }
    return true;
}

// ComputeReprojectionErrorInFrame (:837-871); the pixel maps mix float and double as the
// reference's expressions do (theta / (2.0f * M_PI) is a double division)
__device__ __forceinline__ float mi_clamp1(float x) { return x < -1.0f ? -1.0f : (1.0f < x ? 1.0f : x); }  // std::clamp

__device__ inline float mi_reproj_error(const float* p, const float* b, int W, int H) {
    const float L = mi_norm3(p);
    if (L < 1e-6f) return 1000.0f;
    const float th_o = atan2f(b[0], b[2]);
    const float ph_o = -asinf(mi_clamp1(b[1]));
    const float u_o = (float)((double)W * ((double)0.5f + (double)th_o / (2.0 * M_PI)));
    const float v_o = (float)((double)H * ((double)0.5f - (double)ph_o / M_PI));
    const float q[3] = {p[0] / L, p[1] / L, p[2] / L};
    const float th_p = atan2f(q[0], q[2]);
    const float ph_p = -asinf(mi_clamp1(q[1]));
    const float u_p = (float)((double)W * ((double)0.5f + (double)th_p / (2.0 * M_PI)));
    const float v_p = (float)((double)H * ((double)0.5f - (double)ph_p / M_PI));
    const float du = u_o - u_p, dv = v_o - v_p;
    return sqrtf(du * du + dv * dv);
}

}  // namespace vio360
