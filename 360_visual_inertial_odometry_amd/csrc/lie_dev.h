// lie_dev.h — f64 SO3/SE3 device maths used inside the BA kernels.
// Restates src/util/LieUtils.cpp:203-370 (SO3d::Exp, SE3d::exp, compose, inverse).  The SVD
// re-orthonormalisation that every SO3d construction performs (LieUtils.cpp:275-288) is applied
// once to the f32-derived input rotations (polar3); products of already-orthonormal matrices are
// orthonormal to ~1e-16, where the projection is a no-op.
#pragma once
#include <hip/hip_runtime.h>

namespace vio360 {

__device__ __forceinline__ void m3mul(const double* a, const double* b, double* c) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}
__device__ __forceinline__ void m3tmul(const double* a, const double* b, double* c) {  // a^T b
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c[3 * i + j] = a[i] * b[j] + a[3 + i] * b[3 + j] + a[6 + i] * b[6 + j];
}
__device__ __forceinline__ void m3vec(const double* a, const double* v, double* o) {
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = a[3 * i] * v[0] + a[3 * i + 1] * v[1] + a[3 * i + 2] * v[2];
}
__device__ __forceinline__ void m3tvec(const double* a, const double* v, double* o) {  // a^T v
#pragma unroll
    for (int i = 0; i < 3; ++i) o[i] = a[i] * v[0] + a[3 + i] * v[1] + a[6 + i] * v[2];
}
__device__ __forceinline__ void hat3(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
__device__ __forceinline__ double det3(const double* a) {
    return a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
}
__device__ __forceinline__ double nrm3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// inverse of a general 3x3 by cofactors; returns false if singular
__device__ __forceinline__ bool inv3(const double* a, double* o) {
    double c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
    double d = a[0] * c00 + a[1] * c01 + a[2] * c02;
    if (d == 0.0) return false;
    double id = 1.0 / d;
    o[0] = c00 * id; o[1] = (a[2] * a[7] - a[1] * a[8]) * id; o[2] = (a[1] * a[5] - a[2] * a[4]) * id;
    o[3] = c01 * id; o[4] = (a[0] * a[8] - a[2] * a[6]) * id; o[5] = (a[2] * a[3] - a[0] * a[5]) * id;
    o[6] = c02 * id; o[7] = (a[1] * a[6] - a[0] * a[7]) * id; o[8] = (a[0] * a[4] - a[1] * a[3]) * id;
    return true;
}

// polar factor (nearest rotation) of a near-orthonormal 3x3 by Newton's iteration
// X <- (X + X^-T)/2, which converges quadratically to the same U V^T the reference's JacobiSVD
// projection yields for det > 0 inputs.
__device__ __forceinline__ void polar3_inl(const double* A, double* R) {
    double X[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) X[i] = A[i];
    for (int it = 0; it < 12; ++it) {
        double Xi[9];
        if (!inv3(X, Xi)) break;
        double diff = 0.0;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double nv = 0.5 * (X[3 * i + j] + Xi[3 * j + i]);
                diff = fmax(diff, fabs(nv - X[3 * i + j]));
                X[3 * i + j] = nv;
            }
        if (diff < 1e-17) break;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = X[i];
}
// (the call form: the compiler decides; polar3_inl where a kernel must stay call-free)
__device__ inline void polar3(const double* A, double* R) { polar3_inl(A, R); }

// SO3d::Exp (LieUtils.cpp:203-219)
__device__ inline void so3_exp(const double* w, double* R) {
    double th = nrm3(w);
    double K[9];
    if (th < 1e-10) {
        hat3(w, K);
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = K[i];
        R[0] += 1; R[4] += 1; R[8] += 1;
        return;
    }
    double k[3] = {w[0] / th, w[1] / th, w[2] / th}, K2[9];
    hat3(k, K);
    m3mul(K, K, K2);
    double s = sin(th), c = 1.0 - cos(th);
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = s * K[i] + c * K2[i];
    R[0] += 1; R[4] += 1; R[8] += 1;
}

// SE3d::exp (LieUtils.cpp:305-333), xi = [rho, phi]
__device__ inline void se3_exp(const double* xi, double* R, double* t) {
    so3_exp(xi + 3, R);
    const double* phi = xi + 3;
    double th = nrm3(phi);
    if (th < 1e-10) {
        t[0] = xi[0]; t[1] = xi[1]; t[2] = xi[2];
        return;
    }
    double P[9], P2[9], V[9];
    hat3(phi, P);
    m3mul(P, P, P2);
    double th2 = th * th, a = (1.0 - cos(th)) / th2, b = (th - sin(th)) / (th2 * th);
#pragma unroll
    for (int i = 0; i < 9; ++i) V[i] = a * P[i] + b * P2[i];
    V[0] += 1; V[4] += 1; V[8] += 1;
    m3vec(V, xi, t);
}

}  // namespace vio360
