// init_host.cpp — host side of the monocular initialisation: the RANSAC sample
// stream, feature selection, parallax and the frame-pose composition of
// Initializer::TryMonocularInitialization (src/processing/Initializer.cpp).  No device work.
#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

#include "vio360.h"

extern "C" int vio_mono_init_samples(uint32_t seed, int n, int iters, int32_t* out) {
    // Initializer.cpp:477-494: mt19937 + uniform_int_distribution<>(0, n-1), 8 distinct per hypothesis
    if (n < 8 || iters < 0 || (iters > 0 && !out)) return VIO_EINVAL;
    std::mt19937 gen(seed);
    std::uniform_int_distribution<> dis(0, n - 1);
    for (int it = 0; it < iters; ++it) {
        int got[8], k = 0;
        while (k < 8) {
            const int idx = dis(gen);
            bool dup = false;
            for (int q = 0; q < k; ++q) dup |= got[q] == idx;
            if (!dup) got[k++] = idx;
        }
        for (int q = 0; q < 8; ++q) out[8 * it + q] = got[q];
    }
    return VIO_OK;
}

extern "C" int vio_init_select_features(const float* uv, const int32_t* obs_count, int n, int width, int height,
                                        int grid_cols, int grid_rows, int min_observations, int min_features,
                                        int32_t* out_idx, int* n_out) {
    // Initializer::SelectFeaturesForInit (:351-433)
    if (n < 0 || !n_out || grid_cols <= 0 || grid_rows <= 0 || width <= 0 || height <= 0 ||
        (n > 0 && (!uv || !obs_count || !out_idx)))
        return VIO_EINVAL;
    *n_out = 0;
    std::vector<int> cand;
    for (int i = 0; i < n; ++i)
        if (obs_count[i] >= min_observations) cand.push_back(i);
    if (cand.size() < (size_t)min_features) return VIO_OK;  // :373-375
    const int total = grid_cols * grid_rows;
    const float cw = static_cast<float>(width) / grid_cols;
    const float ch = static_cast<float>(height) / grid_rows;
    std::vector<std::vector<int>> grid(total);
    for (int i : cand) {
        int col = static_cast<int>(uv[2 * i] / cw);
        int row = static_cast<int>(uv[2 * i + 1] / ch);
        col = std::max(0, std::min(col, grid_cols - 1));
        row = std::max(0, std::min(row, grid_rows - 1));
        grid[row * grid_cols + col].push_back(i);
    }
    const int max_per_cell = 5;  // :414
    int m = 0;
    for (int g = 0; g < total; ++g) {
        if (grid[g].empty()) continue;
        // std::sort (not stable) with the reference's comparator: the same libstdc++ permutation
        std::sort(grid[g].begin(), grid[g].end(), [&](int a, int b) { return obs_count[a] > obs_count[b]; });
        const int c = std::min(max_per_cell, static_cast<int>(grid[g].size()));
        for (int j = 0; j < c; ++j) out_idx[m++] = grid[g][j];
    }
    *n_out = m;
    return VIO_OK;
}

extern "C" int vio_init_parallax(const int32_t* ids1, const float* uv1, int n1, const int32_t* ids2, const float* uv2,
                                 int n2, float* parallax) {
    // Initializer::ComputeParallax (:293-349)
    if (!parallax || n1 < 0 || n2 < 0 || (n1 > 0 && (!ids1 || !uv1)) || (n2 > 0 && (!ids2 || !uv2)))
        return VIO_EINVAL;
    *parallax = 0.f;
    if (n1 == 0 || n2 == 0) return VIO_OK;
    std::vector<float> p;
    for (int i = 0; i < n1; ++i)
        for (int j = 0; j < n2; ++j)
            if (ids1[i] == ids2[j]) {
                const float dx = uv2[2 * j] - uv1[2 * i];
                const float dy = uv2[2 * j + 1] - uv1[2 * i + 1];
                p.push_back(std::sqrt(dx * dx + dy * dy));
                break;
            }
    if (p.empty()) return VIO_OK;
    std::sort(p.begin(), p.end());
    const size_t mid = p.size() / 2;
    *parallax = (p.size() % 2 == 0) ? (p[mid - 1] + p[mid]) / 2.0f : p[mid];
    return VIO_OK;
}

namespace {
// rigid inverse of a 4x4 row-major f32 transform [R t; 0 1] -> [R^T -R^T t; 0 1]
void rigid_inverse(const float* T, float* Ti) {
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) Ti[4 * r + c] = T[4 * c + r];
        Ti[4 * r + 3] = -((T[r] * T[3] + T[4 + r] * T[7]) + T[8 + r] * T[11]);
    }
    Ti[12] = Ti[13] = Ti[14] = 0.f;
    Ti[15] = 1.f;
}
void mul4(const float* A, const float* B, float* C) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            C[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
}
}  // namespace

extern "C" int vio_init_compose(const float* T_BC, const float* R, const float* t, float* T_wb1, float* T_wb2,
                                float* points, int n) {
    // Initializer.cpp:174-224 (the reference inverts general 4x4 matrices; these are rigid)
    if (!T_BC || !R || !t || !T_wb1 || !T_wb2 || n < 0 || (n > 0 && !points)) return VIO_EINVAL;
    float T_CB[16], T12[16], T21[16], tmp[16];
    rigid_inverse(T_BC, T_CB);
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) T12[4 * r + c] = R[3 * r + c];
        T12[4 * r + 3] = t[r];
    }
    T12[12] = T12[13] = T12[14] = 0.f;
    T12[15] = 1.f;
    rigid_inverse(T12, T21);
    for (int k = 0; k < 16; ++k) T_wb1[k] = (k % 5 == 0) ? 1.f : 0.f;
    mul4(T_BC, T21, tmp);    // T_wc2 = T_wc1 * T_c2c1 with T_wc1 = T_BC
    mul4(tmp, T_CB, T_wb2);  // T_wb2 = T_wc2 * T_CB
    for (int i = 0; i < n; ++i) {
        float* p = points + 3 * i;
        float q[3];
        for (int r = 0; r < 3; ++r) q[r] = ((T_BC[4 * r] * p[0] + T_BC[4 * r + 1] * p[1]) + T_BC[4 * r + 2] * p[2]) + T_BC[4 * r + 3];
        p[0] = q[0]; p[1] = q[1]; p[2] = q[2];
    }
    return VIO_OK;
}
