/*
 * tracker_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline, never shipped).
 *
 * CPU restatement, in plain C99, of the numeric path of FeatureTracker::TrackFeatures
 * (src/processing/FeatureTracker.cpp:61-379):
 *   - cv::calcOpticalFlowPyrLK as called by TrackOpticalFlow (:228-251): buildOpticalFlowPyramid
 *     (pyrDown 5x5 Gaussian, BORDER_REFLECT_101 pads of winSize), calcSharrDeriv (BORDER_CONSTANT
 *     pads) and LKTrackerInvoker (fixed-point W_BITS = 14 bilinear weights, minEig test with
 *     minEigThreshold = 0.01 as the reference passes criteria.epsilon there, eps^2 stop,
 *     oscillation guard, final error / status re-check) — OpenCV 4.x modules/video/src/lkpyramid.cpp.
 *   - cv::goodFeaturesToTrack(blockSize 3, Sobel 3, useHarris false) as called by
 *     DetectNewFeatures (:208-226) — OpenCV 4.x modules/imgproc/src/featureselect.cpp, corner.cpp.
 *   - RejectOutliersRotationRANSAC / EstimateRotation / ComputeRotationInliers (:253-379) with
 *     Camera::PixelToBearing / AngularDistance (src/database/Camera.cpp:22-47, 89-98), on an
 *     injected sample stream (the reference seeds mt19937 from std::random_device, :273-275).
 *
 * OpenCV is a third-party dependency that is NOT in /root/reference and not in this image
 * (CMakeLists.txt:20 pins only "OpenCV 4"), and no reference test or fixture pins its outputs on
 * this path: parity against the reference binary is UNPINNED.  The restatement is pinned by
 * closed-form properties instead (pure-rotation ERP frames with analytic flow, known-corner
 * images, synthetic rotations with planted outliers; tests/test_tracker_oracle.py).
 *
 * Deliberate, documented deviations (all below float resolution of the reference's own output):
 *   - LK gradient / mismatch sums (A11, A12, A22, b1, b2) are accumulated exactly in int64, where
 *     OpenCV-x86 accumulates the same integer products in float SIMD lanes;
 *   - Sobel derivatives are the exact integer Sobel sums times (float)(1/3060) (OpenCV folds the
 *     scale into the smoothing taps), the 3x3 box sum is a direct double sum (OpenCV: running
 *     double sums);
 *   - bearings and the RANSAC rotation use double trigonometry / a double polar decomposition
 *     rounded to float (Eigen: float sinf/cosf and a float JacobiSVD).
 * The HIP kernels implement exactly these definitions, so oracle and GPU agree bitwise.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/vio360.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

int oracle_get_threads(void); /* ba_oracle.c: host threads of the CPU-baseline leg (1 for every parity test) */

static inline int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

/* ------------------------------------------------------------------------------------------ */
/* pyrDown: 5x5 [1 4 6 4 1]^2 / 256, BORDER_REFLECT_101, dst = ((w+1)/2, (h+1)/2)              */
void oracle_pyr_down(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dstride) {
    static const int wk[5] = {1, 4, 6, 4, 1};
    int dw = (sw + 1) / 2, dh = (sh + 1) / 2;
#pragma omp parallel for num_threads(oracle_get_threads()) schedule(static) if (oracle_get_threads() > 1)
    for (int y = 0; y < dh; ++y)
        for (int x = 0; x < dw; ++x) {
            int tot = 0;
            for (int ky = 0; ky < 5; ++ky) {
                const uint8_t* row = src + (size_t)reflect101(2 * y - 2 + ky, sh) * sstride;
                int rs = 0;
                for (int kx = 0; kx < 5; ++kx) rs += wk[kx] * row[reflect101(2 * x - 2 + kx, sw)];
                tot += wk[ky] * rs;
            }
            dst[(size_t)y * dstride + x] = (uint8_t)((tot + 128) >> 8);
        }
}

typedef struct {
    int w, h;
    uint8_t* img;   /* w*h */
    int16_t* dx;    /* w*h (prev pyramid only) */
    int16_t* dy;
} level_t;

/* calcSharrDeriv: [3 10 3]^T x [-1 0 1] and transpose, BORDER_REFLECT_101 inside the image */
static void scharr(const level_t* L, int16_t* dx, int16_t* dy) {
    int w = L->w, h = L->h;
#pragma omp parallel for num_threads(oracle_get_threads()) schedule(static) if (oracle_get_threads() > 1)
    for (int y = 0; y < h; ++y) {
        const uint8_t* r0 = L->img + (size_t)reflect101(y - 1, h) * w;
        const uint8_t* r1 = L->img + (size_t)y * w;
        const uint8_t* r2 = L->img + (size_t)reflect101(y + 1, h) * w;
        for (int x = 0; x < w; ++x) {
            int xm = reflect101(x - 1, w), xp = reflect101(x + 1, w);
            int t0m = (r0[xm] + r2[xm]) * 3 + r1[xm] * 10, t0p = (r0[xp] + r2[xp]) * 3 + r1[xp] * 10;
            int t1m = r2[xm] - r0[xm], t1c = r2[x] - r0[x], t1p = r2[xp] - r0[xp];
            dx[(size_t)y * w + x] = (int16_t)(t0p - t0m);
            dy[(size_t)y * w + x] = (int16_t)((t1p + t1m) * 3 + t1c * 10);
        }
    }
}

/* image read with the REFLECT_101 pad of winSize (buildOpticalFlowPyramid) */
static inline int img_at(const level_t* L, int x, int y) {
    return L->img[(size_t)reflect101(y, L->h) * L->w + reflect101(x, L->w)];
}
/* derivative read with the BORDER_CONSTANT (zero) pad of winSize */
static inline void der_at(const level_t* L, int x, int y, int* gx, int* gy) {
    if (x < 0 || y < 0 || x >= L->w || y >= L->h) { *gx = 0; *gy = 0; return; }
    *gx = L->dx[(size_t)y * L->w + x];
    *gy = L->dy[(size_t)y * L->w + x];
}

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

static int build_pyramid(const uint8_t* img, int W, int H, int stride, int win, int max_level, int with_deriv,
                         level_t* lv) {
    int levels = 0;
    int w = W, h = H;
    for (int l = 0; l <= max_level; ++l) {
        lv[l].w = w; lv[l].h = h;
        lv[l].img = (uint8_t*)malloc((size_t)w * h);
        if (l == 0) {
            for (int y = 0; y < h; ++y) memcpy(lv[0].img + (size_t)y * w, img + (size_t)y * stride, w);
        } else {
            oracle_pyr_down(lv[l - 1].img, lv[l - 1].w, lv[l - 1].h, lv[l - 1].w, lv[l].img, w);
        }
        lv[l].dx = lv[l].dy = NULL;
        if (with_deriv) {
            lv[l].dx = (int16_t*)malloc(sizeof(int16_t) * (size_t)w * h);
            lv[l].dy = (int16_t*)malloc(sizeof(int16_t) * (size_t)w * h);
            scharr(&lv[l], lv[l].dx, lv[l].dy);
        }
        levels = l;
        int nw = (w + 1) / 2, nh = (h + 1) / 2;
        if (nw <= win || nh <= win) break; /* buildOpticalFlowPyramid returns `level` here */
        w = nw; h = nh;
    }
    return levels;
}
static void free_pyramid(level_t* lv, int levels) {
    for (int l = 0; l <= levels; ++l) { free(lv[l].img); free(lv[l].dx); free(lv[l].dy); }
}

/* one LKTrackerInvoker step for point i at `level` (lkpyramid.cpp) */
static void lk_point(const level_t* I, const level_t* J, int level, int max_level, const float* prev_pt, float* next_pt,
                     uint8_t* status, float* err, int win, int max_iters, double eps2, float min_eig_thr,
                     int16_t* Iw, int16_t* dIw) {
    const float hw = (win - 1) * 0.5f;
    const int W_BITS = 14;
    const float FLT_SCALE = 1.f / (1 << 20);
    float sc = (float)(1. / (1 << level));
    float px = prev_pt[0] * sc, py = prev_pt[1] * sc;
    float nx, ny;
    if (level == max_level) { nx = px; ny = py; }
    else { nx = next_pt[0] * 2.f; ny = next_pt[1] * 2.f; }
    next_pt[0] = nx; next_pt[1] = ny;
    px -= hw; py -= hw;
    int ipx = (int)floorf(px), ipy = (int)floorf(py);
    if (ipx < -win || ipx >= I->w || ipy < -win || ipy >= I->h) {
        if (level == 0) { *status = 0; *err = 0; }
        return;
    }
    float a = px - ipx, b = py - ipy;
    int iw00 = (int)rintf((1.f - a) * (1.f - b) * (1 << W_BITS));
    int iw01 = (int)rintf(a * (1.f - b) * (1 << W_BITS));
    int iw10 = (int)rintf((1.f - a) * b * (1 << W_BITS));
    int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
    int64_t iA11 = 0, iA12 = 0, iA22 = 0;
    for (int y = 0; y < win; ++y)
        for (int x = 0; x < win; ++x) {
            int X = ipx + x, Y = ipy + y;
            int ival = DESCALE(img_at(I, X, Y) * iw00 + img_at(I, X + 1, Y) * iw01 + img_at(I, X, Y + 1) * iw10 +
                                   img_at(I, X + 1, Y + 1) * iw11, W_BITS - 5);
            int g00x, g00y, g01x, g01y, g10x, g10y, g11x, g11y;
            der_at(I, X, Y, &g00x, &g00y);
            der_at(I, X + 1, Y, &g01x, &g01y);
            der_at(I, X, Y + 1, &g10x, &g10y);
            der_at(I, X + 1, Y + 1, &g11x, &g11y);
            int ixv = DESCALE(g00x * iw00 + g01x * iw01 + g10x * iw10 + g11x * iw11, W_BITS);
            int iyv = DESCALE(g00y * iw00 + g01y * iw01 + g10y * iw10 + g11y * iw11, W_BITS);
            Iw[y * win + x] = (int16_t)ival;
            dIw[2 * (y * win + x)] = (int16_t)ixv;
            dIw[2 * (y * win + x) + 1] = (int16_t)iyv;
            iA11 += (int64_t)ixv * ixv;
            iA12 += (int64_t)ixv * iyv;
            iA22 += (int64_t)iyv * iyv;
        }
    float A11 = (float)iA11 * FLT_SCALE, A12 = (float)iA12 * FLT_SCALE, A22 = (float)iA22 * FLT_SCALE;
    float D = A11 * A22 - A12 * A12;
    float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
    if (minEig < min_eig_thr || D < FLT_EPSILON) {
        if (level == 0) *status = 0;
        return;
    }
    D = 1.f / D;
    nx -= hw; ny -= hw;
    float pdx = 0.f, pdy = 0.f;
    for (int j = 0; j < max_iters; ++j) {
        int inx = (int)floorf(nx), iny = (int)floorf(ny);
        if (inx < -win || inx >= J->w || iny < -win || iny >= J->h) {
            if (level == 0) *status = 0;
            break;
        }
        a = nx - inx; b = ny - iny;
        iw00 = (int)rintf((1.f - a) * (1.f - b) * (1 << W_BITS));
        iw01 = (int)rintf(a * (1.f - b) * (1 << W_BITS));
        iw10 = (int)rintf((1.f - a) * b * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        int64_t ib1 = 0, ib2 = 0;
        for (int y = 0; y < win; ++y)
            for (int x = 0; x < win; ++x) {
                int X = inx + x, Y = iny + y;
                int diff = DESCALE(img_at(J, X, Y) * iw00 + img_at(J, X + 1, Y) * iw01 + img_at(J, X, Y + 1) * iw10 +
                                       img_at(J, X + 1, Y + 1) * iw11, W_BITS - 5) - Iw[y * win + x];
                ib1 += (int64_t)diff * dIw[2 * (y * win + x)];
                ib2 += (int64_t)diff * dIw[2 * (y * win + x) + 1];
            }
        float b1 = (float)ib1 * FLT_SCALE, b2 = (float)ib2 * FLT_SCALE;
        float ddx = (A12 * b2 - A22 * b1) * D;
        float ddy = (A12 * b1 - A11 * b2) * D;
        nx += ddx; ny += ddy;
        next_pt[0] = nx + hw; next_pt[1] = ny + hw;
        if ((double)ddx * ddx + (double)ddy * ddy <= eps2) break;
        if (j > 0 && fabs((double)(ddx + pdx)) < 0.01 && fabs((double)(ddy + pdy)) < 0.01) {
            next_pt[0] -= ddx * 0.5f;
            next_pt[1] -= ddy * 0.5f;
            break;
        }
        pdx = ddx; pdy = ddy;
    }
    if (*status && level == 0) {
        float fx = next_pt[0] - hw, fy = next_pt[1] - hw;
        int ix = (int)floorf(fx), iy = (int)floorf(fy);
        if (ix < -win || ix >= J->w || iy < -win || iy >= J->h) {
            *status = 0;
            return;
        }
        float aa = fx - ix, bb = fy - iy;
        iw00 = (int)rintf((1.f - aa) * (1.f - bb) * (1 << W_BITS));
        iw01 = (int)rintf(aa * (1.f - bb) * (1 << W_BITS));
        iw10 = (int)rintf((1.f - aa) * bb * (1 << W_BITS));
        iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
        int64_t es = 0;
        for (int y = 0; y < win; ++y)
            for (int x = 0; x < win; ++x) {
                int X = ix + x, Y = iy + y;
                int diff = DESCALE(img_at(J, X, Y) * iw00 + img_at(J, X + 1, Y) * iw01 + img_at(J, X, Y + 1) * iw10 +
                                       img_at(J, X + 1, Y + 1) * iw11, W_BITS - 5) - Iw[y * win + x];
                es += diff < 0 ? -diff : diff;
            }
        *err = (float)es * (1.f / (32 * win * win));
    }
}

int oracle_klt_track(const uint8_t* prev, const uint8_t* curr, int W, int H, int stride, const float* pts, int n,
                     float* next, uint8_t* status, float* err, const erp_klt_params* p) {
    if (!prev || !curr || W <= 0 || H <= 0 || n < 0 || !p) return VIO_EINVAL;
    int win = p->win, max_level = p->max_level;
    int max_iters = p->max_iters < 0 ? 0 : (p->max_iters > 100 ? 100 : p->max_iters);
    double eps = p->epsilon < 0 ? 0 : (p->epsilon > 10 ? 10 : p->epsilon);
    double eps2 = eps * eps;
    level_t I[16], J[16];
    int lv = build_pyramid(prev, W, H, stride, win, max_level, 1, I);
    build_pyramid(curr, W, H, stride, win, max_level, 0, J);
    for (int i = 0; i < n; ++i) { status[i] = 1; err[i] = 0.f; }
    /* points are independent (LKTrackerInvoker is a parallel_for over them); per-thread window scratch */
    for (int level = lv; level >= 0; --level) {
#pragma omp parallel num_threads(oracle_get_threads()) if (oracle_get_threads() > 1)
        {
            int16_t* Iw = (int16_t*)malloc(sizeof(int16_t) * win * win);
            int16_t* dIw = (int16_t*)malloc(sizeof(int16_t) * 2 * win * win);
#pragma omp for schedule(dynamic, 4)
            for (int i = 0; i < n; ++i)
                lk_point(&I[level], &J[level], level, lv, pts + 2 * i, next + 2 * i, status + i, err + i, win,
                         max_iters, eps2, p->min_eig_threshold, Iw, dIw);
            free(Iw); free(dIw);
        }
    }
    free_pyramid(I, lv);
    free_pyramid(J, lv);
    return VIO_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* goodFeaturesToTrack                                                                         */

/* cornerMinEigenVal(blockSize 3, ksize 3) at every pixel -> eig (float, W*H) */
void oracle_min_eig_map(const uint8_t* img, int W, int H, int stride, float* eig) {
    const float scale = (float)(1.0 / 3060.0); /* 1 / (2^(3-1) * 3 * 255) */
    float* cov = (float*)malloc(sizeof(float) * 3 * (size_t)W * H);
#pragma omp parallel for num_threads(oracle_get_threads()) schedule(static) if (oracle_get_threads() > 1)
    for (int y = 0; y < H; ++y) {
        const uint8_t* r0 = img + (size_t)reflect101(y - 1, H) * stride;
        const uint8_t* r1 = img + (size_t)y * stride;
        const uint8_t* r2 = img + (size_t)reflect101(y + 1, H) * stride;
        for (int x = 0; x < W; ++x) {
            int xm = reflect101(x - 1, W), xp = reflect101(x + 1, W);
            int sx = (r0[xp] - r0[xm]) + 2 * (r1[xp] - r1[xm]) + (r2[xp] - r2[xm]);
            int sy = (r2[xm] + 2 * r2[x] + r2[xp]) - (r0[xm] + 2 * r0[x] + r0[xp]);
            float dx = (float)sx * scale, dy = (float)sy * scale;
            float* c = cov + 3 * ((size_t)y * W + x);
            c[0] = dx * dx; c[1] = dx * dy; c[2] = dy * dy;
        }
    }
#pragma omp parallel for num_threads(oracle_get_threads()) schedule(static) if (oracle_get_threads() > 1)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            double s0 = 0, s1 = 0, s2 = 0;
            for (int ky = -1; ky <= 1; ++ky) {
                int yy = reflect101(y + ky, H);
                for (int kx = -1; kx <= 1; ++kx) {
                    const float* c = cov + 3 * ((size_t)yy * W + reflect101(x + kx, W));
                    s0 += c[0]; s1 += c[1]; s2 += c[2];
                }
            }
            float a = (float)s0 * 0.5f, b = (float)s1, c = (float)s2 * 0.5f;
            eig[(size_t)y * W + x] = (a + c) - sqrtf((a - c) * (a - c) + b * b);
        }
    free(cov);
}

typedef struct { float v; int idx; } cand_t;
static int cand_cmp(const void* pa, const void* pb) { /* greaterThanPtr: value desc, then address desc */
    const cand_t* a = (const cand_t*)pa;
    const cand_t* b = (const cand_t*)pb;
    if (a->v > b->v) return -1;
    if (a->v < b->v) return 1;
    return (a->idx > b->idx) ? -1 : (a->idx < b->idx ? 1 : 0);
}

int oracle_gftt(const uint8_t* img, const uint8_t* mask, int W, int H, int stride, int max_corners, double quality,
                double min_dist, float* out_xy, int* n_out) {
    if (!img || W < 3 || H < 3 || !n_out || quality <= 0 || min_dist < 0 || max_corners < 0) return VIO_EINVAL;
    float* eig = (float*)malloc(sizeof(float) * (size_t)W * H);
    oracle_min_eig_map(img, W, H, stride, eig);
    double maxv = 0.0;
#pragma omp parallel for num_threads(oracle_get_threads()) schedule(static) reduction(max : maxv) if (oracle_get_threads() > 1)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            if (!mask || mask[(size_t)y * stride + x]) { double v = eig[(size_t)y * W + x]; if (v > maxv) maxv = v; }
    float thr = (float)(maxv * quality);
    for (size_t i = 0; i < (size_t)W * H; ++i)
        if (!(eig[i] > thr)) eig[i] = 0.f; /* THRESH_TOZERO */
    size_t cap = 1024, nc = 0;
    cand_t* cand = (cand_t*)malloc(sizeof(cand_t) * cap);
    for (int y = 1; y < H - 1; ++y)
        for (int x = 1; x < W - 1; ++x) {
            float v = eig[(size_t)y * W + x];
            if (v == 0.f) continue;
            if (mask && !mask[(size_t)y * stride + x]) continue;
            float m = v;
            for (int ky = -1; ky <= 1; ++ky)
                for (int kx = -1; kx <= 1; ++kx) { float u = eig[(size_t)(y + ky) * W + x + kx]; if (u > m) m = u; }
            if (v != m) continue;
            if (nc == cap) { cap *= 2; cand = (cand_t*)realloc(cand, sizeof(cand_t) * cap); }
            cand[nc].v = v; cand[nc].idx = y * W + x; nc++;
        }
    qsort(cand, nc, sizeof(cand_t), cand_cmp);
    int ncorners = 0;
    if (min_dist >= 1) {
        int cell = (int)lrint(min_dist);
        int gw = (W + cell - 1) / cell, gh = (H + cell - 1) / cell;
        int* head = (int*)malloc(sizeof(int) * gw * gh);
        for (int i = 0; i < gw * gh; ++i) head[i] = -1;
        int* nxt = (int*)malloc(sizeof(int) * (max_corners > 0 ? max_corners : (int)nc + 1));
        float* acc = (float*)malloc(sizeof(float) * 2 * (max_corners > 0 ? max_corners : (int)nc + 1));
        double md2 = min_dist * min_dist;
        for (size_t i = 0; i < nc; ++i) {
            int y = cand[i].idx / W, x = cand[i].idx % W;
            int xc = x / cell, yc = y / cell;
            int x1 = xc - 1 < 0 ? 0 : xc - 1, y1 = yc - 1 < 0 ? 0 : yc - 1;
            int x2 = xc + 1 > gw - 1 ? gw - 1 : xc + 1, y2 = yc + 1 > gh - 1 ? gh - 1 : yc + 1;
            int good = 1;
            for (int yy = y1; yy <= y2 && good; ++yy)
                for (int xx = x1; xx <= x2 && good; ++xx)
                    for (int j = head[yy * gw + xx]; j >= 0; j = nxt[j]) {
                        float ddx = (float)x - acc[2 * j], ddy = (float)y - acc[2 * j + 1];
                        if ((double)(ddx * ddx + ddy * ddy) < md2) { good = 0; break; }
                    }
            if (!good) continue;
            acc[2 * ncorners] = (float)x; acc[2 * ncorners + 1] = (float)y;
            /* grid lists are scanned completely, so insertion order within a cell is irrelevant */
            nxt[ncorners] = head[yc * gw + xc];
            head[yc * gw + xc] = ncorners;
            if (out_xy) { out_xy[2 * ncorners] = (float)x; out_xy[2 * ncorners + 1] = (float)y; }
            ncorners++;
            if (max_corners > 0 && ncorners == max_corners) break;
        }
        free(head); free(nxt); free(acc);
    } else {
        for (size_t i = 0; i < nc; ++i) {
            if (out_xy) { out_xy[2 * ncorners] = (float)(cand[i].idx % W); out_xy[2 * ncorners + 1] = (float)(cand[i].idx / W); }
            ncorners++;
            if (max_corners > 0 && ncorners == max_corners) break;
        }
    }
    *n_out = ncorners;
    free(cand);
    free(eig);
    return VIO_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* rotation-only RANSAC on ERP bearings                                                        */

/* Camera::PixelToBearing (Camera.cpp:22-47): f32 lon/lat as the reference forms them, double trig
   rounded to float, Eigen normalize() */
void oracle_pixel_to_bearing(float u, float v, int W, int H, float* b) {
    float un = u / (float)W, vn = v / (float)H;
    float lon = (float)((double)((un - 0.5f) * 2.0f) * M_PI);
    float lat = (float)((double)(-(vn - 0.5f)) * M_PI);
    float cl = (float)cos((double)lat), sl = (float)sin((double)lat);
    float so = (float)sin((double)lon), co = (float)cos((double)lon);
    float x = cl * so, y = -sl, z = cl * co;
    float sq = (x * x + y * y) + z * z;
    if (sq > 0.f) {
        float nr = sqrtf(sq);
        x /= nr; y /= nr; z /= nr;
    }
    b[0] = x; b[1] = y; b[2] = z;
}

/* nearest rotation (Kabsch, det fixed on the smallest singular direction) of a float 3x3, computed
   in double by a fixed-sweep Jacobi eigen-solver of H^T H, rounded to float */
static void jacobi3(double* A, double* V) {
    for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 12; ++sweep) {
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double apq = A[3 * p + q];
                if (apq == 0.0) continue;
                double app = A[3 * p + p], aqq = A[3 * q + q];
                double theta = (aqq - app) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) {
                    double akp = A[3 * k + p], akq = A[3 * k + q];
                    A[3 * k + p] = c * akp - s * akq;
                    A[3 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    double apk = A[3 * p + k], aqk = A[3 * q + k];
                    A[3 * p + k] = c * apk - s * aqk;
                    A[3 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    double vkp = V[3 * k + p], vkq = V[3 * k + q];
                    V[3 * k + p] = c * vkp - s * vkq;
                    V[3 * k + q] = s * vkp + c * vkq;
                }
            }
    }
}

void oracle_kabsch_rotation(const float* Hf, float* Rf) {
    double H[9], HtH[9], V[9];
    for (int i = 0; i < 9; ++i) H[i] = Hf[i];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) HtH[3 * i + j] = H[i] * H[j] + H[3 + i] * H[3 + j] + H[6 + i] * H[6 + j];
    jacobi3(HtH, V);
    double w[3] = {HtH[0], HtH[4], HtH[8]};
    int idx[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (w[idx[j]] > w[idx[i]]) { int t = idx[i]; idx[i] = idx[j]; idx[j] = t; }
    double v[3][3], u[3][3];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) v[c][r] = V[3 * r + idx[c]];
    for (int c = 0; c < 2; ++c) {
        for (int r = 0; r < 3; ++r) u[c][r] = H[3 * r] * v[c][0] + H[3 * r + 1] * v[c][1] + H[3 * r + 2] * v[c][2];
        double nn = sqrt(u[c][0] * u[c][0] + u[c][1] * u[c][1] + u[c][2] * u[c][2]);
        if (nn > 0) { u[c][0] /= nn; u[c][1] /= nn; u[c][2] /= nn; }
    }
    double d01 = u[0][0] * u[1][0] + u[0][1] * u[1][1] + u[0][2] * u[1][2];
    for (int r = 0; r < 3; ++r) u[1][r] -= d01 * u[0][r];
    double n1 = sqrt(u[1][0] * u[1][0] + u[1][1] * u[1][1] + u[1][2] * u[1][2]);
    if (n1 > 0) { u[1][0] /= n1; u[1][1] /= n1; u[1][2] /= n1; }
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    double dV = v[0][0] * (v[1][1] * v[2][2] - v[1][2] * v[2][1]) - v[1][0] * (v[0][1] * v[2][2] - v[0][2] * v[2][1]) +
                v[2][0] * (v[0][1] * v[1][2] - v[0][2] * v[1][1]);
    double d = dV < 0 ? -1.0 : 1.0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Rf[3 * r + c] = (float)(u[0][r] * v[0][c] + u[1][r] * v[1][c] + d * u[2][r] * v[2][c]);
}

static float det3f(const float* m) { /* Eigen 3x3 cofactor determinant */
    return m[0] * (m[4] * m[8] - m[7] * m[5]) - m[3] * (m[1] * m[8] - m[7] * m[2]) + m[6] * (m[1] * m[5] - m[4] * m[2]);
}

int oracle_rot_ransac(const float* p0, const float* p1, int n, int W, int H, const int32_t* samples, int iters,
                      float thresh_rad, uint8_t* mask, int* n_in) {
    if (n < 0 || !mask || !n_in) return VIO_EINVAL;
    if (n < 3) {
        for (int i = 0; i < n; ++i) mask[i] = 1;
        *n_in = n;
        return VIO_OK;
    }
    float* b0 = (float*)malloc(sizeof(float) * 3 * n);
    float* b1 = (float*)malloc(sizeof(float) * 3 * n);
    for (int i = 0; i < n; ++i) {
        oracle_pixel_to_bearing(p0[2 * i], p0[2 * i + 1], W, H, b0 + 3 * i);
        oracle_pixel_to_bearing(p1[2 * i], p1[2 * i + 1], W, H, b1 + 3 * i);
    }
    int best = 0, best_it = -1;
    uint8_t* cur = (uint8_t*)malloc(n);
    for (int it = 0; it < iters; ++it) {
        float Hm[9] = {0};
        for (int s = 0; s < 3; ++s) {
            int k = samples[3 * it + s];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) Hm[3 * r + c] += b1[3 * k + r] * b0[3 * k + c];
        }
        float R[9];
        oracle_kabsch_rotation(Hm, R);
        if (fabsf(det3f(R) - 1.0f) > 0.1f) continue;
        int cnt = 0;
        for (int i = 0; i < n; ++i) {
            const float* a = b0 + 3 * i;
            float r0 = (R[0] * a[0] + R[1] * a[1]) + R[2] * a[2];
            float r1 = (R[3] * a[0] + R[4] * a[1]) + R[5] * a[2];
            float r2 = (R[6] * a[0] + R[7] * a[1]) + R[8] * a[2];
            const float* q = b1 + 3 * i;
            float c = (r0 * q[0] + r1 * q[1]) + r2 * q[2];
            c = c < -1.f ? -1.f : (c > 1.f ? 1.f : c);
            float ang = (float)acos((double)c);
            cur[i] = ang < thresh_rad;
            cnt += cur[i];
        }
        if (cnt > best) {
            best = cnt;
            best_it = it;
            memcpy(mask, cur, n);
        }
    }
    if (best_it < 0) for (int i = 0; i < n; ++i) mask[i] = 1;
    *n_in = best;
    free(cur); free(b0); free(b1);
    return VIO_OK;
}
