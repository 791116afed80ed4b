// tracker.hip — ERP feature tracking on MI355X (gfx950): the numeric path of
// FeatureTracker::TrackFeatures (src/processing/FeatureTracker.cpp:61-379).
//
//   pyr_down_kernel      cv::pyrDown inside buildOpticalFlowPyramid: 5x5 [1 4 6 4 1]^2/256,
//                        BORDER_REFLECT_101; both frames of a pair in one launch (blockIdx.z).
//   lk_kernel            cv::calcOpticalFlowPyrLK's LKTrackerInvoker, one wavefront per point,
//                        all pyramid levels in one launch; the Scharr derivatives of the previous
//                        frame are computed on the fly from an LDS-staged 24x24 tile (never
//                        materialised for the whole image), the 21x21 patch, its derivatives and
//                        every 22x22 next-frame tile live in LDS; gradient/mismatch sums are exact
//                        int64 wave reductions.
//   ransac_*             RejectOutliersRotationRANSAC: one wavefront per hypothesis.
//   gftt_*               cv::goodFeaturesToTrack(blockSize 3, Sobel 3): pass 1 computes the
//                        min-eigenvalue map on LDS tiles (Sobel, 3x3 box, eigenvalue), writes it
//                        (f32, W x H) and reduces its masked maximum; pass 2 reads a haloed tile of
//                        the map back, applies THRESH_TOZERO + 3x3 dilate NMS + mask and appends
//                        (response, address) keys; a top-K histogram cut, a sort and one
//                        workgroup's greedy min-distance pass finish.  (Recomputing the map in
//                        pass 2 cost more than its 2 x 4 B/px round trip through HBM / MALL.)
// Float expressions follow tracker_oracle.c literally and the file is built with
// -ffp-contract=off, so results are bitwise those of the oracle.
#include <float.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <hipcub/hipcub.hpp>

#include "tracker_types.h"

namespace vio360 {

// LDS writes of this wave visible to its own later reads (no workgroup barrier)
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Tile of linear block b of an n-block grid such that each XCD works on one contiguous range of tiles:
// blocks b and b + 8 share an XCD (round-robin dispatch, MI355X_MICROARCH.md "Workgroup dispatch"), so
// neighbouring tiles read their shared halo lines through one L2 instead of fetching them once per XCD
// (speed only: any placement gives the same results)
__device__ __forceinline__ int xcd_tile(int b, int n) {
    const int x = b & 7, s = b >> 3, q = n >> 3, r = n & 7;
    return x < r ? x * (q + 1) + s : r * (q + 1) + (x - r) * q + s;
}

__device__ __forceinline__ int reflect101(int p, int n) {
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

__device__ __forceinline__ bool lm_static_in(const GfArgs& G, int x, int y) {
    return y >= G.top_rows && y < G.bottom_start && x >= G.margin && x < G.W - G.margin;
}
__device__ __forceinline__ bool lm_disc(const GfArgs& G, int x, int y) {
    return G.disc_bits && ((G.disc_bits[(size_t)y * G.disc_words + (x >> 5)] >> (x & 31)) & 1u);
}

// ------------------------------------------------------------------------------------------
// pyrDown.  Block = 64 x BY outputs; LDS tile of the (2*BY+4) REFLECT_101 source rows, columns
// [2 ox - 16, 2 ox + 144), staged with 16-B loads (all of a thread's loads issued before its LDS stores; the
// few reflected columns at the left / right image edge are patched bytewise); each thread makes two adjacent
// outputs in BY / 8 rows.  BY = 8 (BY = 32 for the large levels -- a quarter of the blocks and of the halo
// rows, the 3840 x 1920 level-1 launch in one round of resident workgroups -- measured 15.0 against 13.2 us,
// profiles/r6c_ab_pyr.log).
constexpr int PD_BX = 64;
constexpr int PD_TW = 160;
template <int BY>
__global__ void __launch_bounds__(256) pyr_down_kernel(PyrLevelPair src, PyrLevelPair dst) {
    constexpr int PD_BY = BY, PD_TH = 2 * PD_BY + 4;
    __shared__ uint8_t tile[PD_TH][PD_TW];
    const int gxy = gridDim.x * gridDim.y;
    const int t = xcd_tile(blockIdx.x + gridDim.x * blockIdx.y + gxy * blockIdx.z, gxy * gridDim.z);
    const int f = t / gxy, bxy = t - f * gxy, bx = bxy % gridDim.x, by = bxy / gridDim.x;
    const uint8_t* s = f == 0 ? src.p0 : src.p1;
    uint8_t* d = f == 0 ? dst.p0 : dst.p1;
    const int sw = src.w, sh = src.h, sp = src.pitch;
    const int dw = dst.w, dh = dst.h, dp = dst.pitch;
    const int ox = bx * PD_BX, oy = by * PD_BY;
    const int cx0 = 2 * ox - 16, sy0 = 2 * oy - 2;  // tile column 0 = source x cx0
    {  // 16-B chunks of the REFLECT_101 rows; chunks beyond the pitch are skipped
        constexpr int NCH = PD_TH * (PD_TW / 16);
        uint4 v[(NCH + 255) / 256];
#pragma unroll
        for (int it = 0; it < (NCH + 255) / 256; ++it) {
            const int e = threadIdx.x + 256 * it;
            const int x0 = cx0 + 16 * (e % (PD_TW / 16));
            v[it] = make_uint4(0u, 0u, 0u, 0u);
            if (e < NCH && x0 >= 0 && x0 + 16 <= sp)
                v[it] = *reinterpret_cast<const uint4*>(s + (size_t)reflect101(sy0 + e / (PD_TW / 16), sh) * sp + x0);
        }
#pragma unroll
        for (int it = 0; it < (NCH + 255) / 256; ++it) {
            const int e = threadIdx.x + 256 * it;
            const int x0 = cx0 + 16 * (e % (PD_TW / 16));
            if (e < NCH && x0 >= 0 && x0 + 16 <= sp)
                *reinterpret_cast<uint4*>(&tile[e / (PD_TW / 16)][16 * (e % (PD_TW / 16))]) = v[it];
        }
    }
    if (2 * ox - 2 < 0 || 2 * ox + 2 * PD_BX + 2 > sw) {  // left / right image edge: reflected columns
        __syncthreads();
        for (int e = threadIdx.x; e < PD_TH * (2 * PD_BX + 4); e += 256) {
            const int ty = e / (2 * PD_BX + 4), x = 2 * ox - 2 + e % (2 * PD_BX + 4);
            if (x < 0 || x >= sw) tile[ty][x - cx0] = s[(size_t)reflect101(sy0 + ty, sh) * sp + reflect101(x, sw)];
        }
    }
    __syncthreads();
    const int q = threadIdx.x % (PD_BX / 2);  // outputs 2q, 2q+1 of rows ty0 + 8 r
#pragma unroll
    for (int rr = 0; rr < PD_BY / 8; ++rr) {
        const int ty = threadIdx.x / (PD_BX / 2) + 8 * rr;
        const int y = oy + ty;
        if (y >= dh) break;
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int tx = 2 * q + j;
            int tot = 0;
#pragma unroll
            for (int ky = 0; ky < 5; ++ky) {
                const uint8_t* r = &tile[2 * ty + ky][2 * tx + 14];
                const int rs = r[0] + 4 * r[1] + 6 * r[2] + 4 * r[3] + r[4];
                tot += (ky == 0 || ky == 4 ? 1 : (ky == 2 ? 6 : 4)) * rs;
            }
            packed |= (uint32_t)((tot + 128) >> 8) << (8 * j);
        }
        const int x = ox + 2 * q;
        if (x + 1 < dw && ((dp & 1) == 0)) {
            *reinterpret_cast<uint16_t*>(d + (size_t)y * dp + x) = (uint16_t)packed;
        } else {
            for (int j = 0; j < 2; ++j)
                if (x + j < dw) d[(size_t)y * dp + x + j] = (uint8_t)(packed >> (8 * j));
        }
    }
}

// ------------------------------------------------------------------------------------------
// LK.  One workgroup per point.
constexpr int LK_WAVES = 4;  // one point per workgroup of LK_WAVES waves
constexpr int LK_THREADS = 64 * LK_WAVES;
constexpr int LK_WIN_MAX = 21;
constexpr int LK_NIT = (LK_WIN_MAX * LK_WIN_MAX + LK_THREADS - 1) / LK_THREADS;  // patch pixels per lane
constexpr int LK_T = LK_WIN_MAX + 3;  // prev tile (patch + 1 bilinear + 1 Scharr each side)
constexpr int LK_D = LK_WIN_MAX + 1;  // derivative / next tile

constexpr int LK_MARGIN = 8;                 // staged next-frame region: the window +- 8 px
constexpr int LK_R = LK_D + 2 * LK_MARGIN;

struct LkShared {
    uint8_t Jr[LK_R * LK_R];                 // next-frame region (reflect-101 values), origin (rx0, ry0)
    uint8_t It[LK_T * LK_T];
    int16_t dx[LK_D * LK_D], dy[LK_D * LK_D];
};

// Wave sum of integer partials, exact while |sum| < 2^53: the partials are summed as doubles
// (integer-valued, so every order gives the same exact value) with DPP row reductions (xor 1, xor 2,
// half-row mirror, row mirror: VALU lane moves, no LDS crossbar) and the four row totals read out.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_d(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

__device__ __forceinline__ void lk_weights(float a, float b, int& w00, int& w01, int& w10, int& w11) {
    w00 = (int)rintf((1.f - a) * (1.f - b) * 16384.f);
    w01 = (int)rintf(a * (1.f - b) * 16384.f);
    w10 = (int)rintf((1.f - a) * b * 16384.f);
    w11 = 16384 - w00 - w01 - w10;
}

// workgroup sum of integer partials (exact: each wave's partials summed as doubles with DPP row
// reductions and the four row totals read out, then the LK_WAVES wave totals
// added in wave order through LDS); every thread gets the total.  red: LK_WAVES doubles of LDS.
__device__ __forceinline__ long long wg_sum_i64(long long v, double* red) {
    double d = (double)v;
    d += dpp_d<0xB1>(d);
    d += dpp_d<0x4E>(d);
    d += dpp_d<0x141>(d);
    d += dpp_d<0x140>(d);
    const double ws = ((lane_d(d, 0) + lane_d(d, 16)) + lane_d(d, 32)) + lane_d(d, 48);
    const int wid = threadIdx.x >> 6;
    __syncthreads();  // red is free (the previous sum's readers are done)
    if ((threadIdx.x & 63) == 0) red[wid] = ws;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < LK_WAVES; ++q) t += red[q];
    return (long long)t;
}

// make the staged region cover the (win+1)^2 window at (ix, iy); restage around it when it does
// not (one global round trip per level instead of one per iteration).  Values are the
// REFLECT_101-padded pixels, exactly what a per-window load would read.  Workgroup-uniform.
__device__ __forceinline__ void lk_region(uint8_t* Jr, int& rx0, int& ry0, const uint8_t* J, int w, int h, int pitch,
                                          int ix, int iy, int win) {
    const int D = win + 1;
    if (ix >= rx0 && iy >= ry0 && ix + D <= rx0 + LK_R && iy + D <= ry0 + LK_R) return;
    rx0 = ix - LK_MARGIN;
    ry0 = iy - LK_MARGIN;
    __syncthreads();  // the previous region's readers are done
    // every global load of the region is issued before the first LDS store
    constexpr int NR = (LK_R * LK_R + LK_THREADS - 1) / LK_THREADS;
    uint32_t v[NR];
#pragma unroll
    for (int it = 0; it < NR; ++it) {
        const int e = threadIdx.x + LK_THREADS * it;
        const int ty = e / LK_R, tx = e - ty * LK_R;
        v[it] = e < LK_R * LK_R ? J[(size_t)reflect101(ry0 + ty, h) * pitch + reflect101(rx0 + tx, w)] : 0u;
    }
#pragma unroll
    for (int it = 0; it < NR; ++it) {
        const int e = threadIdx.x + LK_THREADS * it;
        if (e < LK_R * LK_R) Jr[e] = (uint8_t)v[it];
    }
    __syncthreads();
}

// calcOpticalFlowPyrLK for one point per workgroup (LK_WAVES waves): the patch pixels are spread over
// all lanes (<= LK_NIT each), the window sums are exact integer workgroup sums, so every order gives
// the sequential values; the per-iteration update is computed by every thread from the same totals.
template <int NT>
__device__ void ransac_raw_body(uint32_t seed, uint32_t* raw, uint32_t* mt);  // (RANSAC section)
__device__ float ransac_cos_bound(float thr);
__device__ void pixel_to_bearing(float u, float v, int W, int H, float* b);
constexpr int LK_AUX_BLOCKS = 17;  // LkAux: one workgroup for the raw draws, 16 for the reset and the bitmap clear
__device__ void lk_aux(const LkAux& X, int b) {
    if (b == 0) {
        __shared__ uint32_t mt[624];
        if (X.raw) ransac_raw_body<LK_THREADS>(X.seed, X.raw, mt);
        if (X.cmin && threadIdx.x == 0) *X.cmin = ransac_cos_bound(X.thresh);
        return;
    }
    const size_t t = (size_t)(b - 1) * LK_THREADS + threadIdx.x, stride = (size_t)(LK_AUX_BLOCKS - 1) * LK_THREADS;
    if (X.hist) {  // gftt_reset_kernel's work
        if (t == 0) {
            X.scal[2] = X.scal[3] = X.scal[4] = 0;
            X.scal[6] = X.scal[7] = X.scal[8] = X.scal[9] = 0;
            X.scal[10] = X.scal[11] = 0;
        }
        for (size_t i = t; i < (size_t)GF_BUCKETS; i += stride) X.hist[i] = 0u;
        for (size_t i = t; i < X.topk_cap; i += stride) X.topk[i] = 0ull;
    }
    if (X.bear0)
        for (size_t i = t; i < (size_t)X.n; i += stride)
            pixel_to_bearing(X.pts[2 * i], X.pts[2 * i + 1], X.W, X.H, X.bear0 + 3 * i);
    if (X.disc) {
        const size_t n4 = X.disc_words / 4;
        uint4* d4p = reinterpret_cast<uint4*>(X.disc);
        for (size_t i = t; i < n4; i += stride) d4p[i] = make_uint4(0u, 0u, 0u, 0u);
        for (size_t i = 4 * n4 + t; i < X.disc_words; i += stride) X.disc[i] = 0u;
    }
}

__global__ void __launch_bounds__(LK_THREADS) lk_kernel(LkArgs A, LkAux X) {
    __shared__ LkShared S;
    __shared__ double red[LK_WAVES];
    const int tid = threadIdx.x;
    const int pt = blockIdx.x;
    if (pt >= A.n) {  // whole workgroup
        lk_aux(X, pt - A.n);
        return;
    }
    const int win = A.win;
    const float hw = (win - 1) * 0.5f;
    const float FLT_SCALE = 1.f / (1 << 20);
    const int np = win * win;
    float prev_x = A.pts[2 * pt], prev_y = A.pts[2 * pt + 1];
    float nxt_x = 0.f, nxt_y = 0.f;
    int status = 1;
    float err = 0.f;
    for (int level = A.levels; level >= 0; --level) {
        const LkLevel& Lv = A.lv[level];
        const int w = Lv.w, h = Lv.h;
        const uint8_t* I = Lv.prev;
        const uint8_t* J = Lv.curr;
        const float sc = (float)(1. / (1 << level));
        float px = prev_x * sc, py = prev_y * sc;
        float nx, ny;
        if (level == A.levels) { nx = px; ny = py; }
        else { nx = nxt_x * 2.f; ny = nxt_y * 2.f; }
        nxt_x = nx; nxt_y = ny;
        px -= hw; py -= hw;
        const int ipx = (int)floorf(px), ipy = (int)floorf(py);
        if (ipx < -win || ipx >= w || ipy < -win || ipy >= h) {
            if (level == 0) { status = 0; err = 0.f; }
            continue;
        }
        // stage the prev tile: rows ipy-1 .. ipy+win+1, cols ipx-1 .. ipx+win+1
        const int T = win + 3;
        __syncthreads();  // the previous level's readers of It / dx / dy are done
        {
            constexpr int NT = (LK_T * LK_T + LK_THREADS - 1) / LK_THREADS;  // loads first, then the LDS stores
            uint32_t v[NT];
#pragma unroll
            for (int it = 0; it < NT; ++it) {
                const int e = tid + LK_THREADS * it;
                const int ty = e / T, tx = e - (e / T) * T;
                v[it] = e < T * T ? I[(size_t)reflect101(ipy - 1 + ty, h) * Lv.pitch + reflect101(ipx - 1 + tx, w)] : 0u;
            }
#pragma unroll
            for (int it = 0; it < NT; ++it) {
                const int e = tid + LK_THREADS * it;
                if (e < T * T) S.It[e] = (uint8_t)v[it];
            }
        }
        __syncthreads();
        // Scharr derivatives at (ipx+tx, ipy+ty), tx,ty in [0, win]; zero outside the image
        const int D = win + 1;
        for (int e = tid; e < D * D; e += LK_THREADS) {
            int ty = e / D, tx = e % D;
            int X = ipx + tx, Y = ipy + ty;
            int gx = 0, gy = 0;
            if (X >= 0 && Y >= 0 && X < w && Y < h) {
                const uint8_t* r0 = &S.It[ty * T + tx];      // (X-1, Y-1)
                const uint8_t* r1 = r0 + T;
                const uint8_t* r2 = r1 + T;
                int t0m = (r0[0] + r2[0]) * 3 + r1[0] * 10, t0p = (r0[2] + r2[2]) * 3 + r1[2] * 10;
                int t1m = r2[0] - r0[0], t1c = r2[1] - r0[1], t1p = r2[2] - r0[2];
                gx = (int16_t)(t0p - t0m);
                gy = (int16_t)((t1p + t1m) * 3 + t1c * 10);
            }
            S.dx[e] = (int16_t)gx;
            S.dy[e] = (int16_t)gy;
        }
        __syncthreads();
        float a = px - ipx, b = py - ipy;
        int w00, w01, w10, w11;
        lk_weights(a, b, w00, w01, w10, w11);
        // the lane's patch pixels e = tid + LK_THREADS it: interpolated I and derivatives stay in registers
        // for all iterations of the level; joff = offset of the pixel in the next-frame window (-1: none)
        int joff[LK_NIT], iwv[LK_NIT], ixr[LK_NIT], iyr[LK_NIT];
        int sA11 = 0, sA12 = 0, sA22 = 0;
#pragma unroll
        for (int it = 0; it < LK_NIT; ++it) {
            const int e = tid + LK_THREADS * it;
            joff[it] = -1;
            iwv[it] = ixr[it] = iyr[it] = 0;
            if (e < np) {
                const int y = e / win, x = e - (e / win) * win;
                const uint8_t* t = &S.It[(y + 1) * T + x + 1];
                const int ival = DESCALE(t[0] * w00 + t[1] * w01 + t[T] * w10 + t[T + 1] * w11, 9);
                const int q = y * D + x;
                const int ixv =
                    DESCALE(S.dx[q] * w00 + S.dx[q + 1] * w01 + S.dx[q + D] * w10 + S.dx[q + D + 1] * w11, 14);
                const int iyv =
                    DESCALE(S.dy[q] * w00 + S.dy[q + 1] * w01 + S.dy[q + D] * w10 + S.dy[q + D + 1] * w11, 14);
                iwv[it] = (int16_t)ival;
                ixr[it] = (int16_t)ixv;
                iyr[it] = (int16_t)iyv;
                joff[it] = y * LK_R + x;
                sA11 += ixv * ixv;
                sA12 += ixv * iyv;
                sA22 += iyv * iyv;
            }
        }
        const long long tA11 = wg_sum_i64(sA11, red), tA12 = wg_sum_i64(sA12, red), tA22 = wg_sum_i64(sA22, red);
        const float A11 = (float)tA11 * FLT_SCALE, A12 = (float)tA12 * FLT_SCALE, A22 = (float)tA22 * FLT_SCALE;
        float Dt = A11 * A22 - A12 * A12;
        const float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
        if (minEig < A.min_eig || Dt < FLT_EPSILON) {
            if (level == 0) status = 0;
            continue;
        }
        Dt = 1.f / Dt;
        nx -= hw; ny -= hw;
        float pdx = 0.f, pdy = 0.f;
        int rx0 = -(1 << 29), ry0 = -(1 << 29);  // no region staged for this level yet
        for (int j = 0; j < A.max_iters; ++j) {
            const int inx = (int)floorf(nx), iny = (int)floorf(ny);
            if (inx < -win || inx >= w || iny < -win || iny >= h) {
                if (level == 0) status = 0;
                break;
            }
            a = nx - inx; b = ny - iny;
            lk_weights(a, b, w00, w01, w10, w11);
            lk_region(S.Jr, rx0, ry0, J, w, h, Lv.pitch, inx, iny, win);
            const uint8_t* Jw = S.Jr + (iny - ry0) * LK_R + (inx - rx0);
            int ib1 = 0, ib2 = 0;
#pragma unroll
            for (int it = 0; it < LK_NIT; ++it) {
                if (joff[it] >= 0) {
                    const uint8_t* t = Jw + joff[it];
                    const int diff = DESCALE(t[0] * w00 + t[1] * w01 + t[LK_R] * w10 + t[LK_R + 1] * w11, 9) - iwv[it];
                    ib1 += diff * ixr[it];
                    ib2 += diff * iyr[it];
                }
            }
            const float b1 = (float)wg_sum_i64(ib1, red) * FLT_SCALE, b2 = (float)wg_sum_i64(ib2, red) * FLT_SCALE;
            const float ddx = (A12 * b2 - A22 * b1) * Dt;
            const float ddy = (A12 * b1 - A11 * b2) * Dt;
            nx += ddx; ny += ddy;
            nxt_x = nx + hw; nxt_y = ny + hw;
            if ((double)ddx * ddx + (double)ddy * ddy <= A.eps2) break;
            if (j > 0 && fabs((double)(ddx + pdx)) < 0.01 && fabs((double)(ddy + pdy)) < 0.01) {
                nxt_x -= ddx * 0.5f;
                nxt_y -= ddy * 0.5f;
                break;
            }
            pdx = ddx; pdy = ddy;
        }
        if (status && level == 0) {
            const float fx = nxt_x - hw, fy = nxt_y - hw;
            const int ix = (int)floorf(fx), iy = (int)floorf(fy);
            if (ix < -win || ix >= w || iy < -win || iy >= h) {
                status = 0;
            } else {
                lk_weights(fx - ix, fy - iy, w00, w01, w10, w11);
                lk_region(S.Jr, rx0, ry0, J, w, h, Lv.pitch, ix, iy, win);
                const uint8_t* Jw = S.Jr + (iy - ry0) * LK_R + (ix - rx0);
                long long es = 0;
#pragma unroll
                for (int it = 0; it < LK_NIT; ++it) {
                    if (joff[it] >= 0) {
                        const uint8_t* t = Jw + joff[it];
                        const int diff =
                            DESCALE(t[0] * w00 + t[1] * w01 + t[LK_R] * w10 + t[LK_R + 1] * w11, 9) - iwv[it];
                        es += diff < 0 ? -diff : diff;
                    }
                }
                es = wg_sum_i64(es, red);
                err = (float)es * (1.f / (32 * win * win));
            }
        }
    }
    if (tid == 0) {
        A.next[2 * pt] = nxt_x;
        A.next[2 * pt + 1] = nxt_y;
        A.status[pt] = (uint8_t)status;
        A.err[pt] = err;
    }
    // the tracked point's bearing (RANSAC's input, FeatureTracker.cpp:262-271) by another wave, beside the stores
    if (A.bear1 && tid == 64) pixel_to_bearing(nxt_x, nxt_y, A.lv[0].w, A.lv[0].h, A.bear1 + 3 * pt);
}

// ------------------------------------------------------------------------------------------
// bearings / filter / RANSAC
__device__ void pixel_to_bearing(float u, float v, int W, int H, float* b) {
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

// order-preserving compaction of the RANSAC input (single workgroup of RP_THREADS: four waves get a CU
// sooner than sixteen while GFTT pass 1 occupies the chip from the side stream):
//   mode 0: all n points (erp_rot_ransac); mode 1: status ∧ !polar ∧ !boundary (pipeline)
constexpr int RP_THREADS = 256;
template <int NT>
__device__ int ransac_prep_body(const RansacArgs& R, int* wsum, int& base) {
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    const int n = R.n;
    for (int c0 = 0; c0 < n; c0 += NT) {
        int i = c0 + threadIdx.x;
        int good = 0;
        if (i < n) {
            if (R.mode == 0) good = 1;
            else {
                float x = R.p1[2 * i], y = R.p1[2 * i + 1];
                float vr = y / (float)R.H;
                bool polar = (vr < R.polar_ratio) || (vr > (1.0f - R.polar_ratio));
                float m = (float)R.margin;
                bool nearb = (x < m) || (x > (float)R.W - m) || (y < m) || (y > (float)R.H - m);
                good = R.status[i] && !polar && !nearb;
            }
            R.kept[i] = 0;
        }
        unsigned long long bal = __ballot(good);
        int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        int pre = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wid] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int k = 0; k < wid; ++k) off += wsum[k];
        if (good) {
            int j = off + pre;
            R.gidx[j] = i;
            if (R.bear0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    R.b0[3 * j + c] = R.bear0[3 * i + c];
                    R.b1[3 * j + c] = R.bear1[3 * i + c];
                }
            } else {
                pixel_to_bearing(R.p0[2 * i], R.p0[2 * i + 1], R.W, R.H, R.b0 + 3 * j);
                pixel_to_bearing(R.p1[2 * i], R.p1[2 * i + 1], R.W, R.H, R.b1 + 3 * j);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int t = 0;
            for (int k = 0; k < NT / 64; ++k) t += wsum[k];
            base += t;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *R.n_good = base;
    return base;
}
// The inlier test (float)acos((double)c) < thr (FeatureTracker.cpp:365-375 + Camera::AngularDistance, Camera.cpp:89-98,
// in the oracle's form) is
// monotone non-increasing in the float cosine c, so it is c >= c_min for the smallest float c in [-1, 1] that
// passes it: found once per run by bisection over the floats' order (31 evaluations of the same acos), every
// hypothesis' inlier count is then a compare per point instead of a double acos.  (Adjacent floats near the
// crossing differ in acos by ~1e-6, far above the double evaluation's error: the two tests agree bit for bit.)
// +inf when no cosine passes (an empty inlier set: no c >= +inf; NaN compares false in both forms).
__device__ float ransac_cos_bound(float thr) {
    auto pass = [&](float c) { return (float)acos((double)c) < thr; };
    auto ord = [](float x) {
        const uint32_t b = __float_as_uint(x);
        return (b >> 31) ? ~b : (b | 0x80000000u);
    };
    auto unord = [](uint32_t m) { return __uint_as_float((m >> 31) ? (m & 0x7fffffffu) : ~m); };
    if (!pass(1.0f)) return INFINITY;
    uint32_t lo = ord(-1.0f), hi = ord(1.0f);  // pass(unord(hi)) holds throughout
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (pass(unord(mid))) hi = mid;
        else lo = mid + 1;
    }
    return unord(hi);
}

__global__ void __launch_bounds__(RP_THREADS) ransac_prep_kernel(RansacArgs R) {
    __shared__ int wsum[RP_THREADS / 64];
    __shared__ int base;
    ransac_prep_body<RP_THREADS>(R, wsum, base);
    if (threadIdx.x == 0) *R.cmin = ransac_cos_bound(R.thresh);
}

// mt19937 + libstdc++-11 uniform_int_distribution (Lemire) — the reference's sampler
// (FeatureTracker.cpp:273-288) with an injected seed; one thread (the stream is sequential).
struct Mt19937 {
    uint32_t mt[624];
    int idx;
    __device__ void seed(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        idx = 624;
    }
    __device__ uint32_t next() {
        if (idx >= 624) {
            for (int i = 0; i < 624; ++i) {
                uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
};
__device__ uint32_t uniform_below(Mt19937& g, uint32_t range) {  // uniform in [0, range)
    uint64_t prod = (uint64_t)g.next() * range;
    uint32_t low = (uint32_t)prod;
    if (low < range) {
        uint32_t thr = (uint32_t)(-range) % range;
        while (low < thr) {
            prod = (uint64_t)g.next() * range;
            low = (uint32_t)prod;
        }
    }
    return (uint32_t)(prod >> 32);
}

// Parallel form of the same stream (one workgroup): the raw mt19937 words of RS_BLOCKS state
// blocks are generated by a three-phase parallel twist (i in [0,227) reads only old words;
// [227,454) and [454,624) read words that the previous phase produced) and tempered in parallel;
// uniform_int_distribution's rejection test depends on a word alone, so accepted draws are a
// prefix-scan compaction; a hypothesis consumes draws until it holds 3 distinct indices, and the
// hypothesis chain is followed one wave at a time, 64 hypotheses per step while each consumes
// exactly 3 draws (the common case).  Bitwise the sequential sampler; if the generated stream runs
// out (tiny n: many duplicate redraws) the sequential sampler runs instead.
constexpr int RS_THREADS = 1024;
constexpr int RS_BLOCKS = 8;
constexpr int RS_RAW = 624 * RS_BLOCKS;
__device__ void ransac_sample_seq(const RansacArgs& R, Mt19937& g, int n) {
    g.seed(R.seed);
    for (int it = 0; it < R.iters; ++it) {
        int got[3];
        int k = 0;
        while (k < 3) {
            int idx = (int)uniform_below(g, (uint32_t)n);
            bool dup = false;
            for (int q = 0; q < k; ++q) dup |= got[q] == idx;
            if (!dup) got[k++] = idx;
        }
        R.samples[3 * it] = got[0];
        R.samples[3 * it + 1] = got[1];
        R.samples[3 * it + 2] = got[2];
    }
}
// the first RS_RAW tempered outputs of mt19937(seed): seeding recurrence, RS_BLOCKS twists of the
// 624-word state (three dependency-free phases each) and tempering.  Depends on the seed only, so
// the tracker pipeline runs it on its side stream while the frames are processed.
template <int NT>
__device__ void ransac_raw_body(uint32_t seed, uint32_t* raw, uint32_t* mt) {
    static_assert(NT >= 227, "one twist element per thread and phase");
    const int tid = threadIdx.x;
    if (tid == 0) {  // seeding recurrence (sequential, 623 steps)
        uint32_t v = seed;
        mt[0] = v;
        for (int i = 1; i < 624; ++i) {
            v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
            mt[i] = v;
        }
    }
    __syncthreads();
    for (int blk = 0; blk < RS_BLOCKS; ++blk) {
        // twist: phases [0,227) [227,454) [454,624)
        const int lo[3] = {0, 227, 454}, hi[3] = {227, 454, 624};
        for (int ph = 0; ph < 3; ++ph) {
            const int i = lo[ph] + tid;
            uint32_t nv = 0;
            if (i < hi[ph]) {
                const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                nv = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            __syncthreads();
            if (i < hi[ph]) mt[i] = nv;
            __syncthreads();
        }
        for (int i = tid; i < 624; i += NT) {
            uint32_t y = mt[i];
            y ^= y >> 11;
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= y >> 18;
            raw[624 * blk + i] = y;
        }
        __syncthreads();  // the next twist overwrites mt
    }
}
__global__ void __launch_bounds__(RS_THREADS) ransac_raw_kernel(uint32_t seed, uint32_t* raw) {
    __shared__ uint32_t mt[624];
    ransac_raw_body<RS_THREADS>(seed, raw, mt);
}

// PREP: the input compaction (ransac_prep_body) first, in the same workgroup (one launch fewer on the
// tracker's critical path); the sampler then reads the count from LDS.  Four waves (a sixteen-wave
// workgroup waits longer for a CU while GFTT pass 1 fills the chip from the side stream): thread t
// tests the RS_CHUNK contiguous stream words [t RS_CHUNK, (t+1) RS_CHUNK), one block scan of the
// per-thread accept counts places its accepted draws in stream order.
constexpr int RS_SAMPLE_THREADS = 256;
constexpr int RS_CHUNK = 20;
static_assert(RS_CHUNK % 4 == 0 && RS_RAW % 4 == 0 && RS_SAMPLE_THREADS * RS_CHUNK >= RS_RAW, "sampler chunks");
template <bool PREP>
__global__ void __launch_bounds__(RS_SAMPLE_THREADS) ransac_sample_kernel(RansacArgs R) {
    __shared__ uint32_t acc[RS_RAW];    // accepted draws (compacted), in stream order
    __shared__ uint8_t len3[RS_RAW];    // 1: a hypothesis starting at draw p consumes exactly 3 draws
    __shared__ int wsum[RS_SAMPLE_THREADS / 64];
    __shared__ int s_fallback, s_base;
#ifdef TRK_STAMPS
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#endif
    const int n = PREP ? ransac_prep_body<RS_SAMPLE_THREADS>(R, wsum, s_base) : *R.n_good;
#ifdef TRK_STAMPS
    const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
#endif
    if (PREP) __syncthreads();  // wsum is reused below
    if (n < 3 || R.iters <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int w0 = tid * RS_CHUNK;
    uint32_t yw[RS_CHUNK];  // the thread's tempered words (raw: a 256-B aligned allocation)
#pragma unroll
    for (int q = 0; q < RS_CHUNK / 4; ++q) {
        const int w = w0 + 4 * q;
        const uint4 v = w < RS_RAW ? *reinterpret_cast<const uint4*>(R.raw + w) : make_uint4(0u, 0u, 0u, 0u);
        yw[4 * q] = v.x;
        yw[4 * q + 1] = v.y;
        yw[4 * q + 2] = v.z;
        yw[4 * q + 3] = v.w;
    }
    const uint32_t range = (uint32_t)n;
    const uint32_t thr = (uint32_t)(-range) % range;
    auto accepted = [&](int u) {  // uniform_int_distribution's rejection test of word u
        const uint32_t low = (uint32_t)((uint64_t)yw[u] * range);
        return w0 + u < RS_RAW && !(low < range && low < thr);
    };
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < RS_CHUNK; ++u) cnt += accepted(u) ? 1 : 0;
    int incl = cnt;  // inclusive scan over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    int pos = incl - cnt;
    for (int q = 0; q < wid; ++q) pos += wsum[q];
#pragma unroll
    for (int u = 0; u < RS_CHUNK; ++u)
        if (accepted(u)) acc[pos++] = (uint32_t)(((uint64_t)yw[u] * range) >> 32);
    const int M = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    for (int p = tid; p < M; p += RS_SAMPLE_THREADS)
        len3[p] = (p + 2 < M && acc[p] != acc[p + 1] && acc[p] != acc[p + 2] && acc[p + 1] != acc[p + 2]) ? 1 : 0;
    __syncthreads();
#ifdef TRK_STAMPS
    const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
#endif
    if (wid == 0) {
        int s = 0, h = 0;
        bool fb = false;
        while (h < R.iters && !fb) {
            const int p = s + 3 * lane;
            const bool ok = h + lane < R.iters && p + 2 < M && len3[p];
            const unsigned long long bad = __ballot(!ok);
            const int f = bad ? __ffsll((long long)bad) - 1 : 64;
            if (lane < f) {
                R.samples[3 * (h + lane)] = (int)acc[p];
                R.samples[3 * (h + lane) + 1] = (int)acc[p + 1];
                R.samples[3 * (h + lane) + 2] = (int)acc[p + 2];
            }
            s += 3 * f;
            h += f;
            if (h >= R.iters) break;
            if (f < 64) {  // hypothesis h consumes more than 3 draws (a duplicate) or the stream ends
                int got[3], k = 0, q = s;
                while (k < 3 && q < M) {
                    const int idx = (int)acc[q++];
                    bool dup = false;
                    for (int u = 0; u < k; ++u) dup |= got[u] == idx;
                    if (!dup) got[k++] = idx;
                }
                if (k < 3) { fb = true; break; }
                if (lane == 0) {
                    R.samples[3 * h] = got[0];
                    R.samples[3 * h + 1] = got[1];
                    R.samples[3 * h + 2] = got[2];
                }
                s = q;
                ++h;
            }
        }
        if (lane == 0) s_fallback = fb ? 1 : 0;
    }
    __syncthreads();
#ifdef TRK_STAMPS
    if (tid == 0)
        printf("ransac_sample: prep %llu draws %llu chain %llu (n %d, M %d)\n", ts1 - ts0, ts2 - ts1,
               __builtin_amdgcn_s_memtime() - ts2, n, M);
#endif
    if (s_fallback && tid == 0) {
        __shared__ Mt19937 g;  // stream exhausted: the sequential sampler from the seed
        ransac_sample_seq(R, g, n);
    }
}

__device__ void jacobi3(double* A, double* V) {
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

// EstimateRotation (FeatureTracker.cpp:330-355): nearest proper rotation of H (see oracle)
__device__ void kabsch_rotation(const float* Hf, float* Rf) {
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

__device__ __forceinline__ float det3f(const float* m) {
    return m[0] * (m[4] * m[8] - m[7] * m[5]) - m[3] * (m[1] * m[8] - m[7] * m[2]) + m[6] * (m[1] * m[5] - m[4] * m[2]);
}

__device__ __forceinline__ bool rot_inlier(const float* R, const float* a, const float* q, float cmin) {
    float r0 = (R[0] * a[0] + R[1] * a[1]) + R[2] * a[2];
    float r1 = (R[3] * a[0] + R[4] * a[1]) + R[5] * a[2];
    float r2 = (R[6] * a[0] + R[7] * a[1]) + R[8] * a[2];
    float c = (r0 * q[0] + r1 * q[1]) + r2 * q[2];
    c = c < -1.f ? -1.f : (c > 1.f ? 1.f : c);
    return c >= cmin;  // (float)acos((double)c) < thr (ransac_cos_bound)
}

// one wavefront per hypothesis: count[it] = inliers, or -1 when |det R - 1| > 0.1 (skipped)
__global__ void __launch_bounds__(256) ransac_hyp_kernel(RansacArgs R) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int it = blockIdx.x * 4 + wid;
    if (it >= R.iters) return;
    const int n = *R.n_good;
    if (n < 3) return;
#ifdef TRK_STAMPS
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#endif
    float Hm[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < 3; ++s) {
        int k = R.samples[3 * it + s];
        const float* q = R.b1 + 3 * k;
        const float* a = R.b0 + 3 * k;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) Hm[3 * r + c] += q[r] * a[c];
    }
    float Rm[9];
#ifdef TRK_STAMPS
    const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
#endif
    kabsch_rotation(Hm, Rm);
#ifdef TRK_STAMPS
    const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
    for (int i = 0; i < 9; ++i)  // ransac_select reads the best one back
        if (lane == i) R.rot[9 * it + i] = Rm[i];
    if (fabsf(det3f(Rm) - 1.0f) > 0.1f) {
        if (lane == 0) R.count[it] = -1;
        return;
    }
    int cnt = 0;
    const float cmin = *R.cmin;
    for (int i = lane; i < n; i += 64) cnt += rot_inlier(Rm, R.b0 + 3 * i, R.b1 + 3 * i, cmin) ? 1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (lane == 0) R.count[it] = cnt;
#ifdef TRK_STAMPS
    if (it == 0 && lane == 0)
        printf("ransac_hyp: loads %llu kabsch %llu count %llu\n", ts1 - ts0, ts2 - ts1, __builtin_amdgcn_s_memtime() - ts2);
#endif
}

// first strictly-best hypothesis (256 threads; its rotation into Rs): returns its index, -1 when none
__device__ int ransac_best(const RansacArgs& R, int n, int* sbest, int* sidx, float* Rs) {
    int best = 0, bi = -1;
    if (n >= 3)
        for (int it = threadIdx.x; it < R.iters; it += 256) {
            int c = R.count[it];
            if (c > best) { best = c; bi = it; }  // strictly greater keeps the earliest of this thread
        }
    sbest[threadIdx.x] = best;
    sidx[threadIdx.x] = bi;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            int b2 = sbest[threadIdx.x + s], i2 = sidx[threadIdx.x + s];
            if (b2 > sbest[threadIdx.x] || (b2 == sbest[threadIdx.x] && b2 > 0 && i2 < sidx[threadIdx.x])) {
                sbest[threadIdx.x] = b2;
                sidx[threadIdx.x] = i2;
            }
        }
        __syncthreads();
    }
    const int bit = sidx[0];
    if (threadIdx.x == 0 && blockIdx.x == 0) *R.n_in = n < 3 ? n : sbest[0];
    if (bit >= 0 && threadIdx.x < 9) Rs[threadIdx.x] = R.rot[9 * bit + threadIdx.x];  // ransac_hyp's rotation
    __syncthreads();
    return bit;
}
// -> mask over the good points, scattered to the input order
__global__ void __launch_bounds__(256) ransac_select_kernel(RansacArgs R) {
    __shared__ int sbest[256], sidx[256];
    __shared__ float Rs[9];
    const int n = *R.n_good;
    const int bit = ransac_best(R, n, sbest, sidx, Rs);
    for (int j = threadIdx.x; j < n; j += 256) {
        uint8_t m = 1;
        if (n >= 3 && bit >= 0) m = rot_inlier(Rs, R.b0 + 3 * j, R.b1 + 3 * j, *R.cmin) ? 1 : 0;
        R.kept[R.gidx[j]] = m;
    }
}

// ------------------------------------------------------------------------------------------
// GFTT.  Tile = 64 x 8 outputs.  Source tile with a halo of H_ (2 for the eig map, 3 when the
// 3x3 NMS needs eig at a 1-pixel halo).
constexpr int GF_BX = 64, GF_BY = 8;

template <int HALO>
struct GfTile {
    static constexpr int EW = GF_BX + 2 * (HALO - 2), EH = GF_BY + 2 * (HALO - 2);  // eig positions
    static constexpr int SW = EW + 4, SH = EH + 4;                                   // source pixels
    static constexpr int CW = EW + 2, CH = EH + 2;                                   // cov positions
};

__device__ __forceinline__ bool gf_masked_in(const GfArgs& G, int x, int y) {
    if (G.mask) return G.mask[(size_t)y * G.mask_pitch + x] != 0;
    if (y < G.top_rows || y >= G.bottom_start || x < G.margin || x >= G.W - G.margin) return false;
    if (G.disc_bits) {
        uint32_t wbits = G.disc_bits[(size_t)y * G.disc_words + (x >> 5)];
        if ((wbits >> (x & 31)) & 1u) return false;
    }
    return true;
}

__device__ __forceinline__ uint32_t ord_f32(float v) {
    uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// compute eig for the EW x EH positions starting at (ex0, ey0) into eig[] (LDS)
template <int HALO>
__device__ void gf_eig_tile(const GfArgs& G, int ex0, int ey0, uint8_t (*src)[GfTile<HALO>::SW + 4],
                            float (*cov)[GfTile<HALO>::CW][3], float (*eig)[GfTile<HALO>::EW]) {
    using T = GfTile<HALO>;
    const int W = G.W, H = G.H;
    const int sx0 = ex0 - 2, sy0 = ey0 - 2;
    {
        constexpr int NS = (T::SW * T::SH + 255) / 256;  // loads first, then the LDS stores
        uint32_t v[NS];
#pragma unroll
        for (int it = 0; it < NS; ++it) {
            const int e = threadIdx.x + 256 * it;
            const int ty = e / T::SW, tx = e % T::SW;
            v[it] = e < T::SW * T::SH ? G.img[(size_t)reflect101(sy0 + ty, H) * G.pitch + reflect101(sx0 + tx, W)] : 0u;
        }
#pragma unroll
        for (int it = 0; it < NS; ++it) {
            const int e = threadIdx.x + 256 * it;
            if (e < T::SW * T::SH) src[e / T::SW][e % T::SW] = (uint8_t)v[it];
        }
    }
    __syncthreads();
    const float scale = (float)(1.0 / 3060.0);
    // interior tile: every Sobel neighbour of every cov position is inside the image, no reflection
    const bool interior = sx0 >= 0 && sy0 >= 0 && sx0 + T::SW <= W && sy0 + T::SH <= H;
    // cov at positions (ex0-1+cx, ey0-1+cy): Sobel of reflect101 neighbours.  The tile holds
    // source rows/cols sy0.. with reflect applied per coordinate, so for a cov position p the
    // neighbours p±1 must be reflected relative to the image, not the tile: re-derive them.
    if (interior) {
        for (int e = threadIdx.x; e < T::CW * T::CH; e += 256) {
            const int cy = e / T::CW, cx = e % T::CW;
            const uint8_t* r0 = src[cy];
            const uint8_t* r1 = src[cy + 1];
            const uint8_t* r2 = src[cy + 2];
            const int sx = (r0[cx + 2] - r0[cx]) + 2 * (r1[cx + 2] - r1[cx]) + (r2[cx + 2] - r2[cx]);
            const int sy = (r2[cx] + 2 * r2[cx + 1] + r2[cx + 2]) - (r0[cx] + 2 * r0[cx + 1] + r0[cx + 2]);
            const float dx = (float)sx * scale, dy = (float)sy * scale;
            cov[cy][cx][0] = dx * dx;
            cov[cy][cx][1] = dx * dy;
            cov[cy][cx][2] = dy * dy;
        }
    } else
    for (int e = threadIdx.x; e < T::CW * T::CH; e += 256) {
        int cy = e / T::CW, cx = e % T::CW;
        int X = reflect101(ex0 - 1 + cx, W), Y = reflect101(ey0 - 1 + cy, H);
        // tile coordinates of X-1, X, X+1 (reflected about the image) — map back into the tile
        int xm = reflect101(X - 1, W) - sx0, xc = X - sx0, xp = reflect101(X + 1, W) - sx0;
        int ym = reflect101(Y - 1, H) - sy0, yc = Y - sy0, yp = reflect101(Y + 1, H) - sy0;
        int sx, sy;
        if (xm >= 0 && xp < T::SW && ym >= 0 && yp < T::SH && xc >= 0 && xc < T::SW && yc >= 0 && yc < T::SH) {
            const uint8_t* r0 = src[ym];
            const uint8_t* r1 = src[yc];
            const uint8_t* r2 = src[yp];
            sx = (r0[xp] - r0[xm]) + 2 * (r1[xp] - r1[xm]) + (r2[xp] - r2[xm]);
            sy = (r2[xm] + 2 * r2[xc] + r2[xp]) - (r0[xm] + 2 * r0[xc] + r0[xp]);
        } else {  // tile edge folded by a reflection: read the image directly
            const uint8_t* r0 = G.img + (size_t)reflect101(Y - 1, H) * G.pitch;
            const uint8_t* r1 = G.img + (size_t)Y * G.pitch;
            const uint8_t* r2 = G.img + (size_t)reflect101(Y + 1, H) * G.pitch;
            int gxm = reflect101(X - 1, W), gxp = reflect101(X + 1, W);
            sx = (r0[gxp] - r0[gxm]) + 2 * (r1[gxp] - r1[gxm]) + (r2[gxp] - r2[gxm]);
            sy = (r2[gxm] + 2 * r2[X] + r2[gxp]) - (r0[gxm] + 2 * r0[X] + r0[gxp]);
        }
        float dx = (float)sx * scale, dy = (float)sy * scale;
        cov[cy][cx][0] = dx * dx;
        cov[cy][cx][1] = dx * dy;
        cov[cy][cx][2] = dy * dy;
    }
    __syncthreads();
    // 3x3 box (reflect101 about the image) + min eigenvalue
    for (int e = threadIdx.x; e < T::EW * T::EH; e += 256) {
        int ey = e / T::EW, ex = e % T::EW;
        int X = ex0 + ex, Y = ey0 + ey;
        if (X < 0 || Y < 0 || X >= W || Y >= H) {  // outside the image: never read (dilate ignores it)
            eig[ey][ex] = 0.f;
            continue;
        }
        double s0 = 0, s1 = 0, s2 = 0;
        if (X >= 1 && X < W - 1 && Y >= 1 && Y < H - 1) {
            for (int ky = 0; ky < 3; ++ky)
                for (int kx = 0; kx < 3; ++kx) {
                    const float* c = cov[ey + ky][ex + kx];
                    s0 += c[0]; s1 += c[1]; s2 += c[2];
                }
        } else {
            // border pixel: neighbours reflect about the image; cov positions of (X+k) live at
            // tile index reflect101(X+k) - (ex0-1), valid for every in-image X of this tile
            for (int ky = -1; ky <= 1; ++ky) {
                int yy = reflect101(Y + ky, H) - (ey0 - 1);
                for (int kx = -1; kx <= 1; ++kx) {
                    int xx = reflect101(X + kx, W) - (ex0 - 1);
                    const float* c = cov[yy][xx];
                    s0 += c[0]; s1 += c[1]; s2 += c[2];
                }
            }
        }
        float a = (float)s0 * 0.5f, b = (float)s1, c = (float)s2 * 0.5f;
        eig[ey][ex] = (a + c) - sqrtf((a - c) * (a - c) + b * b);
    }
    __syncthreads();
}

// Pass 1a: the min-eigenvalue map, independent of the mask (so it can run concurrently with LK /
// RANSAC / the disc mask).  Each workgroup walks GF_SUB tiles down the image.
constexpr int GF_SUB = 4;
__global__ void __launch_bounds__(256) gftt_eig_kernel(GfArgs G) {
    using T = GfTile<2>;
    __shared__ uint8_t src[T::SH][T::SW + 4];
    __shared__ float cov[T::CH][T::CW][3];
    __shared__ float eig[T::EH][T::EW];
    for (int sub = 0; sub < GF_SUB; ++sub) {
        const int ex0 = blockIdx.x * GF_BX, ey0 = (blockIdx.y * GF_SUB + sub) * GF_BY;
        if (ey0 >= G.H) break;
        gf_eig_tile<2>(G, ex0, ey0, src, cov, eig);
        for (int e = threadIdx.x; e < T::EW * T::EH; e += 256) {
            const int ey = e / T::EW, ex = e % T::EW;
            const int X = ex0 + ex, Y = ey0 + ey;
            if (X < G.W && Y < G.H) G.eig[(size_t)Y * G.W + X] = eig[ey][ex];
        }
        __syncthreads();  // eig / src are rewritten by the next tile
    }
}

// Pass 1b: masked maximum of the map (minMaxLoc over the mask), streamed row by row; rows the
// analytic polar mask removes are skipped.  One global atomic per workgroup.
constexpr int GM_BLOCKS = 1024;
__global__ void __launch_bounds__(256) gftt_max_kernel(GfArgs G) {
    __shared__ uint32_t red[4];
    uint32_t m = 0;  // ord(-inf-ish): any value beats 0
    constexpr int U = 8;  // loads in flight per lane
    for (int y = blockIdx.x; y < G.H; y += gridDim.x) {
        if (!G.mask && (y < G.top_rows || y >= G.bottom_start)) continue;
        const float* row = G.eig + (size_t)y * G.W;
        for (int x0 = threadIdx.x; x0 < G.W; x0 += 256 * U) {
            float v[U];
            bool in[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int x = x0 + 256 * u;
                in[u] = x < G.W && gf_masked_in(G, x, y);
                v[u] = x < G.W ? row[x] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (in[u]) m = max(m, ord_f32(v[u]));
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = max(max(red[0], red[1]), max(red[2], red[3]));
        if (t) atomicMax(G.max_ord, t);
    }
}

__global__ void __launch_bounds__(256) gftt_cand_kernel(GfArgs G) {
    using T = GfTile<3>;  // eig positions of the tile with a 1-pixel halo
    __shared__ float eig[T::EH][T::EW];
    __shared__ unsigned long long keys[GF_SUB * GF_BX * GF_BY];
    __shared__ unsigned int s_cnt, s_base;
    if (threadIdx.x == 0) s_cnt = 0;
    // threshold (THRESH_TOZERO with the float threshold)
    const uint32_t mo = *G.max_ord;
    double maxv = mo ? (double)unord_f32(mo) : 0.0;  // minMaxLoc over the mask, 0 when empty
    if (maxv < 0.0) maxv = 0.0;
    const float thr = (float)(maxv * G.quality);
    // the map of pass 1 for all GF_SUB haloed sub-tiles, every load issued up front (positions
    // outside the image read as 0: the dilation ignores them)
    constexpr int NE = (T::EW * T::EH + 255) / 256;
    float vmap[GF_SUB][NE];
#pragma unroll
    for (int sub = 0; sub < GF_SUB; ++sub)
#pragma unroll
        for (int it = 0; it < NE; ++it) {
            const int e = threadIdx.x + 256 * it;
            const int ey = e / T::EW, ex = e % T::EW;
            const int X = blockIdx.x * GF_BX - 1 + ex, Y = (blockIdx.y * GF_SUB + sub) * GF_BY - 1 + ey;
            vmap[sub][it] = (e < T::EW * T::EH && X >= 0 && Y >= 0 && X < G.W && Y < G.H)
                                ? G.eig[(size_t)Y * G.W + X] : 0.f;
        }
    for (int sub = 0; sub < GF_SUB; ++sub) {
        const int ox = blockIdx.x * GF_BX, oy = (blockIdx.y * GF_SUB + sub) * GF_BY;
        if (oy >= G.H) break;
        // thresholded to zero (THRESH_TOZERO)
#pragma unroll
        for (int it = 0; it < NE; ++it) {
            const int e = threadIdx.x + 256 * it;
            if (e < T::EW * T::EH) {
                const float v = vmap[sub][it];
                eig[e / T::EW][e % T::EW] = v > thr ? v : 0.f;
            }
        }
        __syncthreads();
        for (int e = threadIdx.x; e < GF_BX * GF_BY; e += 256) {
            int ty = e / GF_BX, tx = e % GF_BX;
            int X = ox + tx, Y = oy + ty;
            bool c = false;
            float v = 0.f;
            if (X >= 1 && X < G.W - 1 && Y >= 1 && Y < G.H - 1) {
                v = eig[ty + 1][tx + 1];
                if (v != 0.f && gf_masked_in(G, X, Y)) {
                    float m = v;
                    for (int ky = 0; ky < 3; ++ky)
                        for (int kx = 0; kx < 3; ++kx) m = fmaxf(m, eig[ty + ky][tx + kx]);
                    c = (v == m);
                }
            }
            unsigned long long bal = __ballot(c);
            int lane = threadIdx.x & 63;
            int cnt = __popcll(bal);
            unsigned int base = 0;
            if (cnt) {
                if (lane == __ffsll((long long)bal) - 1) base = atomicAdd(&s_cnt, (unsigned int)cnt);  // LDS
                base = __shfl(base, __ffsll((long long)bal) - 1, 64);
            }
            if (c)
                keys[base + __popcll(bal & ((1ull << lane) - 1ull))] =
                    ((unsigned long long)__float_as_uint(v) << 32) | (unsigned int)(Y * G.W + X);
        }
        __syncthreads();  // eig / src are rewritten by the next tile
    }
    const unsigned int n = s_cnt;
    if (n == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(G.n_cand, n);
    __syncthreads();
    const unsigned int base = s_base;
    for (unsigned int i = threadIdx.x; i < n; i += 256)
        if (base + i < G.cand_cap) G.cand[base + i] = keys[i];
}

// the response threshold of a masked maximum mo (ordered-int; 0: empty mask)
__device__ __forceinline__ float lm_thr_of(const GfArgs& G, uint32_t mo) {
    double maxv = mo ? (double)unord_f32(mo) : 0.0;  // minMaxLoc over the mask, 0 when empty
    if (maxv < 0.0) maxv = 0.0;
    return (float)(maxv * G.quality);
}

// greedy min-distance selection over the sorted candidates (goodFeaturesToTrack tail).
// One workgroup.  Accepted corners live in a grid of cell = round(min_dist) with <= 3 per cell.
constexpr int GS_THREADS = 256;
constexpr int GS_SLOTS = 3;
// HASH: the batch's survivors are also chained per grid cell (head[cell] -> s_next[rank], dynamic LDS
// after the grid), so a survivor compares only with the survivors of its 3x3 cells (every pair within
// min_dist lies there, as for the grid test) and the insertion walks only its own cell: the same
// conflict masks and slots as the all-pairs walks, in O(cell occupancy) instead of O(batch).
// G.presel (tracker pipeline, local-maximum path): `keys` is the presorted prefix of EVERY local maximum
// of the static region (gftt_presort on the side stream, before the disc mask exists), so the pre-filter
// also drops the keys inside a disc, and the threshold is bounded from above by thr_hi = quality x the
// static region's maximum (the masked maximum is at most that): a key above thr_hi is a candidate whatever
// the exact threshold, the first key at or below it ends the walk.  A walk that ends there (or runs out of
// a prefix that does not hold every local maximum) before max_corners raises `incomplete` and the host runs
// the exact tail (masked maximum, candidate top-K, this kernel); otherwise the corners are those of the
// exact tail by construction (the same keys in the same order reach the greedy pass).  The prefix is staged
// GS_STAGE keys at a time: their disc / threshold tests run in parallel (two memory round trips per stage
// instead of per batch) and the batches are formed from the staged survivors only.
constexpr int GS_STAGE = 4 * GS_THREADS;
template <bool GLOBAL_GRID, bool HASH>
__global__ void __launch_bounds__(GS_THREADS) gftt_select_kernel(GfArgs G, const unsigned long long* keys,
                                                                  const unsigned int* n_keys, unsigned int cap,
                                                                  int fast) {
    extern __shared__ uint32_t grid_lds[];
    __shared__ int s_next[GS_THREADS];
    __shared__ int s_good[GS_THREADS];
    __shared__ unsigned int s_idx[GS_THREADS];  // the batch's candidate addresses
    __shared__ unsigned int s_sv[GS_THREADS];   // survivors of the pre-filter, batch order: y << 16 | x
    __shared__ int s_cell[GS_THREADS];          // their grid cells (yc * gw + xc)
    __shared__ unsigned long long s_conf[GS_THREADS][GS_THREADS / 64];
    __shared__ int s_wcnt[GS_THREADS / 64];
    __shared__ unsigned long long s_am[GS_THREADS / 64];  // accepted survivors of the batch
    __shared__ unsigned long long s_dm[GS_THREADS / 64];  // decided survivors
    __shared__ uint32_t s_slot_val[GS_THREADS];
    __shared__ int s_slot_idx[GS_THREADS];
    __shared__ int s_acc;
    __shared__ int s_stop;
    __shared__ int s_trunc;
    __shared__ float s_thr;
    __shared__ unsigned int s_st[GS_STAGE + GS_THREADS];  // presel: staged survivors (addresses, key order)
    __shared__ int s_nst;                                  // presel: staged survivors
    __shared__ unsigned int s_kpos;                        // presel: keys staged so far
    uint32_t* grid = GLOBAL_GRID ? G.grid_global : grid_lds;  // static address space (no flat access)
    const int ncell = G.gw * G.gh;
    int* head = reinterpret_cast<int*>(grid_lds + (GLOBAL_GRID ? 0 : ncell * GS_SLOTS));
    for (int e = threadIdx.x; e < ncell * GS_SLOTS; e += GS_THREADS) grid[e] = 0xffffffffu;
    if (HASH)
        for (int e = threadIdx.x; e < ncell; e += GS_THREADS) head[e] = -1;
    const bool presel = G.presel != 0;
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        s_acc = 0; s_stop = 0; s_trunc = 0; s_nst = 0; s_kpos = 0;
        int ok = 1;
        if (G.wait_ctr) {  // the presort's hand-off (the grid's initialisation above runs meanwhile)
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while ((int)(__hip_atomic_load(G.wait_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - G.wait_target) < 0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz: the exact tail decides
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        s_ok = ok;
        if (presel && ok) s_thr = lm_thr_of(G, *G.smax);  // thr_hi: the static region's maximum (the presort's)
    }
    __syncthreads();
    if (!s_ok) {
        if (threadIdx.x == 0) {
            *G.n_out = 0;
            *G.incomplete = 1;
        }
        return;
    }
    const unsigned int total = min(*n_keys, cap);
    const int cell = G.cell;
    const double md2 = G.min_dist * G.min_dist;
    auto conflicts = [&](int x, int y, int slot_lane_only) -> bool {
        const int xc = x / cell, yc = y / cell;
        bool hit = false;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const int xx = xc + dx, yy = yc + dy;
                if (xx < 0 || yy < 0 || xx >= G.gw || yy >= G.gh) continue;
#pragma unroll
                for (int s = 0; s < GS_SLOTS; ++s) {  // every slot read (independent loads), empty = 0xffffffff
                    const uint32_t p = grid[(yy * G.gw + xx) * GS_SLOTS + s];
                    const float ddx = (float)x - (float)(p & 0xffffu), ddy = (float)y - (float)(p >> 16);
                    hit |= p != 0xffffffffu && (double)(ddx * ddx + ddy * ddy) < md2;
                }
            }
        return hit;
    };
#ifdef GFTT_DEBUG
    unsigned long long t_start = __builtin_amdgcn_s_memtime(), t_pre = 0, t_mask = 0, t_greedy = 0, tq;
    int nb_dbg = 0, nsv_dbg = 0;
    unsigned long long dbgv[4][4] = {}, dbgs[4] = {};
#endif
    int sb = 0;  // presel: the batch's first staged survivor
    for (unsigned int c0 = 0;; c0 += GS_THREADS) {
        int nb = GS_THREADS;  // presel: survivors in this batch
        if (!presel) {
            if (c0 >= total) break;
        } else {
            if (s_nst - sb < GS_THREADS && !s_trunc && s_kpos < total) {
                // stage the next GS_STAGE keys behind the survivors still staged: thread t tests keys
                // s_kpos + 4t .. +3 (threshold bound, then the disc bit), one block scan places the survivors
                const int rem = s_nst - sb;
                const unsigned int mv = (int)threadIdx.x < rem ? s_st[sb + threadIdx.x] : 0u;
                const unsigned int k0 = s_kpos + 4 * threadIdx.x;
                unsigned long long kv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) kv[u] = k0 + u < total ? keys[k0 + u] : 0ull;
                bool pass[4];
                int cnt = 0;
                bool tr = false;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const unsigned int idx = (unsigned int)(kv[u] & 0xffffffffu);
                    const bool in = k0 + u < total;
                    const bool above = __uint_as_float((unsigned int)(kv[u] >> 32)) > s_thr;
                    tr |= in && !above;  // this key and every later one: undecided against the exact threshold
                    pass[u] = in && above && !lm_disc(G, (int)(idx % G.W), (int)(idx / G.W));
                    cnt += pass[u] ? 1 : 0;
                }
                const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
                int incl = cnt;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int v = __shfl_up(incl, off, 64);
                    if (lane >= off) incl += v;
                }
                if (lane == 63) s_wcnt[wid] = incl;
                __syncthreads();  // (every thread's read of s_st / s_nst / s_kpos above is done)
                if ((int)threadIdx.x < rem) s_st[threadIdx.x] = mv;
                int pos = rem + incl - cnt, tot = 0;
#pragma unroll
                for (int q = 0; q < GS_THREADS / 64; ++q) {
                    pos += q < wid ? s_wcnt[q] : 0;
                    tot += s_wcnt[q];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (pass[u]) s_st[pos++] = (unsigned int)(kv[u] & 0xffffffffu);
                if (tr) s_trunc = 1;
                __syncthreads();  // s_wcnt is reused by the batch
                if (threadIdx.x == 0) {
                    s_nst = rem + tot;
                    s_kpos += GS_STAGE;
                }
                sb = 0;
                __syncthreads();
            }
            nb = min(GS_THREADS, s_nst - sb);
            if (nb <= 0) break;
        }
        // (1) parallel pre-filter against the corners accepted in earlier batches
        unsigned int ci = c0 + threadIdx.x;
        int good = 0;
#ifdef GFTT_DEBUG
        if (nb_dbg < 4) dbgs[nb_dbg] = __builtin_amdgcn_s_memtime() - t_start;  // (presel: staging so far)
#endif
        if (presel) {
            if ((int)threadIdx.x < nb) {
                const unsigned int idx = s_st[sb + threadIdx.x];
                good = s_acc == 0 || !conflicts((int)(idx % G.W), (int)(idx / G.W), 0);  // (empty grid: no test)
                s_idx[threadIdx.x] = idx;
            }
        } else if (ci < total) {
            unsigned int idx = (unsigned int)(keys[ci] & 0xffffffffu);
            good = !conflicts((int)(idx % G.W), (int)(idx / G.W), 0);
            s_idx[threadIdx.x] = idx;
        }
        s_good[threadIdx.x] = good;
        __syncthreads();
#ifdef GFTT_DEBUG
        tq = __builtin_amdgcn_s_memtime(); t_pre += tq - t_start;
        if (nb_dbg < 4) dbgv[nb_dbg][0] = tq - t_start;
        t_start = tq;
#endif
        // (2) in-order resolution inside the batch.  Survivors of (1) are compacted (batch order);
        // survivor r gets a bitmask of the earlier survivors within min_dist of it; thread 0 walks
        // the masks in order (accept r iff none of its conflicts was accepted) and inserts the
        // accepted corners into the grid in acceptance order.
        {
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            const unsigned long long bal = __ballot(good);
            if (lane == 0) s_wcnt[wid] = __popcll(bal);
            __syncthreads();
            int rank = __popcll(bal & ((1ull << lane) - 1ull));
            for (int q = 0; q < wid; ++q) rank += s_wcnt[q];
            int nsv = 0;
            for (int q = 0; q < GS_THREADS / 64; ++q) nsv += s_wcnt[q];
#ifdef GFTT_DEBUG
            nb_dbg++; nsv_dbg += nsv;
#endif
            int x = 0, y = 0;
            if (good) {
                const unsigned int idx = s_idx[threadIdx.x];
                x = (int)(idx % G.W);
                y = (int)(idx / G.W);
                s_sv[rank] = ((unsigned int)y << 16) | (unsigned int)x;
                s_cell[rank] = (y / cell) * G.gw + x / cell;
                if (HASH) s_next[rank] = atomicExch(&head[s_cell[rank]], rank);
            }
            __syncthreads();
            if (HASH && good) {
                unsigned long long m[GS_THREADS / 64];
#pragma unroll
                for (int q = 0; q < GS_THREADS / 64; ++q) m[q] = 0ull;
                const int xc = x / cell, yc = y / cell;
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int xx = xc + dx, yy = yc + dy;
                        if (xx < 0 || yy < 0 || xx >= G.gw || yy >= G.gh) continue;
                        for (int bq = head[yy * G.gw + xx]; bq >= 0; bq = s_next[bq]) {
                            if (bq >= rank) continue;
                            const unsigned int pj = s_sv[bq];
                            const float ddx = (float)x - (float)(pj & 0xffff), ddy = (float)y - (float)(pj >> 16);
                            if ((double)(ddx * ddx + ddy * ddy) < md2) m[bq >> 6] |= 1ull << (bq & 63);
                        }
                    }
#pragma unroll
                for (int q = 0; q < GS_THREADS / 64; ++q) s_conf[rank][q] = m[q];
            }
            if (!HASH && good) {
#pragma unroll
                for (int q = 0; q < GS_THREADS / 64; ++q) {  // word q of the mask stays in a register
                    unsigned long long m = 0ull;
                    const int jend = min(rank - 64 * q, 64);
#pragma unroll 8
                    for (int b = 0; b < jend; ++b) {
                        const unsigned int pj = s_sv[64 * q + b];
                        const float ddx = (float)x - (float)(pj & 0xffff), ddy = (float)y - (float)(pj >> 16);
                        if ((double)(ddx * ddx + ddy * ddy) < md2) m |= 1ull << b;
                    }
                    s_conf[rank][q] = m;
                }
            }
            __syncthreads();
#ifdef GFTT_DEBUG
            tq = __builtin_amdgcn_s_memtime(); t_mask += tq - t_start; if (nb_dbg < 5 && nb_dbg > 0) dbgv[nb_dbg - 1][1] = tq - t_start; t_start = tq;
#endif
            // greedy in batch order, resolved in rounds: a survivor is accepted once none of its earlier
            // conflicting survivors can still be accepted (all decided rejected), rejected once one of
            // them is accepted.  Identical to the sequential walk; rounds = longest conflict chain.
            if (threadIdx.x < GS_THREADS / 64) { s_am[threadIdx.x] = 0ull; s_dm[threadIdx.x] = 0ull; }
            __syncthreads();
            bool decided = !good;
            unsigned long long cf[GS_THREADS / 64];
#pragma unroll
            for (int q = 0; q < GS_THREADS / 64; ++q) cf[q] = good ? s_conf[rank][q] : 0ull;
            for (;;) {
                bool acc_now = false, dec_now = false;
                if (!decided) {
                    unsigned long long hit = 0ull, open = 0ull;
#pragma unroll
                    for (int q = 0; q < GS_THREADS / 64; ++q) {
                        hit |= cf[q] & s_am[q];
                        open |= cf[q] & ~s_dm[q];
                    }
                    if (hit) dec_now = true;
                    else if (!open) { dec_now = true; acc_now = true; }
                }
                const int any = __syncthreads_or(dec_now ? 1 : 0);
                if (!any) break;
                if (dec_now) {
                    decided = true;
                    atomicOr(&s_dm[rank >> 6], 1ull << (rank & 63));
                    if (acc_now) atomicOr(&s_am[rank >> 6], 1ull << (rank & 63));
                }
                __syncthreads();
            }
#ifdef GFTT_DEBUG
            tq = __builtin_amdgcn_s_memtime(); t_greedy += tq - t_start;
            if (nb_dbg < 5 && nb_dbg > 0) dbgv[nb_dbg - 1][2] = tq - t_start;
            t_start = tq;
#endif
            // max_corners: keep the first (max_corners - s_acc) accepted in order
            if (threadIdx.x == 0 && G.max_corners > 0) {
                int room = G.max_corners - s_acc;
                for (int q = 0; q < GS_THREADS / 64; ++q) {
                    unsigned long long m = s_am[q];
                    const int c = __popcll(m);
                    if (c >= room) {
                        while (__popcll(m) > room) m &= ~(1ull << (63 - __clzll(m)));  // drop the highest bits
                        s_am[q] = m;
                        for (int q2 = q + 1; q2 < GS_THREADS / 64; ++q2) s_am[q2] = 0ull;
                        if (__popcll(m) == room) s_stop = 1;
                        break;
                    }
                    room -= c;
                }
            }
            __syncthreads();
            // accepted survivors in acceptance (= batch) order: corners[s_acc + rank]; grid slots as the
            // sequential insertion would leave them (the i-th insertion into a cell holding e0 entries
            // goes to slot min(e0 + i, GS_SLOTS - 1); an overflowing slot keeps the last one)
            const int nacc_before = s_acc;
            int nacc = 0;
#pragma unroll
            for (int q = 0; q < GS_THREADS / 64; ++q) nacc += __popcll(s_am[q]);
            if (good && ((s_am[rank >> 6] >> (rank & 63)) & 1ull)) {
                int before = 0;
                for (int q = 0; q < (rank >> 6); ++q) before += __popcll(s_am[q]);
                before += __popcll(s_am[rank >> 6] & ((1ull << (rank & 63)) - 1ull));
                const int kk = nacc_before + before;
                G.corners[2 * kk] = (float)x;
                G.corners[2 * kk + 1] = (float)y;
                const int mycell = s_cell[rank];
                int i_cell = 0, m_cell = 0;
                if (HASH) {
                    for (int r = head[mycell]; r >= 0; r = s_next[r]) {
                        if (!((s_am[r >> 6] >> (r & 63)) & 1ull)) continue;
                        if (r < rank) ++i_cell;
                        ++m_cell;
                    }
                } else {
                    for (int r = 0; r < nsv; ++r) {
                        if (!((s_am[r >> 6] >> (r & 63)) & 1ull)) continue;
                        if (s_cell[r] == mycell) {
                            if (r < rank) ++i_cell;
                            ++m_cell;
                        }
                    }
                }
                uint32_t* cellp = &grid[mycell * GS_SLOTS];
                int e0 = 0;
                while (e0 < GS_SLOTS && cellp[e0] != 0xffffffffu) ++e0;  // entries from earlier batches
                const int slot = min(e0 + i_cell, GS_SLOTS - 1);
                if (e0 + i_cell < GS_SLOTS - 1 || i_cell == m_cell - 1) s_slot_val[rank] = ((uint32_t)y << 16) | (uint32_t)x, s_slot_idx[rank] = mycell * GS_SLOTS + slot;
                else s_slot_idx[rank] = -1;
            }
            __syncthreads();
            if (good && ((s_am[rank >> 6] >> (rank & 63)) & 1ull) && s_slot_idx[rank] >= 0)
                grid[s_slot_idx[rank]] = s_slot_val[rank];
            if (HASH && good) head[s_cell[rank]] = -1;  // every chain of the batch emptied (read above)
            if (threadIdx.x == 0) s_acc = nacc_before + nacc;
#ifdef GFTT_DEBUG
            __syncthreads();
            tq = __builtin_amdgcn_s_memtime();
            if (nb_dbg < 5 && nb_dbg > 0) dbgv[nb_dbg - 1][3] = tq - t_start;
            t_start = tq;
#endif
        }
        __syncthreads();
        if (s_stop) break;
        sb += nb;
    }
#ifdef GFTT_DEBUG
    if (threadIdx.x == 0)
        printf("gftt_select: total %u batches %d survivors %d pre %llu mask %llu greedy %llu rest %llu\n", total, nb_dbg, nsv_dbg,
               t_pre, t_mask, t_greedy, __builtin_amdgcn_s_memtime() - t_start);
    if (threadIdx.x == 0)
        for (int q = 0; q < 2; ++q)
            printf("gftt_select batch %d: stage %llu pre %llu mask %llu rounds %llu insert %llu\n", q, dbgs[q], dbgv[q][0], dbgv[q][1], dbgv[q][2], dbgv[q][3]);
#endif
    if (threadIdx.x == 0) {
        *G.n_out = s_acc;
        // the top-K subset ran dry before max_corners: the exact pass over every candidate must decide
        if (fast) *G.incomplete = (!s_stop && (s_trunc || G.cut[1] == 0)) ? 1 : 0;
    }
}

// histogram of candidate responses (bucket = float bits >> 20), grid-stride over the candidates
__global__ void __launch_bounds__(256) gftt_hist_kernel(GfArgs G) {
    __shared__ unsigned int h[GF_BUCKETS];
    for (int b = threadIdx.x; b < GF_BUCKETS; b += 256) h[b] = 0;
    __syncthreads();
    const unsigned int n = min(*G.n_cand, G.cand_cap);
    for (unsigned int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        atomicAdd(&h[(unsigned int)(G.cand[i] >> 52)], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < GF_BUCKETS; b += 256)
        if (h[b]) atomicAdd(&G.hist[b], h[b]);
}

// cut bucket: the highest buckets holding >= topk_target candidates (never more than topk_cap), the
// same top-down walk as a sequential loop would make (first bucket from the top where the running
// count reaches the target, or where the next nonempty bucket would overflow the buffer).  Computed
// by every workgroup of the top-K gather from the final histogram (8 KB from L2) instead of a
// one-workgroup launch between the histogram and the gather: thread t owns buckets [8t, 8t+8), suffix
// sums by a wave scan plus the four wave totals, the stopping bucket by a max over threads.  Returns
// the cut; *below_empty: no candidate below it.  cs: LDS scratch of the workgroup.
constexpr int CUT_PER = GF_BUCKETS / 256;
struct CutShared {
    unsigned int wtot[4], wmax[4], suf_cut;
    int cut;
};
__device__ int gftt_cut_block(const GfArgs& G, CutShared& cs, unsigned int& below_empty) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    unsigned int h[CUT_PER];
    unsigned int loc = 0;
#pragma unroll
    for (int i = CUT_PER - 1; i >= 0; --i) {
        h[i] = G.hist[t * CUT_PER + i];
        loc += h[i];
    }
    unsigned int sfx = loc;  // sum of loc over lanes >= lane of the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned int v = (unsigned int)__shfl_down((int)sfx, off, 64);
        if (lane + off < 64) sfx += v;
    }
    if (lane == 0) cs.wtot[wid] = sfx;
    __syncthreads();
    unsigned int above = 0;  // threads of later waves
    for (int q = wid + 1; q < 4; ++q) above += cs.wtot[q];
    const unsigned int total = cs.wtot[0] + cs.wtot[1] + cs.wtot[2] + cs.wtot[3];  // every candidate
    const unsigned int run0 = sfx + above - loc;  // buckets above this thread's
    // the thread's highest stopping bucket (nonempty, cum + c over the buffer or at the target)
    int cand = -1;
    unsigned int cum_c = 0, c_c = 0;
    {
        unsigned int cum = run0;
#pragma unroll
        for (int i = CUT_PER - 1; i >= 0; --i) {
            const unsigned int c = h[i];
            if (cand < 0 && c != 0 && (cum + c > G.topk_cap || cum + c >= G.topk_target)) {
                cand = t * CUT_PER + i;
                cum_c = cum;
                c_c = c;
            }
            cum += c;
        }
    }
    unsigned int m = (unsigned int)(cand + 1);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, off, 64));
    if (lane == 0) cs.wmax[wid] = m;
    if (t == 0) cs.cut = 0;  // never stopped: the walk reaches bucket 0 (every bucket taken or empty)
    __syncthreads();
    const int bstop = (int)max(max(cs.wmax[0], cs.wmax[1]), max(cs.wmax[2], cs.wmax[3])) - 1;
    __syncthreads();  // cs.cut = 0 before the owner's store
    // not taken (over the buffer): the lowest bucket above bstop reached by the walk, bstop + 1;
    // taken: the target is reached at bstop
    if (bstop >= 0 && cand == bstop) cs.cut = cum_c + c_c > G.topk_cap ? bstop + 1 : bstop;
    if (t == 0) cs.suf_cut = 0;
    __syncthreads();
    const int cut = cs.cut;
    if (cut < GF_BUCKETS && t == cut / CUT_PER) {  // candidates at or above the cut
        unsigned int sc = run0;
#pragma unroll
        for (int i = CUT_PER - 1; i >= 0; --i)
            if (t * CUT_PER + i >= cut) sc += h[i];
        cs.suf_cut = sc;
    }
    __syncthreads();
    below_empty = total - cs.suf_cut == 0 ? 1u : 0u;
    return cut;
}

__global__ void __launch_bounds__(256) gftt_topk_compact_kernel(GfArgs G) {
    __shared__ CutShared cs;
    unsigned int below_empty;
    const unsigned int cut = (unsigned int)gftt_cut_block(G, cs, below_empty);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // for the selection pass
        G.cut[0] = (int)cut;
        G.cut[1] = (int)below_empty;
    }
    const unsigned int n = min(*G.n_cand, G.cand_cap);
    const int lane = threadIdx.x & 63;
    constexpr int U = 4;  // candidate loads in flight per lane
    const unsigned int stride = gridDim.x * 256;
    for (unsigned int i0 = blockIdx.x * 256; i0 < n; i0 += U * stride) {  // wave-uniform trip count
        unsigned long long kv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned int i = i0 + u * stride + threadIdx.x;
            kv[u] = i < n ? G.cand[i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned int i = i0 + u * stride + threadIdx.x;
            const unsigned long long k = kv[u];
            const bool take = i < n && (unsigned int)(k >> 52) >= cut;
            const unsigned long long bal = __ballot(take);  // one counter atomic per wave
            if (!bal) continue;
            const int leader = __ffsll((long long)bal) - 1;
            unsigned int base = 0;
            if (lane == leader) base = atomicAdd(G.n_top, (unsigned int)__popcll(bal));
            base = __shfl(base, leader, 64);
            if (take) {
                const unsigned int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
                if (pos < G.topk_cap) G.topk[pos] = k;
            }
        }
    }
}

// per-frame reset of the GFTT counters, histogram and top-K buffer (one launch instead of memsets)
__global__ void __launch_bounds__(256) gftt_reset_kernel(GfArgs G, int* scal) {
    const unsigned int t = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
    if (t == 0) {
        scal[2] = scal[3] = scal[4] = 0;             // max_ord, n_cand, n_out
        scal[6] = scal[7] = scal[8] = scal[9] = 0;   // n_top, cut[2], incomplete
        scal[10] = scal[11] = 0;                     // lmax overflow, flatten counter
    }
    for (unsigned int i = t; i < GF_BUCKETS; i += stride) G.hist[i] = 0u;
    for (unsigned int i = t; i < G.topk_cap; i += stride) G.topk[i] = 0ull;
}
hipError_t launch_gftt_reset(const GfArgs& g, int* scal, hipStream_t st) {
    hipLaunchKernelGGL(gftt_reset_kernel, dim3(64), dim3(256), 0, st, g, scal);
    return hipGetLastError();
}

// rasterise the discs of CreateFeatureMask (cv::circle filled, LINE_8; half-widths precomputed
// on the host from OpenCV's midpoint Circle()) into a 1-bit-per-pixel exclusion mask
__device__ __forceinline__ void disc_raster(const DiscArgs& D, int i, int nthreads) {
    const float fx = D.pts[2 * i], fy = D.pts[2 * i + 1];
    const int cx = (int)rintf(fx), cy = (int)rintf(fy);  // Point2f -> Point (cvRound)
    const int r = D.radius;
    for (int dy = -r + (int)threadIdx.x; dy <= r; dy += nthreads) {
        int y = cy + dy;
        if (y < 0 || y >= D.H) continue;
        int hwd = D.halfw[dy < 0 ? -dy : dy];
        int x0 = max(cx - hwd, 0), x1 = min(cx + hwd, D.W - 1);
        for (int x = x0; x <= x1;) {
            int wi = x >> 5;
            int b0 = x & 31;
            int b1 = min(31, x1 - (wi << 5));
            uint32_t m = (b1 - b0 == 31) ? 0xffffffffu : (((1u << (b1 - b0 + 1)) - 1u) << b0);
            atomicOr(&D.bits[(size_t)y * D.words + wi], m);
            x = (wi + 1) << 5;
        }
    }
}
__global__ void __launch_bounds__(128) disc_mask_kernel(DiscArgs D) {
    const int k = blockIdx.x;
    if (D.n_pts_dev && k >= *D.n_pts_dev) return;  // null: the grid is exactly the point count
    if (D.kept && !D.kept[D.src_index ? D.src_index[k] : k]) return;
    disc_raster(D, D.src_index ? D.src_index[k] : k, 128);
}

// tracker pipeline: RANSAC's selection and CreateFeatureMask's discs in one launch (one launch fewer on the
// critical path).  Workgroup j (compacted point j < n_good; the grid covers every input point) finds the best
// hypothesis itself -- the same reduction in every workgroup -- tests its point, scatters the kept flag and,
// when kept, rasterises the point's disc (disc_mask_kernel's rows; D.radius <= 0: no discs)
__global__ void __launch_bounds__(256) ransac_select_disc_kernel(RansacArgs R, DiscArgs D) {
    __shared__ int sbest[256], sidx[256];
    __shared__ float Rs[9];
    __shared__ int s_m;
    const int n = *R.n_good;
    if ((int)blockIdx.x >= max(n, 1)) return;  // (workgroup 0 always runs: it writes n_in)
    const int bit = ransac_best(R, n, sbest, sidx, Rs);
    const int j = blockIdx.x;
    if (j >= n) return;
    if (threadIdx.x == 0) {
        uint8_t m = 1;
        if (n >= 3 && bit >= 0) m = rot_inlier(Rs, R.b0 + 3 * j, R.b1 + 3 * j, *R.cmin) ? 1 : 0;
        R.kept[R.gidx[j]] = m;
        s_m = m;
    }
    __syncthreads();
    if (s_m && D.radius > 0) disc_raster(D, R.gidx[j], 256);
}

// ------------------------------------------------------------------------------------------
// GFTT, local-maximum path (no explicit mask).  The candidate test of pass 2 — v > thr after
// THRESH_TOZERO and v == the 3x3 dilation — is, for v > thr, the same as v >= each of its eight
// raw neighbours (a neighbour u <= thr is zeroed but then u < v anyway).  So the 3x3 local maxima
// do not depend on the threshold and the mask's static part (polar rows, side margins) is known
// up front: pass 1 keeps them per tile together with the tile's maximum over the static region,
// concurrently with LK / RANSAC.  After the disc mask: the masked maximum is the largest tile
// maximum of the tiles no disc touches, raised by an exact recount of the touched tiles whose
// maximum could exceed it; candidates are the kept local maxima above the threshold outside the
// discs.  The eigenvalue map is never materialised.
constexpr int LM_SRC_W = 96;                     // 16-B aligned source span [ox-16, ox+80)
constexpr int LM_CW = LM_TX + 4, LM_EW = LM_TX + 2;  // cov x [ox-2, ox+66), eig x [ox-1, ox+65)

template <int TY>  // tile height: eig rows [oy-1, oy+TY+1), cov rows [oy-2, oy+TY+2), source [oy-3, oy+TY+3)
struct LmShared {
    static constexpr int CH = TY + 4, EH = TY + 2, SH = TY + 6;
    uint8_t src[SH][LM_SRC_W];
    float d[2][CH][LM_CW];  // the scaled Sobel derivatives dx, dy (planar); the box sums form their products
    float eig[EH][LM_EW];
};


// Tiles whose eig positions all lie at least one pixel inside the image (no reflected box positions):
// the Sobel sums roll down a column (three source reads per cov position instead of nine: the
// horizontal difference / smoothing of each source row kept for the next two), dx / dy in planar LDS (2
// floats per position instead of the 3 products: 4 workgroups per CU), and eig from rolling vertical sums
// of horizontal triple sums of the products (the same f32 products dx*dx, dx*dy, dy*dy as before).
// The box sums are exact, so any summation order gives the ky / kx order's bits: each f32 product is a
// multiple of 2^-47 (|Sobel| <= 1020 and the scale 1/3060 make a nonzero product >= scale^2 > 2^-24,
// whose ulp is >= 2^-47) below 1/8 in magnitude, so every partial sum of nine fits 53 bits.
template <int TY>
__device__ void lm_eig_interior(LmShared<TY>& S) {
    constexpr int CH = LmShared<TY>::CH, EH = LmShared<TY>::EH, CG = 3;  // CG row groups per column
    static_assert(CG * LM_CW <= 256 && CG * LM_EW <= 256, "one column of a row group per thread");
    float(*cv)[CH][LM_CW] = S.d;
    const float scale = (float)(1.0 / 3060.0);
    const int t = threadIdx.x;
    if (t < CG * LM_CW) {  // cov column cx (image x = ox-2+cx: source columns cx+13 .. cx+15), rows [r0, r1)
        const int cx = t % LM_CW, g = t / LM_CW, r0 = g * CH / CG, r1 = (g + 1) * CH / CG;
        const int c0 = cx + 13;
        int d[3], m[3];  // per source row: x difference, x smoothing
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint8_t* r = S.src[r0 + i];
            d[i] = r[c0 + 2] - r[c0];
            m[i] = r[c0] + 2 * r[c0 + 1] + r[c0 + 2];
        }
        for (int cy = r0; cy < r1; ++cy) {
            const uint8_t* r = S.src[cy + 2];
            d[2] = r[c0 + 2] - r[c0];
            m[2] = r[c0] + 2 * r[c0 + 1] + r[c0 + 2];
            const int sx = d[0] + 2 * d[1] + d[2], sy = m[2] - m[0];
            cv[0][cy][cx] = (float)sx * scale;
            cv[1][cy][cx] = (float)sy * scale;
            d[0] = d[1]; d[1] = d[2];
            m[0] = m[1]; m[1] = m[2];
        }
    }
    __syncthreads();
    if (t < CG * LM_EW) {  // eig column ex (cov columns ex .. ex+2), rows [e0, e1) (cov rows ey .. ey+2)
        const int ex = t % LM_EW, g = t / LM_EW, e0 = g * EH / CG, e1 = (g + 1) * EH / CG;
        double h[3][3];  // [cov row slot][component]: horizontal triple sums
        auto hsum = [&](int cy, double* o) {
            float p[3][3];  // [column][component]: dx*dx, dx*dy, dy*dy
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float dx = cv[0][cy][ex + i], dy = cv[1][cy][ex + i];
                p[i][0] = dx * dx;
                p[i][1] = dx * dy;
                p[i][2] = dy * dy;
            }
#pragma unroll
            for (int j = 0; j < 3; ++j) o[j] = ((double)p[0][j] + (double)p[1][j]) + (double)p[2][j];
        };
        hsum(e0, h[0]);
        hsum(e0 + 1, h[1]);
        for (int ey = e0; ey < e1; ++ey) {
            hsum(ey + 2, h[2]);
            const double s0 = (h[0][0] + h[1][0]) + h[2][0], s1 = (h[0][1] + h[1][1]) + h[2][1],
                         s2 = (h[0][2] + h[1][2]) + h[2][2];
            const float a = (float)s0 * 0.5f, b = (float)s1, c = (float)s2 * 0.5f;
            S.eig[ey][ex] = (a + c) - sqrtf((a - c) * (a - c) + b * b);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                h[0][j] = h[1][j];
                h[1][j] = h[2][j];
            }
        }
    }
    __syncthreads();
}

// eig at the LM_EW x LM_EH positions of the tile at (ox, oy) into S.eig (the gf_eig_tile
// arithmetic: Sobel on reflect101 neighbours, f32 products, f64 3x3 box sums in ky / kx order)
template <int TY>
__device__ void lm_eig_tile(const GfArgs& G, int ox, int oy, LmShared<TY>& S) {
    constexpr int LM_CH = LmShared<TY>::CH, LM_EH = LmShared<TY>::EH, LM_SH = LmShared<TY>::SH;
    const int W = G.W, H = G.H;
    {  // 16-B chunks of the REFLECT_101 source rows (chunks beyond the pitch skipped), then the
       // columns outside the image patched with their reflected pixels
        constexpr int NCH = LM_SH * (LM_SRC_W / 16);
        static_assert(NCH <= 256, "one 16-B load per thread");
        const int x0 = ox - 16 + 16 * (threadIdx.x % (LM_SRC_W / 16));
        const bool ld = threadIdx.x < NCH && x0 >= 0 && x0 + 16 <= G.pitch;
        uint4 v;
        if (ld) v = *reinterpret_cast<const uint4*>(G.img + (size_t)reflect101(oy - 3 + threadIdx.x / (LM_SRC_W / 16), H) * G.pitch + x0);
        if (ld) *reinterpret_cast<uint4*>(&S.src[threadIdx.x / (LM_SRC_W / 16)][16 * (threadIdx.x % (LM_SRC_W / 16))]) = v;
        if (ox - 3 < 0 || ox + LM_TX + 3 > W) {
            __syncthreads();
            for (int e = threadIdx.x; e < LM_SH * (LM_TX + 6); e += 256) {
                const int r = e / (LM_TX + 6), x = ox - 3 + e % (LM_TX + 6);
                if (x < 0 || x >= W) S.src[r][x - (ox - 16)] = G.img[(size_t)reflect101(oy - 3 + r, H) * G.pitch + reflect101(x, W)];
            }
        }
        __syncthreads();
    }
    if (ox >= 2 && ox + LM_EW <= W && oy >= 2 && oy + LM_EH <= H) {  // every eig position >= 1 px inside
        lm_eig_interior(S);
        return;
    }
    const float scale = (float)(1.0 / 3060.0);
    for (int e = threadIdx.x; e < LM_CW * LM_CH; e += 256) {
        // image x = ox-2+cx: source columns x-1, x, x+1 at cx+13 .. cx+15 (REFLECT_101 pixels; cov
        // positions outside the image are never read: the box below reflects its positions)
        const int cy = e / LM_CW, cx = e % LM_CW;
        const uint8_t* r0 = S.src[cy];
        const uint8_t* r1 = S.src[cy + 1];
        const uint8_t* r2 = S.src[cy + 2];
        const int c0 = cx + 13, c1 = cx + 14, c2 = cx + 15;
        const int sx = (r0[c2] - r0[c0]) + 2 * (r1[c2] - r1[c0]) + (r2[c2] - r2[c0]);
        const int sy = (r2[c0] + 2 * r2[c1] + r2[c2]) - (r0[c0] + 2 * r0[c1] + r0[c2]);
        S.d[0][cy][cx] = (float)sx * scale;
        S.d[1][cy][cx] = (float)sy * scale;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < LM_EW * LM_EH; e += 256) {
        const int ey = e / LM_EW, ex = e % LM_EW;
        const int X = ox - 1 + ex, Y = oy - 1 + ey;
        if (X < 0 || Y < 0 || X >= W || Y >= H) {
            S.eig[ey][ex] = 0.f;
            continue;
        }
        double s0 = 0, s1 = 0, s2 = 0;
        if (X >= 1 && X < W - 1 && Y >= 1 && Y < H - 1) {
            for (int ky = 0; ky < 3; ++ky)
                for (int kx = 0; kx < 3; ++kx) {
                    const float dx = S.d[0][ey + ky][ex + kx], dy = S.d[1][ey + ky][ex + kx];
                    const float c0 = dx * dx, c1 = dx * dy, c2 = dy * dy;
                    s0 += c0; s1 += c1; s2 += c2;
                }
        } else {
            for (int ky = -1; ky <= 1; ++ky) {
                const int yy = reflect101(Y + ky, H) - (oy - 2);
                for (int kx = -1; kx <= 1; ++kx) {
                    const int xx = reflect101(X + kx, W) - (ox - 2);
                    const float dx = S.d[0][yy][xx], dy = S.d[1][yy][xx];
                    const float c0 = dx * dx, c1 = dx * dy, c2 = dy * dy;
                    s0 += c0; s1 += c1; s2 += c2;
                }
            }
        }
        const float a = (float)s0 * 0.5f, b = (float)s1, c = (float)s2 * 0.5f;
        S.eig[ey][ex] = (a + c) - sqrtf((a - c) * (a - c) + b * b);
    }
    __syncthreads();
}

// block max of an ordered-int value (every thread passes its value; thread 0 gets the result)
__device__ __forceinline__ uint32_t lm_block_max(uint32_t m, uint32_t* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    const uint32_t t = max(max(red[0], red[1]), max(red[2], red[3]));
    __syncthreads();
    return t;
}

// pass 1: per tile, the 3x3 local maxima inside the static region and the region's maximum
__global__ void __launch_bounds__(256) gftt_lmax_kernel(GfArgs G) {
    __shared__ LmShared<LM_TY> S;
    // the tile's local maxima over the derivative planes (dead once the eigenvalues are formed): 4 workgroups per CU
    static_assert(sizeof(S.d) >= LM_CAP * sizeof(unsigned long long) && offsetof(LmShared<LM_TY>, d) % 8 == 0, "keys in S.d");
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(&S.d[0][0][0]);
    __shared__ unsigned int s_cnt;
    __shared__ uint32_t red[4];
    const int tile = xcd_tile(blockIdx.x, G.tiles_x * G.tiles_y);
    const int ox = (tile % G.tiles_x) * LM_TX, oy = (tile / G.tiles_x) * LM_TY;
    if (G.clear && blockIdx.x == 0)
        for (int i = threadIdx.x; i < G.clear_n; i += 256) G.clear[i] = 0u;
    if (threadIdx.x == 0) s_cnt = 0;
    lm_eig_tile<LM_TY>(G, ox, oy, S);
    uint32_t m = 0, kmax = 0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // lane = tile column, wave = a band of LM_TY / 4 rows: the 3x3 maximum from rolling row maxima of
    // three eig values (no NaN: "no neighbour > v" is "v >= the 3x3 maximum", v included)
    static_assert(LM_TX == 64 && LM_TY % 4 == 0, "one tile column per lane, four row bands");
    constexpr int RB = LM_TY / 4;
    const int tx = lane, X = ox + tx;
    auto rmax = [&](int ey) { return fmaxf(fmaxf(S.eig[ey][tx], S.eig[ey][tx + 1]), S.eig[ey][tx + 2]); };
    float hm0 = rmax(wid * RB), hm1 = rmax(wid * RB + 1);
    for (int ty = wid * RB; ty < wid * RB + RB; ++ty) {
        const float hm2 = rmax(ty + 2);
        const int Y = oy + ty;
        bool c = false;
        float v = 0.f;
        if (X < G.W && Y < G.H && lm_static_in(G, X, Y)) {
            v = S.eig[ty + 1][tx + 1];
            m = max(m, ord_f32(v));
            c = v > 0.f && X >= 1 && X < G.W - 1 && Y >= 1 && Y < G.H - 1 && !(fmaxf(fmaxf(hm0, hm1), hm2) > v);
        }
        hm0 = hm1;
        hm1 = hm2;
        const unsigned long long bal = __ballot(c);
        const int cnt = __popcll(bal);
        unsigned int base = 0;
        if (cnt) {
            const int leader = __ffsll((long long)bal) - 1;
            if (lane == leader) base = atomicAdd(&s_cnt, (unsigned int)cnt);  // LDS
            base = __shfl(base, leader, 64);
        }
        if (c) {
            const unsigned int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
            if (pos < LM_CAP) keys[pos] = ((unsigned long long)__float_as_uint(v) << 32) | (unsigned int)(Y * G.W + X);
            kmax = max(kmax, __float_as_uint(v) >> 20);  // histogram bucket of the key
        }
    }
    m = lm_block_max(m, red);
    kmax = lm_block_max(kmax, red);
    const unsigned int n = s_cnt;
    unsigned long long* out = G.lmax + (size_t)tile * LM_CAP;
    for (unsigned int i = threadIdx.x; i < min(n, (unsigned int)LM_CAP); i += 256) out[i] = keys[i];
    if (threadIdx.x == 0) {
        G.lmax_n[tile] = n;
        G.tile_max[tile] = m;
        G.tile_kmax[tile] = kmax;
    }
}

// the masked maximum, part 1: tiles no disc touches contribute their static-region maximum
// (one wave per tile; one atomic per workgroup)
__global__ void __launch_bounds__(256) gftt_tmax_kernel(GfArgs G) {
    __shared__ uint32_t red[4];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + wid;
    const int n_tiles = G.tiles_x * G.tiles_y;
    uint32_t m = 0;
    if (tile < n_tiles) {
        const int ox = (tile % G.tiles_x) * LM_TX, oy = (tile / G.tiles_x) * LM_TY;
        const int x0 = max(ox, G.margin), x1 = min(min(ox + LM_TX, G.W), G.W - G.margin);  // [x0, x1)
        const int y0 = max(oy, G.top_rows), y1 = min(min(oy + LM_TY, G.H), G.bottom_start);
        bool hit = false;
        if (G.disc_bits && x0 < x1 && y0 < y1) {
            const int w0 = x0 >> 5, w1 = (x1 - 1) >> 5, nw = w1 - w0 + 1;
            for (int q = lane; q < (y1 - y0) * nw; q += 64) {
                const int y = y0 + q / nw, w = w0 + q % nw;
                uint32_t bits = G.disc_bits[(size_t)y * G.disc_words + w];
                const int lo = max(x0 - 32 * w, 0), hi = min(x1 - 32 * w, 32);  // [lo, hi) inside the word
                const uint32_t rm = (hi - lo == 32) ? 0xffffffffu : (((1u << (hi - lo)) - 1u) << lo);
                hit |= (bits & rm) != 0u;
            }
        }
        const bool dirty = __ballot(hit) != 0ull;
        if (lane == 0) G.tile_dirty[tile] = dirty ? 1 : 0;
        if (!dirty) m = G.tile_max[tile];
    }
    m = lm_block_max(m, red);
    if (threadIdx.x == 0 && m) atomicMax(G.max_ord, m);
}

// the masked maximum, part 2: a touched tile whose static maximum exceeds the running maximum is
// recounted exactly over static-region pixels outside the discs, in LM_TY / 8 strips of 64 x 8
constexpr int LM_STRIP = 8;
__global__ void __launch_bounds__(256) gftt_dirty_kernel(GfArgs G) {
    __shared__ LmShared<LM_STRIP> S;
    __shared__ uint32_t red[4];
    __shared__ int s_go;
    constexpr int NS = LM_TY / LM_STRIP;
    const int tile = blockIdx.x / NS, strip = blockIdx.x % NS;
    if (threadIdx.x == 0) s_go = G.tile_dirty[tile] && G.tile_max[tile] > *(volatile uint32_t*)G.max_ord;
    __syncthreads();
    if (!s_go) return;
    const int ox = (tile % G.tiles_x) * LM_TX, oy = (tile / G.tiles_x) * LM_TY + strip * LM_STRIP;
    if (oy >= G.H) return;
    lm_eig_tile<LM_STRIP>(G, ox, oy, S);
    uint32_t m = 0;
    for (int e = threadIdx.x; e < LM_TX * LM_STRIP; e += 256) {
        const int ty = e / LM_TX, tx = e % LM_TX;
        const int X = ox + tx, Y = oy + ty;
        if (X < G.W && Y < G.H && lm_static_in(G, X, Y) && !lm_disc(G, X, Y)) m = max(m, ord_f32(S.eig[ty + 1][tx + 1]));
    }
    m = lm_block_max(m, red);
    if (threadIdx.x == 0 && m) atomicMax(G.max_ord, m);
}

__device__ __forceinline__ float lm_threshold(const GfArgs& G) { return lm_thr_of(G, *G.max_ord); }
__device__ __forceinline__ bool lm_survives(const GfArgs& G, unsigned long long k, float thr) {
    const float v = __uint_as_float((unsigned int)(k >> 32));
    const unsigned int a = (unsigned int)k;
    return v > thr && !lm_disc(G, (int)(a % (unsigned int)G.W), (int)(a / (unsigned int)G.W));
}

// candidates = kept local maxima above the threshold outside the discs: their response histogram
// and count (grid-stride over the tiles, one wave per tile and step)
__global__ void __launch_bounds__(256) gftt_lm_hist_kernel(GfArgs G) {
    __shared__ unsigned int h[GF_BUCKETS];
    __shared__ unsigned int s_n;
    for (int b = threadIdx.x; b < GF_BUCKETS; b += 256) h[b] = 0;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const float thr = lm_threshold(G);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n_tiles = G.tiles_x * G.tiles_y;
    unsigned int cnt = 0;
    uint32_t sm = 0;  // (the presort: the static region's maximum over the wave's tiles)
    // the tile's count and its first 64 key slots are requested together (the slots lie inside the tile's
    // LM_CAP block; those at or past the count are read and ignored), the next tile's one step ahead
    const int stride = gridDim.x * 4;
    int tile = blockIdx.x * 4 + wid;
    unsigned int nk_n = 0;
    unsigned long long k_n = 0ull;
    if (tile < n_tiles) {
        nk_n = G.lmax_n[tile];
        k_n = G.lmax[(size_t)tile * LM_CAP + lane];
    }
    for (; tile < n_tiles; tile += stride) {
        const unsigned int nk = nk_n;
        const unsigned long long k0 = k_n;
        if (tile + stride < n_tiles) {
            nk_n = G.lmax_n[tile + stride];
            k_n = G.lmax[(size_t)(tile + stride) * LM_CAP + lane];
        }
        if (G.smax) sm = max(sm, G.tile_max[tile]);
        if (nk > LM_CAP && lane == 0) *G.lmax_over = 1;
        const unsigned long long* keys = G.lmax + (size_t)tile * LM_CAP;
        for (unsigned int i = lane; i < min(nk, (unsigned int)LM_CAP); i += 64) {
            const unsigned long long k = i < 64 ? k0 : keys[i];
            if (lm_survives(G, k, thr)) {
                atomicAdd(&h[(unsigned int)(k >> 52)], 1u);
                ++cnt;
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += (unsigned int)__shfl_xor((int)cnt, off, 64);
    if (lane == 0 && cnt) atomicAdd(&s_n, cnt);
    if (G.smax && lane == 0 && sm) atomicMax(G.smax, sm);
    __syncthreads();
    for (int b = threadIdx.x; b < GF_BUCKETS; b += 256)
        if (h[b]) atomicAdd(&G.hist[b], h[b]);
    if (threadIdx.x == 0 && s_n) atomicAdd(G.n_cand, s_n);
}

// the candidates at or above the cut bucket into the top-K buffer: gathered in LDS per workgroup,
// one counter atomic per workgroup (a returning atomic per wave serialises on the one word)
constexpr int LM_TOPK_LDS = 2048;
__global__ void __launch_bounds__(256) gftt_lm_topk_kernel(GfArgs G) {
    __shared__ unsigned long long buf[LM_TOPK_LDS];
    __shared__ unsigned int s_n, s_base;
    __shared__ CutShared cs;
    if (threadIdx.x == 0) s_n = 0;
    // the first tile's bucket bound, count and first 64 key slots requested before the cut is formed (the slots
    // lie inside the tile's LM_CAP block; those past the count are ignored), the next tile's one step ahead
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n_tiles = G.tiles_x * G.tiles_y;
    const int stride = gridDim.x * 4;
    int tile = blockIdx.x * 4 + wid;
    uint32_t km_n = 0;
    unsigned int nk_n = 0;
    unsigned long long k_n = 0ull;
    if (tile < n_tiles) {
        km_n = G.tile_kmax[tile];
        nk_n = G.lmax_n[tile];
        k_n = G.lmax[(size_t)tile * LM_CAP + lane];
    }
    unsigned int below_empty;
    const unsigned int cut = (unsigned int)gftt_cut_block(G, cs, below_empty);  // (its barriers order s_n = 0)
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // for the selection pass
        G.cut[0] = (int)cut;
        G.cut[1] = (int)below_empty;
    }
    const float thr = lm_threshold(G);
    for (; tile < n_tiles; tile += stride) {
        const uint32_t km = km_n;
        const unsigned int nk = min(nk_n, (unsigned int)LM_CAP);
        const unsigned long long k0 = k_n;
        if (tile + stride < n_tiles) {
            km_n = G.tile_kmax[tile + stride];
            nk_n = G.lmax_n[tile + stride];
            k_n = G.lmax[(size_t)(tile + stride) * LM_CAP + lane];
        }
        if (km < cut) continue;  // no key of the tile reaches the cut bucket
        const unsigned long long* keys = G.lmax + (size_t)tile * LM_CAP;
        for (unsigned int i0 = 0; i0 < nk; i0 += 64) {  // wave-uniform trip count
            const unsigned int i = i0 + lane;
            unsigned long long k = 0ull;
            bool take = false;
            if (i < nk) {
                k = i0 == 0 ? k0 : keys[i];
                take = (unsigned int)(k >> 52) >= cut && lm_survives(G, k, thr);
            }
            const unsigned long long bal = __ballot(take);
            if (!bal) continue;
            const int leader = __ffsll((long long)bal) - 1;
            unsigned int base = 0;
            if (lane == leader) base = atomicAdd(&s_n, (unsigned int)__popcll(bal));  // LDS
            base = __shfl(base, leader, 64);
            if (take) {
                const unsigned int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
                if (pos < LM_TOPK_LDS) {
                    buf[pos] = k;
                } else {  // the workgroup's buffer is full: straight to the global list
                    const unsigned int g = atomicAdd(G.n_top, 1u);
                    if (g < G.topk_cap) G.topk[g] = k;
                }
            }
        }
    }
    __syncthreads();
    const unsigned int n = min(s_n, (unsigned int)LM_TOPK_LDS);
    if (n == 0) return;
    if (threadIdx.x == 0) s_base = atomicAdd(G.n_top, n);
    __syncthreads();
    for (unsigned int i = threadIdx.x; i < n; i += 256)
        if (s_base + i < G.topk_cap) G.topk[s_base + i] = buf[i];
}

// exact fallback of this path: every surviving candidate into the flat candidate list
__global__ void __launch_bounds__(256) gftt_lm_flatten_kernel(GfArgs G) {
    const float thr = lm_threshold(G);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n_tiles = G.tiles_x * G.tiles_y;
    for (int tile = blockIdx.x * 4 + wid; tile < n_tiles; tile += gridDim.x * 4) {
        const unsigned int nk = min(G.lmax_n[tile], (unsigned int)LM_CAP);
        const unsigned long long* keys = G.lmax + (size_t)tile * LM_CAP;
        for (unsigned int i0 = 0; i0 < nk; i0 += 64) {
            const unsigned int i = i0 + lane;
            unsigned long long k = 0ull;
            bool take = false;
            if (i < nk) {
                k = keys[i];
                take = lm_survives(G, k, thr);
            }
            const unsigned long long bal = __ballot(take);
            if (!bal) continue;
            const int leader = __ffsll((long long)bal) - 1;
            unsigned int base = 0;
            if (lane == leader) base = atomicAdd(G.n_flat, (unsigned int)__popcll(bal));
            base = __shfl(base, leader, 64);
            if (take) {
                const unsigned int pos = base + __popcll(bal & ((1ull << lane) - 1ull));
                if (pos < G.cand_cap) G.cand[pos] = k;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// launchers
hipError_t launch_pyr_down(const PyrLevelPair& s, const PyrLevelPair& d, int frames, hipStream_t st) {
    constexpr int by = 8;
    dim3 g((d.w + PD_BX - 1) / PD_BX, (d.h + by - 1) / by, frames);
    hipLaunchKernelGGL(pyr_down_kernel<by>, g, dim3(256), 0, st, s, d);
    return hipGetLastError();
}
hipError_t launch_lk(const LkArgs& a, hipStream_t st, const LkAux* aux) {
    LkAux x;
    std::memset(&x, 0, sizeof x);
    if (aux) x = *aux;
    const int n = a.n > 0 ? a.n : 0, blocks = n + (aux ? LK_AUX_BLOCKS : 0);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(lk_kernel, dim3(blocks), dim3(LK_THREADS), 0, st, a, x);
    return hipGetLastError();
}
size_t ransac_raw_words() { return RS_RAW; }
hipError_t launch_ransac_raw(uint32_t seed, uint32_t* raw, hipStream_t st) {
    hipLaunchKernelGGL(ransac_raw_kernel, dim3(1), dim3(RS_THREADS), 0, st, seed, raw);
    return hipGetLastError();
}
hipError_t launch_ransac(const RansacArgs& r, bool gen_samples, hipStream_t st) {
    // with samples to draw: the compaction and the sampler in one 4-wave workgroup (a 16-wave one waits
    // longer for a CU while GFTT pass 1 fills the chip from the side stream)
    if (gen_samples)
        hipLaunchKernelGGL(ransac_sample_kernel<true>, dim3(1), dim3(RS_SAMPLE_THREADS), 0, st, r);
    else
        hipLaunchKernelGGL(ransac_prep_kernel, dim3(1), dim3(RP_THREADS), 0, st, r);
    if (r.iters > 0) hipLaunchKernelGGL(ransac_hyp_kernel, dim3((r.iters + 3) / 4), dim3(256), 0, st, r);
    hipLaunchKernelGGL(ransac_select_kernel, dim3(1), dim3(256), 0, st, r);
    return hipGetLastError();
}
hipError_t launch_ransac_pipeline(const RansacArgs& r, const DiscArgs& d, hipStream_t st) {
    hipLaunchKernelGGL(ransac_sample_kernel<true>, dim3(1), dim3(RS_SAMPLE_THREADS), 0, st, r);
    if (r.iters > 0) hipLaunchKernelGGL(ransac_hyp_kernel, dim3((r.iters + 3) / 4), dim3(256), 0, st, r);
    hipLaunchKernelGGL(ransac_select_disc_kernel, dim3(r.n > 0 ? r.n : 1), dim3(256), 0, st, r, d);
    return hipGetLastError();
}
hipError_t launch_disc_mask(const DiscArgs& d, int max_pts, hipStream_t st) {
    if (max_pts <= 0) return hipSuccess;
    hipLaunchKernelGGL(disc_mask_kernel, dim3(max_pts), dim3(128), 0, st, d);
    return hipGetLastError();
}
hipError_t launch_gftt_eig(const GfArgs& g, hipStream_t st) {
    dim3 grd((g.W + GF_BX - 1) / GF_BX, (g.H + GF_BY * GF_SUB - 1) / (GF_BY * GF_SUB));
    hipLaunchKernelGGL(gftt_eig_kernel, grd, dim3(256), 0, st, g);
    return hipGetLastError();
}
// after the map (launch_gftt_eig, on this stream or joined into it): masked max, then candidates
static hipError_t gftt_candidates(const GfArgs& g, hipStream_t st) {
    dim3 grd((g.W + GF_BX - 1) / GF_BX, (g.H + GF_BY * GF_SUB - 1) / (GF_BY * GF_SUB));
    hipLaunchKernelGGL(gftt_max_kernel, dim3(GM_BLOCKS), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_cand_kernel, grd, dim3(256), 0, st, g);
    return hipGetLastError();
}
static size_t gftt_select_lds(const GfArgs& g, bool hash) {
    const size_t ncell = (size_t)g.gw * g.gh;
    return (g.grid_global ? 0 : ncell * GS_SLOTS * sizeof(uint32_t)) + (hash ? ncell * sizeof(int) : 0);
}
// greedy selection over n_keys sorted keys: the cell-chained variant when its chain heads fit next to
// the grid in LDS, else the all-pairs walks
static hipError_t launch_select(const GfArgs& g, const unsigned long long* keys, const unsigned int* n_keys,
                                unsigned int cap, int fast, hipStream_t st) {
    const bool hash = gftt_select_lds(g, true) <= GF_SELECT_LDS_MAX;
    const size_t lds = gftt_select_lds(g, hash);
    if (g.grid_global) {
        if (hash) hipLaunchKernelGGL((gftt_select_kernel<true, true>), dim3(1), dim3(GS_THREADS), lds, st, g, keys, n_keys, cap, fast);
        else hipLaunchKernelGGL((gftt_select_kernel<true, false>), dim3(1), dim3(GS_THREADS), lds, st, g, keys, n_keys, cap, fast);
    } else {
        if (hash) hipLaunchKernelGGL((gftt_select_kernel<false, true>), dim3(1), dim3(GS_THREADS), lds, st, g, keys, n_keys, cap, fast);
        else hipLaunchKernelGGL((gftt_select_kernel<false, false>), dim3(1), dim3(GS_THREADS), lds, st, g, keys, n_keys, cap, fast);
    }
    return hipGetLastError();
}
// Descending sort of the top-K buffer (n = min(n_top, topk_cap) keys) by rank: the keys are unique
// (response bits << 32 | pixel address), so key i belongs at position #{keys > key i} -- the order
// a descending radix sort of the buffer gives.  64 keys per workgroup (one per lane); each of the 16
// waves counts over one sixteenth of the list, staged through LDS in 512-key chunks (coalesced 8-key-per-
// lane loads of the next chunk in flight while the current one is compared; ds_read_b128 broadcasts,
// two comparands per read); the partial counts are summed in LDS and the key written to its position.
// TS_WAVES = 16 for the masked tail's top-K (~5 k keys); the presort's prefix (~2-4 k keys) uses 8-wave
// workgroups: 17 -> 11.5 us against 4-wave ones beside the RANSAC kernels (config-1 pipeline 0.159-0.163 ->
// 0.154-0.156 ms; 16 waves 0.158-0.160 ms: profiles/r6x_ab_presort_sort_waves.log)
constexpr int TS_CHUNK = 512;
template <int TS_WAVES>
__global__ void __launch_bounds__(64 * TS_WAVES) gftt_topk_sort_kernel(GfArgs G) {
    __shared__ unsigned int part[TS_WAVES][64];
    __shared__ __align__(16) unsigned long long buf[TS_WAVES][TS_CHUNK];
    const unsigned int n = min(*G.n_top, G.topk_cap);
    const unsigned int i0 = blockIdx.x * 64;
    auto signal = [&]() {  // presort: this workgroup's stores are done (every storing wave drained, then one release)
        if (!G.done) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(G.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    if (i0 >= n) {
        signal();
        return;
    }
    const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
    const unsigned int i = i0 + lane;
    const unsigned long long k = i < n ? G.topk[i] : ~0ull;
    const unsigned int per = ((n + TS_WAVES - 1) / TS_WAVES + 7) & ~7u;
    const unsigned int j0 = min(n, wid * per), j1 = min(n, j0 + per);
    const unsigned long long* src = G.topk;
    unsigned long long* mine = buf[wid];
    unsigned int cnt = 0;
    unsigned long long nx[TS_CHUNK / 64];
#pragma unroll
    for (int u = 0; u < TS_CHUNK / 64; ++u) {  // key 0 (never > k) pads the last chunk
        const unsigned int j = j0 + 64 * u + lane;
        nx[u] = j < j1 ? src[j] : 0ull;
    }
    for (unsigned int base = j0; base < j1; base += TS_CHUNK) {
#pragma unroll
        for (int u = 0; u < TS_CHUNK / 64; ++u) mine[64 * u + lane] = nx[u];
        wave_lds_fence();
        if (base + TS_CHUNK < j1) {
#pragma unroll
            for (int u = 0; u < TS_CHUNK / 64; ++u) {
                const unsigned int j = base + TS_CHUNK + 64 * u + lane;
                nx[u] = j < j1 ? src[j] : 0ull;
            }
        }
        const ulonglong2* c2 = reinterpret_cast<const ulonglong2*>(mine);
#pragma unroll 8
        for (int q = 0; q < TS_CHUNK / 2; ++q) {
            const ulonglong2 c = c2[q];
            cnt += (c.x > k) + (c.y > k);
        }
        wave_lds_fence();  // every lane's reads of the chunk before the next chunk's writes
    }
    part[wid][lane] = cnt;
    __syncthreads();
    if (wid == 0 && i < n) {
        unsigned int r = 0;
#pragma unroll
        for (int q = 0; q < TS_WAVES; ++q) r += part[q][lane];
        G.topk_sorted[r] = k;
    }
    signal();
}
static hipError_t gftt_sort_topk(const GfArgs& g, void*, size_t, hipStream_t st) {
    hipLaunchKernelGGL(gftt_topk_sort_kernel<16>, dim3((g.topk_cap + 63) / 64), dim3(64 * 16), 0, st, g);
    return hipGetLastError();
}
// fast path: candidates -> histogram -> top-K compaction -> sort of the top-K keys -> greedy
hipError_t launch_gftt(const GfArgs& g, void* sort_tmp, size_t sort_tmp_bytes, hipStream_t st) {
    hipError_t e = gftt_candidates(g, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gftt_hist_kernel, dim3(256), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_topk_compact_kernel, dim3(256), dim3(256), 0, st, g);
    e = gftt_sort_topk(g, sort_tmp, sort_tmp_bytes, st);
    if (e != hipSuccess) return e;
    return launch_select(g, (const unsigned long long*)g.topk_sorted, (const unsigned int*)g.n_top, g.topk_cap, 1, st);
}
hipError_t launch_gftt_lmax(const GfArgs& g, hipStream_t st) {
    hipLaunchKernelGGL(gftt_lmax_kernel, dim3(g.tiles_x * g.tiles_y), dim3(256), 0, st, g);
    return hipGetLastError();
}
// after pass 1 and the disc mask: masked maximum (clean tiles, then the touched tiles that could
// raise it), candidate histogram, cut, top-K, sort, greedy selection
hipError_t launch_gftt_after_lmax(const GfArgs& g, void* sort_tmp, size_t sort_tmp_bytes, hipStream_t st) {
    const int n_tiles = g.tiles_x * g.tiles_y;
    hipLaunchKernelGGL(gftt_tmax_kernel, dim3((n_tiles + 3) / 4), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_dirty_kernel, dim3(n_tiles * (LM_TY / LM_STRIP)), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_lm_hist_kernel, dim3(256), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_lm_topk_kernel, dim3(256), dim3(256), 0, st, g);
    hipError_t e = gftt_sort_topk(g, sort_tmp, sort_tmp_bytes, st);
    if (e != hipSuccess) return e;
    return launch_select(g, (const unsigned long long*)g.topk_sorted, (const unsigned int*)g.n_top, g.topk_cap, 1, st);
}
hipError_t launch_gftt_presort(const GfArgs& g, hipStream_t st) {
    // grid sizes (experiment overrides VIO_TRK_HIST_WGS / VIO_TRK_TOPK_WGS): the histogram on 128 workgroups -- half
    // the workgroups' LDS-histogram flushes beside the RANSAC kernels: config-1 pipeline 0.166-0.169 -> 0.160-0.164
    // ms (64: 0.165, 32: 0.179, 512: 0.179; profiles/r6l_ab_hist_grid.log); the gather stays at 256
    static const int hw = [] { const char* v = std::getenv("VIO_TRK_HIST_WGS"); return v ? std::max(1, std::atoi(v)) : 128; }();
    static const int tw = [] { const char* v = std::getenv("VIO_TRK_TOPK_WGS"); return v ? std::max(1, std::atoi(v)) : 256; }();
    hipLaunchKernelGGL(gftt_lm_hist_kernel, dim3(hw), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_lm_topk_kernel, dim3(tw), dim3(256), 0, st, g);
    hipLaunchKernelGGL(gftt_topk_sort_kernel<8>, dim3((g.topk_cap + 63) / 64), dim3(64 * 8), 0, st, g);
    return hipGetLastError();
}
hipError_t launch_gftt_presel(const GfArgs& g, const unsigned long long* keys, const unsigned int* n_keys,
                              hipStream_t st) {
    return launch_select(g, keys, n_keys, g.topk_cap, 1, st);
}
hipError_t launch_gftt_flatten(const GfArgs& g, hipStream_t st) {
    hipLaunchKernelGGL(gftt_lm_flatten_kernel, dim3(256), dim3(256), 0, st, g);
    return hipGetLastError();
}
// exact fallback: sort every candidate slot (unused slots hold 0 and sort to the end) and redo the
// greedy pass from the strongest candidate
hipError_t launch_gftt_full(const GfArgs& g, unsigned int count, void* sort_tmp, size_t sort_tmp_bytes,
                            hipStream_t st) {
    size_t tb = sort_tmp_bytes;
    count = count < g.cand_cap ? count : g.cand_cap;
    hipError_t e = hipcub::DeviceRadixSort::SortKeysDescending(sort_tmp, tb, g.cand, g.cand_sorted, (int)count, 0, 64,
                                                               st);
    if (e != hipSuccess) return e;
    return launch_select(g, (const unsigned long long*)g.cand_sorted, (const unsigned int*)g.n_cand, g.cand_cap, 0, st);
}
size_t gftt_sort_tmp_bytes(unsigned int cap) {
    size_t tb = 0;
    (void)hipcub::DeviceRadixSort::SortKeysDescending((void*)nullptr, tb, (unsigned long long*)nullptr,
                                                (unsigned long long*)nullptr, (int)cap, 0, 64, (hipStream_t)0);
    return tb;
}
// the dynamic-LDS limit only grows (per device, under a lock): trackers of different sizes on one
// device, on one or several host threads, never lower the limit another one launches with
hipError_t gftt_select_set_lds(size_t bytes) {
    static std::mutex mu;
    static size_t cur[64] = {};
    std::lock_guard<std::mutex> lock(mu);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (bytes <= cur[dev]) return hipSuccess;
    const void* fns[4] = {(const void*)gftt_select_kernel<false, false>, (const void*)gftt_select_kernel<false, true>,
                          (const void*)gftt_select_kernel<true, false>, (const void*)gftt_select_kernel<true, true>};
    for (const void* f : fns) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) return e;
    }
    cur[dev] = bytes;
    return hipSuccess;
}

}  // namespace vio360
