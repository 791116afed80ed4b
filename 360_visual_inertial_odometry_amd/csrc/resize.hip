// resize.hip — cv::resize(..., INTER_AREA) of the grayscale ERP frames before tracking.
//
// Reference: app/main.cpp:199-204 resizes every frame to (camera_width, camera_height) with
// INTER_AREA when the image size differs (3840x1920 -> 960x480 in the demo configuration).
// OpenCV 4.x takes its integer-factor "area fast" path there (modules/imgproc/src/resize.cpp,
// resizeAreaFast_ for uchar): dst = saturate_cast<uchar>(Σ block · (1.f / (fx·fy))), i.e. the block
// sum times the f32 reciprocal, rounded half-to-even — except 2x2 blocks, which OpenCV's
// ResizeAreaFastVec handles as (a + b + c + d + 2) >> 2 (round half up).  Integer factors only (fx = W / dW,
// fy = H / dH exact); other sizes return VIO_ENOSYS.  OpenCV is not in /root/reference nor in
// this image, so parity with it is unpinned; the oracle restates that formula
// (oracle/resize_oracle.py) and the GPU matches it bitwise.
//
// Roofline: HBM-bound streaming, 1 + 1/(fx·fy) bytes per source pixel.  The factor-4 fast path gives
// each lane 4 output pixels on two output rows: eight 16-byte non-temporal row loads (two 16x4
// source blocks), no LDS; the grid covers (output row pair, 4-pixel group, frame).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ctx.h"

namespace vio360 {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct ResizeArgs {
    const uint8_t* src;
    int W, H, stride;
    long long frame_bytes_src;
    uint8_t* dst;
    int dW, dH, dstride;
    long long frame_bytes_dst;
    int fx, fy;
    float scale;  // 1.f / (fx * fy)
};

__device__ __forceinline__ uint8_t area_round(int sum, float scale) {
    const float v = rintf((float)sum * scale);  // cvRound: half to even
    return (uint8_t)fminf(fmaxf(v, 0.f), 255.f);
}

__device__ __forceinline__ int sum_bytes4(uint32_t w) {
    return (int)(w & 0xff) + (int)((w >> 8) & 0xff) + (int)((w >> 16) & 0xff) + (int)(w >> 24);
}

// fx = fy = 4, dst width a multiple of 4, dst height even and 16-byte aligned source rows: lane ->
// 4 output pixels on each of two output rows (eight 16-byte streaming loads in flight per lane)
__global__ __launch_bounds__(256) void resize_area4_kernel(ResizeArgs a) {
    const int groups = a.dW >> 2;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int y0 = 2 * blockIdx.y;
    const int f = blockIdx.z;
    if (g >= groups) return;
    const uint8_t* s = a.src + f * a.frame_bytes_src + (long long)(4 * y0) * a.stride + 16 * g;
    u32x4 r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s + (long long)k * a.stride));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t out = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            int sum = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 v = r[4 * h + k];
                const uint32_t w = c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
                sum += sum_bytes4(w);
            }
            out |= (uint32_t)area_round(sum, a.scale) << (8 * c);
        }
        *reinterpret_cast<uint32_t*>(a.dst + f * a.frame_bytes_dst + (long long)(y0 + h) * a.dstride + 4 * g) = out;
    }
}

// any integer factors: lane -> 1 output pixel
__global__ __launch_bounds__(256) void resize_area_kernel(ResizeArgs a) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int f = blockIdx.z;
    if (x >= a.dW) return;
    const uint8_t* s = a.src + f * a.frame_bytes_src + (long long)(a.fy * y) * a.stride + a.fx * x;
    int sum = 0;
    for (int k = 0; k < a.fy; ++k)
        for (int j = 0; j < a.fx; ++j) sum += s[(long long)k * a.stride + j];
    // 2x2: ResizeAreaFastVec's (sum + 2) >> 2; every other factor: sum * (1.f / (fx fy)), cvRound
    a.dst[f * a.frame_bytes_dst + (long long)y * a.dstride + x] =
        (a.fx == 2 && a.fy == 2) ? (uint8_t)((sum + 2) >> 2) : area_round(sum, a.scale);
}

}  // namespace vio360

using namespace vio360;

static int resize_check(int W, int H, int stride, int dW, int dH, int dstride, int n_frames) {
    if (W <= 0 || H <= 0 || dW <= 0 || dH <= 0 || stride < W || dstride < dW || n_frames < 0) return VIO_EINVAL;
    if (W % dW || H % dH) return VIO_ENOSYS;
    if ((long long)(W / dW) * (H / dH) > (1 << 23)) return VIO_ENOSYS;  // int block sums
    return VIO_OK;
}

extern "C" int erp_resize_area_device(vio_ctx* ctx, const uint8_t* src, int W, int H, int stride, int n_frames,
                                      uint8_t* dst, int dW, int dH, int dst_stride) {
    if (!ctx || !src || !dst) return VIO_EINVAL;
    int rc = resize_check(W, H, stride, dW, dH, dst_stride, n_frames);
    if (rc) {
        set_error(ctx, rc == VIO_ENOSYS ? "erp_resize_area: only integer downscale factors are supported"
                                        : "erp_resize_area: bad sizes");
        return rc;
    }
    if (n_frames == 0) return VIO_OK;
    ResizeArgs a;
    a.src = src;
    a.W = W;
    a.H = H;
    a.stride = stride;
    a.frame_bytes_src = (long long)stride * H;
    a.dst = dst;
    a.dW = dW;
    a.dH = dH;
    a.dstride = dst_stride;
    a.frame_bytes_dst = (long long)dst_stride * dH;
    a.fx = W / dW;
    a.fy = H / dH;
    a.scale = 1.f / (float)(a.fx * a.fy);
    VIO_DEVICE(ctx);
    for (hipEvent_t& ev : ctx->rsz_ev)
        if (!ev) VIO_HIP(ctx, hipEventCreate(&ev));
    VIO_HIP(ctx, hipEventRecord(ctx->rsz_ev[0], ctx->stream));
    const bool fast = a.fx == 4 && a.fy == 4 && dW % 4 == 0 && dH % 2 == 0 && stride % 16 == 0 && dst_stride % 4 == 0 &&
                      (reinterpret_cast<uintptr_t>(src) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 3) == 0;
    if (fast) {
        const int groups = dW / 4;
        hipLaunchKernelGGL(resize_area4_kernel, dim3((groups + 255) / 256, dH / 2, n_frames), dim3(256), 0, ctx->stream,
                           a);
    } else {
        hipLaunchKernelGGL(resize_area_kernel, dim3((dW + 255) / 256, dH, n_frames), dim3(256), 0, ctx->stream, a);
    }
    VIO_HIP(ctx, hipGetLastError());
    VIO_HIP(ctx, hipEventRecord(ctx->rsz_ev[1], ctx->stream));
    return VIO_OK;
}

extern "C" int erp_resize_area(vio_ctx* ctx, const uint8_t* src, int W, int H, int stride, uint8_t* dst, int dW,
                               int dH, int dst_stride) {
    if (!ctx || !src || !dst) return VIO_EINVAL;
    int rc = resize_check(W, H, stride, dW, dH, dst_stride, 1);
    if (rc) {
        set_error(ctx, rc == VIO_ENOSYS ? "erp_resize_area: only integer downscale factors are supported"
                                        : "erp_resize_area: bad sizes");
        return rc;
    }
    // device copies with 16-byte-aligned pitches (fast path)
    const int sp = (W + 15) & ~15, dp = (dW + 3) & ~3;
    uint8_t* d_src = static_cast<uint8_t*>(ctx_buffer(ctx, kSlotResizeSrc, (size_t)sp * H));
    uint8_t* d_dst = static_cast<uint8_t*>(ctx_buffer(ctx, kSlotResizeDst, (size_t)dp * dH));
    if (!d_src || !d_dst) {
        set_error(ctx, "erp_resize_area: device allocation failed");
        return VIO_ENOMEM;
    }
    VIO_DEVICE(ctx);
    VIO_HIP(ctx, hipMemcpy2DAsync(d_src, sp, src, stride, W, H, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = erp_resize_area_device(ctx, d_src, W, H, sp, 1, d_dst, dW, dH, dp))) return rc;
    VIO_HIP(ctx, hipMemcpy2DAsync(dst, dst_stride, d_dst, dp, dW, dH, hipMemcpyDeviceToHost, ctx->stream));
    VIO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return VIO_OK;
}

extern "C" int erp_resize_area_kernel_ms(vio_ctx* ctx, double* ms) {
    if (!ctx || !ms || !ctx->rsz_ev[1]) return VIO_EINVAL;
    float f = 0.f;
    VIO_HIP(ctx, hipEventSynchronize(ctx->rsz_ev[1]));
    VIO_HIP(ctx, hipEventElapsedTime(&f, ctx->rsz_ev[0], ctx->rsz_ev[1]));
    *ms = f;
    return VIO_OK;
}
