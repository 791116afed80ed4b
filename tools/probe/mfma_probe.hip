// Micro-probe: cycles per v_mfma_f64_16x16x4_f64 (independent / dependent accumulators) and per
// v_fma_f64 at one wave per SIMD.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
using d4 = __attribute__((ext_vector_type(4))) double;
__global__ void __launch_bounds__(1024) probe(double* out, unsigned long long* cyc, int n, int mode) {
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double f[8];
    for (int i = 0; i < 8; ++i) f[i] = i;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {
        for (int i = 0; i < n; ++i) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        }
    } else if (mode == 1) {
        for (int i = 0; i < 4 * n; ++i) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    } else {
        for (int i = 0; i < n; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fma(f[j], b, a);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = c0[0] + c1[1] + c2[2] + c3[3];
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    double* out; unsigned long long* cyc;
    (void)hipMalloc(&out, 256 * 1024 * 8); (void)hipMalloc(&cyc, 256 * 8);
    const int n = 4096;
    for (int mode = 0; mode < 3; ++mode) for (int thr : {256, 512, 1024}) { const int blocks = 256;
        probe<<<blocks, thr>>>(out, cyc, n, mode);
        (void)hipDeviceSynchronize();
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        probe<<<blocks, thr>>>(out, cyc, n, mode);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[256];
        (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
        const double ninst = mode == 2 ? 8.0 * n : 4.0 * n;
        const double flops = (double)blocks * (thr / 64) * ninst * (mode == 2 ? 128.0 : 2048.0);
        printf("mode %d (%s) threads %d: %.1f cycles/instr, wall %.3f ms, %.2f TFLOP/s, memtime/wall %.2f GHz\n", mode,
               mode == 0 ? "mfma f64 4 indep acc" : mode == 1 ? "mfma f64 dependent" : "v_fma_f64 8 chains", thr,
               h[0] / ninst, ms, flops / ms / 1e9, h[0] / (ms * 1e6));
    }
    return 0;
}
