// Micro-probe: shader cycles per f64 atan2 / asin / sqrt / division at one wave per SIMD (the BA
// window kernel's occupancy), dependent chains.  Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
__global__ void __launch_bounds__(256) probe(double* out, unsigned long long* cyc, int n, int mode) {
    double x = 0.3 + threadIdx.x * 1e-4, z = 0.9 - threadIdx.x * 1e-4, acc = 0.0;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        double r;
        if (mode == 0) r = atan2(x, z);
        else if (mode == 1) r = asin(x);
        else if (mode == 2) r = sqrt(x);
        else if (mode == 3) r = z / x;
        else if (mode == 4) r = fma(x, z, 0.1);
        else if (mode == 5) {  // 8 dependent FMAs
            double y = x;
#pragma unroll
            for (int j = 0; j < 8; ++j) y = fma(y, z, 0.1);
            r = y;
        } else if (mode == 6) {  // 8 independent FMAs
            double y[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) y[j] = fma(x + j, z, 0.1);
            r = ((y[0] + y[1]) + (y[2] + y[3])) + ((y[4] + y[5]) + (y[6] + y[7]));
        } else if (mode == 7) {  // two independent atan2
            r = atan2(x, z) + atan2(z, x + 0.25);
        } else {  // atan2 + asin independent
            r = atan2(x, z) + asin(0.5 * x);
        }
        acc += r;
        x = 0.5 * x + 1e-3 * r;  // dependent chain
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    double* out;
    unsigned long long* cyc;
    (void)hipMalloc(&out, 256 * 256 * 8);
    (void)hipMalloc(&cyc, 256 * 8);
    const char* names[] = {"atan2", "asin", "sqrt", "div", "fma", "8fma-dep", "8fma-ind", "2atan2", "at+as"};
    const int n = 2000;
    for (int mode = 0; mode < 9; ++mode) {
        probe<<<256, 256>>>(out, cyc, n, mode);
        (void)hipDeviceSynchronize();
        unsigned long long c[256];
        (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < 256; ++i) s += c[i];
        printf("%-9s %.1f cycles per dependent evaluation (1 wave/SIMD)\n", names[mode], s / 256 / n);
    }
    return 0;
}
