// Micro-probe: do the device's f32 sqrt / division and f64 sin / cos (rounded to f32) agree bitwise
// with the host's?  (The IMU preintegration parity depends on it.)  Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>
__global__ void k(const float* x, const float* y, float* o, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    o[6 * i + 0] = __fsqrt_rn(x[i]);
    o[6 * i + 1] = y[i] / x[i];
    o[6 * i + 2] = (float)sin((double)x[i]);
    o[6 * i + 3] = (float)cos((double)x[i]);
    o[6 * i + 4] = sqrtf(x[i]);
    o[6 * i + 5] = (1.f - (float)cos((double)x[i])) / x[i];
}
int main() {
    const int n = 1 << 20;
    std::vector<float> x(n), y(n), o(6 * n);
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        x[i] = 1e-6f + (s >> 8) * (0.5f / 16777216.f);
        s = s * 1664525u + 1013904223u;
        y[i] = -1.f + (s >> 8) * (2.f / 16777216.f);
    }
    float *dx, *dy, *dout;
    hipMalloc(&dx, 4 * n); hipMalloc(&dy, 4 * n); hipMalloc(&dout, 24 * n);
    hipMemcpy(dx, x.data(), 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(dy, y.data(), 4 * n, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, dy, dout, n);
    hipMemcpy(o.data(), dout, 24 * n, hipMemcpyDeviceToHost);
    int bad[6] = {0};
    for (int i = 0; i < n; ++i) {
        float h[6] = {sqrtf(x[i]), y[i] / x[i], (float)sin((double)x[i]), (float)cos((double)x[i]), sqrtf(x[i]),
                      (1.f - (float)cos((double)x[i])) / x[i]};
        for (int j = 0; j < 6; ++j)
            if (memcmp(&h[j], &o[6 * i + j], 4)) {
                if (bad[j] < 3) printf("op %d x=%.9g dev=%.9g host=%.9g\n", j, x[i], o[6 * i + j], h[j]);
                bad[j]++;
            }
    }
    printf("mismatches of %d: fsqrt_rn %d div %d sin %d cos %d sqrtf %d (1-cos)/x %d\n", n, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5]);
    return 0;
}
