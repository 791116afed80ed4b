// Micro-probe: shader-clock latency of the operations on the window Cholesky's pivot chain -- a dependent
// f64 FMA, rsq + two Newton steps (chol_dev.h rsq_nr), a v_readlane broadcast of a double, an LDS
// write -> wave sync -> broadcast read round trip, a 4-wave s_barrier, a 1-wave s_barrier.  Each is a
// chain of R dependent repetitions timed with s_memtime by lane 0 of wave 0; cycles per repetition.
// Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../360_visual_inertial_odometry_amd/csrc/chol_dev.h"

using namespace vio360;

template <int V>
__global__ void __launch_bounds__(256, 1) lat(double seed, int R, double* out, unsigned long long* cyc) {
    __shared__ double buf[2][64];
    const int lane = threadIdx.x & 63;
    double v = seed + lane * 1e-3;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < R; ++r) {
        if (V == 0) {  // dependent f64 fma
            v = fma(v, 0.999999, 1e-7);
        } else if (V == 1) {  // rsq + Newton chain
            v = rsq_nr(v) + 1.0;
        } else if (V == 2) {  // readlane broadcast chain
            v = readlane_d(v, (r & 63)) * 0.5 + 0.5;
        } else if (V == 3) {  // LDS publish -> wave sync -> read another lane's value
            buf[r & 1][lane] = v;
            wave_lds_sync();
            v = buf[r & 1][(lane + 1) & 63] * 0.5 + 0.5;
        } else if (V == 4) {  // 4-wave barrier with an LDS exchange
            buf[r & 1][lane] = v;
            __syncthreads();
            v = buf[r & 1][(lane + 1) & 63] * 0.5 + 0.5;
        } else if (V == 5) {  // 4-wave bare barrier
            __syncthreads();
            v = v * 0.5 + 0.5;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) *cyc = (t1 - t0);
    out[threadIdx.x] = v;
}

int main() {
    const int R = 4096;
    double* d;
    unsigned long long* c;
    hipMalloc(&d, 256 * 8);
    hipMalloc(&c, 8);
    void (*fns[6])(double, int, double*, unsigned long long*) = {lat<0>, lat<1>, lat<2>, lat<3>, lat<4>, lat<5>};
    const char* names[6] = {"f64 fma (dependent)", "rsq_nr chain", "readlane_d chain", "lds write+wave sync+read",
                            "lds write+__syncthreads (4 waves)+read", "__syncthreads (4 waves)"};
    for (int v = 0; v < 6; ++v) {
        unsigned long long cyc = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(fns[v], dim3(1), dim3(256), 0, 0, 1.5, R, d, c);
            if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 1; }
            if (hipMemcpy(&cyc, c, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        }
        printf("%-42s %8.1f cycles per repetition\n", names[v], (double)cyc / R);
    }
    return 0;
}
