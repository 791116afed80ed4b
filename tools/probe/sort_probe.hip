// Micro-probe: one-workgroup bitonic sort of 8192 u64 keys (GFTT top-K), time per stage class.
// Diagnostic only (tools/, not shipped).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

template <int J>
__device__ __forceinline__ void bitonic_regs(unsigned long long (&v)[16], unsigned int base, unsigned int k) {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        if (e & J) continue;
        const unsigned long long a = v[e], b = v[e | J];
        const bool desc = ((base + e) & k) == 0;
        const bool sw = desc ? a < b : a > b;
        v[e] = sw ? b : a;
        v[e | J] = sw ? a : b;
    }
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long x, int m) {
    const int lo = __shfl_xor((int)(unsigned int)x, m, 64), hi = __shfl_xor((int)(unsigned int)(x >> 32), m, 64);
    return ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
}
__global__ void __launch_bounds__(1024) sortk(const unsigned long long* keys, unsigned int n, unsigned long long* out,
                                              int mode, long long* cyc) {
    extern __shared__ unsigned long long sk[];
    unsigned int P = 16;
    while (P < n) P <<= 1;
    const unsigned int t = threadIdx.x, T = P >> 4, base = 16 * t;
    const bool act = t < T;
    unsigned long long v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = act && base + e < n ? keys[base + e] : 0ull;
    long long c[3] = {0, 0, 0};
    for (unsigned int k = 2; k <= P; k <<= 1) {
        for (unsigned int j = k >> 1; j > 0; j >>= 1) {
            int cls;
            if (j >= 1024) {
                cls = 2;
                if (mode & 4) {
                __syncthreads();
                if (act) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) sk[base + e] = v[e];
                }
                __syncthreads();
                if (act) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        const unsigned int i = base + e, lo = i & ~j;
                        const unsigned long long p = sk[i ^ j];
                        const bool keep_max = ((lo & k) == 0) == (i == lo);
                        v[e] = keep_max ? (v[e] > p ? v[e] : p) : (v[e] < p ? v[e] : p);
                    }
                }
                }
            } else if (j >= 16) {
                cls = 1;
                if (mode & 2) {
                const int m = (int)(j >> 4);
                const bool is_lo = (t & (unsigned int)m) == 0;
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const unsigned long long p = shfl_xor_u64(v[e], m);
                    const unsigned int lo = (base + e) & ~j;
                    const bool keep_max = ((lo & k) == 0) == is_lo;
                    v[e] = keep_max ? (v[e] > p ? v[e] : p) : (v[e] < p ? v[e] : p);
                }
                }
            } else {
                cls = 0;
                if (mode & 1) {
                switch (j) {
                    case 8: bitonic_regs<8>(v, base, k); break;
                    case 4: bitonic_regs<4>(v, base, k); break;
                    case 2: bitonic_regs<2>(v, base, k); break;
                    default: bitonic_regs<1>(v, base, k); break;
                }
                }
            }
            c[cls] += 1;
        }
    }
    if (act) {
#pragma unroll
        for (int e = 0; e < 16; ++e)
            if (base + e < n) out[base + e] = v[e];
    }
    if (t == 0) { cyc[0] = c[0]; cyc[1] = c[1]; cyc[2] = c[2]; }
}
int main() {
    const unsigned int n = 6609;
    std::vector<unsigned long long> h(n);
    srand(1);
    for (auto& x : h) x = ((unsigned long long)rand() << 32) | (unsigned long long)rand();
    unsigned long long *dk, *dout;
    long long* dc;
    (void)hipMalloc(&dk, n * 8);
    (void)hipMalloc(&dout, n * 8);
    (void)hipMalloc(&dc, 64);
    (void)hipMemcpy(dk, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipFuncSetAttribute((const void*)sortk, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    for (int mode : {7, 1, 2, 4, 0, 8}) {
        const size_t lds = mode == 8 ? 0 : 65536;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        sortk<<<1, 1024, lds>>>(dk, n, dout, mode, dc);
        (void)hipEventRecord(e0);
        sortk<<<1, 1024, lds>>>(dk, n, dout, mode, dc);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        long long c[3];
        (void)hipMemcpy(c, dc, 24, hipMemcpyDeviceToHost);
        std::vector<unsigned long long> o(n);
        (void)hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost);
        std::vector<unsigned long long> r = h;
        std::sort(r.begin(), r.end(), [](auto a, auto b) { return a > b; });
        printf("mode %d: %.1f us; cycles regs %lld shfl %lld lds %lld; sorted %s\n", mode, ms * 1e3, c[0], c[1], c[2],
               o == r ? "yes" : "no");
    }
    return 0;
}
