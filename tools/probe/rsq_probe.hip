#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
#include "chol_dev.h"
__device__ double rsq_old(double p) { double r = __builtin_amdgcn_rsq(p); const double h = 0.5 * p; r = r * fma(-h * r, r, 1.5); r = r * fma(-h * r, r, 1.5); return r; }
__global__ void k(const double* p, double* o, int n, int v) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) o[i] = v ? rsq_old(p[i]) : vio360::rsq_nr(p[i]); }
int main() {
  const int n = 1 << 20; double *hp = (double*)malloc(n * 8), *ho = (double*)malloc(n * 8);
  srand(1); for (int i = 0; i < n; ++i) hp[i] = ldexp(1.0 + rand() / (double)RAND_MAX, (rand() % 200) - 100);
  double *dp, *dout; hipMalloc(&dp, n * 8); hipMalloc(&dout, n * 8); hipMemcpy(dp, hp, n * 8, hipMemcpyHostToDevice);
  for (int v = 0; v < 2; ++v) {
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dp, dout, n, v); hipMemcpy(ho, dout, n * 8, hipMemcpyDeviceToHost);
  double worst = 0; int over1 = 0;
  for (int i = 0; i < n; ++i) { long double t = 1.0L / sqrtl((long double)hp[i]); double ulp = nextafter((double)t, INFINITY) - (double)t;
    double err = fabs((double)((long double)ho[i] - t)) / ulp; if (err > worst) worst = err; if (err > 1.0) ++over1; }
  printf("%s: worst %.3f ulp, %d of %d above 1 ulp\n", v ? "two Newton steps" : "third-order step", worst, over1, n); }
  return 0; }
