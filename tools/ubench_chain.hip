// Dev micro-benchmark: per-step latency of the building blocks on the 32x32 factor's chain
// (single wave, s_memtime cycles). Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <int MODE>
__global__ void k_chain(const double* in, double* out, unsigned long long* cyc, int n) {
  const int lane = threadIdx.x;
  double x = in[lane];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (MODE == 0) {  // rsq + Newton chain
      double r = __builtin_amdgcn_rsq(x);
      r = r * (1.5 - 0.5 * x * r * r);
      x = r + 1.0;
    } else if (MODE == 1) {  // readlane chain
      x = rlane(x, i & 63) * 1.0000001 + 0.5;
    } else if (MODE == 2) {  // fma chain
      x = x * 1.0000001 + 0.5;
    } else if (MODE == 3) {  // readlane -> rsq -> newton -> mul -> readlane -> fma
      const double d = rlane(x, i & 31) + 2.0;
      double r = __builtin_amdgcn_rsq(d);
      r = r * (1.5 - 0.5 * d * r * r);
      const double l = x * r;
      x = x - l * rlane(l, (i + 1) & 31);
    } else if (MODE == 4) {  // sqrt-based reciprocal
      x = 1.0 / sqrt(x) + 1.0;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = x;
  if (lane == 0) cyc[MODE] = t1 - t0;
}
int main() {
  double *in, *out; unsigned long long* cyc;
  CK(hipMalloc(&in, 64 * 8)); CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&cyc, 64));
  double h[64]; for (int i = 0; i < 64; ++i) h[i] = 1.0 + i * 0.01;
  CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
  const int n = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_chain<0>, 1, 64, 0, 0, in, out, cyc, n);
    hipLaunchKernelGGL(k_chain<1>, 1, 64, 0, 0, in, out, cyc, n);
    hipLaunchKernelGGL(k_chain<2>, 1, 64, 0, 0, in, out, cyc, n);
    hipLaunchKernelGGL(k_chain<3>, 1, 64, 0, 0, in, out, cyc, n);
    hipLaunchKernelGGL(k_chain<4>, 1, 64, 0, 0, in, out, cyc, n);
    CK(hipDeviceSynchronize());
  }
  unsigned long long c[8]; CK(hipMemcpy(c, cyc, 64, hipMemcpyDeviceToHost));
  const char* names[] = {"rsq+newton", "readlane+fma", "fma", "pivot chain", "1/sqrt"};
  for (int m = 0; m < 5; ++m) printf("%-14s %7.1f cycles/step\n", names[m], (double)c[m] / n);
  return 0;
}
