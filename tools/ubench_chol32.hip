// Dev micro-benchmark: the 32x32 diagonal factor (cholesky.hip chol32) in isolation, one wave,
// s_memtime cycles per call, with variants switched off to see what the time is made of.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int NB = 32;
__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// V bits: 1 no deferred update, 2 no look-ahead, 4 no forward solve, 8 no Newton
template <int V>
__device__ __forceinline__ bool chol32(double (&row)[NB], double& y, int lane, double* col, double* dinv) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double2 cc[NB / 2];
    const int c0 = (j + 2) & ~1;
    if (j >= 1 && !(V & 1)) {
      const double* cb = col + ((j - 1) & 1) * 2 * NB;
#pragma unroll
      for (int c = c0; c < NB; c += 2) cc[c >> 1] = *reinterpret_cast<const double2*>(cb + c);
    }
    const double djj = rlane(row[j], j);
    ok &= djj > 0.0;
    const double d = djj > 0.0 ? djj : 1.0;
    double r = __builtin_amdgcn_rsq(d);
    if (!(V & 8)) r = r * (1.5 - 0.5 * d * r * r);
    const double lj = row[j] * r;
    row[j] = lj;
    if (j + 1 < NB) {
      if (!(V & 2)) {
        row[j + 1] -= lj * rlane(lj, j + 1);
        if (j + 2 < NB) row[j + 2] -= lj * rlane(lj, j + 2);
      }
      col[(j & 1) * 2 * NB + lane] = lj;
    }
    if (!(V & 4)) {
      const double yj = rlane(y, j) * r;
      y = lane == j ? yj : (lane > j ? y - lj * yj : y);
    }
    if (j >= 1 && !(V & 1)) {
      const double lp = row[j - 1];
#pragma unroll
      for (int c = c0; c < NB; c += 2) {
        if (c > j + 1) row[c] -= lp * cc[c >> 1].x;
        row[c + 1] -= lp * cc[c >> 1].y;
      }
    }
#pragma unroll
    for (int c = j + 1; c < NB; ++c) asm volatile("" : "+v"(row[c]));
  }
  return ok;
}
template <int V>
__global__ void __launch_bounds__(64) k_bench(const double* A, double* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  __shared__ double dinv[NB];
  const int lane = threadIdx.x;
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? A[lane * NB + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
  double y = lane < NB ? 1.0 : 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok = chol32<V>(row, y, lane, col, dinv);
  asm volatile("" : "+v"(row[NB - 1]), "+v"(y));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = y + (ok ? 0.0 : 1.0);
#pragma unroll
  for (int c = 0; c < NB; ++c) s += row[c];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int V>
int run(const double* A, double* out, unsigned long long* cyc, const char* name) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL(k_bench<V>, 1, 64, 0, 0, A, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    if (c < best) best = c;
  }
  printf("%-28s %7llu cycles  (%5.1f per column)\n", name, best, best / 32.0);
  return 0;
}
int main() {
  double h[NB * NB];
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) h[i * NB + j] = (i == j ? NB + 1.0 : 0.0) + 1.0 / (1 + i + j);
  double *A, *out; unsigned long long* cyc;
  CK(hipMalloc(&A, sizeof h)); CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&cyc, 8));
  CK(hipMemcpy(A, h, sizeof h, hipMemcpyHostToDevice));
  run<0>(A, out, cyc, "full");
  run<8>(A, out, cyc, "no Newton");
  run<4>(A, out, cyc, "no forward solve");
  run<2>(A, out, cyc, "no look-ahead (wrong)");
  run<1>(A, out, cyc, "no deferred update (wrong)");
  run<3>(A, out, cyc, "pivot chain only (wrong)");
  run<15>(A, out, cyc, "bare (wrong)");
  return 0;
}
