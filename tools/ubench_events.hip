// Dev micro-benchmark: what a timing event costs on a dependent chain of short kernels. hipEventRecord puts a marker
// between two kernels; hipExtLaunchKernelGGL attaches the event to the kernel's own dispatch. Not product code.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// runs ~`ticks` x 10 ns (s_memrealtime is a 100 MHz counter) on 64 workgroups, then writes one value
__global__ void k_spin(double* p, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {}
  if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

int main() {
  double* p;
  CK(hipMalloc(&p, 1 << 20));
  CK(hipMemset(p, 0, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int N = 400, EVERY = 10, NE = N / EVERY;
  std::vector<hipEvent_t> ev(NE + 1);
  for (auto& evk : ev) CK(hipEventCreate(&evk));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const unsigned long long ticks = 500;  // 5 us per kernel
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < 4; ++mode) {
      // 0: no events, 1: hipEventRecord every EVERY kernels, 2: start event on every EVERY-th dispatch,
      // 3: stop event on every EVERY-th dispatch
      CK(hipEventRecord(t0, s));
      int k = 0;
      for (int i = 0; i < N; ++i) {
        const bool mark = i % EVERY == 0;
        if (mode == 1 && mark) CK(hipEventRecord(ev[k++], s));
        if ((mode == 2 || mode == 3) && mark) {
          hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, mode == 2 ? ev[k] : nullptr,
                                mode == 3 ? ev[k] : nullptr, 0, p, ticks);
          ++k;
        } else {
          hipLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, p, ticks);
        }
      }
      CK(hipEventRecord(t1, s));
      CK(hipEventSynchronize(t1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      float sub = 0;
      if (mode > 0) CK(hipEventElapsedTime(&sub, ev[0], ev[k - 1]));
      printf("rep %d mode %d: %7.2f us per kernel, %2d events, first..last event %8.1f us (%.2f us per kernel)\n", rep,
             mode, ms * 1e3 / N, k, sub * 1e3, sub * 1e3 / ((k - 1) * EVERY));
    }
  }
  // host wait on a stop event attached to a dispatch
  hipExtLaunchKernelGGL(k_spin, dim3(64), dim3(64), 0, s, nullptr, ev[0], 0, p, 100000ULL);
  CK(hipEventSynchronize(ev[0]));
  CK(hipStreamQuery(s));
  printf("host wait on a dispatch stop event: stream idle after hipEventSynchronize: %s\n",
         hipStreamQuery(s) == hipSuccess ? "yes" : "no");
  return 0;
}
