// Dev micro-benchmark: cost of a kernel boundary on a dependent chain vs a device-side handoff between
// two workgroups (same XCD / different XCDs). Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_tiny(double* p, int nwrite) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = i; k < nwrite; k += gridDim.x * blockDim.x) p[k] += 1.0;
}

// ping-pong between block a and block b through a flag word; agent-scope release/acquire
template <int SCOPE>  // 0: workgroup->agent atomics with explicit cache ops (default HIP atomics), 1: relaxed + nothing
__global__ void k_pingpong(unsigned* flag, int iters, int a, int b, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  const int me = blockIdx.x;
  if (me != a && me != b) return;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    const unsigned want = 2 * i + (me == a ? 0 : 1);
    if (SCOPE == 0) {
      while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != want) {}
      __hip_atomic_store(flag, want + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {}
      __hip_atomic_store(flag, want + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (me == a) out[0] = t1 - t0;
}

int main() {
  double* p; CK(hipMalloc(&p, 64 << 20)); CK(hipMemset(p, 0, 64 << 20));
  unsigned* flag; CK(hipMalloc(&flag, 4));
  unsigned long long* out; CK(hipMalloc(&out, 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int N = 400;
  struct { int grid, nwrite; const char* name; } cfg[] = {{1, 64, "1 WG, 512 B"}, {1, 8192, "1 WG, 64 KB"},
      {64, 64 * 4096, "64 WG, 2 MB"}, {300, 300 * 4096, "300 WG, 9.6 MB"}, {1024, 1024 * 4096, "1024 WG, 32 MB"}};
  for (auto& c : cfg) {
    hipLaunchKernelGGL(k_tiny, c.grid, 256, 0, 0, p, c.nwrite);
    CK(hipEventRecord(e0));
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_tiny, c.grid, 256, 0, 0, p, c.nwrite);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("chain of launches, %-16s %6.2f us per launch\n", c.name, ms * 1e3 / N);
  }
  // the same chains captured into a hipGraph and replayed
  for (auto& c : cfg) {
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_tiny, c.grid, 256, 0, st, p, c.nwrite);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st)); CK(hipStreamSynchronize(st));
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("graph of launches, %-16s %6.2f us per launch\n", c.name, ms * 1e3 / N);
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g)); CK(hipStreamDestroy(st));
  }
  const int iters = 2000;
  for (int sc = 0; sc < 2; ++sc)
    for (int pair = 0; pair < 2; ++pair) {
      const int a = 0, b = pair == 0 ? 8 : 1;  // blocks 0 and 8: same XCD (round-robin dispatch); 0 and 1: different
      CK(hipMemset(flag, 0, 4));
      if (sc == 0) hipLaunchKernelGGL(k_pingpong<0>, 16, 64, 0, 0, flag, iters, a, b, out);
      else hipLaunchKernelGGL(k_pingpong<1>, 16, 64, 0, 0, flag, iters, a, b, out);
      CK(hipDeviceSynchronize());
      unsigned long long t; CK(hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost));
      printf("ping-pong %s, %s: %.3f us per one-way handoff\n", sc == 0 ? "acq/rel agent" : "relaxed agent",
             pair == 0 ? "same XCD" : "cross XCD", t / 100.0 / (2.0 * iters));
    }
  return 0;
}
