// Measured roofline peaks of the GPU this library runs on (bench.py prints every roofline fraction against both the
// spec peaks of MI355X_MICROARCH.md and these): a streaming HBM copy and the FP64 MFMA / VALU issue rates.
//   HBM:  16-byte-per-lane grid-stride copy of a buffer far larger than the 256 MB Infinity Cache; bytes = read +
//         written per pass (the guide's "float4 copy" measurement, 6.29 TB/s there).
//   MFMA: v_mfma_f64_16x16x4f64 with 8 independent accumulators per wave and no memory traffic (2048 flop each).
//   VALU: v_fma_f64 with 8 independent chains per lane.
// Each figure is the best of several timed launches after one warm-up launch (HIP events on a private stream).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"

namespace g2ohip {
namespace {

typedef double pdx4 __attribute__((ext_vector_type(4)));
typedef double pdx2 __attribute__((ext_vector_type(2)));

// U pieces of 16 B in flight per thread per iteration; NT: nontemporal loads and stores (no L2 / MALL allocation)
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_peak_copy(const pdx2* __restrict__ in, pdx2* __restrict__ out, long long n) {
  const long long stride = (long long)gridDim.x * 256 * U;
  for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
    pdx2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long k = i + 256LL * u;
      if (k < n) v[u] = NT ? __builtin_nontemporal_load(in + k) : in[k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long k = i + 256LL * u;
      if (k < n) {
        if (NT) __builtin_nontemporal_store(v[u], out + k);
        else out[k] = v[u];
      }
    }
  }
}

constexpr int PEAK_NACC = 8;
__global__ void __launch_bounds__(256) k_peak_mfma(double* out, int iters, double seed) {
  pdx4 acc[PEAK_NACC];
#pragma unroll
  for (int i = 0; i < PEAK_NACC; ++i) acc[i] = pdx4{0.0, 0.0, 0.0, 0.0};
  const double a = seed + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < PEAK_NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < PEAK_NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[blockIdx.x * 256 + threadIdx.x] = s;  // keeps the loop alive; never true in practice
}

__global__ void __launch_bounds__(256) k_peak_valu(double* out, int iters, double seed) {
  double x[PEAK_NACC];
#pragma unroll
  for (int i = 0; i < PEAK_NACC; ++i) x[i] = seed + threadIdx.x * 1e-3 + i;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < PEAK_NACC; ++i) x[i] = __builtin_fma(x[i], m, c);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < PEAK_NACC; ++i) s += x[i];
  if (s == 12345.678) out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class F>
double best_ms(hipStream_t s, int reps, F launch) {
  hipEvent_t a, b;
  HIP_CHECK(hipEventCreate(&a));
  HIP_CHECK(hipEventCreate(&b));
  launch();  // warm-up (clocks, code object, TLB)
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    HIP_CHECK(hipEventRecord(a, s));
    launch();
    HIP_CHECK(hipEventRecord(b, s));
    HIP_CHECK(hipEventSynchronize(b));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  HIP_CHECK(hipEventDestroy(a));
  HIP_CHECK(hipEventDestroy(b));
  return best;
}

}  // namespace

namespace launch {
// out[0] HBM copy GB/s (read + write bytes), out[1] FP64 MFMA TFLOP/s, out[2] FP64 VALU TFLOP/s, out[3] CUs
void measure_peaks(int device, double* out) {
  HIP_CHECK(hipSetDevice(device));
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, device));
  const int cus = p.multiProcessorCount;
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  {
    const long long bytes = 2LL << 30;  // 2 GiB each way: 8x the Infinity Cache
    const long long n = bytes / (long long)sizeof(pdx2);
    DevBuf<pdx2> in(n), o(n);
    HIP_CHECK(hipMemsetAsync(in.get(), 0, bytes, s));
    // the best of a few shapes (pieces in flight per thread, grid, nontemporal)
    double best = 1e30;
    auto tryc = [&](auto kern, int grid, int U) {
      (void)U;
      best = std::min(best, best_ms(s, 3, [&] {
        hipLaunchKernelGGL(kern, grid, 256, 0, s, in.get(), o.get(), n);
        KERNEL_CHECK();
      }));
    };
    tryc(k_peak_copy<2, false>, cus * 16, 2);
    tryc(k_peak_copy<4, false>, cus * 8, 4);
    tryc(k_peak_copy<4, true>, cus * 8, 4);
    tryc(k_peak_copy<8, true>, cus * 4, 8);
    out[0] = 2.0 * bytes / (best * 1e-3) / 1e9;
  }
  {
    DevBuf<double> sink((size_t)cus * 8 * 256);
    const int grid = cus * 8, iters = 4000;  // 2 waves per SIMD
    const double ms = best_ms(s, 5, [&] {
      hipLaunchKernelGGL(k_peak_mfma, grid, 256, 0, s, sink.get(), iters, 0.5);
      KERNEL_CHECK();
    });
    out[1] = (double)grid * 4 * iters * PEAK_NACC * 2048.0 / (ms * 1e-3) / 1e12;
    const double mv = best_ms(s, 5, [&] {
      hipLaunchKernelGGL(k_peak_valu, grid, 256, 0, s, sink.get(), iters, 0.5);
      KERNEL_CHECK();
    });
    out[2] = (double)grid * 256 * iters * PEAK_NACC * 2.0 / (mv * 1e-3) / 1e12;
  }
  out[3] = cus;
  HIP_CHECK(hipStreamDestroy(s));
}
}  // namespace launch
}  // namespace g2ohip
