// Dev probe: the lane layout of v_mfma_f64_4x4x4f64 (four independent 4x4x4 blocks per instruction) on gfx950, found
// by experiment rather than assumed. For every candidate assignment of (block, row, k) / (block, k, col) /
// (block, row, col) to lanes, one random product per block is computed on the device and checked on the host; the
// candidates that reproduce every block are printed. Also times a dependent and an independent issue loop.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mfma4x4.hip -o tools/ubench_mfma4x4
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

typedef double dx1 __attribute__((ext_vector_type(1)));

__global__ void k_one(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(A[l], B[l], 0.0, 0, 0, 0);
  D[l] = d;
}

template <int NACC>
__global__ void k_rate(double* out, int iters) {
  const int l = threadIdx.x & 63;
  double a = 1.0 + 1e-9 * l, b = 1.0 - 1e-9 * l;
  double acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// lane of (b, x, y) under a candidate: 16 b + perm of (x, y) in {x + 4 y, y + 4 x}, or the block index inside
static int lane_of(int cand, int b, int x, int y) {
  switch (cand) {
    case 0: return 16 * b + x + 4 * y;
    case 1: return 16 * b + y + 4 * x;
    case 2: return b + 4 * x + 16 * y;
    case 3: return b + 4 * y + 16 * x;
    case 4: return x + 4 * b + 16 * y;
    default: return y + 4 * b + 16 * x;
  }
}

int main() {
  std::vector<double> hA(64), hB(64), hD(64);
  for (int i = 0; i < 64; ++i) {
    hA[i] = std::sin(1.0 + 1.7 * i);
    hB[i] = std::cos(0.3 + 2.3 * i);
  }
  double *A, *B, *D, *O;
  (void)hipMalloc(&A, 64 * 8);
  (void)hipMalloc(&B, 64 * 8);
  (void)hipMalloc(&D, 64 * 8);
  (void)hipMalloc(&O, 1024 * 256 * 8);
  (void)hipMemcpy(A, hA.data(), 64 * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(B, hB.data(), 64 * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_one, 1, 64, 0, 0, A, B, D);
  (void)hipMemcpy(hD.data(), D, 64 * 8, hipMemcpyDeviceToHost);
  int found = 0;
  for (int ca = 0; ca < 6; ++ca)      // A: (b, i, k) -> lane_of(ca, b, i, k)
    for (int cb = 0; cb < 6; ++cb)    // B: (b, k, j) -> lane_of(cb, b, k, j)
      for (int cd = 0; cd < 6; ++cd) {  // D: (b, i, j) -> lane_of(cd, b, i, j)
        double err = 0.0;
        for (int b = 0; b < 4; ++b)
          for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
              double s = 0.0;
              for (int k = 0; k < 4; ++k) s += hA[lane_of(ca, b, i, k)] * hB[lane_of(cb, b, k, j)];
              err = std::fmax(err, std::fabs(s - hD[lane_of(cd, b, i, j)]));
            }
        if (err < 1e-12) {
          printf("layout: A(b,i,k) cand %d, B(b,k,j) cand %d, D(b,i,j) cand %d  (max err %.1e)\n", ca, cb, cd, err);
          ++found;
        }
      }
  if (!found) {
    printf("no candidate layout matched; raw D:");
    for (int l = 0; l < 64; ++l) printf(" %.4f", hD[l]);
    printf("\nA:");
    for (int l = 0; l < 64; ++l) printf(" %.4f", hA[l]);
    printf("\nB:");
    for (int l = 0; l < 64; ++l) printf(" %.4f", hB[l]);
    printf("\n");
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 4096, grid = 1024;
  auto rate = [&](auto kern, int nacc, const char* name) {
    hipLaunchKernelGGL(kern, grid, 256, 0, 0, O, 16);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern, grid, 256, 0, 0, O, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fl = 2.0 * 256 * (double)grid * 4 * iters * nacc;  // 4 waves x 256 FMA per instruction
    printf("%-34s %8.3f ms  %6.2f TF/s  %.1f cycles per instruction per SIMD at 2.4 GHz\n", name, ms, fl / (ms * 1e-3) / 1e12,
           (ms * 1e-3 * 2.4e9) / ((double)grid * 4 / 1024.0 * iters * nacc));
  };
  rate(k_rate<1>, 1, "4x4x4 f64, 1 accumulator (dependent)");
  rate(k_rate<4>, 4, "4x4x4 f64, 4 accumulators");
  rate(k_rate<16>, 16, "4x4x4 f64, 16 accumulators");
  return 0;
}
