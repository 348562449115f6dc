// Dev micro-benchmark: the GemmNT tile update (gemm_nt.hpp) on one lower-triangular SYRK
// C -= A A^T (m x m, K), TFLOP/s per tile shape, against rocBLAS dsyrk/dgemm on the same sizes, plus an
// fp64 host check of sampled entries. Not product code.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "gemm_nt.hpp"
using namespace g2ohip;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int BM, int BN, int WM, int WN, int OCC, int KC = 16, int XCD = 0>
__global__ void __launch_bounds__(64 * WM * WN, OCC) k_tri(const int* tiles, const double* A, int lda, double* C, int m, int K) {
  extern __shared__ double lds[];
  const int t = tiles[XCD ? xcd_item(blockIdx.x, gridDim.x) : blockIdx.x];
  const int ti = t & 0xffff, tj = t >> 16;
  GemmNT<BM, BN, WM, WN, KC>::run(A, lda, C, m, m, m, ti * BM, tj * BN, 0, K, lds);
}

template <int BM, int BN, int WM = 2, int WN = 2, int OCC = 1, int KC = 16, int XCD = 0>
double run(const double* dA, double* dC, int m, int K, int reps, double* flops_out) {
  std::vector<int> tl;
  for (int tj = 0; tj * BN < m; ++tj)
    for (int ti = 0; ti * BM < m; ++ti)
      if (ti * BM + BM > tj * BN) tl.push_back(ti | (tj << 16));
  int* dt; CK(hipMalloc(&dt, tl.size() * 4)); CK(hipMemcpy(dt, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
  const size_t lds = GemmNT<BM, BN, WM, WN, KC>::LDS_DOUBLES * 8;
  const int nt = 64 * WM * WN;
  CK(hipFuncSetAttribute((const void*)k_tri<BM, BN, WM, WN, OCC, KC, XCD>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k_tri<BM, BN, WM, WN, OCC, KC, XCD><<<(unsigned)tl.size(), nt, lds, 0>>>(dt, dA, m, dC, m, K);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) k_tri<BM, BN, WM, WN, OCC, KC, XCD><<<(unsigned)tl.size(), nt, lds, 0>>>(dt, dA, m, dC, m, K);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  double fl = (double)m * (m + 1) * K;  // useful flops of the lower triangle
  *flops_out = fl;
  CK(hipFree(dt));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 2048, reps = 5;
  std::vector<double> hA((size_t)m * K);
  srand(1);
  for (auto& x : hA) x = rand() / (double)RAND_MAX - 0.5;
  double *dA, *dC, *dC2;
  CK(hipMalloc(&dA, hA.size() * 8)); CK(hipMalloc(&dC, (size_t)m * m * 8)); CK(hipMalloc(&dC2, (size_t)m * m * 8));
  CK(hipMemcpy(dA, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
  double fl;
  auto report = [&](const char* name, double ms) { printf("m %d K %d %-12s %8.3f ms  %6.2f TF/s\n", m, K, name, ms, fl / ms * 1e-9); };
  // correctness: C = 0 - A A^T after one launch
  CK(hipMemset(dC, 0, (size_t)m * m * 8));
  {
    std::vector<int> tl;
    for (int tj = 0; tj * 128 < m; ++tj) for (int ti = 0; ti * 128 < m; ++ti) if (ti * 128 + 128 > tj * 128) tl.push_back(ti | (tj << 16));
    int* dt; CK(hipMalloc(&dt, tl.size() * 4)); CK(hipMemcpy(dt, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
    const size_t lds = GemmNT<128, 128, 4, 2>::LDS_DOUBLES * 8;
    CK(hipFuncSetAttribute((const void*)k_tri<128, 128, 4, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    k_tri<128, 128, 4, 2, 1><<<(unsigned)tl.size(), 512, lds, 0>>>(dt, dA, m, dC, m, K);
    CK(hipDeviceSynchronize());
    std::vector<double> hC((size_t)m * m);
    CK(hipMemcpy(hC.data(), dC, hC.size() * 8, hipMemcpyDeviceToHost));
    double maxerr = 0; int bad_upper = 0;
    for (int s = 0; s < 2000; ++s) {
      int i = rand() % m, j = rand() % m;
      double ref = 0; for (int k = 0; k < K; ++k) ref -= hA[(size_t)k * m + i] * hA[(size_t)k * m + j];
      double g = hC[(size_t)j * m + i];
      if (i >= j) maxerr = std::max(maxerr, std::fabs(g - ref) / (1 + std::fabs(ref)));
      else if (g != 0.0) bad_upper++;
    }
    printf("check: max rel err %.3e, upper entries touched %d\n", maxerr, bad_upper);
    CK(hipFree(dt));
  }
  report("128x128w4o2", run<128, 128, 2, 2, 2>(dA, dC, m, K, reps, &fl));
  report("128x128w8", run<128, 128, 4, 2, 1>(dA, dC, m, K, reps, &fl));
  report("128x128w8o2", run<128, 128, 4, 2, 2>(dA, dC, m, K, reps, &fl));
  report("128x64w4o2", run<128, 64, 2, 2, 2>(dA, dC, m, K, reps, &fl));
  report("128x64w8", run<128, 64, 4, 2, 1>(dA, dC, m, K, reps, &fl));
  report("256x128w8", run<256, 128, 4, 2, 1>(dA, dC, m, K, reps, &fl));
  report("64x64", run<64, 64>(dA, dC, m, K, reps, &fl));
  report("64x64k32", run<64, 64, 2, 2, 1, 32>(dA, dC, m, K, reps, &fl));
  report("64x64xcd", run<64, 64, 2, 2, 1, 16, 1>(dA, dC, m, K, reps, &fl));
  report("128x128w4o2xcd", run<128, 128, 2, 2, 2, 16, 1>(dA, dC, m, K, reps, &fl));
  report("128x64w8xcd", run<128, 64, 4, 2, 1, 16, 1>(dA, dC, m, K, reps, &fl));
  report("128x64w8k32", run<128, 64, 4, 2, 1, 32>(dA, dC, m, K, reps, &fl));
  report("128x128w8k32", run<128, 128, 4, 2, 1, 32>(dA, dC, m, K, reps, &fl));
  rocblas_handle h; rocblas_create_handle(&h);
  const double alpha = -1.0, beta = 1.0;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, m, K, &alpha, dA, m, &beta, dC2, m);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, m, K, &alpha, dA, m, &beta, dC2, m);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b)); report("rocblas_syrk", ms / reps);
  rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, m, K, &alpha, dA, m, dA, m, &beta, dC2, m);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, m, m, K, &alpha, dA, m, dA, m, &beta, dC2, m);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  printf("m %d K %d %-12s %8.3f ms  %6.2f TF/s (full gemm flops)\n", m, K, "rocblas_gemm", ms / reps, 2.0 * m * m * K / (ms / reps) * 1e-9);
  return 0;
}
