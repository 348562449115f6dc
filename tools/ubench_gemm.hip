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

namespace g2ohip {

// Experimental: the same tile update on the FP64 vector ALU (v_fma_f64 sustains ≈ 65 TFLOP/s against ≈ 46 for
// v_mfma_f64_16x16x4f64 in the pure issue-rate loops below); this register-blocked form reaches only
// ≈ 25-27 TFLOP/s (occupancy 2, exposed LDS latency) and is not used by the product. 256 threads own a 128 x 128 tile, each an 8 x 8 register block: rows {4 ty + i, 64 + 4 ty + i},
// columns {4 tx + j, 64 + 4 tx + j} (ty = tid / 16, tx = tid % 16), so the four ds_read_b128 of A and of
// B per k are contiguous 512-byte rows across a wave's lanes. K in double-buffered LDS chunks of 16 as in
// GemmNT.
struct GemmNTv {
  static constexpr int BM = 128, BN = 128, NT = 256, KC = 16;
  static constexpr int S = 128 + 8;  // k-major LDS stride (doubles); 16-byte aligned rows
  static constexpr int LDS_DOUBLES = 2 * 2 * KC * S;
  static constexpr int LA = BM * KC / NT;  // 8 global loads per thread per chunk and matrix

  __device__ static void run(const double* __restrict__ A, int lda, double* __restrict__ C, int ldc, int mrows,
                             int climit, int I0, int J0, int ka, int kb, double* lds) {
    const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
    constexpr int BUF = 2 * KC * S;  // buffer b: A image at b BUF, B image at b BUF + KC S
    double ra[LA], rb[LA];
    unsigned oka = 0, okb = 0;
    auto fetch = [&](int kc) {
      oka = okb = 0;
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int e = tid + NT * u, r = e & (BM - 1), k = kc + e / BM;
        const bool oa = k < kb && I0 + r < mrows, ob = k < kb && J0 + r < mrows;
        ra[u] = A[oa ? k * lda + I0 + r : 0];
        rb[u] = A[ob ? k * lda + J0 + r : 0];
        oka |= (unsigned)oa << u;
        okb |= (unsigned)ob << u;
      }
    };
    auto stash = [&](int b) {
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int e = tid + NT * u, r = e & (BM - 1), k = e / BM;
        lds[b * BUF + k * S + r] = (oka >> u) & 1 ? ra[u] : 0.0;
        lds[b * BUF + KC * S + k * S + r] = (okb >> u) & 1 ? rb[u] : 0.0;
      }
    };
    double acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.0;
    fetch(ka);
    stash(0);
    __syncthreads();
    const int nch = (kb - ka + KC - 1) / KC;
    for (int c = 0; c < nch; ++c) {
      const int b = c & 1;
      fetch(ka + (c + 1) * KC);
      const double* pa = lds + b * BUF + 4 * ty;
      const double* pb = lds + b * BUF + KC * S + 4 * tx;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        double a[8], bb[8];
        const double2* a2 = reinterpret_cast<const double2*>(pa + k * S);
        const double2* b2 = reinterpret_cast<const double2*>(pb + k * S);
        const double2 a0 = a2[0], a1 = a2[1], a4 = a2[32], a5 = a2[33];
        const double2 b0 = b2[0], b1 = b2[1], b4 = b2[32], b5 = b2[33];
        a[0] = a0.x; a[1] = a0.y; a[2] = a1.x; a[3] = a1.y; a[4] = a4.x; a[5] = a4.y; a[6] = a5.x; a[7] = a5.y;
        bb[0] = b0.x; bb[1] = b0.y; bb[2] = b1.x; bb[3] = b1.y; bb[4] = b4.x; bb[5] = b4.y; bb[6] = b5.x; bb[7] = b5.y;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_fma(a[i], bb[j], acc[i][j]);
      }
      stash(b ^ 1);
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int gj = J0 + (j < 4 ? 4 * tx + j : 64 + 4 * tx + j - 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int gi = I0 + (i < 4 ? 4 * ty + i : 64 + 4 * ty + i - 4);
        if (gi < mrows && gj < climit && gi >= gj) C[(size_t)gj * ldc + gi] -= acc[i][j];
      }
    }
  }
};

}  // namespace g2ohip

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int BM, int BN, int WM, int WN, int OCC, int KC = 16, int XCD = 0>
__global__ void __launch_bounds__(64 * WM * WN, OCC) k_tri(const int* tiles, const double* A, int lda, double* C, int m, int K) {
  extern __shared__ double lds[];
  const int t = tiles[XCD ? xcd_item(blockIdx.x, gridDim.x) : blockIdx.x];
  const int ti = t & 0xffff, tj = t >> 16;
  GemmNT<BM, BN, WM, WN, KC>::run(A, lda, C, m, m, m, ti * BM, tj * BN, 0, K, lds);
}

template <int BM, int BN, int WM, int WN, int OCC, int KC, int NS>
__global__ void __launch_bounds__(64 * WM * WN, OCC) k_tri_d(const int* tiles, const double* A, int lda, double* C, int m, int K) {
  extern __shared__ double lds[];
  const int t = tiles[blockIdx.x];
  const int ti = t & 0xffff, tj = t >> 16;
  GemmNTd<BM, BN, WM, WN, KC, NS>::run(A, lda, C, m, m, m, ti * BM, tj * BN, 0, K, lds);
}
template <int BM, int BN, int WM = 2, int WN = 2, int OCC = 2, int KC = 16, int NS = 3>
double run_d(const double* dA, double* dC, int m, int K, int reps, double* flops_out) {
  std::vector<int> tl;
  for (int tj = 0; tj * BN < m; ++tj)
    for (int ti = 0; ti * BM < m; ++ti)
      if (ti * BM + BM > tj * BN) tl.push_back(ti | (tj << 16));
  int* dt; CK(hipMalloc(&dt, tl.size() * 4)); CK(hipMemcpy(dt, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
  const size_t lds = GemmNTd<BM, BN, WM, WN, KC, NS>::LDS_DOUBLES * 8;
  const int nt = 64 * WM * WN;
  CK(hipFuncSetAttribute((const void*)k_tri_d<BM, BN, WM, WN, OCC, KC, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k_tri_d<BM, BN, WM, WN, OCC, KC, NS><<<(unsigned)tl.size(), nt, lds, 0>>>(dt, dA, m, dC, m, K);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) k_tri_d<BM, BN, WM, WN, OCC, KC, NS><<<(unsigned)tl.size(), nt, lds, 0>>>(dt, dA, m, dC, m, K);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  *flops_out = (double)m * (m + 1) * K;
  CK(hipFree(dt));
  return ms / reps;
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


// pure v_mfma_f64_16x16x4f64 issue rate: NACC independent accumulators per wave, no memory traffic
template <int NACC>
__global__ void __launch_bounds__(256) k_mfma_peak(double* out, int iters) {
  gdx4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = gdx4{0.0, 0.0, 0.0, 0.0};
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NACC>
void peak(double* buf) {
  const int grid = 1024, iters = 2000;
  k_mfma_peak<NACC><<<grid, 256>>>(buf, iters);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  k_mfma_peak<NACC><<<grid, 256>>>(buf, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double fl = (double)grid * 4 * iters * NACC * 2048.0;
  printf("mfma f64 16x16x4, %2d accumulators/wave, 4 waves/CU-slot: %6.2f TF/s\n", NACC, fl / (ms * 1e-3) * 1e-12);
}

typedef double gdx2 __attribute__((ext_vector_type(2)));
// FP64 VALU FMA issue rate: NCH independent chains per lane (scalar double or double2 vector FMAs)
template <int NCH, int VEC>
__global__ void __launch_bounds__(256) k_valu_peak(double* out, int iters) {
  gdx2 x[NCH];
  for (int i = 0; i < NCH; ++i) x[i] = gdx2{threadIdx.x * 1e-3 + i, 1.0 + i};
  const gdx2 m = {0.999999, 0.999998}, c = {1e-7, 2e-7};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (VEC) x[i] = __builtin_elementwise_fma(x[i], m, c);
      else { x[i].x = __builtin_fma(x[i].x, m.x, c.x); x[i].y = __builtin_fma(x[i].y, m.y, c.y); }
    }
  }
  double s = 0;
  for (int i = 0; i < NCH; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int NCH, int VEC>
void vpeak(double* buf) {
  const int grid = 1024, iters = 4000;
  k_valu_peak<NCH, VEC><<<grid, 256>>>(buf, iters);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  k_valu_peak<NCH, VEC><<<grid, 256>>>(buf, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  const double fl = (double)grid * 256 * iters * NCH * 2 * 2.0;
  printf("valu f64 fma %s, %d chains x2: %6.2f TF/s\n", VEC ? "double2" : "scalar", NCH, fl / (ms * 1e-3) * 1e-12);
}

__global__ void __launch_bounds__(256, 2) k_tri_v(const int* tiles, const double* A, int lda, double* C, int m, int K) {
  extern __shared__ double lds[];
  const int t = tiles[blockIdx.x];
  const int ti = t & 0xffff, tj = t >> 16;
  GemmNTv::run(A, lda, C, m, m, m, ti * 128, tj * 128, 0, K, lds);
}
double run_v(const double* dA, double* dC, int m, int K, int reps, double* flops_out) {
  std::vector<int> tl;
  for (int tj = 0; tj * 128 < m; ++tj)
    for (int ti = 0; ti * 128 < m; ++ti)
      if (ti >= tj) tl.push_back(ti | (tj << 16));
  int* dt; CK(hipMalloc(&dt, tl.size() * 4)); CK(hipMemcpy(dt, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
  const size_t lds = GemmNTv::LDS_DOUBLES * 8;
  CK(hipFuncSetAttribute((const void*)k_tri_v, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k_tri_v<<<(unsigned)tl.size(), 256, lds, 0>>>(dt, dA, m, dC, m, K);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) k_tri_v<<<(unsigned)tl.size(), 256, lds, 0>>>(dt, dA, m, dC, m, K);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  *flops_out = (double)m * (m + 1) * K;
  CK(hipFree(dt));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int m = argc > 1 ? atoi(argv[1]) : 4096, K = argc > 2 ? atoi(argv[2]) : 2048, reps = 5;
  if (m == 0) {
    double* buf; CK(hipMalloc(&buf, 1024 * 256 * 8));
    peak<1>(buf); peak<2>(buf); peak<4>(buf); peak<8>(buf);
    vpeak<4, 0>(buf); vpeak<4, 1>(buf); vpeak<8, 0>(buf); vpeak<8, 1>(buf);
    return 0;
  }
  std::vector<double> hA((size_t)m * K);
  srand(1);
  for (auto& x : hA) x = rand() / (double)RAND_MAX - 0.5;
  double *dA, *dC, *dC2;
  CK(hipMalloc(&dA, hA.size() * 8 + 64)); CK(hipMalloc(&dC, (size_t)m * m * 8)); CK(hipMalloc(&dC2, (size_t)m * m * 8));
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
  {  // GemmNTv correctness: C = 0 - A A^T
    CK(hipMemset(dC, 0, (size_t)m * m * 8));
    double f0; run_v(dA, dC, m, K, 0, &f0);
    CK(hipDeviceSynchronize());
    std::vector<double> hC((size_t)m * m);
    CK(hipMemcpy(hC.data(), dC, hC.size() * 8, hipMemcpyDeviceToHost));
    double maxerr = 0; int bad_upper = 0;
    for (int s2 = 0; s2 < 2000; ++s2) {
      int i = rand() % m, j = rand() % m;
      double ref = 0; for (int k = 0; k < K; ++k) ref -= hA[(size_t)k * m + i] * hA[(size_t)k * m + j];
      double g = hC[(size_t)j * m + i];
      if (i >= j) maxerr = std::max(maxerr, std::fabs(g - ref) / (1 + std::fabs(ref)));
      else if (g != 0.0) bad_upper++;
    }
    printf("check v: max rel err %.3e, upper entries touched %d\n", maxerr, bad_upper);
  }
  auto check = [&](const char* name, auto runner) {  // C = 0 - A A^T after one launch, sampled against the host
    CK(hipMemset(dC, 0, (size_t)m * m * 8));
    double f0; runner(0, &f0);
    CK(hipDeviceSynchronize());
    std::vector<double> hC((size_t)m * m);
    CK(hipMemcpy(hC.data(), dC, hC.size() * 8, hipMemcpyDeviceToHost));
    double maxerr = 0; int bad_upper = 0;
    for (int s2 = 0; s2 < 3000; ++s2) {
      int i = rand() % m, j = rand() % m;
      if (s2 < 64) { i = m - 1 - (s2 & 7); j = m - 1 - (s2 >> 3); }  // the ragged corner
      double ref = 0; for (int k = 0; k < K; ++k) ref -= hA[(size_t)k * m + i] * hA[(size_t)k * m + j];
      double g = hC[(size_t)j * m + i];
      if (i >= j) maxerr = std::max(maxerr, std::fabs(g - ref) / (1 + std::fabs(ref)));
      else if (g != 0.0) bad_upper++;
    }
    printf("check %s: max rel err %.3e, upper entries touched %d\n", name, maxerr, bad_upper);
  };
  check("d64", [&](int r, double* f) { return run_d<64, 64>(dA, dC, m, K, r, f); });
  check("d128x64", [&](int r, double* f) { return run_d<128, 64, 4, 2, 1>(dA, dC, m, K, r, f); });
  check("d128", [&](int r, double* f) { return run_d<128, 128, 4, 2, 1>(dA, dC, m, K, r, f); });
  report("d64x64k16s2o4", run_d<64, 64, 2, 2, 4, 16, 2>(dA, dC, m, K, reps, &fl));  // the k_syrk default
  report("d64x64o2", run_d<64, 64, 2, 2, 2>(dA, dC, m, K, reps, &fl));
  report("d64x64o3", run_d<64, 64, 2, 2, 3>(dA, dC, m, K, reps, &fl));
  report("d64x64s4", run_d<64, 64, 2, 2, 2, 16, 4>(dA, dC, m, K, reps, &fl));
  report("d64x64k8s3o4", run_d<64, 64, 2, 2, 4, 8, 3>(dA, dC, m, K, reps, &fl));
  report("d64x64k8s4o3", run_d<64, 64, 2, 2, 3, 8, 4>(dA, dC, m, K, reps, &fl));
  report("d64x64k32s2", run_d<64, 64, 2, 2, 2, 32, 2>(dA, dC, m, K, reps, &fl));
  report("d64x64k32s3", run_d<64, 64, 2, 2, 1, 32, 3>(dA, dC, m, K, reps, &fl));
  report("d128x64w8", run_d<128, 64, 4, 2, 1>(dA, dC, m, K, reps, &fl));
  report("d128x64w4", run_d<128, 64, 2, 2, 1>(dA, dC, m, K, reps, &fl));
  report("d128x128w8", run_d<128, 128, 4, 2, 1>(dA, dC, m, K, reps, &fl));
  report("d128x128w4", run_d<128, 128, 2, 2, 1>(dA, dC, m, K, reps, &fl));
  report("valu128", run_v(dA, dC, m, K, reps, &fl));
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
