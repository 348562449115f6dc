// Dev micro-benchmark: a barrier-free, LDS-free f64 MFMA tile (operands streamed global -> registers through a
// P-deep register ring, each wave loading its own fragments) against the product's LDS-DMA ring tile
// (GemmNTd<64,64,2,2,16,2>, k_syrk's default) on lower-triangular SYRKs C -= A A^T (m x m, K), sampled against an fp64
// host reference. Not product code. Measured on MI355X (profiles/r06_ubench_gemm_reg.log): 40.4-42.0 TF/s for the
// P = 6 / 8 rings against 45.9 for GemmNTd on 4096^2 at K = 2048 — the LDS-DMA ring stays. The asm-load ring is fragile:
// at P = 4 the results were wrong (the compiler may copy an asm load's destination before its counted wait) and a
// 128 x 128 variant (256 VGPRs) faulted; both were removed from this file.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 -Ig2o_amd/csrc -Iinclude \
//     tools/ubench_gemm_reg.hip -o tools/ubench_gemm_reg
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gemm_nt.hpp"
using namespace g2ohip;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);             \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// C(I, J) -= A(I, K) A(J, K)^T, lower triangle. Wave (wr, wc) owns MI x NJ 16x16 blocks; every k-step (4 columns) it
// loads its MI + NJ fragments straight from global memory (lane lr + 16 lk: row lr, column lk of the 16x4 fragment,
// 16 lanes = one 128-byte column segment) into ring slot s, P k-steps ahead of their MFMAs. No LDS, no barrier.
template <int P, int MI = 2, int NJ = 2, int WM = 2, int WN = 2>
struct GemmNTr {
  static constexpr int BM = WM * 16 * MI, BN = WN * 16 * NJ, NT = 64 * WM * WN;
  __device__ __forceinline__ static void run(const double* __restrict__ A, int lda, double* __restrict__ C, int ldc,
                                             int mrows, int I0, int J0, int ka, int kb) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w % WM, wc = w / WM, lr = lane & 15, lk = lane >> 4;
    const int r0 = I0 + wr * (BM / WM), c0 = J0 + wc * (BN / WN);
    if (r0 + BM / WM <= c0) return;  // block wholly above the diagonal
    gdx4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = gdx4{0.0, 0.0, 0.0, 0.0};
    int ra[MI], rb[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) ra[i] = min(r0 + 16 * i + lr, mrows - 1);
#pragma unroll
    for (int j = 0; j < NJ; ++j) rb[j] = min(c0 + 16 * j + lr, mrows - 1);
    double fa[P][MI], fb[P][NJ];
    // loads by inline asm (the compiler sinks plain loads next to their MFMAs), completion by counted waits that take
    // the ring registers as in/out operands (so no MFMA reads a slot before its wait)
    auto load = [&](int step, int s) {
      const int k = min(ka + 4 * step + lk, kb - 1);
      const double* col = A + (size_t)k * lda;
#pragma unroll
      for (int i = 0; i < MI; ++i) asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(fa[s][i]) : "v"(col + ra[i]) : "memory");
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(fb[s][j]) : "v"(col + rb[j]) : "memory");
    };
    constexpr int LATER = (P - 1) * (MI + NJ);  // loads issued after a slot's: the other P - 1 slots'
    static_assert(LATER < 64, "vmcnt range");
    const int ns = (kb - ka + 3) / 4, ng = (ns + P - 1) / P;
#pragma unroll
    for (int s = 0; s < P; ++s) load(s, s);
    for (int g = 0; g < ng; ++g) {
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const int step = g * P + s;
        if constexpr (MI == 2 && NJ == 2)
          asm volatile("s_waitcnt vmcnt(%4)" : "+v"(fa[s][0]), "+v"(fa[s][1]), "+v"(fb[s][0]), "+v"(fb[s][1]) : "n"(LATER));
        else if constexpr (MI == 4 && NJ == 2)
          asm volatile("s_waitcnt vmcnt(%6)" : "+v"(fa[s][0]), "+v"(fa[s][1]), "+v"(fa[s][2]), "+v"(fa[s][3]), "+v"(fb[s][0]),
                       "+v"(fb[s][1]) : "n"(LATER));
        else
          asm volatile("s_waitcnt vmcnt(%8)" : "+v"(fa[s][0]), "+v"(fa[s][1]), "+v"(fa[s][2]), "+v"(fa[s][3]), "+v"(fb[s][0]),
                       "+v"(fb[s][1]), "+v"(fb[s][2]), "+v"(fb[s][3]) : "n"(LATER));
        const bool kv = ka + 4 * step + lk < kb;
        double a[MI], b[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) a[i] = kv ? fa[s][i] : 0.0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) b[j] = fb[s][j];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
        load(step + P, s);  // past kb: clamped (masked at use)
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's last (unused) loads land before its registers are reused
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gj = c0 + 16 * j + lr;
      double cv[MI][4];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gi = r0 + 16 * i + lk + 4 * q;
          cv[i][q] = gi < mrows && gj < mrows && gi >= gj ? C[(size_t)gj * ldc + gi] : 0.0;
        }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gi = r0 + 16 * i + lk + 4 * q;
          if (gi < mrows && gj < mrows && gi >= gj) C[(size_t)gj * ldc + gi] = cv[i][q] - acc[i][j][q];
        }
    }
  }
};

template <class T, int OCC>
__global__ void __launch_bounds__(T::NT, OCC) k_reg(const int* tiles, const double* A, int lda, double* C, int m, int K) {
  const int t = tiles[blockIdx.x];
  T::run(A, lda, C, m, m, (t & 0xffff) * T::BM, (t >> 16) * T::BN, 0, K);
}
__global__ void __launch_bounds__(256, 4) k_dma(const int* tiles, const double* A, int lda, double* C, int m, int K) {
  extern __shared__ double lds[];
  const int t = tiles[blockIdx.x];
  using T = GemmNTd<64, 64, 2, 2, 16, 2>;
  T::run(A, lda, C, m, m, m, (t & 0xffff) * 64, (t >> 16) * 64, 0, K, lds);
}

static std::vector<int> tile_list(int m, int BM, int BN) {
  std::vector<int> tl;
  for (int tj = 0; tj * BN < m; ++tj)
    for (int ti = 0; ti * BM < m; ++ti)
      if (ti * BM + BM > tj * BN) tl.push_back(ti | (tj << 16));
  return tl;
}

int main(int argc, char** argv) {
  const int shapes[][2] = {{4096, 2048}, {3072, 2760}, {2048, 384}, {1152, 256}, {6144, 512}};
  for (auto& sh : shapes) {
    const int m = sh[0], K = sh[1], reps = 5;
    std::vector<double> hA((size_t)m * K);
    srand(1);
    for (auto& x : hA) x = rand() / (double)RAND_MAX - 0.5;
    double *dA, *dC;
    CK(hipMalloc(&dA, hA.size() * 8 + 64));
    CK(hipMalloc(&dC, (size_t)m * m * 8));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
    const double fl = (double)m * (m + 1) * K;
    auto bench = [&](const char* name, int BM, int BN, auto launch) {
      std::vector<int> tl = tile_list(m, BM, BN);
      int* dt;
      CK(hipMalloc(&dt, tl.size() * 4));
      CK(hipMemcpy(dt, tl.data(), tl.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemset(dC, 0, (size_t)m * m * 8));
      launch(dt, (unsigned)tl.size());
      CK(hipDeviceSynchronize());
      std::vector<double> hC((size_t)m * m);
      CK(hipMemcpy(hC.data(), dC, hC.size() * 8, hipMemcpyDeviceToHost));
      double maxerr = 0;
      int bad = 0;
      for (int s = 0; s < 1500; ++s) {
        int i = rand() % m, j = rand() % m;
        if (s < 64) { i = m - 1 - (s & 7); j = m - 1 - (s >> 3); }
        double ref = 0;
        for (int k = 0; k < K; ++k) ref -= hA[(size_t)k * m + i] * hA[(size_t)k * m + j];
        const double g = hC[(size_t)j * m + i];
        if (i >= j) maxerr = std::fmax(maxerr, std::fabs(g - ref) / (1 + std::fabs(ref)));
        else if (g != 0.0) ++bad;
      }
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a));
      for (int r = 0; r < reps; ++r) launch(dt, (unsigned)tl.size());
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= reps;
      printf("m %5d K %5d %-16s %5zu tiles %8.3f ms %6.2f TF/s  err %.1e upper %d\n", m, K, name, tl.size(), ms,
             fl / ms * 1e-9, maxerr, bad);
      CK(hipFree(dt));
    };
    const size_t lds = GemmNTd<64, 64, 2, 2, 16, 2>::LDS_DOUBLES * 8;
    CK(hipFuncSetAttribute((const void*)k_dma, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    bench("dma64 (k_syrk)", 64, 64, [&](int* dt, unsigned n) { k_dma<<<n, 256, lds, 0>>>(dt, dA, m, dC, m, K); });
    bench("reg64 P8", 64, 64, [&](int* dt, unsigned n) { k_reg<GemmNTr<8>, 2><<<n, 256, 0, 0>>>(dt, dA, m, dC, m, K); });
    bench("reg64 P8 o3", 64, 64, [&](int* dt, unsigned n) { k_reg<GemmNTr<8>, 3><<<n, 256, 0, 0>>>(dt, dA, m, dC, m, K); });
    bench("reg64 P6", 64, 64, [&](int* dt, unsigned n) { k_reg<GemmNTr<6>, 3><<<n, 256, 0, 0>>>(dt, dA, m, dC, m, K); });
    CK(hipFree(dA));
    CK(hipFree(dC));
  }
  return 0;
}
