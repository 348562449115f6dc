// Dev micro-benchmark: the Schur complement's panel-times-panel product on MFMA.
// Per landmark l with k = 10 observations, P_l = [G_l,c1; ...; G_l,ck] (60 x 3, G = Hpl U^-T) and the Schur
// update is P_l P_l^T (60 x 60; its 55 lower 6x6 blocks land in S). C4 shape: 100k landmarks.
//   A  MFMA  v_mfma_f64_16x16x4f64, K = 3 padded to 4, the 10 lower 16x16 tiles of the 64x64 product per
//            landmark, one wave per landmark; the 55 blocks written out (the minimum a per-landmark formulation
//            must move before any reduction into S)
//   B  VALU  the same 55 blocks with v_fma_f64 (one lane per output entry row), written out the same way
//   A0 / B0  the same products without the output writes (sums kept in registers): pure compute
// Prints the time per pass; compare with k_schur_rows (150 us at C4) and the stage's 173 MB algorithmic bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e = (x);                                                                         \
    if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } \
  } while (0)

typedef double dx4 __attribute__((ext_vector_type(4)));
constexpr int K = 10, R = 6 * K;  // observations per landmark, rows of P_l
constexpr int NBLK = K * (K + 1) / 2;

// P stored per landmark row-major 60 x 3 (as 10 stacked 6x3 G blocks, row-major here for simple indexing)
template <bool WRITE>
__global__ void __launch_bounds__(256) k_mfma(int nl, const double* __restrict__ P, double* __restrict__ out,
                                              double* __restrict__ sink) {
  __shared__ double Ps[4][64 * 4];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l = blockIdx.x * 4 + w;
  if (l >= nl) return;
  const double* p = P + (size_t)l * R * 3;
  // stage P_l as 64 x 4 (rows >= 60 and column 3 zero)
  for (int e = lane; e < 64 * 4; e += 64) {
    const int r = e >> 2, c = e & 3;
    Ps[w][e] = (r < R && c < 3) ? p[r * 3 + c] : 0.0;
  }
  __builtin_amdgcn_s_waitcnt(0);
  const int lr = lane & 15, lk = lane >> 4;
  double keep = 0.0;
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int tj = 0; tj <= ti; ++tj) {
      dx4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Ps[w][(16 * ti + lr) * 4 + lk], Ps[w][(16 * tj + lr) * 4 + lk], acc,
                                                  0, 0, 0);
      if (WRITE) {  // entry (16 ti + lk + 4 i, 16 tj + lr) -> its 6x6 block (bi, bj), bi >= bj, col-major
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * ti + lk + 4 * i, c = 16 * tj + lr;
          if (r < R && c < R) {
            const int bi = r / 6, bj = c / 6;
            if (bi >= bj) {
              const int b = bi * (bi + 1) / 2 + bj;
              out[((size_t)l * NBLK + b) * 36 + (c % 6) * 6 + r % 6] = acc[i];
            }
          }
        }
      } else {
        keep += acc[0] + acc[1] + acc[2] + acc[3];
      }
    }
  if (!WRITE) sink[(size_t)l * 64 + lane] = keep;
}

template <bool WRITE>
__global__ void __launch_bounds__(256) k_valu(int nl, const double* __restrict__ P, double* __restrict__ out,
                                              double* __restrict__ sink) {
  // one wave per landmark; lane r < 60 owns row r of P_l P_l^T and computes its entries c <= r block-wise
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l = blockIdx.x * 4 + w;
  if (l >= nl) return;
  __shared__ double Ps[4][R * 3];
  const double* p = P + (size_t)l * R * 3;
  for (int e = lane; e < R * 3; e += 64) Ps[w][e] = p[e];
  __builtin_amdgcn_s_waitcnt(0);
  if (lane >= R) return;
  const double a0 = Ps[w][lane * 3], a1 = Ps[w][lane * 3 + 1], a2 = Ps[w][lane * 3 + 2];
  const int bi = lane / 6;
  double keep = 0.0;
  for (int c = 0; c < 6 * (bi + 1); ++c) {
    const double v = a0 * Ps[w][c * 3] + a1 * Ps[w][c * 3 + 1] + a2 * Ps[w][c * 3 + 2];
    if (WRITE) {
      const int bj = c / 6, b = bi * (bi + 1) / 2 + bj;
      out[((size_t)l * NBLK + b) * 36 + (c % 6) * 6 + lane % 6] = v;
    } else {
      keep += v;
    }
  }
  if (!WRITE) sink[(size_t)l * 64 + lane] = keep;
}

template <class F>
float timeit(F f, hipEvent_t a, hipEvent_t b) {
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a, 0);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 20;
}

int main() {
  const int nl = 100000;
  std::vector<double> h((size_t)nl * R * 3);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5;
  double *P, *out, *sink;
  CK(hipMalloc(&P, h.size() * 8));
  CK(hipMalloc(&out, (size_t)nl * NBLK * 36 * 8));
  CK(hipMalloc(&sink, (size_t)nl * 64 * 8));
  CK(hipMemcpy(P, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = (nl + 3) / 4;
  const double in_mb = h.size() * 8 / 1e6, out_mb = (double)nl * NBLK * 36 * 8 / 1e6;
  const double fl = 2.0 * nl * (double)NBLK * 36 * 3;
  float t;
  t = timeit([&] { hipLaunchKernelGGL((k_mfma<true>), grid, 256, 0, 0, nl, P, out, sink); }, a, b);
  printf("A  MFMA + 55 blocks written : %8.1f us  (in %.0f MB, out %.0f MB, %.2f TF/s useful)\n", t * 1e3, in_mb, out_mb,
         fl / (t * 1e-3) / 1e12);
  t = timeit([&] { hipLaunchKernelGGL((k_valu<true>), grid, 256, 0, 0, nl, P, out, sink); }, a, b);
  printf("B  VALU + 55 blocks written : %8.1f us  (%.2f TF/s useful)\n", t * 1e3, fl / (t * 1e-3) / 1e12);
  t = timeit([&] { hipLaunchKernelGGL((k_mfma<false>), grid, 256, 0, 0, nl, P, out, sink); }, a, b);
  printf("A0 MFMA products only        : %8.1f us  (%.2f TF/s useful, MFMA tiles 64x64x4 per landmark)\n", t * 1e3,
         fl / (t * 1e-3) / 1e12);
  t = timeit([&] { hipLaunchKernelGGL((k_valu<false>), grid, 256, 0, 0, nl, P, out, sink); }, a, b);
  printf("B0 VALU products only        : %8.1f us  (%.2f TF/s useful)\n", t * 1e3, fl / (t * 1e-3) / 1e12);
  return 0;
}
