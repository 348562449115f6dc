// Solver::computeMarginals (core/solver.h; BlockSolver::computeMarginals block_solver.hpp:448-460 ->
// LinearSolverCSparse::solvePattern linear_solver_csparse.h:190-225 -> MarginalCovarianceCholesky) from the device
// factor: the requested blocks of A^-1 (A = Hpp, as the reference) come from multi-right-hand-side solves
// A X = E_c with the supernodal L the factorization left in HBM (lbuf: [L11; L21] per front, linv: L_kk^-1 per
// 32-column panel), block columns batched into one set of K <= 64 right-hand sides:
//   k_mfwd (per tree level, ascending)  children's below-diagonal parts are added into the front's own rows /
//            below part in fixed child order (the multifrontal extend-add of the right-hand sides), the own rows
//            solved panel by panel with L_kk^-1, the below part updated: W_f = W_f - L21 Y_f
//   k_mbwd (per level, descending)      t = Y_f - L21^T X(rows below), then x panel by panel from the last with L_kk^-T
// One workgroup per front, threads over (row, right-hand side): exact arithmetic order per entry, deterministic.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"

namespace g2ohip {
namespace {
constexpr int NB = 32;
constexpr int B = 256;
}  // namespace

__global__ void __launch_bounds__(B) k_mfwd(const int* __restrict__ lfronts, const launch::FrontDesc* __restrict__ fd,
                                            const int* __restrict__ children, const int* __restrict__ relmap,
                                            const double* __restrict__ lbuf, const double* __restrict__ linv,
                                            const long long* __restrict__ woff, double* __restrict__ W,
                                            double* __restrict__ Y, double* __restrict__ T, int n, int K) {
  const int f = lfronts[blockIdx.x];
  const launch::FrontDesc me = fd[f];
  const int ns = me.ns, nr = me.nr, m = ns + nr, c0 = me.c0;
  const double* L = lbuf + me.l_off;
  double* Wf = W + woff[f];
  const int tid = threadIdx.x;
  for (int i = tid; i < nr * K; i += B) Wf[i] = 0.0;
  __syncthreads();
  // extend-add of the children's update parts, children in fixed order
  for (int ci = me.child_begin; ci < me.child_end; ++ci) {
    const int c = children[ci];
    const launch::FrontDesc ch = fd[c];
    const double* Wc = W + woff[c];
    for (int i = tid; i < ch.nr * K; i += B) {
      const int j = i % ch.nr, k = i / ch.nr;
      const int pos = relmap[ch.rows_off + j];
      const double v = Wc[(size_t)k * ch.nr + j];
      if (pos < ns) Y[(size_t)k * n + c0 + pos] += v;
      else Wf[(size_t)k * nr + pos - ns] += v;
    }
    __syncthreads();
  }
  // own rows, panel by panel: y_p = L_pp^-1 (y_p - sum_{j < p} L(p, j) y_j)
  for (int k0 = 0; k0 < ns; k0 += NB) {
    const int kb = min(NB, ns - k0);
    const double* Li = linv + (size_t)(c0 + k0) * (NB * NB);
    for (int i = tid; i < kb * K; i += B) {
      const int r = i % kb, k = i / kb;
      double t = Y[(size_t)k * n + c0 + k0 + r];
      for (int j = 0; j < k0; ++j) t -= L[(size_t)j * m + k0 + r] * Y[(size_t)k * n + c0 + j];
      T[(size_t)k * n + c0 + k0 + r] = t;
    }
    __syncthreads();
    for (int i = tid; i < kb * K; i += B) {
      const int r = i % kb, k = i / kb;
      double y = 0.0;
      for (int j = 0; j < kb; ++j) y += Li[r * NB + j] * T[(size_t)k * n + c0 + k0 + j];
      Y[(size_t)k * n + c0 + k0 + r] = y;
    }
    __syncthreads();
  }
  // below part: W_f -= L21 y_f
  for (int i = tid; i < nr * K; i += B) {
    const int r = i % nr, k = i / nr;
    double t = Wf[(size_t)k * nr + r];
    for (int j = 0; j < ns; ++j) t -= L[(size_t)j * m + ns + r] * Y[(size_t)k * n + c0 + j];
    Wf[(size_t)k * nr + r] = t;
  }
}

__global__ void __launch_bounds__(B) k_mbwd(const int* __restrict__ lfronts, const launch::FrontDesc* __restrict__ fd,
                                            const int* __restrict__ rows, const double* __restrict__ lbuf,
                                            const double* __restrict__ linv, double* __restrict__ Y,
                                            double* __restrict__ T, int n, int K) {
  const int f = lfronts[blockIdx.x];
  const launch::FrontDesc me = fd[f];
  const int ns = me.ns, nr = me.nr, m = ns + nr, c0 = me.c0;
  const double* L = lbuf + me.l_off;
  const int* R = rows + me.rows_off;
  const int tid = threadIdx.x;
  // t = y_f - L21^T x(rows below): the rows below belong to ancestors, solved at an earlier (higher) level
  for (int i = tid; i < ns * K; i += B) {
    const int j = i % ns, k = i / ns;
    double t = Y[(size_t)k * n + c0 + j];
    for (int r = 0; r < nr; ++r) t -= L[(size_t)j * m + ns + r] * Y[(size_t)k * n + R[r]];
    T[(size_t)k * n + c0 + j] = t;
  }
  __syncthreads();
  const int np = (ns + NB - 1) / NB;
  for (int p = np - 1; p >= 0; --p) {  // x_p = L_pp^-T (t_p - sum_{j' beyond p} L(j', p)^T x_j')
    const int k0 = p * NB, kb = min(NB, ns - k0);
    const double* Li = linv + (size_t)(c0 + k0) * (NB * NB);
    for (int i = tid; i < kb * K; i += B) {
      const int r = i % kb, k = i / kb;
      double t = T[(size_t)k * n + c0 + k0 + r];
      for (int j = k0 + kb; j < ns; ++j) t -= L[(size_t)(k0 + r) * m + j] * Y[(size_t)k * n + c0 + j];
      T[(size_t)k * n + c0 + k0 + r] = t;
    }
    __syncthreads();
    for (int i = tid; i < kb * K; i += B) {
      const int r = i % kb, k = i / kb;
      double x = 0.0;
      for (int j = 0; j < kb; ++j) x += Li[j * NB + r] * T[(size_t)k * n + c0 + k0 + j];
      Y[(size_t)k * n + c0 + k0 + r] = x;
    }
    __syncthreads();
  }
}

// Y(:, k) = e_{pinv[col_k]}, everything else 0 (Y zeroed by the caller)
__global__ void k_munit(int K, const int* __restrict__ prow, double* __restrict__ Y, int n) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < K) Y[(size_t)k * n + prow[k]] = 1.0;
}
// out[i] = Y[idx[i]]
__global__ void k_mgather(long long cnt, const long long* __restrict__ idx, const double* __restrict__ Y,
                          double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < cnt) out[i] = Y[idx[i]];
}

namespace launch {
void marg_forward(int nf, const int* lfronts, const FrontDesc* fd, const int* children, const int* relmap,
                  const double* lbuf, const double* linv, const long long* woff, double* W, double* Y, double* T, int n,
                  int K, hipStream_t s) {
  if (nf <= 0) return;
  hipLaunchKernelGGL(k_mfwd, nf, B, 0, s, lfronts, fd, children, relmap, lbuf, linv, woff, W, Y, T, n, K);
  KERNEL_CHECK();
}
void marg_backward(int nf, const int* lfronts, const FrontDesc* fd, const int* rows, const double* lbuf,
                   const double* linv, double* Y, double* T, int n, int K, hipStream_t s) {
  if (nf <= 0) return;
  hipLaunchKernelGGL(k_mbwd, nf, B, 0, s, lfronts, fd, rows, lbuf, linv, Y, T, n, K);
  KERNEL_CHECK();
}
void marg_unit(int K, const int* prow, double* Y, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_munit, 1, 64, 0, s, K, prow, Y, n);
  KERNEL_CHECK();
}
void marg_gather(long long cnt, const long long* idx, const double* Y, double* out, hipStream_t s) {
  if (cnt <= 0) return;
  hipLaunchKernelGGL(k_mgather, grid_for(cnt, 256), 256, 0, s, cnt, idx, Y, out);
  KERNEL_CHECK();
}
}  // namespace launch
}  // namespace g2ohip
