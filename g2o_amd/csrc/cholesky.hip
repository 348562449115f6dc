// Supernodal multifrontal LL^T on gfx950 — numeric factorization and triangular solves.
//
// Replaces the reference's serial up-looking factorization
// (csparse_extension.cpp:64-119 cs_chol_workspace; cs_lsolve/cs_ltsolve/cs_ipvec/cs_pvec
// at :47-52) behind LinearSolver::solve (linear_solver.h:65): the symbolic
// analysis (symbolic.cpp) fixes the ordering, the supernodes and the frontal
// maps once per structure; every LM trial runs
//   scatter  (input blocks -> fronts, + lambda on the diagonal for pose graphs)
//   level l = 0..L-1:  k_chol_level   (extend-add of the children's update matrices,
//                                      dense partial LL^T of the front)
//   forward  level 0..L-1, backward level L-1..0 (front-wise triangular solves)
// All fronts of one level are independent; one workgroup owns one front, so every
// front entry is written by exactly one workgroup in a fixed order: the factor is
// bitwise reproducible run to run (no atomics anywhere).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"

namespace g2ohip {

using launch::FrontDesc;

constexpr int CT = 256;  // threads per front workgroup
constexpr int NB = 16;   // panel width

__global__ void __launch_bounds__(256) k_chol_scatter(long long nent, const double* __restrict__ vals,
                                                      const long long* __restrict__ dst,
                                                      const unsigned char* __restrict__ is_diag,
                                                      const double* __restrict__ lam, double* __restrict__ fronts) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nent) return;
  const long long d = dst[k];
  if (d < 0) return;
  double v = vals[k];
  if (is_diag[k]) v += *lam;
  fronts[d] = v;
}

// Dense partial Cholesky of a front F (m x m col-major, lower triangle), first ns columns.
__device__ void front_factor(double* __restrict__ F, int m, int ns, int* __restrict__ fail) {
  __shared__ double Ld[NB][NB + 1];
  __shared__ double Pi[64][NB + 1];
  __shared__ double Pj[64][NB + 1];
  const int tid = threadIdx.x;
  for (int k0 = 0; k0 < ns; k0 += NB) {
    const int kb = min(NB, ns - k0);
    // (a) diagonal block
    if (tid < kb * kb) {
      const int r = tid % kb, c = tid / kb;
      Ld[r][c] = r >= c ? F[(size_t)(k0 + c) * m + k0 + r] : 0.0;
    }
    __syncthreads();
    for (int j = 0; j < kb; ++j) {
      if (tid == 0) {
        const double d = Ld[j][j];
        if (!(d > 0.0)) *fail = 1;
        Ld[j][j] = sqrt(d > 0.0 ? d : 1.0);
      }
      __syncthreads();
      if (tid > j && tid < kb) Ld[tid][j] /= Ld[j][j];
      __syncthreads();
      {
        const int r = tid % kb, c = tid / kb;
        if (tid < kb * kb && c > j && r >= c) Ld[r][c] -= Ld[r][j] * Ld[c][j];
      }
      __syncthreads();
    }
    if (tid < kb * kb) {
      const int r = tid % kb, c = tid / kb;
      if (r >= c) F[(size_t)(k0 + c) * m + k0 + r] = Ld[r][c];
    }
    // (b) panel rows below: x L^T = row
    const int r0 = k0 + kb;
    for (int i = r0 + tid; i < m; i += CT) {
      double x[NB];
#pragma unroll
      for (int t = 0; t < NB; ++t) x[t] = t < kb ? F[(size_t)(k0 + t) * m + i] : 0.0;
#pragma unroll
      for (int t = 0; t < NB; ++t) {
        if (t < kb) {
          double s = x[t];
#pragma unroll
          for (int u = 0; u < NB; ++u)
            if (u < t) s -= x[u] * Ld[t][u];
          x[t] = s / Ld[t][t];
        }
      }
#pragma unroll
      for (int t = 0; t < NB; ++t)
        if (t < kb) F[(size_t)(k0 + t) * m + i] = x[t];
    }
    __syncthreads();
    // (c) trailing update of the lower triangle [r0, m)
    const int nt = m - r0;
    const int ntiles = (nt + 63) / 64;
    for (int tj = 0; tj < ntiles; ++tj) {
      for (int ti = tj; ti < ntiles; ++ti) {
        const int i0 = r0 + ti * 64, j0 = r0 + tj * 64;
        for (int idx = tid; idx < 64 * NB; idx += CT) {
          const int rr = idx % 64, t = idx / 64;
          Pi[rr][t] = (i0 + rr < m && t < kb) ? F[(size_t)(k0 + t) * m + i0 + rr] : 0.0;
          Pj[rr][t] = (j0 + rr < m && t < kb) ? F[(size_t)(k0 + t) * m + j0 + rr] : 0.0;
        }
        __syncthreads();
        const int tx = tid % 16, ty = tid / 16;
        double acc[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[a][c] = 0.0;
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          double pa[4], pb[4];
#pragma unroll
          for (int a = 0; a < 4; ++a) { pa[a] = Pi[tx * 4 + a][t]; pb[a] = Pj[ty * 4 + a][t]; }
#pragma unroll
          for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[a][c] += pa[a] * pb[c];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int j = j0 + ty * 4 + c;
          if (j >= m) continue;
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const int i = i0 + tx * 4 + a;
            if (i < m && i >= j) F[(size_t)j * m + i] -= acc[a][c];
          }
        }
        __syncthreads();
      }
    }
  }
}

__global__ void __launch_bounds__(CT) k_chol_level(const int* __restrict__ level_list, const FrontDesc* __restrict__ fd,
                                                   const int* __restrict__ children, const int* __restrict__ relmap,
                                                   double* __restrict__ fronts, int* __restrict__ fail) {
  const int s = level_list[blockIdx.x];
  const FrontDesc me = fd[s];
  const int m = me.ns + me.nr;
  double* F = fronts + me.front_off;
  const int tid = threadIdx.x;
  // extend-add of the children's update matrices (children in fixed order)
  for (int k = me.child_begin; k < me.child_end; ++k) {
    const FrontDesc cd = fd[children[k]];
    const int mc = cd.ns + cd.nr, nrc = cd.nr;
    const double* U = fronts + cd.front_off;
    const int* rel = relmap + cd.rows_off;
    for (int j = 0; j < nrc; ++j) {
      const int pj = rel[j];
      const double* uc = U + (size_t)(cd.ns + j) * mc + cd.ns;
      double* fc = F + (size_t)pj * m;
      for (int i = j + tid; i < nrc; i += CT) fc[rel[i]] += uc[i];
    }
    __syncthreads();
  }
  front_factor(F, m, me.ns, fail);
}

__global__ void k_permute(int n, const int* __restrict__ perm, const double* __restrict__ in, double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = in[perm[k]];
}
__global__ void k_ipermute(int n, const int* __restrict__ perm, const double* __restrict__ in, double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[perm[k]] = in[k];
}

// forward: v_s = [rhs(own cols); 0] + extend-add of children's u; L11 y = v1; v2 -= L21 y
__global__ void __launch_bounds__(CT) k_chol_forward(const int* __restrict__ level_list, const FrontDesc* __restrict__ fd,
                                                     const int* __restrict__ children, const int* __restrict__ relmap,
                                                     const double* __restrict__ fronts, double* __restrict__ vecs,
                                                     const double* __restrict__ rhs) {
  const int s = level_list[blockIdx.x];
  const FrontDesc me = fd[s];
  const int m = me.ns + me.nr;
  const double* F = fronts + me.front_off;
  double* v = vecs + me.vec_off;
  const int tid = threadIdx.x;
  for (int i = tid; i < m; i += CT) v[i] = i < me.ns ? rhs[me.c0 + i] : 0.0;
  __syncthreads();
  for (int k = me.child_begin; k < me.child_end; ++k) {
    const FrontDesc cd = fd[children[k]];
    const double* u = vecs + cd.vec_off + cd.ns;
    const int* rel = relmap + cd.rows_off;
    for (int r = tid; r < cd.nr; r += CT) v[rel[r]] += u[r];
    __syncthreads();
  }
  __shared__ double yj;
  for (int j = 0; j < me.ns; ++j) {
    if (tid == 0) {
      yj = v[j] / F[(size_t)j * m + j];
      v[j] = yj;
    }
    __syncthreads();
    const double y = yj;
    const double* col = F + (size_t)j * m;
    for (int i = j + 1 + tid; i < m; i += CT) v[i] -= col[i] * y;
    __syncthreads();
  }
}

// backward: x_s = L11^-T (y_s - L21^T x_rows)
__global__ void __launch_bounds__(CT) k_chol_backward(const int* __restrict__ level_list, const FrontDesc* __restrict__ fd,
                                                      const int* __restrict__ rows, const double* __restrict__ fronts,
                                                      double* __restrict__ vecs, double* __restrict__ xsol) {
  const int s = level_list[blockIdx.x];
  const FrontDesc me = fd[s];
  const int m = me.ns + me.nr;
  const double* F = fronts + me.front_off;
  double* v = vecs + me.vec_off;
  const int* rw = rows + me.rows_off;
  const int tid = threadIdx.x;
  for (int j = tid; j < me.ns; j += CT) {
    const double* col = F + (size_t)j * m + me.ns;
    double r = v[j];
    for (int i = 0; i < me.nr; ++i) r -= col[i] * xsol[rw[i]];
    v[j] = r;
  }
  __syncthreads();
  __shared__ double xj;
  for (int j = me.ns - 1; j >= 0; --j) {
    if (tid == 0) {
      xj = v[j] / F[(size_t)j * m + j];
      xsol[me.c0 + j] = xj;
    }
    __syncthreads();
    const double x = xj;
    for (int i = tid; i < j; i += CT) v[i] -= F[(size_t)i * m + j] * x;
    __syncthreads();
  }
}

namespace launch {

void chol_scatter(long long nent, const double* vals, const long long* dst, const unsigned char* is_diag,
                  const double* lam, double* fronts, hipStream_t s) {
  if (nent <= 0) return;
  hipLaunchKernelGGL(k_chol_scatter, grid_for(nent, 256), 256, 0, s, nent, vals, dst, is_diag, lam, fronts);
  KERNEL_CHECK();
}
void chol_level(int nfronts, const int* level_list, const FrontDesc* fd, const int* children, const int* relmap,
                double* fronts, int* fail, int /*max_m*/, hipStream_t s) {
  if (nfronts <= 0) return;
  hipLaunchKernelGGL(k_chol_level, nfronts, CT, 0, s, level_list, fd, children, relmap, fronts, fail);
  KERNEL_CHECK();
}
void chol_permute(int n, const int* perm, const double* in, double* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_permute, grid_for(n, 256), 256, 0, s, n, perm, in, out);
  KERNEL_CHECK();
}
void chol_ipermute(int n, const int* perm, const double* in, double* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_ipermute, grid_for(n, 256), 256, 0, s, n, perm, in, out);
  KERNEL_CHECK();
}
void chol_forward(int nfronts, const int* level_list, const FrontDesc* fd, const int* children, const int* relmap,
                  const double* fronts, double* vecs, const double* rhs, hipStream_t s) {
  if (nfronts <= 0) return;
  hipLaunchKernelGGL(k_chol_forward, nfronts, CT, 0, s, level_list, fd, children, relmap, fronts, vecs, rhs);
  KERNEL_CHECK();
}
void chol_backward(int nfronts, const int* level_list, const FrontDesc* fd, const int* rows, const double* fronts,
                   const double* vecs, double* xsol, hipStream_t s) {
  if (nfronts <= 0) return;
  hipLaunchKernelGGL(k_chol_backward, nfronts, CT, 0, s, level_list, fd, rows, fronts, const_cast<double*>(vecs), xsol);
  KERNEL_CHECK();
}

}  // namespace launch
}  // namespace g2ohip
