// Supernodal multifrontal LL^T on gfx950 — numeric factorization fused with the forward
// solve, and the backward solve.
//
// Replaces the reference's serial up-looking factorization
// (csparse_extension.cpp:64-119 cs_chol_workspace; cs_lsolve/cs_ltsolve/cs_ipvec/cs_pvec
// at :47-52) behind LinearSolver::solve (linear_solver.h:65).  The symbolic
// analysis (symbolic.cpp) fixes ordering, supernodes and frontal maps once per
// structure; each LM trial runs
//   k_permute + k_vec_init   rhs -> P rhs -> front vectors (own rows)
//   k_chol_scatter           input blocks -> fronts (+ lambda on the diagonal for pose graphs)
//   per level l (all fronts of a level are independent):
//     k_extend_add     children's update matrices AND update vectors -> parent fronts;
//                      one workgroup per (front, 32-column slab), children in fixed order
//     per 32-wide panel p:
//       k_panel        POTRF of the 32x32 diagonal block in registers of one wave
//                      (every workgroup of the front recomputes it), forward-solve of the
//                      block's rhs, TRSM of 256 rows per workgroup fused with the rhs update
//       k_trail        SYRK/GEMM of the trailing lower triangle in 64x64 tiles on
//                      v_mfma_f64_16x16x4f64 (4 waves x 2x2 MFMA tiles, K = 32)
//   k_chol_backward level L-1..0: one workgroup per front, LDS-resident solution slice.
// Every front entry is written by exactly one workgroup per step in a fixed order: the
// factor and the solution are bitwise reproducible run to run (no atomics).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"

namespace g2ohip {

using launch::FrontDesc;
using launch::Task;

constexpr int NB = 32;   // panel width
constexpr int TT = 64;   // trailing tile
constexpr int PS = 34;   // LDS row stride (doubles) for the P tiles: conflict-free ds_read_b64
constexpr int EA = 32;   // extend-add column slab

typedef double dx4 __attribute__((ext_vector_type(4)));

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

// front vectors: v_s = [P rhs (own columns); 0]
__global__ void __launch_bounds__(256) k_vec_init(const FrontDesc* __restrict__ fd, const double* __restrict__ rhs_p,
                                                  double* __restrict__ vecs) {
  const FrontDesc me = fd[blockIdx.x];
  const int m = me.ns + me.nr;
  double* v = vecs + me.vec_off;
  for (int i = threadIdx.x; i < m; i += 256) v[i] = i < me.ns ? rhs_p[me.c0 + i] : 0.0;
}

// ---------------------------------------------------------------------------- extend-add
__global__ void __launch_bounds__(256) k_extend_add(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                                    const int* __restrict__ children, const int* __restrict__ relmap,
                                                    double* __restrict__ fronts, double* __restrict__ vecs) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr;
  double* F = fronts + me.front_off;
  double* v = vecs + me.vec_off;
  const int a = t.a, b = t.b;
  for (int k = me.child_begin; k < me.child_end; ++k) {
    const FrontDesc cd = fd[children[k]];
    const int mc = cd.ns + cd.nr, nrc = cd.nr;
    const double* U = fronts + cd.front_off + (size_t)cd.ns * mc + cd.ns;  // U(i,j) = U[j*mc + i]
    const double* u = vecs + cd.vec_off + cd.ns;
    const int* rel = relmap + cd.rows_off;
    // child columns whose parent column lies in [a, b) (rel is increasing)
    int lo = 0, hi = nrc;
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (rel[mid] < a) lo = mid + 1; else hi = mid; }
    const int j0 = lo;
    hi = nrc;
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (rel[mid] < b) lo = mid + 1; else hi = mid; }
    const int j1 = lo;
    for (int j = j0 + (int)threadIdx.x; j < j1; j += 256) v[rel[j]] += u[j];
    // (j, i >= j) pairs of the slab flattened over the workgroup, 4 loads in flight per thread
    const long long tot = (long long)(j1 - j0) * nrc;
    for (long long p0 = threadIdx.x; p0 < tot; p0 += 1024) {
      double val[4];
      long long dsti[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long long p = p0 + q * 256;
        dsti[q] = -1;
        val[q] = 0.0;
        if (p < tot) {
          const int j = j0 + (int)(p / nrc), i = (int)(p % nrc);
          if (i >= j) {
            val[q] = U[(size_t)j * mc + i];
            dsti[q] = (long long)rel[j] * m + rel[i];
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (dsti[q] >= 0) F[dsti[q]] += val[q];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------- wave helpers
// Wave-uniform broadcast of lane `l` (compile-time after unrolling): v_readlane, no LDS.
__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// order this wave's LDS traffic (in-order per wave in hardware; this stops compiler motion)
__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Factor the 32x32 diagonal block held row-wise by lanes 0..31 (row[c] = A(lane, c), c <= lane;
// rows >= kb padded with the identity). Column j of L is broadcast through LDS (col, 32 doubles,
// read back two at a time). On return row[c] = L(lane, c), dinv[lane] = 1 / L(lane, lane).
// Returns false if a pivot was not positive (cs_chol's `d <= 0` test).
__device__ __forceinline__ bool chol32(double (&row)[NB], int lane, double* col, double* dinv) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double djj = rlane(row[j], j);
    ok &= djj > 0.0;
    const double ljj = sqrt(djj > 0.0 ? djj : 1.0);
    const double inv = 1.0 / ljj;
    const double lrj = lane == j ? ljj : (lane > j ? row[j] * inv : 0.0);
    row[j] = lrj;
    if (lane == j) dinv[j] = inv;
    if (j + 1 < NB) {
      if (lane < NB) col[lane] = lrj;
      lds_fence();
#pragma unroll
      for (int c = ((j + 1) & ~1); c < NB; c += 2) {
        const double2 cc = *reinterpret_cast<const double2*>(col + c);
        if (c > j) row[c] -= lrj * cc.x;
        if (c + 1 > j) row[c + 1] -= lrj * cc.y;
      }
      lds_fence();
    }
  }
  return ok;
}

// ---------------------------------------------------------------------------- panel
// Task: s, a = k0, b = first row of this workgroup's row block, c = kb.
// Wave 0 factors the (identity-padded) diagonal block in registers and forward-solves the
// block's rhs; then every wave solves X L_kk^T = P for its 64 rows against the LDS copy of L_kk
// and applies the rhs update v_i -= X_i y.
__global__ void __launch_bounds__(256) k_panel(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                               double* __restrict__ fronts, double* __restrict__ vecs,
                                               double* __restrict__ ysol, double* __restrict__ ldiag,
                                               int* __restrict__ fail) {
  __shared__ __attribute__((aligned(16))) double Lk[NB][NB + 2];  // L_kk, row stride 34 (16-B aligned rows)
  __shared__ __attribute__((aligned(16))) double col[NB];
  __shared__ double dinv[NB];
  __shared__ double yv[NB];
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr;
  double* F = fronts + me.front_off;
  double* v = vecs + me.vec_off;
  const int k0 = t.a, row0 = t.b, kb = t.c;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = k0 + kb;
  const int i = row0 + w * 64 + lane;
  const bool act = i < m;
  double x[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) x[q] = (act && q < kb) ? F[(size_t)(k0 + q) * m + i] : 0.0;
  if (w == 0) {
    double row[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      double a = 0.0;
      if (lane < kb && c <= lane) a = F[(size_t)(k0 + c) * m + k0 + lane];
      if (lane >= kb && c == lane) a = 1.0;
      row[c] = a;
    }
    const bool ok = chol32(row, lane, col, dinv);
    if (lane < NB) {
#pragma unroll
      for (int c = 0; c < NB; ++c) Lk[lane][c] = row[c];
    }
    lds_fence();
    // L_kk y = v(k0 .. k0+kb)
    double y = lane < kb ? v[k0 + lane] : 0.0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const double yj = rlane(y, j) * dinv[j];
      y = lane == j ? yj : (lane > j ? y - row[j] * yj : y);
    }
    if (lane < NB) yv[lane] = y;
    if (row0 == r0) {  // first workgroup of the front publishes L_kk and y_k
      // L_kk goes to the (unused) upper triangle of the diagonal block, transposed, and its
      // diagonal to ldiag: the lower triangle keeps A_kk, which the other workgroups of this
      // launch may still be reading.
      if (lane == 0 && !ok) *fail = 1;
      if (lane < kb) {
        double dg = 0.0;
#pragma unroll
        for (int c = 0; c < NB; ++c) {
          if (c < lane) F[(size_t)(k0 + lane) * m + k0 + c] = row[c];
          dg = c == lane ? row[c] : dg;
        }
        ldiag[me.c0 + k0 + lane] = dg;
        ysol[me.c0 + k0 + lane] = y;
      }
    }
  }
  __syncthreads();
  double s2 = 0.0;
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    double s = x[q];
#pragma unroll
    for (int u = 0; u + 1 < q; u += 2) {
      const double2 l2 = *reinterpret_cast<const double2*>(&Lk[q][u]);
      s -= x[u] * l2.x;
      s -= x[u + 1] * l2.y;
    }
    if (q & 1) s -= x[q - 1] * Lk[q][q - 1];
    x[q] = s * dinv[q];
    s2 += x[q] * yv[q];
  }
  if (act) {
#pragma unroll
    for (int q = 0; q < NB; ++q)
      if (q < kb) F[(size_t)(k0 + q) * m + i] = x[q];
    v[i] -= s2;
  }
}

// ---------------------------------------------------------------------------- trailing update (MFMA)
// Task: s, a = k0, b = ti | tj << 16, c = kb.  C[I,J] -= P_I P_J^T on the lower triangle.
__global__ void __launch_bounds__(256) k_trail(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                               double* __restrict__ fronts) {
  __shared__ double sh[2 * TT * PS];  // Pa | Pb, reused as the 64 x 65 result tile
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr;
  double* F = fronts + me.front_off;
  const int k0 = t.a, kb = t.c;
  const int ti = t.b & 0xffff, tj = t.b >> 16;
  const int r0 = k0 + kb;
  const int I0 = r0 + ti * TT, J0 = r0 + tj * TT;
  const int tid = threadIdx.x;
  double* Pa = sh;
  double* Pb = sh + TT * PS;
  for (int idx = tid; idx < TT * NB; idx += 256) {
    const int r = idx % TT, k = idx / TT;
    const bool kin = k < kb;
    Pa[r * PS + k] = (kin && I0 + r < m) ? F[(size_t)(k0 + k) * m + I0 + r] : 0.0;
    Pb[r * PS + k] = (kin && J0 + r < m) ? F[(size_t)(k0 + k) * m + J0 + r] : 0.0;
  }
  __syncthreads();
  const int lane = tid & 63, w = tid >> 6;
  const int wr = (w & 1) * 32, wc = (w >> 1) * 32;
  const int lr = lane & 15, lk = lane >> 4;
  dx4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = dx4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int k = kk * 4 + lk;
    const double a0 = Pa[(wr + lr) * PS + k], a1 = Pa[(wr + 16 + lr) * PS + k];
    const double b0 = Pb[(wc + lr) * PS + k], b1 = Pb[(wc + 16 + lr) * PS + k];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
  __syncthreads();
  // D layout of v_mfma_f64_16x16x4f64: lane l holds D[(l>>4) + 4*i][l & 15], i = 0..3
  constexpr int CS = TT + 1;
  double* Ct = sh;  // [row][col] with stride CS
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wr + x * 16 + lk + 4 * i, col = wc + y * 16 + lr;
        Ct[row * CS + col] = acc[x][y][i];
      }
  __syncthreads();
  for (int idx = tid; idx < TT * TT; idx += 256) {
    const int r = idx % TT, c = idx / TT;
    const int gi = I0 + r, gj = J0 + c;
    if (gi < m && gj < m && gi >= gj) F[(size_t)gj * m + gi] -= Ct[r * CS + c];
  }
}

__global__ void k_permute(int n, const int* __restrict__ perm, const double* __restrict__ in, double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] = in[perm[k]];
}
__global__ void k_ipermute(int n, const int* __restrict__ perm, const double* __restrict__ in, double* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[perm[k]] = in[k];
}


// ---------------------------------------------------------------------------- backward solve
// x_s = L11^-T (y_s - L21^T x_rows): first the L21^T x_rows GEMV with one thread per column
// (sequential, cache-line friendly column reads), then 32-column blocks from the last: the
// in-supernode column dots by 8 threads per column, the 32x32 triangle by one wave in registers.
__global__ void __launch_bounds__(256) k_chol_backward(const int* __restrict__ level_list, const FrontDesc* __restrict__ fd,
                                                       const int* __restrict__ rows, const double* __restrict__ fronts,
                                                       const double* __restrict__ ysol, const double* __restrict__ ldiag,
                                                       double* __restrict__ xsol) {
  extern __shared__ __attribute__((aligned(16))) double xs[];  // [m]: own x (being solved) then x_rows
  __shared__ double red[8][NB];
  const int s = level_list[blockIdx.x];
  const FrontDesc me = fd[s];
  const int m = me.ns + me.nr, ns = me.ns;
  const double* F = fronts + me.front_off;
  const int* rw = rows + me.rows_off;
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < m; i += 256) xs[i] = i < ns ? ysol[me.c0 + i] : xsol[rw[i - ns]];
  __syncthreads();
  for (int j = tid; j < ns; j += 256) {
    const double* col = F + (size_t)j * m + ns;
    double acc = 0.0;
    for (int i = 0; i < me.nr; ++i) acc += col[i] * xs[ns + i];
    xs[j] -= acc;
  }
  __syncthreads();
  const int nblk = (ns + NB - 1) / NB;
  const int q = tid & (NB - 1), g = tid >> 5;
  for (int bk = nblk - 1; bk >= 0; --bk) {
    const int k0 = bk * NB, kb = min(NB, ns - k0);
    double part = 0.0;
    if (q < kb) {
      const double* col = F + (size_t)(k0 + q) * m;
      for (int i = k0 + kb + g; i < ns; i += 8) part += col[i] * xs[i];
    }
    red[g][q] = part;
    __syncthreads();
    if (tid < 64) {
      double Lc[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        double a = 0.0;
        if (lane < kb && j > lane && j < kb) a = F[(size_t)(k0 + j) * m + k0 + lane];  // L(j, lane), upper storage
        if (lane < kb && j == lane) a = ldiag[me.c0 + k0 + lane];
        if (lane >= kb && j == lane) a = 1.0;
        Lc[j] = a;
      }
      double v = 0.0;
      if (lane < kb) {
        double r = xs[k0 + lane];
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) r -= red[gg][lane];
        v = r;
      }
      double dg = 1.0;
#pragma unroll
      for (int j = 0; j < NB; ++j) dg = j == lane ? Lc[j] : dg;
      const double rinv = 1.0 / dg;
#pragma unroll
      for (int j = NB - 1; j >= 0; --j) {
        const double xj = rlane(v, j) * rlane(rinv, j);
        v = lane == j ? xj : (lane < j ? v - Lc[j] * xj : v);
      }
      if (lane < kb) xs[k0 + lane] = v;
    }
    __syncthreads();
  }
  for (int j = tid; j < ns; j += 256) xsol[me.c0 + j] = xs[j];
}

namespace launch {

void chol_scatter(long long nent, const double* vals, const long long* dst, const unsigned char* is_diag,
                  const double* lam, double* fronts, hipStream_t s) {
  if (nent <= 0) return;
  hipLaunchKernelGGL(k_chol_scatter, grid_for(nent, 256), 256, 0, s, nent, vals, dst, is_diag, lam, fronts);
  KERNEL_CHECK();
}
void chol_vec_init(int nfronts, const FrontDesc* fd, const double* rhs_p, double* vecs, hipStream_t s) {
  if (nfronts <= 0) return;
  hipLaunchKernelGGL(k_vec_init, nfronts, 256, 0, s, fd, rhs_p, vecs);
  KERNEL_CHECK();
}
void chol_extend_add(int ntasks, const Task* tasks, const FrontDesc* fd, const int* children, const int* relmap,
                     double* fronts, double* vecs, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_extend_add, ntasks, 256, 0, s, tasks, fd, children, relmap, fronts, vecs);
  KERNEL_CHECK();
}
void chol_panel(int ntasks, const Task* tasks, const FrontDesc* fd, double* fronts, double* vecs, double* ysol,
                double* ldiag, int* fail, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_panel, ntasks, 256, 0, s, tasks, fd, fronts, vecs, ysol, ldiag, fail);
  KERNEL_CHECK();
}
void chol_trail(int ntasks, const Task* tasks, const FrontDesc* fd, double* fronts, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_trail, ntasks, 256, 0, s, tasks, fd, fronts);
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
void chol_backward(int nfronts, const int* level_list, const FrontDesc* fd, const int* rows, const double* fronts,
                   const double* ysol, const double* ldiag, double* xsol, int max_m, hipStream_t s) {
  if (nfronts <= 0) return;
  const size_t bytes = (size_t)max_m * sizeof(double);
  if (bytes > 150 * 1024) throw DeviceError("front larger than LDS for the backward solve");
  if (bytes > 64 * 1024)
    HIP_CHECK(hipFuncSetAttribute((const void*)k_chol_backward, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  hipLaunchKernelGGL(k_chol_backward, nfronts, 256, bytes, s, level_list, fd, rows, fronts, ysol, ldiag, xsol);
  KERNEL_CHECK();
}

}  // namespace launch
}  // namespace g2ohip
