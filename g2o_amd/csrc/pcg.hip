// Block-Jacobi PCG (linear_solver_pcg.hpp:80-159) on gfx950.
//
// One PCG iteration is four launches on the solver stream:
//   k_pcg_spmv    q = A d (thread per scalar row, its block row's entries, upper blocks used directly or
//                 transposed, linear_solver_pcg.hpp:180-197); d itself is never materialised by a separate
//                 pass: d = s + β d_prev is formed on the fly from s and the previous direction (double
//                 buffered), and each workgroup leaves its partial of d·q
//   k_pcg_alpha   α = dn / d·q (one workgroup, partials summed in a fixed order)
//   k_pcg_update  x += α d, r -= α q, s = J r (thread per block row), partial of r·s
//   k_pcg_beta    dn' = r·s, β = dn'/dn, iteration count, convergence flag (dn' <= d0 or maxIter)
// Every launch returns at once when the flag is set, so the host enqueues CHUNK iterations between
// convergence checks. All reductions use fixed trees: results are bitwise reproducible.
#include "pcg.hpp"

#include <cmath>

namespace g2ohip {
namespace {

constexpr int PB = 256;
constexpr int CHUNK = 16;
enum { SC_DN = 0, SC_D0, SC_A, SC_BA, SC_ITER, SC_DONE, SC_RESID, SC_NAN, SC_N };

__device__ inline double block_sum(double v, double* sh) {
  __syncthreads();  // sh may still be read from a previous call
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int s = PB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  return sh[0];
}
__device__ inline double sum_partials(const double* p, int np, double* sh) {
  double v = 0.0;
  for (int k = threadIdx.x; k < np; k += PB) v += p[k];
  return block_sum(v, sh);
}

// J_i = (D_i + λ I)^-1 (linear_solver_pcg.hpp:92-96: Eigen's inverse() of the diagonal block, i.e. an LU with
// partial pivoting). Gauss-Jordan with row pivoting, pivot rows exchanged by selects so the register arrays
// keep compile-time indices. Indefinite blocks invert like the reference's (no Cholesky NaN).
template <int PD>
__global__ void __launch_bounds__(PB) k_pcg_jacobi(int nb, const int* __restrict__ diag, const double* __restrict__ vals,
                                                   const double* __restrict__ lam, double* __restrict__ J) {
  const int i = blockIdx.x * PB + threadIdx.x;
  if (i >= nb) return;
  const double* D = vals + (size_t)diag[i] * PD * PD;
  const double l = *lam;
  double M[PD][PD], V[PD][PD];
#pragma unroll
  for (int r = 0; r < PD; ++r)
#pragma unroll
    for (int c = 0; c < PD; ++c) {
      M[r][c] = D[c * PD + r] + (r == c ? l : 0.0);
      V[r][c] = r == c ? 1.0 : 0.0;
    }
#pragma unroll
  for (int c = 0; c < PD; ++c) {
    int p = c;
    double best = fabs(M[c][c]);
#pragma unroll
    for (int r = c + 1; r < PD; ++r)
      if (fabs(M[r][c]) > best) { best = fabs(M[r][c]); p = r; }
#pragma unroll
    for (int r = c + 1; r < PD; ++r) {
      const bool sw = r == p;
#pragma unroll
      for (int k = 0; k < PD; ++k) {
        const double m0 = M[c][k], m1 = M[r][k], v0 = V[c][k], v1 = V[r][k];
        M[c][k] = sw ? m1 : m0; M[r][k] = sw ? m0 : m1;
        V[c][k] = sw ? v1 : v0; V[r][k] = sw ? v0 : v1;
      }
    }
    const double inv = 1.0 / M[c][c];
#pragma unroll
    for (int k = 0; k < PD; ++k) { M[c][k] *= inv; V[c][k] *= inv; }
#pragma unroll
    for (int r = 0; r < PD; ++r) {
      if (r == c) continue;
      const double f = M[r][c];
#pragma unroll
      for (int k = 0; k < PD; ++k) { M[r][k] -= f * M[c][k]; V[r][k] -= f * V[c][k]; }
    }
  }
  double* Jo = J + (size_t)i * PD * PD;
#pragma unroll
  for (int c = 0; c < PD; ++c)
#pragma unroll
    for (int r = 0; r < PD; ++r) Jo[c * PD + r] = V[r][c];
}

// x = 0, r = b, s = J r (= the first direction), d_prev = 0, partial of r·s (linear_solver_pcg.hpp:118-123)
template <int PD>
__global__ void __launch_bounds__(PB) k_pcg_init(int nb, const double* __restrict__ J, const double* __restrict__ b,
                                                 double* __restrict__ x, double* __restrict__ r, double* __restrict__ s,
                                                 double* __restrict__ dprev, double* __restrict__ part) {
  __shared__ double sh[PB];
  const int i = blockIdx.x * PB + threadIdx.x;
  double rs = 0.0;
  if (i < nb) {
    double rv[PD];
#pragma unroll
    for (int c = 0; c < PD; ++c) {
      const size_t k = (size_t)i * PD + c;
      rv[c] = b[k];
      r[k] = rv[c];
      x[k] = 0.0;
      dprev[k] = 0.0;
    }
    const double* Ji = J + (size_t)i * PD * PD;
#pragma unroll
    for (int rr = 0; rr < PD; ++rr) {
      double t = 0.0;
#pragma unroll
      for (int c = 0; c < PD; ++c) t += Ji[c * PD + rr] * rv[c];
      s[(size_t)i * PD + rr] = t;
      rs += rv[rr] * t;
    }
  }
  const double t = block_sum(rs, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// dn = r·s, d0 = tol dn (or the carried absolute residual), linear_solver_pcg.hpp:123-130
__global__ void __launch_bounds__(PB) k_pcg_start(const double* __restrict__ part, int np, double tol, int abs_tol,
                                                  int maxit, double* __restrict__ sc) {
  __shared__ double sh[PB];
  const double dn = sum_partials(part, np, sh);
  if (threadIdx.x == 0) {
    double d0 = tol * dn;
    const double res = sc[SC_RESID];
    if (abs_tol && res > 0.0 && res > d0) d0 = res;
    sc[SC_DN] = dn;
    sc[SC_D0] = d0;
    sc[SC_BA] = 0.0;
    sc[SC_ITER] = 0.0;
    // a NaN residual never satisfies dn <= d0: the reference keeps iterating to maxIter and returns a NaN
    // x (every later x += a d is NaN); stop here and poison x instead (k_pcg_finish), same result
    const bool nan = dn != dn;
    sc[SC_NAN] = nan ? 1.0 : 0.0;
    sc[SC_DONE] = (dn <= d0 || maxit <= 0 || nan) ? 1.0 : 0.0;
  }
}

template <int PD>
__global__ void __launch_bounds__(PB)
    k_pcg_spmv(int n, const int* __restrict__ rptr, const int2* __restrict__ ent, const int* __restrict__ diag,
               const double* __restrict__ vals, const double* __restrict__ lam, const double* __restrict__ s,
               const double* __restrict__ dprev, double* __restrict__ dcur, double* __restrict__ q,
               double* __restrict__ part, const double* __restrict__ sc) {
  __shared__ double sh[PB];
  if (sc[SC_DONE] != 0.0) return;
  const double ba = sc[SC_BA];
  const int row = blockIdx.x * PB + threadIdx.x;
  double dq = 0.0;
  if (row < n) {
    const int i = row / PD, rr = row - i * PD;
    auto dv = [&](int j, int c) {
      const size_t k = (size_t)j * PD + c;
      return s[k] + ba * dprev[k];
    };
    const double d = dv(i, rr);
    const double* D = vals + (size_t)diag[i] * PD * PD;
    double y = *lam * d;
#pragma unroll
    for (int c = 0; c < PD; ++c) y += D[c * PD + rr] * dv(i, c);
    const int e1 = rptr[i + 1];
    for (int e = rptr[i]; e < e1; ++e) {
      const int2 t = ent[e];
      const int j = t.y & 0x7fffffff;
      const double* B = vals + (size_t)t.x * PD * PD;
      if (t.y < 0) {
#pragma unroll
        for (int c = 0; c < PD; ++c) y += B[rr * PD + c] * dv(j, c);
      } else {
#pragma unroll
        for (int c = 0; c < PD; ++c) y += B[c * PD + rr] * dv(j, c);
      }
    }
    dcur[row] = d;
    q[row] = y;
    dq = d * y;
  }
  const double t = block_sum(dq, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void __launch_bounds__(PB) k_pcg_alpha(const double* __restrict__ part, int np, double* __restrict__ sc) {
  __shared__ double sh[PB];
  if (sc[SC_DONE] != 0.0) return;
  const double dq = sum_partials(part, np, sh);
  if (threadIdx.x == 0) sc[SC_A] = sc[SC_DN] / dq;
}

template <int PD>
__global__ void __launch_bounds__(PB)
    k_pcg_update(int nb, const double* __restrict__ J, const double* __restrict__ d, const double* __restrict__ q,
                 double* __restrict__ x, double* __restrict__ r, double* __restrict__ s, double* __restrict__ part,
                 const double* __restrict__ sc) {
  __shared__ double sh[PB];
  if (sc[SC_DONE] != 0.0) return;
  const double a = sc[SC_A];
  const int i = blockIdx.x * PB + threadIdx.x;
  double rs = 0.0;
  if (i < nb) {
    double rv[PD];
#pragma unroll
    for (int c = 0; c < PD; ++c) {
      const size_t k = (size_t)i * PD + c;
      x[k] += a * d[k];
      rv[c] = r[k] - a * q[k];
      r[k] = rv[c];
    }
    const double* Ji = J + (size_t)i * PD * PD;
#pragma unroll
    for (int rr = 0; rr < PD; ++rr) {
      double t = 0.0;
#pragma unroll
      for (int c = 0; c < PD; ++c) t += Ji[c * PD + rr] * rv[c];
      s[(size_t)i * PD + rr] = t;
      rs += rv[rr] * t;
    }
  }
  const double t = block_sum(rs, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void __launch_bounds__(PB) k_pcg_beta(const double* __restrict__ part, int np, int maxit,
                                                 double* __restrict__ sc) {
  __shared__ double sh[PB];
  if (sc[SC_DONE] != 0.0) return;
  const double dn = sum_partials(part, np, sh);
  if (threadIdx.x == 0) {
    const double it = sc[SC_ITER] + 1.0;
    sc[SC_BA] = dn / sc[SC_DN];
    sc[SC_DN] = dn;
    sc[SC_ITER] = it;
    const bool nan = dn != dn;
    if (nan) sc[SC_NAN] = 1.0;
    sc[SC_DONE] = (dn <= sc[SC_D0] || it >= (double)maxit || nan) ? 1.0 : 0.0;
  }
}

// _residual = 0.5 dn (:153); a NaN recurrence leaves x NaN, as the reference's maxIter NaN iterations would
__global__ void __launch_bounds__(PB) k_pcg_finish(int n, double* __restrict__ x, double* __restrict__ sc) {
  const bool nan = sc[SC_NAN] != 0.0;
  if (nan)
    for (int k = blockIdx.x * PB + threadIdx.x; k < n; k += gridDim.x * PB) x[k] = __builtin_nan("");
  if (blockIdx.x == 0 && threadIdx.x == 0) sc[SC_RESID] = 0.5 * sc[SC_DN];
}

// stream capture that always ends (and frees its graph) even when a capture call throws
struct CaptureGuard {
  hipStream_t st;
  hipGraph_t g = nullptr;
  bool open = true;
  explicit CaptureGuard(hipStream_t s) : st(s) { HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal)); }
  hipGraph_t end() {
    open = false;
    HIP_CHECK(hipStreamEndCapture(st, &g));
    return g;
  }
  ~CaptureGuard() {
    if (open) (void)hipStreamEndCapture(st, &g);
    if (g) (void)hipGraphDestroy(g);
  }
};

template <int PD>
void run(int nb, int n, int npa, int npb, int maxit, double tol, int abs_tol, const int* rptr, const int2* ent,
         const int* diag, const double* vals, const double* lam, const double* b, double* x, double* J, double* r,
         double* sv, double* q, double* dbuf, double* part, double* sc, int& iters, hipGraphExec_t& exec,
         const void* (&key)[4], hipStream_t st) {
  double* pa = part;
  double* pbp = part + npa;
  double* dA = dbuf;
  double* dB = dbuf + n;
  const unsigned gb = grid_for(nb, PB), gn = grid_for(n, PB);
  hipLaunchKernelGGL(k_pcg_jacobi<PD>, gb, PB, 0, st, nb, diag, vals, lam, J);
  hipLaunchKernelGGL(k_pcg_init<PD>, gb, PB, 0, st, nb, J, b, x, r, sv, dA, pbp);
  hipLaunchKernelGGL(k_pcg_start, 1, PB, 0, st, pbp, npb, tol, abs_tol, maxit, sc);
  KERNEL_CHECK();
  double h[SC_N];
  auto enqueue = [&](int k0, int cnt) {
    for (int k = k0; k < k0 + cnt; ++k) {
      double* dprev = (k & 1) ? dB : dA;
      double* dcur = (k & 1) ? dA : dB;
      hipLaunchKernelGGL(k_pcg_spmv<PD>, gn, PB, 0, st, n, rptr, ent, diag, vals, lam, sv, dprev, dcur, q, pa, sc);
      hipLaunchKernelGGL(k_pcg_alpha, 1, PB, 0, st, pa, npa, sc);
      hipLaunchKernelGGL(k_pcg_update<PD>, gb, PB, 0, st, nb, J, dcur, q, x, r, sv, pbp, sc);
      hipLaunchKernelGGL(k_pcg_beta, 1, PB, 0, st, pbp, npb, maxit, sc);
    }
  };
  // full chunks (always starting at an even k) replay one captured graph of CHUNK iterations
  const void* want[4] = {vals, lam, x, (const void*)(size_t)maxit};
  for (int k = 0; k < maxit;) {
    const int cnt = maxit - k < CHUNK ? maxit - k : CHUNK;
    if (cnt == CHUNK) {
      if (!exec || key[0] != want[0] || key[1] != want[1] || key[2] != want[2] || key[3] != want[3]) {
        if (exec) HIP_CHECK(hipGraphExecDestroy(exec));
        exec = nullptr;
        for (auto& k : key) k = nullptr;  // set only once a graph is instantiated
        {
          CaptureGuard cap(st);
          enqueue(0, CHUNK);
          hipGraph_t g = cap.end();
          hipGraphExec_t ex = nullptr;
          HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
          exec = ex;
        }
        for (int u = 0; u < 4; ++u) key[u] = want[u];
      }
      HIP_CHECK(hipGraphLaunch(exec, st));
    } else {
      enqueue(k, cnt);
    }
    k += cnt;
    KERNEL_CHECK();
    HIP_CHECK(hipMemcpyAsync(h, sc, sizeof h, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h[SC_DONE] != 0.0) break;
  }
  hipLaunchKernelGGL(k_pcg_finish, grid_for(n, PB) < 1024 ? grid_for(n, PB) : 1024, PB, 0, st, n, x, sc);
  KERNEL_CHECK();
  HIP_CHECK(hipMemcpyAsync(h, sc, sizeof h, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  iters = (int)h[SC_ITER];
}

}  // namespace

void DevicePCG::setup(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj, hipStream_t s) {
  if (bdim != 3 && bdim != 6) throw std::runtime_error("DevicePCG: block dimension must be 3 or 6");
  if (chunk_exec) HIP_CHECK(hipGraphExecDestroy(chunk_exec));
  chunk_exec = nullptr;
  nb = nblocks;
  pd = bdim;
  n = nb * pd;
  std::vector<int> dg(nb, -1), cnt(nb + 1, 0);
  for (size_t t = 0; t < bi.size(); ++t) {
    if (bi[t] == bj[t]) dg[bi[t]] = (int)t;
    else { ++cnt[bi[t] + 1]; ++cnt[bj[t] + 1]; }
  }
  for (int i = 0; i < nb; ++i) {
    if (dg[i] < 0) throw std::runtime_error("DevicePCG: missing diagonal block " + std::to_string(i));
    cnt[i + 1] += cnt[i];
  }
  std::vector<int2> e(cnt[nb]);
  std::vector<int> fill(cnt.begin(), cnt.end() - 1);
  for (size_t t = 0; t < bi.size(); ++t) {
    if (bi[t] == bj[t]) continue;
    e[fill[bi[t]]++] = make_int2((int)t, bj[t]);                                 // A(bi, bj) = B
    e[fill[bj[t]]++] = make_int2((int)t, (int)((unsigned)bi[t] | 0x80000000u));  // A(bj, bi) = B^T
  }
  rptr.upload(cnt, s);
  diag.upload(dg, s);
  ent.upload(e.empty() ? std::vector<int2>{make_int2(0, 0)} : e, s);
  npa = (int)grid_for(n, PB);
  npb = (int)grid_for(nb, PB);
  J.resize((size_t)nb * pd * pd);
  r.resize(n);
  sv.resize(n);
  q.resize(n);
  dbuf.resize(2 * (size_t)n);
  part.resize(npa + npb);
  sc.resize(SC_N);
  reset(s);
}

void DevicePCG::reset(hipStream_t s) {
  const double init[SC_N] = {0, 0, 0, 0, 0, 0, -1.0, 0};  // _residual = -1 (linear_solver_pcg.h:56,66)
  HIP_CHECK(hipMemcpyAsync(sc.get(), init, sizeof init, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

void DevicePCG::solve(const double* vals, const double* lam, const double* b, double* x, hipStream_t s) {
  if (nb <= 0) return;
  const int maxit = max_iter < 0 ? n : max_iter;  // :132
  if (pd == 6)
    run<6>(nb, n, npa, npb, maxit, tolerance, absolute_tolerance, rptr.get(), ent.get(), diag.get(), vals, lam, b, x,
           J.get(), r.get(), sv.get(), q.get(), dbuf.get(), part.get(), sc.get(), last_iterations, chunk_exec, chunk_key, s);
  else
    run<3>(nb, n, npa, npb, maxit, tolerance, absolute_tolerance, rptr.get(), ent.get(), diag.get(), vals, lam, b, x,
           J.get(), r.get(), sv.get(), q.get(), dbuf.get(), part.get(), sc.get(), last_iterations, chunk_exec, chunk_key, s);
}

}  // namespace g2ohip
