// Matrix-free preconditioned CGLS of the fork's LinearSolverPCGEigen (see cgls.hpp) on gfx950.
//
// Per LM iteration (buildSystem): k_cgls_jac stores every observation's two Jacobian rows scaled by sqrt(Omega00)
// (point 2x3 and camera 2x6 blocks, the camera block again in camera-major order), k_cgls_gram_* the block Gram
// matrices J_b^T J_b. Per LM trial (solve): k_cgls_prec factors J_b^T J_b + lambda I = R^T R per camera / point and
// keeps R^-1; five init launches build y0, p = s = R^-T (b - J^T J R^-1 y0), q = J R^-1 p; then five launches per CG
// iteration, the active block alternating (odd: cameras, even: points):
//   k_cgls_alpha   stop test gamma < eta gamma0, alpha = gamma / q.q   (one workgroup, fixed-order sums)
//   k_cgls_grad_*  s_b = R_b^-T (-alpha J_b^T q) for the active block type, partials of s.s
//   k_cgls_beta    gamma' = s.s, beta = gamma'/gamma
//   k_cgls_dir     y += alpha p, p = s + beta p, z = R^-1 s (active block)
//   k_cgls_q       q = beta q + J_b z (edge rows and lambda rows), partials of q.q
// All reductions are fixed trees: bitwise reproducible. Iterations run in captured chunks between host checks.
#include "cgls.hpp"

#include <cmath>

#include "device_types.hpp"
#include "device_util.hpp"

namespace g2ohip {
namespace {

constexpr int B = 256;
constexpr int CHUNK = 16;  // even: a chunk always starts on a point (even) iteration
enum { SC_GAMMA = 0, SC_THR, SC_ALPHA, SC_BETA, SC_DONE, SC_ITER, SC_SQL, SC_MAXIT, SC_N };

__device__ inline double block_sum(double v, double* sh) {
  __syncthreads();
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int s = B / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] += sh[threadIdx.x + s];
    __syncthreads();
  }
  return sh[0];
}
__device__ inline double sum_parts(const double* p, int np, double* sh) {
  double v = 0.0;
  for (int k = threadIdx.x; k < np; k += B) v += p[k];
  return block_sum(v, sh);
}
// 6 values summed over a workgroup in a fixed tree
__device__ inline void wg_sum6(double (&a)[6], double (*red)[6]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < 6; ++k) a[k] += __shfl_xor(a[k], m, 64);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) red[w][k] = a[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 6; ++k) a[k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
}
// y = R^-1 x (tr = false) or R^-T x (tr = true), R^-1 row-major D x D
template <int D, bool TR>
__device__ inline void rmul(const double* Ri, const double* x, double* y) {
#pragma unroll
  for (int r = 0; r < D; ++r) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < D; ++c) s += (TR ? Ri[c * D + r] : Ri[r * D + c]) * x[c];
    y[r] = s;
  }
}

// ---- buildSystem: J blocks ----
__global__ void __launch_bounds__(B) k_cgls_jac(dev::EdgeData d, int ne, const int* __restrict__ h0,
                                                const int* __restrict__ h1, double* __restrict__ JA,
                                                double* __restrict__ JB) {
  const int e = blockIdx.x * B + threadIdx.x;
  if (e >= ne) return;
  double err[2], A[6], Bm[12];
  dev::FamilyBA::linearize(d, e, err, A, Bm);
  const double si = sqrt(dev::info_rec(d, e, dev::FamilyBA::INFO)[0]);  // sqrt(Omega(0,0)) (jacobi_solver.hpp:563)
  const bool fa = h0[d.v0[e]] >= 0, fb = h1[d.v1[e]] >= 0;
#pragma unroll
  for (int k = 0; k < 6; ++k) JA[(size_t)e * 6 + k] = fa ? A[k] * si : 0.0;
#pragma unroll
  for (int k = 0; k < 12; ++k) JB[(size_t)e * 12 + k] = fb ? Bm[k] * si : 0.0;
}
__global__ void __launch_bounds__(B) k_cgls_gather_cam(int nce, const int* __restrict__ cam_e,
                                                       const double* __restrict__ JB, double* __restrict__ JBc) {
  const int k = blockIdx.x * B + threadIdx.x;
  if (k >= nce) return;
  const double* s = JB + (size_t)cam_e[k] * 12;
#pragma unroll
  for (int u = 0; u < 12; ++u) JBc[(size_t)k * 12 + u] = s[u];
}
// camera Gram blocks: one workgroup per camera, 21 sums (upper) in a fixed tree
__global__ void __launch_bounds__(B) k_cgls_gram_cam(int ncam, const int* __restrict__ cam_ptr,
                                                     const double* __restrict__ JBc, double* __restrict__ Gc) {
  __shared__ double red[4][21];
  const int c = blockIdx.x;
  double a[21];
#pragma unroll
  for (int k = 0; k < 21; ++k) a[k] = 0.0;
  for (int p = cam_ptr[c] + threadIdx.x; p < cam_ptr[c + 1]; p += B) {
    const double* J = JBc + (size_t)p * 12;
    int k = 0;
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i) a[k++] += J[i] * J[j] + J[6 + i] * J[6 + j];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < 21; ++k) a[k] += __shfl_xor(a[k], m, 64);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 21; ++k) red[w][k] = a[k];
  __syncthreads();
  if (threadIdx.x < 21) {
    const int t = threadIdx.x;
    const double v = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
    int j = 0, base = 0;
    while (t >= base + j + 1) base += ++j;
    const int i = t - base;
    Gc[(size_t)c * 36 + i * 6 + j] = v;
    Gc[(size_t)c * 36 + j * 6 + i] = v;
  }
}
__global__ void __launch_bounds__(B) k_cgls_gram_pt(int npt, const int* __restrict__ pt_ptr,
                                                    const double* __restrict__ JA, double* __restrict__ Gp) {
  const int l = blockIdx.x * B + threadIdx.x;
  if (l >= npt) return;
  double a[6] = {0, 0, 0, 0, 0, 0};
  for (int e = pt_ptr[l]; e < pt_ptr[l + 1]; ++e) {
    const double* J = JA + (size_t)e * 6;
    int k = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int i = 0; i <= j; ++i) a[k++] += J[i] * J[j] + J[3 + i] * J[3 + j];
  }
  int k = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      Gp[(size_t)l * 9 + i * 3 + j] = a[k];
      Gp[(size_t)l * 9 + j * 3 + i] = a[k];
      ++k;
    }
}

// ---- per trial: R^-1 of every block, R^T R = G + lambda I (R upper, positive diagonal) ----
template <int D>
__global__ void __launch_bounds__(B) k_cgls_prec(int nb, const double* __restrict__ G, const double* __restrict__ lam,
                                                 double* __restrict__ Ri, double* __restrict__ sc) {
  const int i = blockIdx.x * B + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) sc[SC_SQL] = sqrt(*lam);
  if (i >= nb) return;
  const double l = *lam;
  const double* g = G + (size_t)i * D * D;
  double R[D][D], V[D][D];
#pragma unroll
  for (int r = 0; r < D; ++r)
#pragma unroll
    for (int c = 0; c < D; ++c) R[r][c] = 0.0;
#pragma unroll
  for (int j = 0; j < D; ++j) {  // upper Cholesky: R(j, c) = (G(j, c) - sum_k R(k, j) R(k, c)) / R(j, j)
    double dj = g[j * D + j] + l;
#pragma unroll
    for (int k = 0; k < j; ++k) dj -= R[k][j] * R[k][j];
    const double rjj = sqrt(dj);
    R[j][j] = rjj;
#pragma unroll
    for (int c = j + 1; c < D; ++c) {
      double t = g[j * D + c];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= R[k][j] * R[k][c];
      R[j][c] = t / rjj;
    }
  }
#pragma unroll
  for (int c = 0; c < D; ++c) {  // V = R^-1 (upper), column by column
#pragma unroll
    for (int r = D - 1; r >= 0; --r) {
      double t = r == c ? 1.0 : 0.0;
#pragma unroll
      for (int k = r + 1; k < D; ++k) t -= R[r][k] * V[k][c];
      V[r][c] = r > c ? 0.0 : t / R[r][r];
    }
  }
  double* o = Ri + (size_t)i * D * D;
#pragma unroll
  for (int r = 0; r < D; ++r)
#pragma unroll
    for (int c = 0; c < D; ++c) o[r * D + c] = V[r][c];
}

// ---- init ----
// cameras: p_C = R^-T b_C (pre-conditioned b), y_C = 0, z_C = 0; points: p_P = R^-T b_P, y_P = p_P, z_P = R^-1 y_P
__global__ void __launch_bounds__(B) k_cgls_init_a(int ncam, int npt, const double* __restrict__ Rc,
                                                   const double* __restrict__ Rp, const double* __restrict__ b,
                                                   double* __restrict__ p, double* __restrict__ y,
                                                   double* __restrict__ z) {
  const int i = blockIdx.x * B + threadIdx.x;
  if (i < ncam) {
    double t[6];
    rmul<6, true>(Rc + (size_t)i * 36, b + (size_t)i * 6, t);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      p[(size_t)i * 6 + k] = t[k];
      y[(size_t)i * 6 + k] = 0.0;
      z[(size_t)i * 6 + k] = 0.0;
    }
  } else if (i < ncam + npt) {
    const int l = i - ncam;
    const size_t o = (size_t)ncam * 6 + (size_t)l * 3;
    double t[3], u[3];
    rmul<3, true>(Rp + (size_t)l * 9, b + o, t);
    rmul<3, false>(Rp + (size_t)l * 9, t, u);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      p[o + k] = t[k];
      y[o + k] = t[k];
      z[o + k] = u[k];
    }
  }
}
// q = J z: edge rows (point block + camera block) and lambda rows; optional partials of q.q
__global__ void __launch_bounds__(B) k_cgls_jz(int ne, int n, int ncam, const int* __restrict__ e_cam,
                                               const int* __restrict__ e_pt, const double* __restrict__ JA,
                                               const double* __restrict__ JB, const double* __restrict__ z,
                                               double* __restrict__ q, const double* __restrict__ sc,
                                               double* __restrict__ part) {
  __shared__ double sh[B];
  const int t = blockIdx.x * B + threadIdx.x;
  double qq = 0.0;
  if (t < ne) {
    const int c = e_cam[t], l = e_pt[t];
    double r0 = 0.0, r1 = 0.0;
    if (l >= 0) {
      const double* A = JA + (size_t)t * 6;
      const double* zp = z + (size_t)ncam * 6 + (size_t)l * 3;
      r0 += A[0] * zp[0] + A[1] * zp[1] + A[2] * zp[2];
      r1 += A[3] * zp[0] + A[4] * zp[1] + A[5] * zp[2];
    }
    if (c >= 0) {
      const double* Bm = JB + (size_t)t * 12;
      const double* zc = z + (size_t)c * 6;
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) { s0 += Bm[k] * zc[k]; s1 += Bm[6 + k] * zc[k]; }
      r0 += s0;
      r1 += s1;
    }
    q[(size_t)t * 2] = r0;
    q[(size_t)t * 2 + 1] = r1;
    qq = r0 * r0 + r1 * r1;
  } else if (t < ne + n) {
    const int k = t - ne;
    const double v = sc[SC_SQL] * z[k];
    q[(size_t)ne * 2 + k] = v;
    qq = v * v;
  }
  if (part) {
    const double s = block_sum(qq, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}
// J^T q per camera (workgroup) into w; INIT: p = p - R^-T w, s = p (+ partial of s.s per camera); ITER: s = R^-T
// (-alpha w) (the camera step of an odd iteration)
template <bool INIT>
__global__ void __launch_bounds__(B) k_cgls_cam_jtq(int ncam, int ne, const int* __restrict__ cam_ptr,
                                                    const int* __restrict__ cam_e, const double* __restrict__ JBc,
                                                    const double* __restrict__ q, const double* __restrict__ Rc,
                                                    double* __restrict__ p, double* __restrict__ s,
                                                    double* __restrict__ part, const double* __restrict__ sc) {
  __shared__ double red[4][6];
  if (!INIT && sc[SC_DONE] != 0.0) return;
  const int c = xcd_item(blockIdx.x, ncam);
  double a[6] = {0, 0, 0, 0, 0, 0};
  for (int k = cam_ptr[c] + threadIdx.x; k < cam_ptr[c + 1]; k += B) {
    const double* J = JBc + (size_t)k * 12;
    const double* qe = q + (size_t)cam_e[k] * 2;
    const double q0 = qe[0], q1 = qe[1];
#pragma unroll
    for (int u = 0; u < 6; ++u) a[u] += J[u] * q0 + J[6 + u] * q1;
  }
  wg_sum6(a, red);
  if (threadIdx.x != 0) return;
  const double sl = sc[SC_SQL];
  double w[6];
#pragma unroll
  for (int u = 0; u < 6; ++u) w[u] = a[u] + sl * q[(size_t)ne * 2 + (size_t)c * 6 + u];
  double t[6], ss = 0.0;
  if (INIT) {
    rmul<6, true>(Rc + (size_t)c * 36, w, t);
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const double v = p[(size_t)c * 6 + u] - t[u];
      p[(size_t)c * 6 + u] = v;
      s[(size_t)c * 6 + u] = v;
      ss += v * v;
    }
  } else {
    const double na = -sc[SC_ALPHA];
#pragma unroll
    for (int u = 0; u < 6; ++u) w[u] *= na;
    rmul<6, true>(Rc + (size_t)c * 36, w, t);
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      s[(size_t)c * 6 + u] = t[u];
      ss += t[u] * t[u];
    }
  }
  part[c] = ss;
}
template <bool INIT>
__global__ void __launch_bounds__(B) k_cgls_pt_jtq(int npt, int ncam, int ne, const int* __restrict__ pt_ptr,
                                                   const double* __restrict__ JA, const double* __restrict__ q,
                                                   const double* __restrict__ Rp, double* __restrict__ p,
                                                   double* __restrict__ s, double* __restrict__ part,
                                                   const double* __restrict__ sc) {
  __shared__ double sh[B];
  if (!INIT && sc[SC_DONE] != 0.0) return;
  const int l = blockIdx.x * B + threadIdx.x;
  double ss = 0.0;
  if (l < npt) {
    double w[3] = {0, 0, 0};
    for (int e = pt_ptr[l]; e < pt_ptr[l + 1]; ++e) {
      const double* A = JA + (size_t)e * 6;
      const double q0 = q[(size_t)e * 2], q1 = q[(size_t)e * 2 + 1];
#pragma unroll
      for (int u = 0; u < 3; ++u) w[u] += A[u] * q0 + A[3 + u] * q1;
    }
    const double sl = sc[SC_SQL];
    const size_t o = (size_t)ncam * 6 + (size_t)l * 3;
#pragma unroll
    for (int u = 0; u < 3; ++u) w[u] += sl * q[(size_t)ne * 2 + o + u];
    double t[3];
    if (INIT) {
      rmul<3, true>(Rp + (size_t)l * 9, w, t);
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const double v = p[o + u] - t[u];
        p[o + u] = v;
        s[o + u] = v;
        ss += v * v;
      }
    } else {
      const double na = -sc[SC_ALPHA];
#pragma unroll
      for (int u = 0; u < 3; ++u) w[u] *= na;
      rmul<3, true>(Rp + (size_t)l * 9, w, t);
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        s[o + u] = t[u];
        ss += t[u] * t[u];
      }
    }
  }
  const double v = block_sum(ss, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}
// z = R^-1 p over every block (init)
__global__ void __launch_bounds__(B) k_cgls_rinv_all(int ncam, int npt, const double* __restrict__ Rc,
                                                     const double* __restrict__ Rp, const double* __restrict__ in,
                                                     double* __restrict__ out) {
  const int i = blockIdx.x * B + threadIdx.x;
  if (i < ncam) {
    rmul<6, false>(Rc + (size_t)i * 36, in + (size_t)i * 6, out + (size_t)i * 6);
  } else if (i < ncam + npt) {
    const size_t o = (size_t)ncam * 6 + (size_t)(i - ncam) * 3;
    rmul<3, false>(Rp + (size_t)(i - ncam) * 9, in + o, out + o);
  }
}
__global__ void __launch_bounds__(B) k_cgls_start(const double* __restrict__ part, int np, const double* __restrict__ lam,
                                                  double eta, long long maxit, double* __restrict__ sc) {
  __shared__ double sh[B];
  const double g = sum_parts(part, np, sh);
  if (threadIdx.x == 0) {
    sc[SC_GAMMA] = g;
    sc[SC_THR] = eta * g;  // scaledInitialError (linear_solver_pcg_eigen.h:170)
    sc[SC_DONE] = 0.0;
    sc[SC_ITER] = 0.0;
    sc[SC_MAXIT] = (double)maxit;
    (void)lam;
  }
}

// ---- iteration ----
__global__ void __launch_bounds__(B) k_cgls_alpha(const double* __restrict__ partq, int npq, double* __restrict__ sc) {
  __shared__ double sh[B];
  if (sc[SC_DONE] != 0.0) return;
  const double qq = sum_parts(partq, npq, sh);
  if (threadIdx.x == 0) {
    const double g = sc[SC_GAMMA];
    if (g < sc[SC_THR] || sc[SC_ITER] >= sc[SC_MAXIT]) {
      sc[SC_DONE] = 1.0;
    } else {
      sc[SC_ALPHA] = g / qq;
      sc[SC_ITER] += 1.0;
    }
  }
}
__global__ void __launch_bounds__(B) k_cgls_beta(const double* __restrict__ part, int np, double* __restrict__ sc) {
  __shared__ double sh[B];
  if (sc[SC_DONE] != 0.0) return;
  const double g = sum_parts(part, np, sh);
  if (threadIdx.x == 0) {
    sc[SC_BETA] = g / sc[SC_GAMMA];
    sc[SC_GAMMA] = g;
  }
}
// y += alpha p; p = s + beta p (active block) or beta p (inactive: s = 0); z = R^-1 s on the active block, 0 else
__global__ void __launch_bounds__(B) k_cgls_dir(int ncam, int npt, int cams_active, const double* __restrict__ Rc,
                                                const double* __restrict__ Rp, const double* __restrict__ s,
                                                double* __restrict__ p, double* __restrict__ y, double* __restrict__ z,
                                                const double* __restrict__ sc) {
  if (sc[SC_DONE] != 0.0) return;
  const int i = blockIdx.x * B + threadIdx.x;
  const double al = sc[SC_ALPHA], be = sc[SC_BETA];
  if (i < ncam) {
    const size_t o = (size_t)i * 6;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      y[o + k] += al * p[o + k];
      p[o + k] = cams_active ? s[o + k] + be * p[o + k] : be * p[o + k];
    }
    if (cams_active) rmul<6, false>(Rc + (size_t)i * 36, s + o, z + o);
  } else if (i < ncam + npt) {
    const size_t o = (size_t)ncam * 6 + (size_t)(i - ncam) * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      y[o + k] += al * p[o + k];
      p[o + k] = cams_active ? be * p[o + k] : s[o + k] + be * p[o + k];
    }
    if (!cams_active) rmul<3, false>(Rp + (size_t)(i - ncam) * 9, s + o, z + o);
  }
}
// q = beta q + J_b z_b for the active block b (edge rows, and that block's lambda rows), partials of q.q
__global__ void __launch_bounds__(B) k_cgls_q(int ne, int n, int ncam, int cams_active, const int* __restrict__ e_cam,
                                              const int* __restrict__ e_pt, const double* __restrict__ JA,
                                              const double* __restrict__ JB, const double* __restrict__ z,
                                              double* __restrict__ q, double* __restrict__ part,
                                              const double* __restrict__ sc) {
  __shared__ double sh[B];
  if (sc[SC_DONE] != 0.0) return;
  const int t = blockIdx.x * B + threadIdx.x;
  const double be = sc[SC_BETA];
  double qq = 0.0;
  if (t < ne) {
    double r0 = 0.0, r1 = 0.0;
    if (cams_active) {
      const int c = e_cam[t];
      if (c >= 0) {
        const double* Bm = JB + (size_t)t * 12;
        const double* zc = z + (size_t)c * 6;
#pragma unroll
        for (int k = 0; k < 6; ++k) { r0 += Bm[k] * zc[k]; r1 += Bm[6 + k] * zc[k]; }
      }
    } else {
      const int l = e_pt[t];
      if (l >= 0) {
        const double* A = JA + (size_t)t * 6;
        const double* zp = z + (size_t)ncam * 6 + (size_t)l * 3;
        r0 = A[0] * zp[0] + A[1] * zp[1] + A[2] * zp[2];
        r1 = A[3] * zp[0] + A[4] * zp[1] + A[5] * zp[2];
      }
    }
    const double v0 = be * q[(size_t)t * 2] + r0, v1 = be * q[(size_t)t * 2 + 1] + r1;
    q[(size_t)t * 2] = v0;
    q[(size_t)t * 2 + 1] = v1;
    qq = v0 * v0 + v1 * v1;
  } else if (t < ne + n) {
    const int k = t - ne;
    const bool act = (k < ncam * 6) == (cams_active != 0);
    const double v = be * q[(size_t)ne * 2 + k] + (act ? sc[SC_SQL] * z[k] : 0.0);
    q[(size_t)ne * 2 + k] = v;
    qq = v * v;
  }
  const double v = block_sum(qq, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = v;
}

}  // namespace

DeviceCGLS::~DeviceCGLS() {
  if (chunk_exec) (void)hipGraphExecDestroy(chunk_exec);
}

void DeviceCGLS::setup(int nc, int np_, int ne_, const std::vector<int>& ptp, const std::vector<int>& cp,
                       const std::vector<int>& ce, const std::vector<int>& ec, const std::vector<int>& ep,
                       hipStream_t s) {
  ncam = nc;
  npt = np_;
  ne = ne_;
  n = 6 * ncam + 3 * npt;
  pt_ptr.upload(ptp, s);
  cam_ptr.upload(cp, s);
  cam_e.upload(ce.empty() ? std::vector<int>{0} : ce, s);
  e_cam.upload(ec.empty() ? std::vector<int>{-1} : ec, s);
  e_pt.upload(ep.empty() ? std::vector<int>{-1} : ep, s);
  JA.resize((size_t)std::max(ne, 1) * 6);
  JB.resize((size_t)std::max(ne, 1) * 12);
  JBc.resize((size_t)std::max<size_t>(ce.size(), 1) * 12);
  Gc.resize((size_t)std::max(ncam, 1) * 36);
  Gp.resize((size_t)std::max(npt, 1) * 9);
  Rc.resize((size_t)std::max(ncam, 1) * 36);
  Rp.resize((size_t)std::max(npt, 1) * 9);
  y.resize(std::max(n, 1));
  p.resize(std::max(n, 1));
  sv.resize(std::max(n, 1));
  z.resize(std::max(n, 1));
  q.resize((size_t)2 * ne + n + 1);
  npart = (int)(ncam + grid_for(npt, B) + grid_for((size_t)ne + n, B) + 8);
  part.resize(npart);
  sc.resize(SC_N);
  if (chunk_exec) HIP_CHECK(hipGraphExecDestroy(chunk_exec));
  chunk_exec = nullptr;
}

void DeviceCGLS::build(const EdgeArgs& a, const int* h0, const int* h1, hipStream_t s) {
  if (ne <= 0) return;
  const dev::EdgeData d{a.v0, a.v1, a.meas, a.info, a.params, a.s0, a.s1, a.rk, a.rk_delta, a.ue};
  hipLaunchKernelGGL(k_cgls_jac, grid_for(ne, B), B, 0, s, d, ne, h0, h1, JA.get(), JB.get());
  const int nce = (int)(JBc.size() / 12);
  hipLaunchKernelGGL(k_cgls_gather_cam, grid_for(nce, B), B, 0, s, nce, cam_e.get(), JB.get(), JBc.get());
  if (ncam > 0) hipLaunchKernelGGL(k_cgls_gram_cam, ncam, B, 0, s, ncam, cam_ptr.get(), JBc.get(), Gc.get());
  if (npt > 0) hipLaunchKernelGGL(k_cgls_gram_pt, grid_for(npt, B), B, 0, s, npt, pt_ptr.get(), JA.get(), Gp.get());
  KERNEL_CHECK();
}

void DeviceCGLS::diag_max(double* partial, double* out, hipStream_t s) {
  launch::diag_absmax(Gc.get(), ncam, 6, npt > 0 ? Gp.get() : nullptr, npt, 3, partial, out, s);
}

// CG iterations k0 .. k0+cnt-1 (the active block alternates: even iterations points, odd cameras)
void DeviceCGLS::iterate(int k0, int cnt, hipStream_t s) {
  const int npP = (int)grid_for(npt, B), npq = (int)grid_for((size_t)ne + n, B), PQ = ncam + npP;
  const unsigned gb = grid_for((size_t)ncam + npt, B), gq = grid_for((size_t)ne + n, B);
  for (int k = k0; k < k0 + cnt; ++k) {
    const int cams = k & 1;
    hipLaunchKernelGGL(k_cgls_alpha, 1, B, 0, s, part.get() + PQ, npq, sc.get());
    if (cams) {
      if (ncam > 0)
        hipLaunchKernelGGL(k_cgls_cam_jtq<false>, ncam, B, 0, s, ncam, ne, cam_ptr.get(), cam_e.get(), JBc.get(),
                           q.get(), Rc.get(), p.get(), sv.get(), part.get(), sc.get());
      hipLaunchKernelGGL(k_cgls_beta, 1, B, 0, s, part.get(), ncam, sc.get());
    } else {
      if (npt > 0)
        hipLaunchKernelGGL(k_cgls_pt_jtq<false>, npP, B, 0, s, npt, ncam, ne, pt_ptr.get(), JA.get(), q.get(),
                           Rp.get(), p.get(), sv.get(), part.get(), sc.get());
      hipLaunchKernelGGL(k_cgls_beta, 1, B, 0, s, part.get(), npP, sc.get());
    }
    hipLaunchKernelGGL(k_cgls_dir, gb, B, 0, s, ncam, npt, cams, Rc.get(), Rp.get(), sv.get(), p.get(), y.get(), z.get(),
                       sc.get());
    hipLaunchKernelGGL(k_cgls_q, gq, B, 0, s, ne, n, ncam, cams, e_cam.get(), e_pt.get(), JA.get(), JB.get(), z.get(),
                       q.get(), part.get() + PQ, sc.get());
  }
  KERNEL_CHECK();
}

namespace {
// stream capture that always ends (and frees its graph), even when a capture call throws
struct Capture {
  hipStream_t st;
  hipGraph_t g = nullptr;
  bool open = true;
  explicit Capture(hipStream_t s) : st(s) { HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal)); }
  hipGraph_t end() {
    open = false;
    HIP_CHECK(hipStreamEndCapture(st, &g));
    return g;
  }
  ~Capture() {
    if (open) (void)hipStreamEndCapture(st, &g);
    if (g) (void)hipGraphDestroy(g);
  }
};
}  // namespace

void DeviceCGLS::solve(const double* lam, const double* b, double* x, hipStream_t s) {
  if (n <= 0) return;
  const int npP = (int)grid_for(npt, B), PQ = ncam + npP;
  const unsigned gb = grid_for((size_t)ncam + npt, B), gq = grid_for((size_t)ne + n, B);
  // preconditioner (computeRc_inverse / computeRp_inverse)
  hipLaunchKernelGGL(k_cgls_prec<6>, grid_for(std::max(ncam, 1), B), B, 0, s, ncam, Gc.get(), lam, Rc.get(), sc.get());
  hipLaunchKernelGGL(k_cgls_prec<3>, grid_for(std::max(npt, 1), B), B, 0, s, npt, Gp.get(), lam, Rp.get(), sc.get());
  // y0 = (0, R_p^-T b_p), p = R^-T (b - J^T J R^-1 y0), s = p, q = J R^-1 p (linear_solver_pcg_eigen.h:100-160)
  hipLaunchKernelGGL(k_cgls_init_a, gb, B, 0, s, ncam, npt, Rc.get(), Rp.get(), b, p.get(), y.get(), z.get());
  hipLaunchKernelGGL(k_cgls_jz, gq, B, 0, s, ne, n, ncam, e_cam.get(), e_pt.get(), JA.get(), JB.get(), z.get(), q.get(),
                     sc.get(), nullptr);
  if (ncam > 0)
    hipLaunchKernelGGL(k_cgls_cam_jtq<true>, ncam, B, 0, s, ncam, ne, cam_ptr.get(), cam_e.get(), JBc.get(), q.get(),
                       Rc.get(), p.get(), sv.get(), part.get(), sc.get());
  if (npt > 0)
    hipLaunchKernelGGL(k_cgls_pt_jtq<true>, npP, B, 0, s, npt, ncam, ne, pt_ptr.get(), JA.get(), q.get(), Rp.get(),
                       p.get(), sv.get(), part.get() + ncam, sc.get());
  hipLaunchKernelGGL(k_cgls_rinv_all, gb, B, 0, s, ncam, npt, Rc.get(), Rp.get(), p.get(), z.get());
  hipLaunchKernelGGL(k_cgls_jz, gq, B, 0, s, ne, n, ncam, e_cam.get(), e_pt.get(), JA.get(), JB.get(), z.get(), q.get(),
                     sc.get(), part.get() + PQ);
  const long long rows = 2LL * ne + n, maxit = rows + rows % 2;  // maxIter = J.rows(), rounded up to even
  hipLaunchKernelGGL(k_cgls_start, 1, B, 0, s, part.get(), PQ, lam, eta, maxit, sc.get());
  KERNEL_CHECK();
  double h[SC_N];
  for (long long k = 0; k < maxit;) {
    const int cnt = (int)std::min<long long>(CHUNK, maxit - k);
    if (cnt == CHUNK) {
      if (!chunk_exec) {
        Capture cap(s);
        iterate(0, CHUNK, s);
        hipGraph_t g = cap.end();
        hipGraphExec_t ex = nullptr;
        HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
        chunk_exec = ex;
      }
      HIP_CHECK(hipGraphLaunch(chunk_exec, s));
    } else {
      iterate((int)(k & 1), cnt, s);
    }
    k += cnt;
    HIP_CHECK(hipMemcpyAsync(h, sc.get(), sizeof h, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (h[SC_DONE] != 0.0) break;
  }
  last_iterations = (int)h[SC_ITER];
  hipLaunchKernelGGL(k_cgls_rinv_all, gb, B, 0, s, ncam, npt, Rc.get(), Rp.get(), y.get(), x);  // x = R^-1 y
  KERNEL_CHECK();
}

}  // namespace g2ohip
