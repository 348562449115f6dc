// Small device helpers shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>

namespace g2ohip {

// Load that never branches: the address is selected and the value masked. A guarded load
// (`ok ? p[i] : 0`) compiles to a branch with its own s_waitcnt, which serialises every load of an
// unrolled batch; this form keeps the whole batch in flight. p[0] must be a valid address.
template <class T>
__device__ __forceinline__ T ld0(const T* p, int idx, bool ok) {
  const T v = p[ok ? idx : 0];
  return ok ? v : T(0);
}

// XCD-aware workgroup order: the dispatcher deals workgroups to the 8 XCDs round-robin; this
// bijection gives XCD x a contiguous range of work items [x*n/8, (x+1)*n/8), so neighbouring items
// (camera rows that share landmarks) run side by side behind the same L2.
__device__ __forceinline__ int xcd_item(int bid, int n) {
  const int xcd = bid & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Landmark block of the Schur complement (block_solver.hpp:341-360), split symmetrically:
//   Hll + lambda I = U U^T,  c = U^-1 b_l,  G_a = Hpl_a U^-T   =>   Hpl Dinv Hpl^T = G G^T,  Hpl Dinv b_l = G c_l.
// a: the LD x LD block, column-major, lambda already on its diagonal. U record (UF doubles, r = reciprocal pivots):
// LD = 3: r0 r1 r2 u10 u20 u21, LD = 2: r0 r1 u10 0. Returns false when a pivot is not positive.
template <int LD>
__device__ __forceinline__ bool lm_ufac(const double* a, const double* bl, double* U, double* c) {
  auto m = [&](int r, int cc) { return a[cc * LD + r]; };
  if constexpr (LD == 3) {
    const double d0 = m(0, 0);
    const double r0 = 1.0 / sqrt(d0);
    const double u10 = m(1, 0) * r0, u20 = m(2, 0) * r0;
    const double d1 = m(1, 1) - u10 * u10;
    const double r1 = 1.0 / sqrt(d1);
    const double u21 = (m(2, 1) - u20 * u10) * r1;
    const double d2 = m(2, 2) - u20 * u20 - u21 * u21;
    const double r2 = 1.0 / sqrt(d2);
    U[0] = r0; U[1] = r1; U[2] = r2; U[3] = u10; U[4] = u20; U[5] = u21;
    const double g0 = bl[0] * r0;
    const double g1 = (bl[1] - u10 * g0) * r1;
    const double g2 = (bl[2] - u20 * g0 - u21 * g1) * r2;
    c[0] = g0; c[1] = g1; c[2] = g2;
    return d0 > 0.0 && d1 > 0.0 && d2 > 0.0;
  } else {
    const double d0 = m(0, 0);
    const double r0 = 1.0 / sqrt(d0);
    const double u10 = m(1, 0) * r0;
    const double d1 = m(1, 1) - u10 * u10;
    const double r1 = 1.0 / sqrt(d1);
    U[0] = r0; U[1] = r1; U[2] = u10; U[3] = 0.0;
    const double g0 = bl[0] * r0;
    c[0] = g0;
    c[1] = (bl[1] - u10 * g0) * r1;
    return d0 > 0.0 && d1 > 0.0;
  }
}

// G = Hpl U^-T in place: g (PD x LD col-major) holds Hpl on entry, G on exit; row r solves U g_r = h_r
template <int PD, int LD>
__device__ __forceinline__ void form_G(double* g, const double* U) {
#pragma unroll
  for (int r = 0; r < PD; ++r) {
    if constexpr (LD == 3) {
      const double g0 = g[r] * U[0];
      const double g1 = (g[PD + r] - U[3] * g0) * U[1];
      g[2 * PD + r] = (g[2 * PD + r] - U[4] * g0 - U[5] * g1) * U[2];
      g[r] = g0;
      g[PD + r] = g1;
    } else {
      const double g0 = g[r] * U[0];
      g[PD + r] = (g[PD + r] - U[2] * g0) * U[1];
      g[r] = g0;
    }
  }
}

}  // namespace g2ohip
