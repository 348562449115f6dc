// Dev micro-benchmark: the production 32x32 diagonal factor (cholesky.hip chol32: one column per pivot step) against a
// two-column variant (chol32p: 2 x 2 pivot blocks whose two reciprocal square roots are issued together), one wave,
// s_memtime cycles per call; both checked against a host Cholesky of the same SPD matrix (L in lanes 0..31, L^-1 in
// lanes 32..63).
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 tools/ubench_chol32p.hip -o tools/ubench_chol32p
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int NB = 32;
__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
#define SB() __builtin_amdgcn_sched_barrier(0)

// ---- production (cholesky.hip) -----------------------------------------------------------------------------------
constexpr int C32_NCH = 3;
struct C32State {
  double dn, a1, b1, c2, lp;
  double2 cc[NB / 2];
  bool ok;
};
template <int J, int K>
__device__ __forceinline__ void c32_fill(double (&row)[NB], const C32State& st) {
  constexpr int c0 = (J + 2) & ~1;
  constexpr int nf = J >= 1 ? (NB - c0) / 2 : 0;
  constexpr int qa = nf * K / C32_NCH, qb = nf * (K + 1) / C32_NCH;
#pragma unroll
  for (int q = qa; q < qb; ++q) {
    const int c = c0 + 2 * q;
    if (c > J + 1) row[c] -= st.lp * st.cc[c >> 1].x;
    row[c + 1] -= st.lp * st.cc[c >> 1].y;
  }
}
template <int J>
__device__ __forceinline__ void c32_step(double (&row)[NB], int lane, double* col, C32State& st) {
  if constexpr (J < NB) {
    const double d = st.dn;
    st.ok &= d > 0.0;
    const double r0 = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    SB(); c32_fill<J, 0>(row, st); SB();
    const double t1 = hd * r0;
    SB(); c32_fill<J, 1>(row, st); SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5);
    SB(); c32_fill<J, 2>(row, st); SB();
    const double r = r0 * t2;
    const double l1 = st.b1 * r, l2 = st.c2 * r;
    if constexpr (J + 1 < NB) st.dn = __builtin_fma(-l1, l1, st.a1);
    SB();
    const double lj = row[J] * r;
    row[J] = lj;
    if constexpr (J + 1 < NB) {
      row[J + 1] -= lj * l1;
      col[(J & 1) * 2 * NB + lane] = lj;
    }
    if constexpr (J + 2 < NB) row[J + 2] -= lj * l2;
    SB();
    if constexpr (J + 1 < NB) {
      constexpr int n0 = (J + 3) & ~1;
      const double* cb = col + (J & 1) * 2 * NB;
#pragma unroll
      for (int c = n0; c < NB; c += 2) st.cc[c >> 1] = *reinterpret_cast<const double2*>(cb + c);
      st.lp = lj;
    }
    if constexpr (J + 2 < NB) { st.a1 = rlane(row[J + 2], J + 2); st.b1 = rlane(row[J + 1], J + 2); }
    if constexpr (J + 3 < NB) st.c2 = rlane(row[J + 1], J + 3);
    SB();
    c32_step<J + 1>(row, lane, col, st);
  }
}
__device__ __forceinline__ bool chol32(double (&row)[NB], int lane, double* col) {
  C32State st;
  st.ok = true;
  st.lp = 0.0;
  st.dn = rlane(row[0], 0);
  st.a1 = rlane(row[1], 1);
  st.b1 = rlane(row[0], 1);
  st.c2 = rlane(row[0], 2);
  c32_step<0>(row, lane, col, st);
  return st.ok;
}

// ---- two-column pivot steps ------------------------------------------------------------------------------------
// Pair J factors columns J, J+1 from the uniform 2 x 2 block (a b; b c) of A' (every update of the pairs before J
// applied): r1 = 1/sqrt(a), and with D = a c - b^2 the second pivot's reciprocal 1/sqrt(c - b^2/a) = (a r1)/sqrt(D), so
// the two reciprocal square roots (and their Newton steps) run side by side. Per lane l0 = A(i,J) r1, l1 = (A(i,J+1)
// - l0 L(J+1,J)) r2 (lanes 32..63 hold identity rows: the same forward substitution builds L^-1).
// Invariant at the top of pair J: columns J..J+3 hold every update of the pairs before J, columns >= J+4 lack pair
// J-2's rank-2 update (its deferred part, applied here in NCH chunks pinned between this pair's dependent chain steps).
// The next pair's block comes from uniform values: rows J+2, J+3 at columns J..J+3 (v_readlane at the top of this
// pair) minus this pair's terms. The pair's own rank-2 update reaches columns J+2..J+5 at once (eager), the rest waits
// for the next pair. The pair's columns are broadcast through LDS as one 16-byte (L(c,J), L(c,J+1)) entry per row.
template <int NCH>
struct P2 {
  struct St {
    double a, b, c;   // this pair's 2 x 2 block
    double l0p, l1p;  // this lane's entries of the previous pair
    bool ok;
  };
  template <int J, int K>
  __device__ __forceinline__ static void fill(double (&row)[NB], const St& st, const double2* cbp) {
    constexpr int c0 = J + 4;  // deferred columns of the previous pair
    constexpr int nf = J >= 2 && c0 < NB ? NB - c0 : 0;
    constexpr int qa = nf * K / NCH, qb = nf * (K + 1) / NCH;
#pragma unroll
    for (int q = qa; q < qb; ++q) {
      const double2 x = cbp[c0 + q];
      row[c0 + q] -= st.l0p * x.x + st.l1p * x.y;
    }
  }
  template <int J>
  __device__ __forceinline__ static void step(double (&row)[NB], int lane, double2* col, St& st) {
    if constexpr (J < NB) {
      const double2* cbp = col + ((J / 2 + 1) & 1) * 64;  // previous pair's columns
      double2* cbo = col + ((J / 2) & 1) * 64;             // this pair's
      // rows J+2, J+3 at columns J..J+3 (complete for every pair before J)
      double A20 = 0, A21 = 0, A22 = 0, A30 = 0, A31 = 0, A32 = 0, A33 = 0;
      if constexpr (J + 2 < NB) {
        A20 = rlane(row[J], J + 2); A21 = rlane(row[J + 1], J + 2); A22 = rlane(row[J + 2], J + 2);
        A30 = rlane(row[J], J + 3); A31 = rlane(row[J + 1], J + 3); A32 = rlane(row[J + 2], J + 3);
        A33 = rlane(row[J + 3], J + 3);
      }
      const double a = st.a, b = st.b, c = st.c;
      const double D = __builtin_fma(a, c, -(b * b));
      st.ok &= a > 0.0 && D > 0.0;
      const double ra0 = __builtin_amdgcn_rsq(a), rd0 = __builtin_amdgcn_rsq(D);
      const double ha = 0.5 * a, hD = 0.5 * D;
      SB(); fill<J, 0>(row, st, cbp); SB();
      const double ta = ha * ra0, td = hD * rd0;
      SB(); if constexpr (NCH > 1) fill<J, 1>(row, st, cbp); SB();
      const double sa = __builtin_fma(-ra0, ta, 1.5), sd = __builtin_fma(-rd0, td, 1.5);
      SB(); if constexpr (NCH > 2) fill<J, 2>(row, st, cbp); SB();
      const double r1 = ra0 * sa, rd = rd0 * sd;
      const double Lb = b * r1, ar = a * r1;
      const double r2 = ar * rd;
      SB(); if constexpr (NCH > 3) fill<J, 3>(row, st, cbp); SB();
      // the next pair's block (uniform)
      const double L20 = A20 * r1, L30 = A30 * r1;
      const double L21 = (A21 - L20 * Lb) * r2, L31 = (A31 - L30 * Lb) * r2;
      const double na = A22 - L20 * L20 - L21 * L21;
      const double nb = A32 - L30 * L20 - L31 * L21;
      const double nc = A33 - L30 * L30 - L31 * L31;
      // this lane's entries of the pair's columns
      const double l0 = row[J] * r1;
      const double l1 = (row[J + 1] - l0 * Lb) * r2;
      row[J] = l0;
      row[J + 1] = l1;
      if constexpr (J + 2 < NB) cbo[lane] = double2{l0, l1};
      SB();
      if constexpr (J + 2 < NB) {  // eager part: the next two pairs' columns
#pragma unroll
        for (int cc = J + 2; cc < J + 6 && cc < NB; ++cc) {
          const double2 x = cbo[cc];
          row[cc] -= l0 * x.x + l1 * x.y;
        }
        st.l0p = l0;
        st.l1p = l1;
        st.a = na; st.b = nb; st.c = nc;
      }
      SB();
      step<J + 2>(row, lane, col, st);
    }
  }
  __device__ __forceinline__ static bool run(double (&row)[NB], int lane, double2* col) {
    St st;
    st.ok = true;
    st.l0p = st.l1p = 0.0;
    st.a = rlane(row[0], 0);
    st.b = rlane(row[0], 1);
    st.c = rlane(row[1], 1);
    step<0>(row, lane, col, st);
    return st.ok;
  }
};

template <int V>
__global__ void __launch_bounds__(64) k_bench(const double* A, double* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[4 * NB * 2];
  const int lane = threadIdx.x;
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? A[lane * NB + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok;
  if constexpr (V == 0) ok = chol32(row, lane, col);
  else ok = P2<V>::run(row, lane, reinterpret_cast<double2*>(col));
  asm volatile("" : "+v"(row[NB - 1]));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int c = 0; c < NB; ++c) out[lane * NB + c] = row[c];
  if (lane == 0) { cyc[0] = t1 - t0; cyc[1] = ok; }
}

template <int V>
int run(const double* A, double* out, unsigned long long* cyc, const char* name, const double* L, const double* Li) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 50; ++r) {
    hipLaunchKernelGGL(k_bench<V>, 1, 64, 0, 0, A, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c[2];
    CK(hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost));
    if (c[0] < best) best = c[0];
  }
  static double h[64 * NB];
  unsigned long long okf[2];
  CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  CK(hipMemcpy(okf, cyc, 16, hipMemcpyDeviceToHost));
  double el = 0, ei = 0;
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j <= i; ++j) el = fmax(el, fabs(h[i * NB + j] - L[i * NB + j]) / fmax(1.0, fabs(L[i * NB + j])));
  for (int c = 0; c < NB; ++c)  // lane 32 + c: column c of L^-1 (row[i] = L^-1(i, c))
    for (int i = c; i < NB; ++i) ei = fmax(ei, fabs(h[(NB + c) * NB + i] - Li[i * NB + c]) / fmax(1.0, fabs(Li[i * NB + c])));
  printf("%-34s %7llu cycles (%5.1f per column)  ok %llu  max rel err L %.2e  L^-1 %.2e\n", name, best, best / 32.0,
         okf[1], el, ei);
  return 0;
}

int main() {
  double h[NB * NB], L[NB * NB] = {0}, Li[NB * NB] = {0};
  srand(7);
  double B[NB * NB];
  for (int i = 0; i < NB * NB; ++i) B[i] = (rand() / (double)RAND_MAX) - 0.5;
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      double s = (i == j) ? 4.0 : 0.0;
      for (int k = 0; k < NB; ++k) s += B[i * NB + k] * B[j * NB + k];
      h[i * NB + j] = s;
    }
  for (int j = 0; j < NB; ++j) {  // host Cholesky (long double accumulation)
    long double d = h[j * NB + j];
    for (int k = 0; k < j; ++k) d -= (long double)L[j * NB + k] * L[j * NB + k];
    L[j * NB + j] = sqrtl(d);
    for (int i = j + 1; i < NB; ++i) {
      long double s = h[i * NB + j];
      for (int k = 0; k < j; ++k) s -= (long double)L[i * NB + k] * L[j * NB + k];
      L[i * NB + j] = s / L[j * NB + j];
    }
  }
  for (int c = 0; c < NB; ++c)  // L^-1 column c by forward substitution
    for (int i = c; i < NB; ++i) {
      long double s = i == c ? 1.0 : 0.0;
      for (int k = c; k < i; ++k) s -= (long double)L[i * NB + k] * Li[k * NB + c];
      Li[i * NB + c] = s / L[i * NB + i];
    }
  double *A, *out;
  unsigned long long* cyc;
  CK(hipMalloc(&A, sizeof h)); CK(hipMalloc(&out, 64 * NB * 8)); CK(hipMalloc(&cyc, 16));
  CK(hipMemcpy(A, h, sizeof h, hipMemcpyHostToDevice));
  run<0>(A, out, cyc, "chol32 (production)", L, Li);
  run<1>(A, out, cyc, "chol32p, deferred in 1 chunk", L, Li);
  run<2>(A, out, cyc, "chol32p, deferred in 2 chunks", L, Li);
  run<3>(A, out, cyc, "chol32p, deferred in 3 chunks", L, Li);
  run<4>(A, out, cyc, "chol32p, deferred in 4 chunks", L, Li);
  run<0>(A, out, cyc, "chol32 (production, again)", L, Li);
  return 0;
}
