// Dev micro-benchmark: the production chol32 column machinery at NB = 16 (one 16 x 16 block per wave; lanes 16..31 build the inverse) — what a blocked 16 + 16 chol32 would pay per half.
// column loop (y from the explicit inverse afterwards), F&2 division-form pivot chain d' = a - b^2/d.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int NB = 16;
#define SB() __builtin_amdgcn_sched_barrier(0)
__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
struct C4State {
  double dn, a1, b1, c2, lp, dinv, bb;
  double2 cc[NB / 2];
  bool ok;
};
template <int F, int NCH, int J, int K>
__device__ __forceinline__ void c4_fill(double (&row)[NB], const C4State& st) {
  constexpr int c0 = (J + 2) & ~1;
  constexpr int nf = J >= 1 ? (NB - c0) / 2 : 0;
  constexpr int qa = nf * K / NCH, qb = nf * (K + 1) / NCH;
#pragma unroll
  for (int q = qa; q < qb; ++q) {
    const int c = c0 + 2 * q;
    if (c > J + 1) row[c] -= st.lp * st.cc[c >> 1].x;
    row[c + 1] -= st.lp * st.cc[c >> 1].y;
  }
}
template <int F, int NCH, int J>
__device__ __forceinline__ void c4_step(double (&row)[NB], double& y, int lane, double* col, C4State& st) {
  if constexpr (J < NB) {
    const double d = st.dn;
    st.ok &= d > 0.0;
    const double r0 = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    if constexpr (F & 2) {  // 1/d: rcp + one Newton step, beside the rsq
      const double q0 = __builtin_amdgcn_rcp(d);
      st.dinv = __builtin_fma(q0, __builtin_fma(-d, q0, 1.0), q0);
      st.bb = st.b1 * st.b1;
    }
    SB();
    c4_fill<F, NCH, J, 0>(row, st);
    SB();
    const double t1 = hd * r0;
    SB();
    if constexpr (NCH > 1) c4_fill<F, NCH, J, 1>(row, st);
    SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5);
    SB();
    if constexpr (NCH > 2) c4_fill<F, NCH, J, 2>(row, st);
    SB();
    const double r = r0 * t2;
    const double l1 = st.b1 * r, l2 = st.c2 * r;  // l_{j+1,j}, l_{j+2,j}
    if constexpr (J + 1 < NB) {
      if constexpr (F & 2) st.dn = __builtin_fma(-st.bb, st.dinv, st.a1);
      else st.dn = __builtin_fma(-l1, l1, st.a1);
    }
    SB();
    if constexpr (NCH > 3) c4_fill<F, NCH, J, 3>(row, st);
    SB();
    const double lj = row[J] * r;
    row[J] = lj;
    if constexpr (J + 1 < NB) {
      row[J + 1] -= lj * l1;
      col[(J & 1) * 2 * NB + lane] = lj;
    }
    if constexpr (J + 2 < NB) row[J + 2] -= lj * l2;
    if constexpr (!(F & 1)) {
      const double yj = rlane(y, J) * r;
      y = lane == J ? yj : (lane > J ? y - lj * yj : y);
    }
    SB();
    if constexpr (NCH > 4) c4_fill<F, NCH, J, 4>(row, st);
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
    c4_step<F, NCH, J + 1>(row, y, lane, col, st);
  }
}
template <int F, int NCH>
__device__ __forceinline__ bool chol32_v4(double (&row)[NB], double& y, int lane, double* col) {
  C4State st;
  st.ok = true;
  st.lp = 0.0;
  st.dn = rlane(row[0], 0);
  st.a1 = rlane(row[1], 1);
  st.b1 = rlane(row[0], 1);
  st.c2 = rlane(row[0], 2);
  c4_step<F, NCH, 0>(row, y, lane, col, st);
  return st.ok;
}
template <int F, int NCH>
__global__ void __launch_bounds__(64) k_bench_v4(const double* A, double* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  const int lane = threadIdx.x;
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? A[lane * NB + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
  double y = lane < NB ? 1.0 : 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok = chol32_v4<F, NCH>(row, y, lane, col);
  asm volatile("" : "+v"(row[NB - 1]), "+v"(y));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = y + (ok ? 0.0 : 1.0);
#pragma unroll
  for (int c = 0; c < NB; ++c) s += row[c];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int F, int NCH>
int run_v4(const double* A, double* out, unsigned long long* cyc, const char* name, const double* ref) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL((k_bench_v4<F, NCH>), 1, 64, 0, 0, A, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    if (c < best) best = c;
  }
  double h[64];
  CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  double md = 0;
  for (int i = 0; i < 64; ++i) md = fmax(md, fabs(h[i] - ref[i]) / fmax(1.0, fabs(ref[i])));
  printf("%-28s %7llu cycles  (%5.1f per column)  max rel diff vs full %.2e\n", name, best, best / (double)NB, md);
  return 0;
}

int main() {
  double h[NB * NB];
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) h[i * NB + j] = (i == j ? NB + 1.0 : 0.0) + 1.0 / (1 + i + j);
  double *A, *out; unsigned long long* cyc;
  CK(hipMalloc(&A, sizeof h)); CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&cyc, 8));
  CK(hipMemcpy(A, h, sizeof h, hipMemcpyHostToDevice));
  double ref[64] = {0};
  run_v4<0, 3>(A, out, cyc, "v3 (production form)", ref);
  CK(hipMemcpy(ref, out, sizeof ref, hipMemcpyDeviceToHost));
  run_v4<0, 3>(A, out, cyc, "v3 again", ref);
  run_v4<1, 3>(A, out, cyc, "no forward solve", ref);
  run_v4<2, 3>(A, out, cyc, "division-form chain", ref);
  run_v4<3, 3>(A, out, cyc, "both", ref);
  run_v4<1, 1>(A, out, cyc, "no fwd, 1 chunk", ref);
  run_v4<1, 5>(A, out, cyc, "no fwd, 5 chunks", ref);
  return 0;
}
