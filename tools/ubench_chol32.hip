// Dev micro-benchmark: the 32x32 diagonal factor (cholesky.hip chol32) in isolation, one wave,
// s_memtime cycles per call, with variants switched off to see what the time is made of.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int NB = 32;
__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// V bits: 1 no deferred update, 2 no look-ahead, 4 no forward solve, 8 no Newton
template <int V>
__device__ __forceinline__ bool chol32(double (&row)[NB], double& y, int lane, double* col, double* dinv) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double2 cc[NB / 2];
    const int c0 = (j + 2) & ~1;
    if (j >= 1 && !(V & 1)) {
      const double* cb = col + ((j - 1) & 1) * 2 * NB;
#pragma unroll
      for (int c = c0; c < NB; c += 2) cc[c >> 1] = *reinterpret_cast<const double2*>(cb + c);
    }
    const double djj = rlane(row[j], j);
    ok &= djj > 0.0;
    const double d = djj > 0.0 ? djj : 1.0;
    double r = __builtin_amdgcn_rsq(d);
    if (!(V & 8)) r = r * (1.5 - 0.5 * d * r * r);
    const double lj = row[j] * r;
    row[j] = lj;
    if (j + 1 < NB) {
      if (!(V & 2)) {
        row[j + 1] -= lj * rlane(lj, j + 1);
        if (j + 2 < NB) row[j + 2] -= lj * rlane(lj, j + 2);
      }
      col[(j & 1) * 2 * NB + lane] = lj;
    }
    if (!(V & 4)) {
      const double yj = rlane(y, j) * r;
      y = lane == j ? yj : (lane > j ? y - lj * yj : y);
    }
    if (j >= 1 && !(V & 1)) {
      const double lp = row[j - 1];
#pragma unroll
      for (int c = c0; c < NB; c += 2) {
        if (c > j + 1) row[c] -= lp * cc[c >> 1].x;
        row[c + 1] -= lp * cc[c >> 1].y;
      }
    }
#pragma unroll
    for (int c = j + 1; c < NB; ++c) asm volatile("" : "+v"(row[c]));
  }
  return ok;
}

// Interleaved variant: the pivot chain of column j is pinned in program order (sched_barrier) with
// the deferred update of column j-1 cut into chunks between its dependent steps, and column j's
// LDS reads for the next iteration issued right after its write.
#define SB() __builtin_amdgcn_sched_barrier(0)
template <int NCH>
__device__ __forceinline__ bool chol32_il(double (&row)[NB], double& y, int lane, double* col) {
  bool ok = true;
  double2 cc[NB / 2];
  double lp = 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int c0 = (j + 2) & ~1;
    const int nf = j >= 1 ? (NB - c0) / 2 : 0;  // column pairs of the deferred update
    // P0: pivot of column j
    const double djj = rlane(row[j], j);
    ok &= djj > 0.0;
    const double d = djj > 0.0 ? djj : 1.0;
    const double r0 = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    SB();
    auto fill = [&](int k) {  // chunk k of NCH of the deferred update of column j-1
      const int a = nf * k / NCH, b = nf * (k + 1) / NCH;
#pragma unroll
      for (int q = a; q < b; ++q) {
        const int c = c0 + 2 * q;
        if (c > j + 1) row[c] -= lp * cc[c >> 1].x;
        row[c + 1] -= lp * cc[c >> 1].y;
      }
    };
    fill(0); SB();
    const double t1 = hd * r0; SB();
    fill(1); SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5); SB();
    fill(2); SB();
    const double r = r0 * t2; SB();
    fill(3); SB();
    const double lj = row[j] * r;
    row[j] = lj;
    double b1 = 0.0, b2 = 0.0;
    if (j + 1 < NB) b1 = rlane(lj, j + 1);
    if (j + 2 < NB) b2 = rlane(lj, j + 2);
    if (j + 1 < NB) col[(j & 1) * 2 * NB + lane] = lj;
    SB();
    fill(4); SB();
    if (j + 1 < NB) row[j + 1] -= lj * b1;
    if (j + 2 < NB) row[j + 2] -= lj * b2;
    const double yj = rlane(y, j) * r;
    y = lane == j ? yj : (lane > j ? y - lj * yj : y);
    SB();
    // column j for the next iteration's deferred update (columns >= j+3)
    if (j + 1 < NB) {
      const int n0 = (j + 3) & ~1;
      const double* cb = col + (j & 1) * 2 * NB;
#pragma unroll
      for (int c = n0; c < NB; c += 2) cc[c >> 1] = *reinterpret_cast<const double2*>(cb + c);
      lp = lj;
    }
    SB();
  }
  return ok;
}
template <int NCH>
__global__ void __launch_bounds__(64) k_bench_il(const double* A, double* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  const int lane = threadIdx.x;
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? A[lane * NB + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
  double y = lane < NB ? 1.0 : 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok = chol32_il<NCH>(row, y, lane, col);
  asm volatile("" : "+v"(row[NB - 1]), "+v"(y));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = y + (ok ? 0.0 : 1.0);
#pragma unroll
  for (int c = 0; c < NB; ++c) s += row[c];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int NCH>
int run_il(const double* A, double* out, unsigned long long* cyc, const char* name, const double* ref) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL(k_bench_il<NCH>, 1, 64, 0, 0, A, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    if (c < best) best = c;
  }
  double h[64];
  CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  double md = 0;
  for (int i = 0; i < 64; ++i) md = fmax(md, fabs(h[i] - ref[i]) / fmax(1.0, fabs(ref[i])));
  printf("%-28s %7llu cycles  (%5.1f per column)  max rel diff vs full %.2e\n", name, best, best / 32.0, md);
  return 0;
}

// v3: the pivot chain runs on wave-uniform values only. d_{j+1} = A(j+1,j+1) - (A(j+1,j) r_j)^2 with
// both entries read (v_readlane) one iteration early, so the chain per column is
// rsq -> 3 Newton/scale ops -> l_{j+1,j} -> d_{j+1}; the look-ahead, deferred update, column
// write and forward solve are off it. NCH chunks of the deferred update are pinned between the
// chain's dependent steps (sched_barrier). One template instance per column: every index is a
// compile-time constant.
struct C32State {
  double dn, a1, b1, c2, lp;
  double2 cc[NB / 2];
  bool ok;
};
template <int NCH, int J, int K>
__device__ __forceinline__ void c32_fill(double (&row)[NB], const C32State& st) {
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
template <int NCH, int J>
__device__ __forceinline__ void c32_step(double (&row)[NB], double& y, int lane, double* col, C32State& st) {
  if constexpr (J < NB) {
    const double d = st.dn;
    st.ok &= d > 0.0;
    const double r0 = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    SB();
    c32_fill<NCH, J, 0>(row, st);
    SB();
    const double t1 = hd * r0;
    SB();
    if constexpr (NCH > 1) c32_fill<NCH, J, 1>(row, st);
    SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5);
    SB();
    if constexpr (NCH > 2) c32_fill<NCH, J, 2>(row, st);
    SB();
    const double r = r0 * t2;
    const double l1 = st.b1 * r, l2 = st.c2 * r;  // l_{j+1,j}, l_{j+2,j}
    if constexpr (J + 1 < NB) st.dn = __builtin_fma(-l1, l1, st.a1);
    SB();
    if constexpr (NCH > 3) c32_fill<NCH, J, 3>(row, st);
    SB();
    const double lj = row[J] * r;
    row[J] = lj;
    if constexpr (J + 1 < NB) {
      row[J + 1] -= lj * l1;
      col[(J & 1) * 2 * NB + lane] = lj;
    }
    if constexpr (J + 2 < NB) row[J + 2] -= lj * l2;
    const double yj = rlane(y, J) * r;
    y = lane == J ? yj : (lane > J ? y - lj * yj : y);
    SB();
    if constexpr (NCH > 4) c32_fill<NCH, J, 4>(row, st);
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
    c32_step<NCH, J + 1>(row, y, lane, col, st);
  }
}
template <int NCH>
__device__ __forceinline__ bool chol32_v3(double (&row)[NB], double& y, int lane, double* col) {
  C32State st;
  st.ok = true;
  st.lp = 0.0;
  st.dn = rlane(row[0], 0);
  st.a1 = rlane(row[1], 1);
  st.b1 = rlane(row[0], 1);
  st.c2 = rlane(row[0], 2);
  c32_step<NCH, 0>(row, y, lane, col, st);
  return st.ok;
}
template <int NCH>
__global__ void __launch_bounds__(64) k_bench_v3(const double* A, double* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  const int lane = threadIdx.x;
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? A[lane * NB + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
  double y = lane < NB ? 1.0 : 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok = chol32_v3<NCH>(row, y, lane, col);
  asm volatile("" : "+v"(row[NB - 1]), "+v"(y));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = y + (ok ? 0.0 : 1.0);
#pragma unroll
  for (int c = 0; c < NB; ++c) s += row[c];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int NCH>
int run_v3(const double* A, double* out, unsigned long long* cyc, const char* name, const double* ref) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL(k_bench_v3<NCH>, 1, 64, 0, 0, A, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    if (c < best) best = c;
  }
  double h[64];
  CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  double md = 0;
  for (int i = 0; i < 64; ++i) md = fmax(md, fabs(h[i] - ref[i]) / fmax(1.0, fabs(ref[i])));
  printf("%-28s %7llu cycles  (%5.1f per column)  max rel diff vs full %.2e\n", name, best, best / 32.0, md);
  return 0;
}
template <int V>
__global__ void __launch_bounds__(64) k_bench(const double* A, double* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  __shared__ double dinv[NB];
  const int lane = threadIdx.x;
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? A[lane * NB + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
  double y = lane < NB ? 1.0 : 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  bool ok = chol32<V>(row, y, lane, col, dinv);
  asm volatile("" : "+v"(row[NB - 1]), "+v"(y));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = y + (ok ? 0.0 : 1.0);
#pragma unroll
  for (int c = 0; c < NB; ++c) s += row[c];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int V>
int run(const double* A, double* out, unsigned long long* cyc, const char* name) {
  unsigned long long best = ~0ull;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL(k_bench<V>, 1, 64, 0, 0, A, out, cyc);
    CK(hipDeviceSynchronize());
    unsigned long long c;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    if (c < best) best = c;
  }
  printf("%-28s %7llu cycles  (%5.1f per column)\n", name, best, best / 32.0);
  return 0;
}
__global__ void k_clock(unsigned long long* o, double* sink) {
  double a = threadIdx.x * 1e-3;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 200000; ++i) a = __builtin_fma(a, 0.999999, 1e-7);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  sink[threadIdx.x] = a;
  if (threadIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; }
}

int main() {
  {
    unsigned long long* o; double* sk;
    CK(hipMalloc(&o, 16)); CK(hipMalloc(&sk, 64 * 8));
    for (int r = 0; r < 3; ++r) {
      hipLaunchKernelGGL(k_clock, 1, 64, 0, 0, o, sk);
      CK(hipDeviceSynchronize());
      unsigned long long h[2];
      CK(hipMemcpy(h, o, 16, hipMemcpyDeviceToHost));
      printf("clock: %llu memtime ticks / %llu realtime ticks (100 MHz) -> %.3f GHz; dependent fma %.1f cycles\n", h[0], h[1],
             h[0] / (h[1] * 1e-2) * 1e-3, h[0] / 200000.0);
    }
  }
  double h[NB * NB];
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) h[i * NB + j] = (i == j ? NB + 1.0 : 0.0) + 1.0 / (1 + i + j);
  double *A, *out; unsigned long long* cyc;
  CK(hipMalloc(&A, sizeof h)); CK(hipMalloc(&out, 64 * 8)); CK(hipMalloc(&cyc, 8));
  CK(hipMemcpy(A, h, sizeof h, hipMemcpyHostToDevice));
  run<0>(A, out, cyc, "full");
  double ref[64];
  CK(hipMemcpy(ref, out, sizeof ref, hipMemcpyDeviceToHost));
  run_il<3>(A, out, cyc, "interleaved 3 chunks", ref);
  run_v3<1>(A, out, cyc, "v3 1 chunk", ref);
  run_v3<3>(A, out, cyc, "v3 3 chunks", ref);
  run_v3<5>(A, out, cyc, "v3 5 chunks", ref);
  run<8>(A, out, cyc, "no Newton");
  run<4>(A, out, cyc, "no forward solve");
  run<2>(A, out, cyc, "no look-ahead (wrong)");
  run<1>(A, out, cyc, "no deferred update (wrong)");
  run<3>(A, out, cyc, "pivot chain only (wrong)");
  run<15>(A, out, cyc, "bare (wrong)");
  return 0;
}
