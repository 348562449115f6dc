// Dev micro-benchmark: the 32x32 diagonal factor split over the four waves of a workgroup (wave w owns columns
// 8w .. 8w+7 of every row, lanes 32..63 the identity rows whose elimination leaves L^-1), against the one-wave chol32
// of cholesky.hip (restated here). s_memtime cycles from the first load to the last wave's finish; L^-1 checked
// against a host factorization. Not product code.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chol32w.hip -o tools/ubench_chol32w
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int NB = 32, DS = NB + 1;

__device__ __forceinline__ double rlane(double v, int l) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double rsq_nr(double d) {
  const double r0 = __builtin_amdgcn_rsq(d);
  const double t1 = 0.5 * d * r0;
  return r0 * __builtin_fma(-r0, t1, 1.5);
}

// ---- one wave, right-looking, no look-ahead (reference shape: row per lane)
__device__ bool chol32_1w(double (&row)[NB], int lane, double* col) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double d = rlane(row[j], j);
    ok &= d > 0.0;
    const double r = rsq_nr(d);
    row[j] *= r;
    col[j * 64 + lane] = row[j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int c = j + 1; c < NB; ++c) row[c] -= row[j] * col[j * 64 + c];
  }
  return ok;
}

// ---- the product's one-wave chol32 (cholesky.hip), restated verbatim for the comparison
#define CHOL_SB() __builtin_amdgcn_sched_barrier(0)
constexpr int C32_NCH = 3;  // chunks of the deferred update per column
struct C32State {
  double dn, a1, b1, c2, lp;  // next pivot; A(j+1,j+1), A(j+1,j), A(j+2,j); column j-1's own entry
  double2 cc[NB / 2];         // column j-1 (entries >= j+2) from LDS
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
    const double r0 = __builtin_amdgcn_rsq(d);  // ~5e-8 relative; one Newton step -> ~4e-15
    const double hd = 0.5 * d;
    CHOL_SB();
    c32_fill<J, 0>(row, st);
    CHOL_SB();
    const double t1 = hd * r0;
    CHOL_SB();
    c32_fill<J, 1>(row, st);
    CHOL_SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5);
    CHOL_SB();
    c32_fill<J, 2>(row, st);
    CHOL_SB();
    const double r = r0 * t2;
    const double l1 = st.b1 * r, l2 = st.c2 * r;  // l_{j+1,j}, l_{j+2,j}
    if constexpr (J + 1 < NB) st.dn = __builtin_fma(-l1, l1, st.a1);
    CHOL_SB();
    // column j of L (or of L^-1 e_c in lanes >= 32); lane j's own row[j] is the pivot d
    const double lj = row[J] * r;
    row[J] = lj;
    if constexpr (J + 1 < NB) {
      row[J + 1] -= lj * l1;
      col[(J & 1) * 2 * NB + lane] = lj;  // every lane writes (lanes >= 32 into the unused half)
    }
    if constexpr (J + 2 < NB) row[J + 2] -= lj * l2;
    CHOL_SB();
    if constexpr (J + 1 < NB) {  // column j for the next column's deferred update (entries >= j+3)
      constexpr int n0 = (J + 3) & ~1;
      const double* cb = col + (J & 1) * 2 * NB;
#pragma unroll
      for (int c = n0; c < NB; c += 2) st.cc[c >> 1] = *reinterpret_cast<const double2*>(cb + c);
      st.lp = lj;
    }
    // pivot inputs of column j+2's step (rows j+1, j+2 hold every update of columns <= j now)
    if constexpr (J + 2 < NB) { st.a1 = rlane(row[J + 2], J + 2); st.b1 = rlane(row[J + 1], J + 2); }
    if constexpr (J + 3 < NB) st.c2 = rlane(row[J + 1], J + 3);
    CHOL_SB();
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


// ---- four waves with the product's scheduling idea inside each wave: column k's chain (rsq, Newton) with the deferred
// update of column k-1 (columns >= k+1 of this wave, broadcast values read from LDS one column early) cut into chunks
// between its dependent steps; the next column's own entry updated right after the scaling (critical)
template <int W, int K>
__device__ __forceinline__ void w4_defer(double (&row)[8], double lp, const double (&lc)[8], int q, int nq) {
  // deferred update of column 8W + K - 1 applied to this wave's columns K + 1 .. 7, chunk q of nq
  constexpr int c0 = K + 1;
  constexpr int n = 8 - c0 > 0 ? 8 - c0 : 0;
#pragma unroll
  for (int t = 0; t < n; ++t)
    if (t * nq / (n > 0 ? n : 1) == q || (n < nq && t == q)) row[c0 + t] -= lp * lc[c0 + t];
}
template <int W>
__device__ __forceinline__ bool chol32_w4b_wave(double (&row)[8], int lane, double* col, volatile int* ready) {
  bool ok = true;
  for (int j = 0; j < 8 * W; ++j) {
    while (ready[0] <= j) __builtin_amdgcn_s_sleep(1);
    const double lij = col[j * 64 + lane];
    double lc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) lc[k] = col[j * 64 + 8 * W + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) row[k] -= lij * lc[k];
  }
  double lp = 0.0, lc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) lc[k] = 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int j = 8 * W + k;
    const double d = rlane(row[k], j);
    ok &= d > 0.0;
    const double r0 = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    CHOL_SB();
    if (k >= 1) {  // deferred: column j-1 into columns k+1.. (row[k] got it at step k-1)
#pragma unroll
      for (int c = k + 1; c < 8; c += 2) row[c] -= lp * lc[c];
    }
    CHOL_SB();
    const double t1 = hd * r0;
    CHOL_SB();
    if (k >= 1) {
#pragma unroll
      for (int c = k + 2; c < 8; c += 2) row[c] -= lp * lc[c];
    }
    CHOL_SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5);
    const double r = r0 * t2;
    row[k] *= r;
    col[j * 64 + lane] = row[k];
    if (k + 1 < 8) row[k + 1] -= row[k] * rlane(row[k], j + 1);  // the next pivot's column first
    CHOL_SB();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) ready[0] = j + 1;
    lp = row[k];
#pragma unroll
    for (int c = k + 2; c < 8; ++c) lc[c] = col[j * 64 + 8 * W + c];  // lands while the next chain runs
  }
  return ok;
}
template <int W>
__device__ __forceinline__ bool w4b_dispatch(double (&row)[8], int lane, double* col, volatile int* ready) {
  return chol32_w4b_wave<W>(row, lane, col, ready);
}

// ---- four waves: wave w owns columns 8w .. 8w+7. ready: number of finished columns (LDS), col: 32 x 64 column buffer
template <int W>
__device__ __forceinline__ bool chol32_w4_wave(double (&row)[8], int lane, double* col, volatile int* ready) {
  bool ok = true;
  // updates from the columns of the earlier waves, as they are published
  for (int j = 0; j < 8 * W; ++j) {
    if (j % 8 == 0 || true) {
      while (ready[0] <= j) __builtin_amdgcn_s_sleep(0);
    }
    const double lij = col[j * 64 + lane];
    double lc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) lc[k] = col[j * 64 + 8 * W + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) row[k] -= lij * lc[k];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int j = 8 * W + k;
    const double d = rlane(row[k], j);
    ok &= d > 0.0;
    const double r = rsq_nr(d);
    row[k] *= r;
    col[j * 64 + lane] = row[k];
    if (k + 1 < 8) row[k + 1] -= row[k] * rlane(row[k], j + 1);  // the next pivot's column first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) ready[0] = j + 1;
#pragma unroll
    for (int kk = k + 2; kk < 8; ++kk) row[kk] -= row[k] * col[j * 64 + 8 * W + kk];
  }
  return ok;
}

__global__ void __launch_bounds__(256) k_w4(const double* A, double* out, unsigned long long* cyc, int reps) {
  __shared__ double D[NB * DS];
  __shared__ __attribute__((aligned(16))) double col[NB * 64];
  __shared__ int ready;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < NB * NB; e += 256) D[(e >> 5) * DS + (e & 31)] = A[e];
    if (tid == 0) ready = 0;
    __syncthreads();
    if (rep == reps - 1) t0 = __builtin_amdgcn_s_memtime();
    double row[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = 8 * w + k;
      row[k] = lane < NB ? (c <= lane ? D[lane * DS + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
    }
    bool ok;
    switch (__builtin_amdgcn_readfirstlane(w)) {
      case 0: ok = chol32_w4_wave<0>(row, lane, col, &ready); break;
      case 1: ok = chol32_w4_wave<1>(row, lane, col, &ready); break;
      case 2: ok = chol32_w4_wave<2>(row, lane, col, &ready); break;
      default: ok = chol32_w4_wave<3>(row, lane, col, &ready); break;
    }
    // L^-1 transposed into D as factor_block leaves it: D[c * DS + i] = L^-1(i, c)
    if (lane >= NB)
#pragma unroll
      for (int k = 0; k < 8; ++k) D[(lane - NB) * DS + 8 * w + k] = row[k];
    (void)ok;
    __syncthreads();
    if (rep == reps - 1) t1 = __builtin_amdgcn_s_memtime();
  }
  for (int e = tid; e < NB * NB; e += 256) out[e] = D[(e & 31) * DS + (e >> 5)];  // out[i * 32 + c] = L^-1(i, c)
  if (tid == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(256) k_1w(const double* A, double* out, unsigned long long* cyc, int reps) {
  __shared__ double D[NB * DS];
  __shared__ __attribute__((aligned(16))) double col[NB * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < NB * NB; e += 256) D[(e >> 5) * DS + (e & 31)] = A[e];
    __syncthreads();
    if (rep == reps - 1) t0 = __builtin_amdgcn_s_memtime();
    if (tid < 64) {
      double row[NB];
#pragma unroll
      for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? D[lane * DS + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
      chol32_1w(row, lane, col);
      if (lane >= NB)
#pragma unroll
        for (int i = 0; i < NB; ++i) D[(lane - NB) * DS + i] = row[i];
    }
    __syncthreads();
    if (rep == reps - 1) t1 = __builtin_amdgcn_s_memtime();
  }
  for (int e = tid; e < NB * NB; e += 256) out[e] = D[(e & 31) * DS + (e >> 5)];
  if (tid == 0) cyc[0] = t1 - t0;
}

__global__ void __launch_bounds__(256) k_prod(const double* A, double* out, unsigned long long* cyc, int reps) {
  __shared__ double D[NB * DS];
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  const int tid = threadIdx.x, lane = tid & 63;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < NB * NB; e += 256) D[(e >> 5) * DS + (e & 31)] = A[e];
    __syncthreads();
    if (rep == reps - 1) t0 = __builtin_amdgcn_s_memtime();
    if (tid < 64) {
      double row[NB];
#pragma unroll
      for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? D[lane * DS + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
      chol32(row, lane, col);
      if (lane >= NB)
#pragma unroll
        for (int i = 0; i < NB; ++i) D[(lane - NB) * DS + i] = row[i];
    }
    __syncthreads();
    if (rep == reps - 1) t1 = __builtin_amdgcn_s_memtime();
  }
  for (int e = tid; e < NB * NB; e += 256) out[e] = D[(e & 31) * DS + (e >> 5)];
  if (tid == 0) cyc[0] = t1 - t0;
}
__global__ void __launch_bounds__(256) k_w4b(const double* A, double* out, unsigned long long* cyc, int reps) {
  __shared__ double D[NB * DS];
  __shared__ __attribute__((aligned(16))) double col[NB * 64];
  __shared__ int ready;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < NB * NB; e += 256) D[(e >> 5) * DS + (e & 31)] = A[e];
    if (tid == 0) ready = 0;
    __syncthreads();
    if (rep == reps - 1) t0 = __builtin_amdgcn_s_memtime();
    double row[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = 8 * w + k;
      row[k] = lane < NB ? (c <= lane ? D[lane * DS + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
    }
    switch (__builtin_amdgcn_readfirstlane(w)) {
      case 0: w4b_dispatch<0>(row, lane, col, &ready); break;
      case 1: w4b_dispatch<1>(row, lane, col, &ready); break;
      case 2: w4b_dispatch<2>(row, lane, col, &ready); break;
      default: w4b_dispatch<3>(row, lane, col, &ready); break;
    }
    if (lane >= NB)
#pragma unroll
      for (int k = 0; k < 8; ++k) D[(lane - NB) * DS + 8 * w + k] = row[k];
    __syncthreads();
    if (rep == reps - 1) t1 = __builtin_amdgcn_s_memtime();
  }
  for (int e = tid; e < NB * NB; e += 256) out[e] = D[(e & 31) * DS + (e >> 5)];
  if (tid == 0) cyc[0] = t1 - t0;
}


// ---- lag-2 deferral: column j's rank-1 update reaches columns j+1..j+3 at once (three chain values l1..l3) and the
// rest two steps later, so the LDS reads of the broadcast column have a whole step to land before their first use
struct C32L {
  double dn, a1, b1, c2, c3;
  double lp[2];
  double2 cc0[NB / 2], cc1[NB / 2];
  bool ok;
};
template <int J, int K>
__device__ __forceinline__ void l2_fill(double (&row)[NB], C32L& st) {
  constexpr int c0 = (J + 2) & ~1;
  constexpr int nf = J >= 2 ? (NB - c0) / 2 : 0;
  constexpr int qa = nf * K / C32_NCH, qb = nf * (K + 1) / C32_NCH;
  const double lp = st.lp[J & 1];
#pragma unroll
  for (int q = qa; q < qb; ++q) {
    const int c = c0 + 2 * q;
    const double2 v = (J & 1) ? st.cc1[c >> 1] : st.cc0[c >> 1];
    if (c > J + 1) row[c] -= lp * v.x;
    row[c + 1] -= lp * v.y;
  }
}
template <int J>
__device__ __forceinline__ void l2_step(double (&row)[NB], int lane, double* col, C32L& st) {
  if constexpr (J < NB) {
    const double d = st.dn;
    st.ok &= d > 0.0;
    const double r0 = __builtin_amdgcn_rsq(d);
    const double hd = 0.5 * d;
    CHOL_SB();
    l2_fill<J, 0>(row, st);
    CHOL_SB();
    const double t1 = hd * r0;
    CHOL_SB();
    l2_fill<J, 1>(row, st);
    CHOL_SB();
    const double t2 = __builtin_fma(-r0, t1, 1.5);
    CHOL_SB();
    l2_fill<J, 2>(row, st);
    CHOL_SB();
    const double r = r0 * t2;
    const double l1 = st.b1 * r, l2 = st.c2 * r, l3 = st.c3 * r;
    if constexpr (J + 1 < NB) st.dn = __builtin_fma(-l1, l1, st.a1);
    CHOL_SB();
    const double lj = row[J] * r;
    row[J] = lj;
    if constexpr (J + 1 < NB) row[J + 1] -= lj * l1;
    if constexpr (J + 2 < NB) row[J + 2] -= lj * l2;
    if constexpr (J + 3 < NB) row[J + 3] -= lj * l3;
    constexpr int n0 = (J + 4) & ~1;
    if constexpr (n0 < NB) {
      double* cb = col + (J & 1) * 2 * NB;
      cb[lane] = lj;
      CHOL_SB();
#pragma unroll
      for (int c = n0; c < NB; c += 2) {
        const double2 v = *reinterpret_cast<const double2*>(cb + c);
        if (J & 1) st.cc1[c >> 1] = v; else st.cc0[c >> 1] = v;
      }
      st.lp[J & 1] = lj;
    }
    if constexpr (J + 2 < NB) { st.a1 = rlane(row[J + 2], J + 2); st.b1 = rlane(row[J + 1], J + 2); }
    if constexpr (J + 3 < NB) st.c2 = rlane(row[J + 1], J + 3);
    if constexpr (J + 4 < NB) st.c3 = rlane(row[J + 1], J + 4);
    CHOL_SB();
    l2_step<J + 1>(row, lane, col, st);
  }
}
__device__ __forceinline__ bool chol32_lag2(double (&row)[NB], int lane, double* col) {
  C32L st;
  st.ok = true;
  st.lp[0] = st.lp[1] = 0.0;
  st.dn = rlane(row[0], 0);
  st.a1 = rlane(row[1], 1);
  st.b1 = rlane(row[0], 1);
  st.c2 = rlane(row[0], 2);
  st.c3 = rlane(row[0], 3);
  l2_step<0>(row, lane, col, st);
  return st.ok;
}
__global__ void __launch_bounds__(256) k_lag2(const double* A, double* out, unsigned long long* cyc, int reps) {
  __shared__ double D[NB * DS];
  __shared__ __attribute__((aligned(16))) double col[4 * NB];
  const int tid = threadIdx.x, lane = tid & 63;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int e = tid; e < NB * NB; e += 256) D[(e >> 5) * DS + (e & 31)] = A[e];
    __syncthreads();
    if (rep == reps - 1) t0 = __builtin_amdgcn_s_memtime();
    if (tid < 64) {
      double row[NB];
#pragma unroll
      for (int c = 0; c < NB; ++c) row[c] = lane < NB ? (c <= lane ? D[lane * DS + c] : 0.0) : (lane - NB == c ? 1.0 : 0.0);
      chol32_lag2(row, lane, col);
      if (lane >= NB)
#pragma unroll
        for (int i = 0; i < NB; ++i) D[(lane - NB) * DS + i] = row[i];
    }
    __syncthreads();
    if (rep == reps - 1) t1 = __builtin_amdgcn_s_memtime();
  }
  for (int e = tid; e < NB * NB; e += 256) out[e] = D[(e & 31) * DS + (e >> 5)];
  if (tid == 0) cyc[0] = t1 - t0;
}

int main() {
  // SPD test block
  std::vector<double> A(NB * NB), L(NB * NB, 0.0), Li(NB * NB, 0.0);
  srand(3);
  std::vector<double> B(NB * NB);
  for (auto& x : B) x = rand() / (double)RAND_MAX - 0.5;
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) {
      double s = i == j ? NB : 0.0;
      for (int k = 0; k < NB; ++k) s += B[i * NB + k] * B[j * NB + k];
      A[i * NB + j] = s;
    }
  for (int j = 0; j < NB; ++j) {  // host Cholesky and inverse
    double s = A[j * NB + j];
    for (int k = 0; k < j; ++k) s -= L[j * NB + k] * L[j * NB + k];
    L[j * NB + j] = std::sqrt(s);
    for (int i = j + 1; i < NB; ++i) {
      double t = A[i * NB + j];
      for (int k = 0; k < j; ++k) t -= L[i * NB + k] * L[j * NB + k];
      L[i * NB + j] = t / L[j * NB + j];
    }
  }
  for (int c = 0; c < NB; ++c)
    for (int i = 0; i < NB; ++i) {
      double t = i == c ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) t -= L[i * NB + k] * Li[k * NB + c];
      Li[i * NB + c] = t / L[i * NB + i];
    }
  double *dA, *dO;
  unsigned long long* dc;
  CK(hipMalloc(&dA, NB * NB * 8)); CK(hipMalloc(&dO, NB * NB * 8)); CK(hipMalloc(&dc, 8));
  CK(hipMemcpy(dA, A.data(), NB * NB * 8, hipMemcpyHostToDevice));
  auto run = [&](const char* name, auto kern) -> int {
    unsigned long long best = ~0ull;
    for (int t = 0; t < 20; ++t) {
      hipLaunchKernelGGL(kern, 1, 256, 0, 0, dA, dO, dc, 3);
      CK(hipDeviceSynchronize());
      unsigned long long c;
      CK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
      best = std::min(best, c);
    }
    std::vector<double> o(NB * NB);
    CK(hipMemcpy(o.data(), dO, NB * NB * 8, hipMemcpyDeviceToHost));
    double md = 0;
    for (int i = 0; i < NB; ++i)
      for (int c = 0; c <= i; ++c) md = std::max(md, std::fabs(o[i * NB + c] - Li[i * NB + c]) / (1e-12 + std::fabs(Li[i * NB + c]) + 1.0));
    printf("%-24s %7llu cycles (memtime units)  max rel diff of L^-1 vs host %.2e\n", name, best, md);
    return 0;
  };
  run("one wave, right-looking", k_1w);
  run("four waves, 8 columns each", k_w4);
  run("product chol32 (one wave)", k_prod);
  run("four waves, deferred chunks", k_w4b);
  run("lag-2 chol32 (one wave)", k_lag2);
  return 0;
}
