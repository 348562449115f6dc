// Supernodal multifrontal LL^T on gfx950 — numeric factorization fused with the forward
// solve, and the backward solve.
//
// Replaces the reference's serial up-looking factorization
// (csparse_extension.cpp:64-119 cs_chol_workspace; cs_lsolve/cs_ltsolve/cs_ipvec/cs_pvec
// at :47-52) behind LinearSolver::solve (linear_solver.h:65).  The symbolic
// analysis (symbolic.cpp) fixes ordering, supernodes and frontal maps once per
// structure.  Storage: `fronts` holds each front (m x m col-major, m = ns + nr) as the
// Schur updates progress; the finished factor columns [L11; L21] (m x ns, ld m) go to `lbuf` (the
// 32x32 diagonal blocks of L11 as their inverses in `linv` only),
// so no kernel ever reads a column another workgroup of the same launch is rewriting.
// Each LM trial runs
//   k_permute + k_vec_init   rhs -> P rhs -> front vectors (own rows)
//   per level l (all fronts of a level are independent):
//     k_extend_add     assembly: input entries (+ lambda) and the children's update matrices AND update
//                      vectors -> the level's fronts, one workgroup per (front, 16-column slab),
//                      children in fixed order; beside them
//                      one workgroup per front assembles, factors and forward-solves its first
//                      32x32 diagonal block (the first panel step's input)
//     k_step (x panels) one launch per 32-column panel step: every workgroup owns one 64x64
//                      tile (I, J) of the panel region, solves the panel rows of I and J
//                      against L_kk (TRSM), updates the tile on v_mfma_f64_16x16x4f64, and the
//                      (I = 0)-column writers store L21 rows + update the front vector; the
//                      workgroup of tile (0, 0) then factors the NEXT 32x32 diagonal block —
//                      one kernel boundary per panel step on the critical path
//     k_syrk           contribution block U = A22 - L21 L21^T once per front, K = ns
//     (inverse tasks)  in the k_step launches: X = L11^-1 block by block, beside the critical chain
//   per level L-1..0: k_bwd_gemv (t = y - L21^T x, one wave per column) + k_bwd_x (x = X^T t, one
//                    wave per column): the backward solve has no sequential chain inside a front.
// Every output entry is written by exactly one workgroup per launch in a fixed order: the
// factor and the solution are bitwise reproducible run to run (no atomics).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "device_util.hpp"
#include "gemm_nt.hpp"
#include "kernels.hpp"

namespace g2ohip {

using launch::FrontDesc;
using launch::StepTask;
using launch::Task;

constexpr int NB = 32;   // panel width
constexpr int TT = 64;   // update tile
constexpr int PS = 34;   // LDS row stride (doubles) for the 64 x 32 panel tiles
constexpr int DS = 33;   // LDS row stride of a 32 x 32 diagonal block
constexpr int CS = TT + 1;

typedef double dx4 __attribute__((ext_vector_type(4)));

// Optional phase stamps (development build, -DG2OHIP_PHASES): workgroup 0 / thread 0 of each
// instrumented launch records s_memtime at phase boundaries; read back by g2ohip_debug_phases.
#ifdef G2OHIP_PHASES
__device__ unsigned long long g_phase[4096][8];
__device__ unsigned int g_phase_n;
#define PH_BEGIN(id)                                                       \
  const bool ph_on_ = threadIdx.x == 0 && blockIdx.x == 0;                 \
  unsigned ph_k_ = 0;                                                      \
  if (ph_on_) {                                                            \
    ph_k_ = atomicAdd(&g_phase_n, 1u) % 4096u;                             \
    g_phase[ph_k_][0] = (id);                                              \
    g_phase[ph_k_][1] = __builtin_amdgcn_s_memtime();                      \
    for (int q_ = 2; q_ < 7; ++q_) g_phase[ph_k_][q_] = 0;                 \
    g_phase[ph_k_][7] = __builtin_amdgcn_s_memrealtime();                  \
  }
#define PH(i) \
  if (ph_on_) g_phase[ph_k_][i] = __builtin_amdgcn_s_memtime();
#define PH_REC (ph_on_ ? g_phase[ph_k_] : nullptr)
// second record for the launch's last workgroup (k_step: when the last-dispatched task starts and ends)
#define PH1_BEGIN(id)                                                      \
  const bool ph1_on_ = threadIdx.x == 0 && blockIdx.x == gridDim.x - 1 && gridDim.x > 1; \
  unsigned ph1_k_ = 0;                                                     \
  if (ph1_on_) {                                                           \
    ph1_k_ = atomicAdd(&g_phase_n, 1u) % 4096u;                            \
    g_phase[ph1_k_][0] = (id);                                             \
    g_phase[ph1_k_][1] = __builtin_amdgcn_s_memtime();                     \
    for (int q_ = 2; q_ < 8; ++q_) g_phase[ph1_k_][q_] = 0;                \
    g_phase[ph1_k_][6] = __builtin_amdgcn_s_memrealtime();                 \
  }
#define PH1(i) \
  if (ph1_on_) g_phase[ph1_k_][i] = __builtin_amdgcn_s_memtime();
#define PH1R(i) \
  if (ph1_on_) g_phase[ph1_k_][i] = __builtin_amdgcn_s_memrealtime();
#else
#define PH1R(i)
#define PH1_BEGIN(id)
#define PH1(i)
#define PH_REC nullptr
#define PH_BEGIN(id)
#define PH(i)
#endif

// Small levels (latency-bound, see DeviceCholesky::setup) are zeroed and receive their input entries
// before the first level, by these two massively parallel passes; their assembly launches then add the
// children only. Zero tasks: (offset, length) ranges of the front pool.
__global__ void __launch_bounds__(256) k_zero_ranges(const long long* __restrict__ rng, double* __restrict__ fronts) {
  const long long off = rng[2 * blockIdx.x], len = rng[2 * blockIdx.x + 1];
  for (long long i = threadIdx.x; i < len; i += 256) fronts[off + i] = 0.0;
}
// front vectors: v_s = [P rhs (own columns); 0], the permutation applied on the fly (one workgroup per front)
__device__ __forceinline__ void vec_init_front(const FrontDesc* __restrict__ fd, int f, const int* __restrict__ perm,
                                               const double* __restrict__ rhs, double* __restrict__ vecs) {
  const FrontDesc me = fd[f];
  const int m = me.ns + me.nr;
  double* v = vecs + me.vec_off;
  for (int i = threadIdx.x; i < m; i += 256) v[i] = i < me.ns ? rhs[perm[me.c0 + i]] : 0.0;
}
__global__ void __launch_bounds__(256) k_vec_init(const FrontDesc* __restrict__ fd, const int* __restrict__ perm,
                                                  const double* __restrict__ rhs, double* __restrict__ vecs) {
  vec_init_front(fd, blockIdx.x, perm, rhs, vecs);
}
// the input entries of the prescattered levels; the workgroups past the entries' own (nsb) initialise the front
// vectors, one per front (disjoint data, one launch instead of two at the start of every factorization)
__global__ void __launch_bounds__(256) k_chol_scatter(long long nent, int nsb, const double* __restrict__ vals,
                                                      const long long* __restrict__ dst, const int* __restrict__ src,
                                                      const double* __restrict__ lam, double* __restrict__ fronts,
                                                      const FrontDesc* __restrict__ fd, const int* __restrict__ perm,
                                                      const double* __restrict__ rhs, double* __restrict__ vecs) {
  if ((int)blockIdx.x >= nsb) {
    vec_init_front(fd, (int)blockIdx.x - nsb, perm, rhs, vecs);
    return;
  }
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nent) return;
  const int sr = src[k];
  const double v = vals[sr & 0x7fffffff];
  fronts[dst[k]] = sr < 0 ? v + *lam : v;
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
// rows >= kb padded with the identity). On return row[c] = L(lane, c).
// Returns false if a pivot was not positive (cs_chol's `d <= 0` test).
// Latency-shaped for one wave, right-looking. The pivot chain runs on wave-uniform values only:
// d_{j+1} = A(j+1,j+1) - (A(j+1,j) r_j)^2, both entries read by v_readlane one column early, so the
// sequential chain per column is rsq -> Newton step -> r_j -> l_{j+1,j} -> d_{j+1}. Off the chain:
// the scaled column l_j = row[j] r_j, its two-column look-ahead (l_{j+1,j}, l_{j+2,j} are chain
// values, no broadcast), the rest of column j-1's rank-1 update (through LDS, one column late,
// columns >= j+2), cut into chunks that sched_barriers pin between the chain's dependent steps.
// The block's forward solve is not in this loop (publish_inverse multiplies by L^-1). Entries
// above a lane's diagonal may collect garbage; they are never read. One template instance per
// column keeps every register index a compile-time constant.
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

// Wave 0: factor the kb x kb block staged in D (LDS, row stride DS, lower triangle valid).
// Lanes 32..63 run the same instruction stream on the identity: lane 32 + c ends holding column c
// of L^-1 (right-looking substitution on the broadcast columns of L), left transposed in D
// (D[c * DS + i] = L^-1(i, c)) for publish_inverse, which the whole workgroup runs after a barrier.
// The diagonal block of L itself is not stored: every consumer of the factor (tile TRSM, next-diagonal
// update, inverse tasks, backward and multi-right-hand-side solves) uses L^-1 for diagonal blocks.
__device__ __forceinline__ void factor_block(double* D, int kb, const double* vy, double* col, int lane, int* fail,
                                             double* ysol, unsigned long long* ph = nullptr, double* ylds = nullptr) {
  double row[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    const double a = ld0(D, lane * DS + c, lane < kb && c <= lane);
    row[c] = ((lane >= kb && c == lane) || lane - NB == c) ? 1.0 : a;
  }
  if (ph) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); ph[5] = __builtin_amdgcn_s_memtime(); }
  const bool ok = chol32(row, lane, col);
  if (ph) { asm volatile("" : "+v"(row[NB - 1])); ph[6] = __builtin_amdgcn_s_memtime(); }
  if (lane == 0 && !ok) *fail = 1;
  if (lane >= NB) {  // every read of D (the row loads above) is done: this wave's LDS traffic is in order
#pragma unroll
    for (int i = 0; i < NB; ++i) D[(lane - NB) * DS + i] = row[i];
  }
  // the block's forward solve y = L^-1 v (v in LDS, kb values) as a product with the inverse the same wave
  // just wrote (in-order LDS traffic, no barrier) — a substitution inside chol32's column loop cost ~50
  // cycles per column on the critical chain; ysol leaves before the inverse stores
  if (lane < NB) {
    double y4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c0 = 0; c0 < NB; c0 += 8) {
      double dv[8], vv[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) { dv[c] = D[(c0 + c) * DS + lane]; vv[c] = vy[c0 + c]; }
#pragma unroll
      for (int c = 0; c < 8; ++c) y4[c & 3] += (c0 + c <= lane ? dv[c] : 0.0) * (c0 + c < kb ? vv[c] : 0.0);
    }
    const double yv = (y4[0] + y4[1]) + (y4[2] + y4[3]);
    if (lane < kb) ysol[lane] = yv;
    if (ylds) ylds[lane] = lane < kb ? yv : 0.0;  // (same wave: in-order LDS traffic for its later readers)
  }
}
// After factor_block and a workgroup barrier: L_kk^-1 row-major to linv and the diagonal block of
// X = L11^-1 (column-major, leading dimension ldx), both coalesced over the 256 threads.
__device__ __forceinline__ void publish_inverse(const double* D, int kb, int tid, double* linv, double* X, int ldx) {
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = tid + 256 * u, i = e >> 5, c = e & (NB - 1);
    linv[e] = D[c * DS + i];  // row i, column c of L^-1 (identity-padded past kb)
  }
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = tid + 256 * u, c = e >> 5, i = e & (NB - 1);
    if (c < kb && i < kb) X[(size_t)c * ldx + i] = D[c * DS + i];
  }
}

// ---------------------------------------------------------------------------- 64-column panel steps
// The launch-per-panel schedule with 64-column panels (DeviceCholesky::setup chooses it per level): half the kernel
// boundaries on the diagonal chain — each boundary costs ~3 us of drain + dispatch and ~2.4 us of reloads at the next
// diagonal task's start (tools/phase_probe.py) against ~4 us for a chol32 — and every trailing update is rank 64 (the
// lagged pairs' traffic without their strip steps). The current panel's inverse L_p^-1 = [A 0; N B] is kept as the two
// per-32-panel inverses A = L_a^-1, B = L_b^-1 (linv, as the 32-column schedule: the backward solve and
// computeMarginals read them) and N = -L_b^-1 L_ba L_a^-1 (linvn, one per 64-panel). Tasks (StepTask, k0kb = k0 | kb << 16,
// kb <= 64):
//   tile (flags & 1 update)  TRSM of the tile's panel rows as X = P L_p^-T in two 32-column halves (X_a = P_a A^T,
//                            X_b = P_a N^T + P_b B^T), then C_IJ -= X_I X_J^T half by half (rank 64); writers store
//                            L rows and update the front vector with X_I y_p;
//   diagonal (flags & 4)     the next 64 x 64 block: D' = D - X X^T with its own X rows, then chol64 (below);
//   inverse (flags & 16)     X = L11^-1 for the backward solve, block row by block row (32-row blocks p, 32-column
//                            blocks j): W_pj += L_pa X_aj + L_pb X_bj for the previous 64-panel (a, b); the two rows of
//                            the current 64-panel finalised as X = -L_p^-1 W.
constexpr int W64_LI = 3 * NB * PS;           // A | N | B of the current panel, row-major, stride PS
constexpr int W64_R = W64_LI;                 // role region
constexpr int W64_COL = W64_R + TT * PS + 3 * NB * DS;
constexpr int W64_VN = W64_COL + 4 * NB, W64_YL = W64_VN + TT, W64_YK = W64_YL + TT;
constexpr int W64_LDS = W64_YK + TT;
static_assert(W64_R + 2 * TT * PS <= W64_COL && TT * (TT + 1) <= 2 * TT * PS, "tile role region");
static_assert(W64_R + TT * PS + NB * PS + TT * (NB + 1) <= W64_LDS, "inverse role region");
static_assert(W64_COL % 2 == 0, "col buffer: 16-byte aligned");

struct Chol64Lds {
  double *Qaa, *Qba, *Qbb;  // quadrants of the block, 32 x DS each (row-major; lower parts valid)
  double *S, *Nb;           // scratch: 64 x PS and 32 x PS
  double *col, *vn, *yl;    // chol32 column buffers, right-hand side (64), y (64)
};
// publish_inverse over threads [t0, t0 + nt) of the workgroup (the others are busy)
__device__ __forceinline__ void publish_inv_part(const double* D, int kb, int t, int nt, double* linv, double* X, int ldx) {
  for (int e = t; e < NB * NB; e += nt) linv[e] = D[(e & (NB - 1)) * DS + (e >> 5)];
  for (int e = t; e < NB * NB; e += nt) {
    const int c = e >> 5, i = e & (NB - 1);
    if (c < kb && i < kb) X[(size_t)c * ldx + i] = D[c * DS + i];
  }
}
struct NoSide {
  __device__ void operator()() const {}
};
// Factor the kbn x kbn (kbn <= 64) block in q.Q* with right-hand side q.vn: L_a = chol(Qaa), L_ba = Qba L_a^-T,
// L_b = chol(Qbb - L_ba L_ba^T), N = -L_b^-1 L_ba L_a^-1, y = L^-1 vn. Publishes L_a^-1, L_b^-1 (linv rows), N (linvn),
// the block's part of X = L11^-1 (X, leading dimension ldx) and y (ysol); L_ba goes to the factor (Lba, leading dimension
// ldl: the only part of L this block owns in lbuf, diagonal 32 x 32 blocks are never stored). Whole workgroup; while
// wave 0 runs each chol32 the other three waves work beside it: side_a() during the first (the caller's updates of Qba,
// Qbb and vn_b), M = L_ba L_a^-1 and the a half's publishing during the second.
template <class SideA>
__device__ __forceinline__ void chol64(const Chol64Lds& q, int kbn, int tid, int* fail, double* ysol, double* linv_a,
                                       double* linv_b, double* linvn, double* X, int ldx, double* Lba, int ldl,
                                       unsigned long long* ph, SideA side_a) {
  const int lane = tid & 63, w = tid >> 6, lr = lane & 15, lk = lane >> 4;
  const int kna = min(NB, kbn), knb = kbn - NB;
  if (tid < 64) factor_block(q.Qaa, kna, q.vn, q.col, tid, fail, ysol, ph, q.yl);
  else side_a();
  __syncthreads();
  if (knb <= 0) {
    publish_inv_part(q.Qaa, kna, tid, 256, linv_a, X, ldx);
    return;
  }
  const int tr = w & 1, tc = w >> 1;
  {  // L_ba = Qba L_a^-T (L_a^-1(c, k) = Qaa[k DS + c]); rows past knb zeroed (N and the tiles rely on it)
    dx4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {
      const int k = kk * 4 + lk;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(q.Qba[(16 * tr + lr) * DS + k], q.Qaa[k * DS + 16 * tc + lr], acc, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * tr + lk + 4 * i, c = 16 * tc + lr;
      const double v = r < knb ? acc[i] : 0.0;
      q.Qba[r * DS + c] = v;
      if (r < knb) Lba[(size_t)c * ldl + r] = v;
    }
  }
  __syncthreads();
  if (w < 3) {  // Qbb -= L_ba L_ba^T on the lower 16 x 16 tiles (0,0), (1,0), (1,1)
    const int ur = (w + 1) >> 1, uc = w >> 1;
    dx4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {
      const int k = kk * 4 + lk;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(q.Qba[(16 * ur + lr) * DS + k], q.Qba[(16 * uc + lr) * DS + k], acc, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) q.Qbb[(16 * ur + lk + 4 * i) * DS + 16 * uc + lr] -= acc[i];
  } else if (lane < NB) {  // the b rows' right-hand side: vn_b -= L_ba y_a
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < NB; ++k) s2 += q.Qba[lane * DS + k] * q.yl[k];
    q.vn[NB + lane] -= s2;
  }
  __syncthreads();
  if (tid < 64) {
    factor_block(q.Qbb, knb, q.vn + NB, q.col, tid, fail, ysol + NB, nullptr, q.yl + NB);
  } else {  // beside it: M = L_ba L_a^-1 (row-major into S; tiles over waves 1..3), the a half published
    for (int tl = w - 1; tl < 4; tl += 3) {
      const int ur = tl & 1, uc = tl >> 1;
      dx4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(q.Qba[(16 * ur + lr) * DS + k], q.Qaa[(16 * uc + lr) * DS + k], acc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) q.S[(16 * ur + lk + 4 * i) * PS + 16 * uc + lr] = acc[i];
    }
    publish_inv_part(q.Qaa, kna, tid - 64, 192, linv_a, X, ldx);
  }
  __syncthreads();
  {  // N = -L_b^-1 M
    dx4 an = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {
      const int k = kk * 4 + lk;
      an = __builtin_amdgcn_mfma_f64_16x16x4f64(q.Qbb[k * DS + 16 * tr + lr], q.S[k * PS + 16 * tc + lr], an, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) q.Nb[(16 * tr + lk + 4 * i) * PS + 16 * tc + lr] = -an[i];
  }
  __syncthreads();
  publish_inv_part(q.Qbb, knb, tid, 256, linv_b, X + (size_t)NB * ldx + NB, ldx);
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = tid + 256 * u;
    linvn[e] = q.Nb[(e >> 5) * PS + (e & (NB - 1))];
  }
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = tid + 256 * u, c = e >> 5, i = e & (NB - 1);
    if (i < knb) X[(size_t)c * ldx + NB + i] = q.Nb[i * PS + c];
  }
}

// stage the current panel's inverses A | N | B (row-major, as in linv / linvn) into Li3; B and N only with a b half
__device__ __forceinline__ void load_li3(const double* la, const double* ln, const double* lb, bool bh, int tid,
                                         double (&v)[3][NB * NB / 256]) {
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    v[0][u] = la[tid + 256 * u];
    v[1][u] = ld0(ln, tid + 256 * u, bh);
    v[2][u] = ld0(lb, tid + 256 * u, bh);
  }
}
__device__ __forceinline__ void store_li3(double* Li3, int tid, const double (&v)[3][NB * NB / 256]) {
#pragma unroll
  for (int h = 0; h < 3; ++h)
#pragma unroll
    for (int u = 0; u < NB * NB / 256; ++u) {
      const int e = tid + 256 * u;
      Li3[h * NB * PS + (e >> 5) * PS + (e & (NB - 1))] = v[h][u];
    }
}
// X rows of a 64-row panel slab (rows 16 w .. 16 w + 15 of this wave), cols [16 h, 16 h + 16) of a 32-column half:
// x[h] += P(rows, 0:32) Lq^T with Lq row-major (stride PS) in LDS
__device__ __forceinline__ void trsm_half(const double* P, const double* Lq, int lane, int w, dx4 (&x)[2]) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int k = kk * 4 + lk;
    const double a = P[(16 * w + lr) * PS + k];
    x[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Lq[lr * PS + k], x[0], 0, 0, 0);
    x[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Lq[(16 + lr) * PS + k], x[1], 0, 0, 0);
  }
}
__device__ __forceinline__ void store_xhalf(double* P, int lane, int w, const dx4 (&x)[2]) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 16 * w + lk + 4 * i;
    P[r * PS + lr] = x[0][i];
    P[r * PS + 16 + lr] = x[1][i];
  }
}

// ---------------------------------------------------------------------------- assembly + extend-add
// One launch per level assembles every front of the level from scratch (no front-pool memset, no
// separate scatter pass), with two kinds of workgroup:
//  * block-0 tasks (t.c == 1, dispatched first, one per front): the front's first kb x kb diagonal block
//    and front-vector head are assembled here (the column's input entries of the reduced system + the
//    children's update-matrix entries that map into it, children in fixed order), factored and
//    forward-solved, and L_00, y_0, L_00^-1 published: the first panel step needs no launch of its own;
//  * slab tasks (t.c == 0): columns [a, b) of one front, every entry outside the first diagonal block:
//    the lower part of each column is written once (zero, or the input entry + lambda on the diagonal;
//    inputs come from a per-column list, `colptr`/`ent_row`/`ent_src`), then the children's update
//    matrices AND update vectors are added, children in fixed order. One wave per column, 4 columns per
//    wave: the column's writes are coalesced runs.
// Every entry is written by exactly one workgroup, in the same order: bitwise reproducible.
__device__ __forceinline__ double input_entry(const double* vals, const int* ent_src, const int* ent_row, int e,
                                              const double* lam, int& row) {
  const int rr = ent_row[e];
  row = rr & 0x3fffffff;
  const double v = vals[ent_src[e]];
  return (rr >> 30) ? v + *lam : v;
}
// ASM: the level's fronts are assembled here (EAC: rows per LDS column chunk); else they were pre-zeroed and
// scattered
// W64: the level runs 64-column panel steps (k_step64): its first-block tasks assemble and factor the first 64 columns
// (chol64), and the slabs leave those 64 x 64 entries to them
template <bool ASM, int EAC, bool W64>
__global__ void __launch_bounds__(256) k_extend_add(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                                    const int* __restrict__ children, const int* __restrict__ relmap,
                                                    const int* __restrict__ jtab, const int* __restrict__ cmptr,
                                                    const int2* __restrict__ cment, const int* __restrict__ colptr, const int* __restrict__ ent_row,
                                                    const int* __restrict__ ent_src, const double* __restrict__ vals,
                                                    const double* __restrict__ lam, double* __restrict__ fronts,
                                                    double* __restrict__ vecs, double* __restrict__ lbuf,
                                                    double* __restrict__ ysol, double* __restrict__ linv,
                                                    double* __restrict__ linvn, double* __restrict__ xinv,
                                                    int* __restrict__ fail) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, kb0 = min(W64 ? TT : NB, me.ns);
  double* F = fronts + me.front_off;
  double* v = vecs + me.vec_off;
  const int tid = threadIdx.x;
  // W64: one buffer for both roles (the 64-wide first block, the slabs' column buffers)
  constexpr int SMU = !W64 ? 1 : (W64_LDS > 4 * EAC ? W64_LDS : 4 * EAC);
  __shared__ __attribute__((aligned(16))) double smu[SMU];
  if constexpr (W64) {
    if (t.c == 1) {
      // ---- first 64 x 64 block: assembled (input entries, children), factored with chol64, published
      Chol64Lds q;
      q.S = smu + W64_R;
      q.Qaa = q.S + TT * PS;
      q.Qba = q.Qaa + NB * DS;
      q.Qbb = q.Qba + NB * DS;
      q.Nb = smu + NB * PS;
      q.col = smu + W64_COL;
      q.vn = smu + W64_VN;
      q.yl = smu + W64_YL;
      int* cp = reinterpret_cast<int*>(smu + W64_YK);  // kb0 + 1 column pointers (64 doubles hold 128 ints)
      auto qp = [&](int r, int c) -> double* {
        return r < NB ? q.Qaa + r * DS + c : (c < NB ? q.Qba + (r - NB) * DS + c : q.Qbb + (r - NB) * DS + c - NB);
      };
      PH_BEGIN(1)
      if constexpr (!ASM) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
          const bool ok = r < kb0 && c <= r;
          const double x = ld0(F, c * m + r, ok);
          if (c <= r) *qp(r, c) = x;
        }
        if (tid < TT) q.vn[tid] = ld0(v, tid, tid < kb0);
      } else {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
          if (c <= r) *qp(r, c) = 0.0;
        }
        if (tid <= kb0) cp[tid] = colptr[me.c0 + tid];
        if (tid < TT) q.vn[tid] = ld0(v, tid, tid < kb0);
        __syncthreads();
        for (int e = cp[0] + tid; e < cp[kb0]; e += 256) {
          int lo = 0, hi = kb0;
          while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (cp[mid] <= e) lo = mid; else hi = mid; }
          int r;
          const double x = input_entry(vals, ent_src, ent_row, e, lam, r);
          if (r < kb0) *qp(r, lo) = x;
        }
      }
      __syncthreads();
      // children two at a time: every load of a pair in flight before the first add, adds in fixed child order
      constexpr int B0C = 2;
      for (int kc = me.child_begin; kc < me.child_end; kc += B0C) {
        double val[B0C][16], vv[B0C];
        int dst[B0C][16], vdst[B0C];
#pragma unroll
        for (int c = 0; c < B0C; ++c) {
          const bool has = kc + c < me.child_end;
          const FrontDesc cd = fd[children[has ? kc + c : kc]];
          const int mc = cd.ns + cd.nr, nrc = cd.nr;
          const double* U = fronts + cd.front_off + (size_t)cd.ns * mc + cd.ns;
          const int* rel = relmap + cd.rows_off;
          const int n0 = has ? jtab[cd.jt_off] : 0;  // child rows mapping into the first 64 x 64 block
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            const int e = tid + 256 * u;
            const int i = e & (TT - 1), j = e >> 6;
            const bool in = i < nrc && j <= i;
            val[c][u] = ld0(U, j * mc + i, in);
            const int ri = ld0(rel, i, in), rj = ld0(rel, j, in);
            dst[c][u] = (in && i < n0) ? (ri | (rj << 8)) : -1;
          }
          vv[c] = ld0(vecs + cd.vec_off + cd.ns, tid, tid < nrc && tid < TT);
          const int rt = ld0(rel, tid, tid < nrc && tid < TT);
          vdst[c] = tid < n0 && tid < TT ? rt : -1;
        }
#pragma unroll
        for (int c = 0; c < B0C; ++c) {
          if (kc + c >= me.child_end) break;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (dst[c][u] >= 0) *qp(dst[c][u] & 0xff, dst[c][u] >> 8) += val[c][u];
          if (vdst[c] >= 0) q.vn[vdst[c]] += vv[c];
          __syncthreads();
        }
      }
      PH(2)
      chol64(q, kb0, tid, fail, ysol + me.c0, linv + (size_t)me.c0 * (NB * NB), linv + (size_t)(me.c0 + NB) * (NB * NB),
             linvn + (size_t)me.c0 * (NB * NB), xinv + me.x_off, me.ns, lbuf + me.l_off + NB, m, PH_REC, NoSide{});
      PH(3)
      PH(4)
      return;
    }
  }
  if constexpr (!W64) {
  if (t.c == 1) {
    __shared__ double D[NB * DS];
    __shared__ __attribute__((aligned(16))) double col[4 * NB];  // two 64-lane column buffers
    __shared__ double vy[NB];
    PH_BEGIN(1)
    if constexpr (!ASM) {
#pragma unroll
      for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
        const int e = tid + 256 * u_;
        const int r = e & (NB - 1), c = e >> 5;
        const bool ok = r < kb0 && c < kb0 && r >= c;
        const double x = ld0(F, c * m + r, ok);
        if (ok) D[r * DS + c] = x;
      }
      if (tid < kb0) vy[tid] = v[tid];
    } else {
      __shared__ int cp[NB + 1];
      for (int i = tid; i < NB * DS; i += 256) D[i] = 0.0;
      if (tid <= kb0) cp[tid] = colptr[me.c0 + tid];
      if (tid < kb0) vy[tid] = v[tid];
      __syncthreads();
      // input entries of the block's columns (one contiguous range), the whole workgroup striding over it
      for (int e = cp[0] + tid; e < cp[kb0]; e += 256) {
        int lo = 0, hi = kb0;  // column of entry e: cp[lo] <= e < cp[lo + 1]
        while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (cp[mid] <= e) lo = mid; else hi = mid; }
        int r;
        const double x = input_entry(vals, ent_src, ent_row, e, lam, r);
        if (r < kb0) D[r * DS + lo] = x;
      }
    }
    __syncthreads();
    // children in groups of B0C: every load of a group (descriptors, n0, rel, update entries) is issued
    // before the first add, so a group costs three dependent round trips instead of three per child;
    // the adds then run child by child in the fixed order (bitwise reproducible)
    constexpr int B0C = 4;
    for (int kc = me.child_begin; kc < me.child_end; kc += B0C) {
      double val[B0C][NB * NB / 256], vv[B0C];
      int dst[B0C][NB * NB / 256], vdst[B0C];
#pragma unroll
      for (int c = 0; c < B0C; ++c) {
        const bool has = kc + c < me.child_end;
        const FrontDesc cd = fd[children[has ? kc + c : kc]];
        const int mc = cd.ns + cd.nr, nrc = cd.nr;
        const double* U = fronts + cd.front_off + (size_t)cd.ns * mc + cd.ns;
        const int* rel = relmap + cd.rows_off;
        const int n0 = has ? jtab[cd.jt_off] : 0;  // child rows mapping into the block (rel is increasing)
#pragma unroll
        for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
          const int e = tid + 256 * u_;
          const int i = e & (NB - 1), j = e >> 5;
          const bool in = i < nrc && j <= i;  // independent of n0: issued together with it
          val[c][u_] = ld0(U, j * mc + i, in);
          const int ri = ld0(rel, i, in), rj = ld0(rel, j, in);
          dst[c][u_] = (in && i < n0) ? ri * DS + rj : -1;
        }
        vv[c] = ld0(vecs + cd.vec_off + cd.ns, tid, tid < nrc && tid < NB);
        const int rt = ld0(rel, tid, tid < nrc && tid < NB);
        vdst[c] = tid < n0 ? rt : -1;
      }
#pragma unroll
      for (int c = 0; c < B0C; ++c) {
        if (kc + c >= me.child_end) break;
#pragma unroll
        for (int u_ = 0; u_ < NB * NB / 256; ++u_)
          if (dst[c][u_] >= 0) D[dst[c][u_]] += val[c][u_];
        if (vdst[c] >= 0) vy[vdst[c]] += vv[c];
        __syncthreads();
      }
    }
    PH(2)
    if (t.a < 0) {  // level factored by k_dag: the assembled block and its right-hand side go into the front
#pragma unroll
      for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
        const int e = tid + 256 * u_, r = e & (NB - 1), c = e >> 5;
        if (r < kb0 && c < kb0 && r >= c) F[c * m + r] = D[r * DS + c];
      }
      if (tid < kb0) v[tid] = vy[tid];
      return;
    }
    if (tid < 64) factor_block(D, kb0, vy, col, tid, fail, ysol + me.c0, PH_REC);
    __syncthreads();
    publish_inverse(D, kb0, tid, linv + (size_t)me.c0 * (NB * NB), xinv + me.x_off, me.ns);
    PH(3)
    PH(4)
    return;
  }
  }
  const int a = t.a, b = t.b;
  const int lane = tid & 63, w = tid >> 6;
  if constexpr (ASM) {
    // In-place assembly: each wave builds its columns in an LDS column buffer (zero, the column's input
    // entries, then every (child, child column) pair mapping to it in child order) and writes each entry
    // of the front once; rows in chunks of EAC. The children's update vectors follow below.
    __shared__ double cbuf_[W64 ? 1 : 4][W64 ? 1 : EAC];
    double(*cbuf)[EAC] = W64 ? reinterpret_cast<double(*)[EAC]>(smu) : reinterpret_cast<double(*)[EAC]>(&cbuf_[0][0]);
    for (int j = a + w; j < b; j += 4) {
      const int rlo = j < kb0 ? kb0 : j;  // rows of the first diagonal block: block-0 task
      double* Fj = F + (size_t)j * m;
      const int q0 = cmptr[me.cm_off + j], q1 = cmptr[me.cm_off + j + 1];
      for (int rc = rlo; rc < m; rc += EAC) {
        const int rce = min(m, rc + EAC);
        double* cb = cbuf[w] - rc;
        for (int i = rc + lane; i < rce; i += 64) cb[i] = 0.0;
        if (j < me.ns)
          for (int e = colptr[me.c0 + j] + lane; e < colptr[me.c0 + j + 1]; e += 64) {
            int r;
            const double x = input_entry(vals, ent_src, ent_row, e, lam, r);
            if (r >= rc && r < rce) cb[r] = x;
          }
        for (int q = q0; q < q1; ++q) {
          const int2 ce = cment[q];
          const FrontDesc cd = fd[ce.x];
          const int mc = cd.ns + cd.nr, nrc = cd.nr;
          const double* Uj = fronts + cd.front_off + (size_t)(cd.ns + ce.y) * mc + cd.ns;
          const int* rel = relmap + cd.rows_off;
          for (int i0 = ce.y + lane; i0 < nrc; i0 += 256) {
            double val[4];
            int ri[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int i = i0 + u * 64;
              const bool ok = i < nrc;
              val[u] = ld0(Uj, i, ok);
              ri[u] = ok ? ld0(rel, i, ok) : -1;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (ri[u] >= rc && ri[u] < rce) cb[ri[u]] += val[u];
          }
        }
        for (int i = rc + lane; i < rce; i += 64) Fj[i] = cb[i];
      }
    }
    for (int k = me.child_begin; k < me.child_end; ++k) {  // update vectors, children in fixed order
      const FrontDesc cd = fd[children[k]];
      const double* u = vecs + cd.vec_off + cd.ns;
      const int* rel = relmap + cd.rows_off;
      const int j0 = jtab[cd.jt_off + t.c - 1], j1 = jtab[cd.jt_off + t.c];
      for (int j = j0 + tid; j < j1; j += 256)
        if (rel[j] >= kb0) v[rel[j]] += u[j];
      __syncthreads();
    }
    return;
  }
  // 2. children in fixed order
  for (int k = me.child_begin; k < me.child_end; ++k) {
    const FrontDesc cd = fd[children[k]];
    const int mc = cd.ns + cd.nr, nrc = cd.nr;
    const double* U = fronts + cd.front_off + (size_t)cd.ns * mc + cd.ns;  // U(i,j) = U[j*mc + i]
    const double* u = vecs + cd.vec_off + cd.ns;
    const int* rel = relmap + cd.rows_off;
    // child columns whose parent column lies in [a, b) (rel is increasing; precomputed per slab)
    const int j0 = jtab[cd.jt_off + t.c - 1], j1 = jtab[cd.jt_off + t.c];
    for (int j = j0 + tid; j < j1; j += 256)
      if (rel[j] >= kb0) v[rel[j]] += u[j];
    // lower triangle: one wave per child column, lanes run down the rows (coalesced U reads,
    // mostly-contiguous F writes), 4 independent loads in flight per lane
    for (int j = j0 + w; j < j1; j += 4) {
      const double* Uj = U + (size_t)j * mc;
      double* Fj = F + (size_t)rel[j] * m;
      const int rlo = rel[j] < kb0 ? kb0 : 0;  // rows of the first diagonal block: block-0 task
      for (int i0 = j + lane; i0 < nrc; i0 += 256) {
        double val[4];
        int ri[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = i0 + q * 64;
          const bool ok = i < nrc;
          val[q] = ld0(Uj, i, ok);
          ri[q] = ok ? ld0(rel, i, ok) : -1;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (ri[q] >= rlo) Fj[ri[q]] += val[q];
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------- panel step
struct MfmaTile {  // 64x64 tile, 4 waves x (2x2) v_mfma_f64_16x16x4f64 tiles, K chunk of 32 in LDS
  dx4 acc[2][2];
  __device__ void zero() {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = dx4{0.0, 0.0, 0.0, 0.0};
  }
  __device__ void step(const double* Pa, const double* Pb, int lane, int w) {
    const int wr = (w & 1) * 32, wc = (w >> 1) * 32;
    const int lr = lane & 15, lk = lane >> 4;
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
  }
  // D layout of v_mfma_f64_16x16x4f64: lane l holds D[(l>>4) + 4*i][l & 15], i = 0..3
  __device__ void store(double* Ct, int lane, int w) const {
    const int wr = (w & 1) * 32, wc = (w >> 1) * 32;
    const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) Ct[(wr + x * 16 + lk + 4 * i) * CS + wc + y * 16 + lr] = acc[x][y][i];
  }
};

// C tile entries owned by a thread: idx = tid + 256 u -> (r = idx % 64, c = idx / 64)
__device__ __forceinline__ void load_ctile(const double* F, int m, int I0, int J0, int climit, int tid, double (&cv)[16]) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = tid + 256 * u, r = idx & (TT - 1), c = idx >> 6;
    const int gi = I0 + r, gj = J0 + c;
    cv[u] = ld0(F, gj * m + gi, gi < m && gj < climit && gi >= gj);
  }
}

// Task flags: 1 update the tile (else TRSM + L21 store only), 4 the step's next-diagonal task,
// 8 the tile may reach into the contribution block (columns >= ns: no separate k_syrk pass),
// 16 an inverse task: block (tj, ti) of X = L11^-1 (see below),
// 64 lagged pair (odd steps of a lagged front, DeviceCholesky::setup): the update also applies the PREVIOUS
//    panel (k0 - 32, whose L rows the strip tiles of the even step stored), so the trailing columns are read and
//    written once per two panels (rank-64); the even steps update only the next panel's strip (clim = r0 + kbn).
// Rows/columns of the tile: I0 = r0 + 64 ti, J0 = r0 + 64 tj, r0 = k0 + kb.
// PAIRS: the launch may hold lagged-pair tasks (flag 64); without them the pair code is compiled out (166 instead of
// ~180 VGPRs: three workgroups per CU instead of two)
template <bool PAIRS>
__global__ void __launch_bounds__(256, 3) k_step(const StepTask* __restrict__ tasks, const launch::StepHead head,
                                              double* __restrict__ fronts,
                                              double* __restrict__ lbuf, double* __restrict__ vecs,
                                              double* __restrict__ ysol, double* __restrict__ linv,
                                              double* __restrict__ xinv, int* __restrict__ fail) {
  __shared__ double Li[NB * PS];      // L_kk^-1, row-major, stride 34
  __shared__ double yk[NB];
  __shared__ double sh[2 * TT * PS];  // Pa | Pb; reused as the 64 x 65 result tile
  __shared__ double Dn[NB * DS];      // next diagonal block
  __shared__ __attribute__((aligned(16))) double col[4 * NB];  // two 64-lane column buffers
  __shared__ double vn[NB];
  PH_BEGIN(2)
  PH1_BEGIN(3)
  const StepTask t = (int)blockIdx.x < head.n ? head.t[blockIdx.x] : tasks[blockIdx.x];
  const int m = t.m, ns = t.ns;
  double* F = fronts + t.f_off;
  double* L = lbuf + t.l_off;
  double* v = vecs + t.v_off;
  const int k0 = t.k0kb & 0xffff, kb = t.k0kb >> 16;
  const int ti = t.tile & 0xffff, tj = t.tile >> 16;
  const bool upd = t.flags & 1, writer = tj == 0;
  const int r0 = k0 + kb;
  const int I0 = r0 + ti * TT, J0 = r0 + tj * TT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double* Pa = sh;
  double* Pb = sh + TT * PS;
  const double* Lin = linv + (size_t)(t.c0 + k0) * (NB * NB);

  if (t.flags & 4) {
    // ---- dedicated next-diagonal task (runs beside the tile tasks of this step): the 32x32 block
    // D' = A(r0:r0+32, r0:r0+32) - X X^T with X = P(r0:r0+32) L_kk^-T, then its factor, inverse
    // and forward solve. Only the critical chain of the panel step lives here.
    const int kbn = min(NB, ns - r0);
    const bool pair = PAIRS && (t.flags & 64);  // the block also lacks the previous panel's update (lagged, odd step)
    double lv[NB * NB / 256], pv[NB * NB / 256], cdv[NB * NB / 256], xpv[NB * NB / 256];
#pragma unroll
    for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
      const int e = tid + 256 * u_, r = e & (NB - 1), c = e >> 5;
      lv[u_] = ld0(Lin, e, kb > 0);  // kb = 0: first block of a big panel, already fully updated
      pv[u_] = ld0(F, (k0 + c) * m + r0 + r, c < kb);
      cdv[u_] = ld0(F, (r0 + c) * m + r0 + r, r >= c && r < kbn);
      xpv[u_] = ld0(L, (k0 - NB + c) * m + r0 + r, pair);  // L rows of the block in the previous panel
    }
    const double ykv = ld0(ysol, t.c0 + k0 + tid, tid < kb);
    const double vo = ld0(v, r0 + tid, tid < kbn);
#pragma unroll
    for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
      const int e = tid + 256 * u_, r = e & (NB - 1), c = e >> 5;
      Li[c * PS + r] = lv[u_];  // e = row * 32 + col of the row-major inverse: (c, r) = (row, col)
      Pa[r * PS + c] = pv[u_];
      Dn[r * DS + c] = cdv[u_];
      Pb[r * PS + c] = xpv[u_];
    }
    if (tid < NB) yk[tid] = ykv;
    __syncthreads();
    const int lr = lane & 15, lk = lane >> 4;
    {  // X = P L_kk^-T: wave w owns the 16x16 tile (w & 1, w >> 1), one MFMA pipe per tile
      const int xr = w & 1, xc = w >> 1;
      dx4 x0 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(Pa[(16 * xr + lr) * PS + k], Li[(16 * xc + lr) * PS + k], x0, 0, 0, 0);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 4; ++i) Pa[(16 * xr + lk + 4 * i) * PS + 16 * xc + lr] = x0[i];
    }
    __syncthreads();
    {  // D' -= X X^T (+ X_prev X_prev^T on a lagged odd step): wave w owns the 16x16 tile (w & 1, w >> 1)
      const int tr = w & 1, tc = w >> 1;
      dx4 acc = {0.0, 0.0, 0.0, 0.0};
      if (pair) {
#pragma unroll
        for (int kk = 0; kk < NB / 4; ++kk) {
          const int k = kk * 4 + lk;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Pb[(16 * tr + lr) * PS + k], Pb[(16 * tc + lr) * PS + k], acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Pa[(16 * tr + lr) * PS + k], Pa[(16 * tc + lr) * PS + k], acc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * tr + lk + 4 * i, c = 16 * tc + lr;
        Dn[r * DS + c] -= acc[i];
      }
    }
    if (tid < NB) {  // rhs of the next block: v - X y_k (same sum, same order as the writer task)
      double s2 = 0.0;
#pragma unroll
      for (int q = 0; q < NB; ++q) s2 += Pa[tid * PS + q] * yk[q];
      vn[tid] = vo - s2;
    }
    __syncthreads();
    PH(2)
    if (tid < 64) factor_block(Dn, kbn, vn, col, tid, fail, ysol + t.c0 + r0, PH_REC);
    __syncthreads();
    publish_inverse(Dn, kbn, tid, linv + (size_t)(t.c0 + r0) * (NB * NB), xinv + t.x_off + (size_t)r0 * ns + r0, ns);
    PH(3)
    PH(4)
    return;
  }

  if (t.flags & 16) {
    // ---- explicit inverse of the supernode's diagonal part, X = L11^-1, for the parallel backward
    // solve (k_bwd_x). Right-looking over the panel steps: the step of panel s adds the term of block
    // row s-1 to every pending block (p, j), p >= s, j < s:  W_pj += L_{p,s-1} X_{s-1,j}, kept in X's
    // own slot; at p = s the block is final: X_sj = -L_ss^-1 W_sj. Every input was written by an
    // earlier launch; one 32x32x32 product (two when finalising) per task, beside the critical chain.
    const int j = ti, pp = tj, kq = k0 / NB - 1;
    const bool fin = pp * NB == k0;
    const int kbp = min(NB, ns - NB * pp);
    double* Xf = xinv + t.x_off;
    double wv[4], lq[4], xq[4], li[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, r = e & (NB - 1), c = e >> 5;
      wv[u] = ld0(Xf, (NB * j + c) * ns + NB * pp + r, kq > j && r < kbp);  // W_pj so far
      lq[u] = ld0(L, (NB * kq + c) * m + NB * pp + r, r < kbp);              // L_{p,kq}(r, c)
      xq[u] = Xf[(NB * j + c) * ns + NB * kq + r];                           // X_{kq,j}(r, c)
      li[u] = ld0(Lin, e, fin);                                              // L_ss^-1, row-major
    }
    double* Ts = Dn;  // 32 x DS
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, r = e & (NB - 1), c = e >> 5;
      Pa[r * PS + c] = lq[u];
      Pb[r * PS + c] = xq[u];
      Ts[r * DS + c] = wv[u];
      Li[(e >> 5) * PS + (e & (NB - 1))] = li[u];
    }
    __syncthreads();
    const int tr = w & 1, tc = w >> 1;
    dx4 acc = {0.0, 0.0, 0.0, 0.0};
    {  // acc = L_{p,kq} X_{kq,j} on the wave's 16x16 tile (B given as rows q of X_{kq,j})
      const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Pa[(16 * tr + lr) * PS + k], Pb[k * PS + 16 * tc + lr], acc, 0, 0, 0);
      }
    }
    const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += Ts[(16 * tr + lk + 4 * i) * DS + 16 * tc + lr];
    if (!fin) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * tr + lk + 4 * i, c = 16 * tc + lr;
        if (r < kbp) Xf[(size_t)(NB * j + c) * ns + NB * pp + r] = acc[i];
      }
      PH1R(7)
      return;
    }
    __syncthreads();  // every read of Ts done
#pragma unroll
    for (int i = 0; i < 4; ++i) Ts[(16 * tr + lk + 4 * i) * DS + 16 * tc + lr] = acc[i];
    __syncthreads();
    dx4 xo = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {  // X_sj = -L_ss^-1 W_sj
      const int k = kk * 4 + lk;
      xo = __builtin_amdgcn_mfma_f64_16x16x4f64(Li[(16 * tr + lr) * PS + k], Ts[k * DS + 16 * tc + lr], xo, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * tr + lk + 4 * i, c = 16 * tc + lr;
      if (r < kbp) Xf[(size_t)(NB * j + c) * ns + NB * pp + r] = -xo[i];
    }
    PH1R(7)
    return;
  }

  // ---- lagged pair: the previous panel's L rows of I and J (stored by the even step's strip tiles) go first
  const bool pair = PAIRS && (t.flags & 64) && upd;
  MfmaTile T;
  T.zero();
  double xpa[8], xpb[8];  // issued with the current panel's loads (one round trip), staged before the C prefetch
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
    xpa[u] = ld0(L, (k0 - NB + q) * m + I0 + r, pair && I0 + r < m);
    xpb[u] = ld0(L, (k0 - NB + q) * m + J0 + r, pair && J0 + r < m);
  }
  // ---- stage L_kk^-1, y_k, the raw panel rows of I (and J), prefetch the C tile: every global
  // load is issued before the first LDS store so the whole batch is in flight at once
  double lv[NB * NB / 256], pav[8], pbv[8], cv[16];
#pragma unroll
  for (int u_ = 0; u_ < NB * NB / 256; ++u_) lv[u_] = Lin[tid + 256 * u_];
  const double ykv = ld0(ysol, t.c0 + k0 + tid, tid < kb);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
    pav[u] = ld0(F, (k0 + q) * m + I0 + r, q < kb && I0 + r < m);
    pbv[u] = ld0(F, (k0 + q) * m + J0 + r, upd && q < kb && J0 + r < m);
  }
  const int climit = t.clim;  // ns; m when the contribution block is fused; the big-panel end when blocked
  if (pair) {  // C[I, J] -= X_prev,I X_prev,J^T into the accumulators first, the current panel's loads in flight
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
      Pa[r * PS + q] = xpa[u];
      Pb[r * PS + q] = xpb[u];
    }
    __syncthreads();
    T.step(Pa, Pb, lane, w);
    __syncthreads();  // Pa / Pb free for the current panel
  }
  if (upd) load_ctile(F, m, I0, J0, climit, tid, cv);
#pragma unroll
  for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
    const int e = tid + 256 * u_;
    Li[(e >> 5) * PS + (e & (NB - 1))] = lv[u_];
  }
  if (tid < NB) yk[tid] = ykv;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
    Pa[r * PS + q] = pav[u];
    Pb[r * PS + q] = pbv[u];
  }
  __syncthreads();

  PH1(2)
  // ---- TRSM as a product: X = P L_kk^-T on v_mfma_f64_16x16x4f64; wave w owns rows 16w..16w+15
  // of both panels (A = P rows, B[k][c] = L_kk^-1(c, k))
  {
    const int lr = lane & 15, lk = lane >> 4;
    dx4 xa0 = {0.0, 0.0, 0.0, 0.0}, xa1 = xa0, xb0 = xa0, xb1 = xa0;
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {
      const int k = kk * 4 + lk;
      const double a = Pa[(16 * w + lr) * PS + k], b = Pb[(16 * w + lr) * PS + k];
      const double l0 = Li[lr * PS + k], l1 = Li[(16 + lr) * PS + k];
      xa0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, l0, xa0, 0, 0, 0);
      xa1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, l1, xa1, 0, 0, 0);
      xb0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, l0, xb0, 0, 0, 0);
      xb1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, l1, xb1, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 16 * w + lk + 4 * i;
      Pa[r * PS + lr] = xa0[i];
      Pa[r * PS + 16 + lr] = xa1[i];
      Pb[r * PS + lr] = xb0[i];
      Pb[r * PS + 16 + lr] = xb1[i];
    }
  }
  __syncthreads();
  // rows/columns of the next diagonal block, [r0, r0 + kbn): this step's diagonal task reads their
  // raw values at its start and applies the panel update itself, so tile tasks never write them
  const int kbn = (t.flags & 32) ? 0 : max(0, min(NB, ns - r0));
  if (writer && tid < 64 && I0 + tid < m && I0 + tid >= r0 + kbn) {  // forward-solve update: v_i -= x_i y_k
    double s2 = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) s2 += Pa[tid * PS + q] * yk[q];
    v[I0 + tid] -= s2;
  }

  // ---- writers store the L21 rows of block I
  if (writer) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
      if (q < kb && I0 + r < m) L[(k0 + q) * m + I0 + r] = Pa[r * PS + q];
    }
  }
  PH1(3)
  if (!upd) { PH1R(7) return; }

  // ---- C[I, J] -= P_I P_J^T (columns inside the supernode, lower triangle)
  T.step(Pa, Pb, lane, w);
  __syncthreads();
  T.store(sh, lane, w);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = tid + 256 * u, r = idx & (TT - 1), c = idx >> 6;
    const int gi = I0 + r, gj = J0 + c;
    const bool dblk = gi < r0 + kbn && gj < r0 + kbn;
    if (gi < m && gj < climit && gi >= gj && !dblk) F[(size_t)gj * m + gi] = cv[u] - sh[r * CS + c];
  }
  PH1(4)
  PH1R(7)
}

// ---------------------------------------------------------------------------- 64-column panel steps (kernel)
// (see the 64-column helpers above k_extend_add)
__global__ void __launch_bounds__(256, 2) k_step64(const StepTask* __restrict__ tasks, const launch::StepHead head,
                                                   double* __restrict__ fronts, double* __restrict__ lbuf,
                                                   double* __restrict__ vecs, double* __restrict__ ysol,
                                                   double* __restrict__ linv, double* __restrict__ linvn,
                                                   double* __restrict__ xinv, int* __restrict__ fail) {
  __shared__ __attribute__((aligned(16))) double sm[W64_LDS];
  PH_BEGIN(2)
  PH1_BEGIN(3)
  const StepTask t = (int)blockIdx.x < head.n ? head.t[blockIdx.x] : tasks[blockIdx.x];
  const int m = t.m, ns = t.ns;
  double* F = fronts + t.f_off;
  double* L = lbuf + t.l_off;
  double* v = vecs + t.v_off;
  const int k0 = t.k0kb & 0xffff, kb = t.k0kb >> 16;  // current panel [k0, k0 + kb), kb <= 64
  const int kbb = kb - NB;                             // columns of its b half (<= 0: none)
  const bool bh = kbb > 0;
  const int r0 = k0 + kb;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double* Li3 = sm;
  const double* la = linv + (size_t)(t.c0 + k0) * (NB * NB);
  const double* lb = linv + (size_t)(t.c0 + k0 + (bh ? NB : 0)) * (NB * NB);
  const double* ln = linvn + (size_t)(t.c0 + k0) * (NB * NB);

  if (t.flags & 4) {
    // ---- next-diagonal task: the 64 x 64 block at r0 with this panel's update applied, then chol64
    const int kbn = min(TT, ns - r0);
    Chol64Lds q;
    q.S = sm + W64_R;
    q.Qaa = q.S + TT * PS;
    q.Qba = q.Qaa + NB * DS;
    q.Qbb = q.Qba + NB * DS;
    q.Nb = Li3 + NB * PS;
    q.col = sm + W64_COL;
    q.vn = sm + W64_VN;
    q.yl = sm + W64_YL;
    double* yk = sm + W64_YK;
    double lv[3][NB * NB / 256], pa[8], pb[8], dq[16];
    load_li3(la, ln, lb, bh, tid, lv);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
      pa[u] = ld0(F, (k0 + c) * m + r0 + r, r < kbn && c < kb);
      pb[u] = ld0(F, (k0 + NB + c) * m + r0 + r, r < kbn && c < kbb);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
      dq[u] = ld0(F, (r0 + c) * m + r0 + r, r < kbn && c <= r);
    }
    const double vo = ld0(v, r0 + tid, tid < kbn);
    const double ykv = ld0(ysol, t.c0 + k0 + tid, tid < kb);
    store_li3(Li3, tid, lv);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
      q.S[r * PS + c] = pa[u];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
      if (c <= r) {
        double* Qp = r < NB ? q.Qaa + r * DS + c : (c < NB ? q.Qba + (r - NB) * DS + c : q.Qbb + (r - NB) * DS + c - NB);
        *Qp = dq[u];
      }
    }
    if (tid < TT) { q.vn[tid] = vo; yk[tid] = ykv; }
    __syncthreads();
    PH(2)
    // X = P L_p^-T: X_a = P_a A^T (S afterwards), X_b = P_a N^T + P_b B^T (X2 = the Li3 region afterwards)
    dx4 xa[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}}, xb[2] = {xa[0], xa[0]};
    trsm_half(q.S, Li3, lane, w, xa);
    trsm_half(q.S, Li3 + NB * PS, lane, w, xb);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
      q.S[r * PS + c] = pb[u];
    }
    __syncthreads();
    trsm_half(q.S, Li3 + 2 * NB * PS, lane, w, xb);
    __syncthreads();
    double* X2 = Li3;  // 64 x PS (A | N | B are dead)
    store_xhalf(q.S, lane, w, xa);
    store_xhalf(X2, lane, w, xb);
    __syncthreads();
    const int lr = lane & 15, lk = lane >> 4;
    // tile (ur, uc) of the 64 x 64 block: Q -= X(rows) X(cols)^T over K = 64 (both halves)
    auto dtile = [&](int ur, int uc) {
      dx4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(q.S[(16 * ur + lr) * PS + k], q.S[(16 * uc + lr) * PS + k], acc, 0, 0, 0);
      }
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X2[(16 * ur + lr) * PS + k], X2[(16 * uc + lr) * PS + k], acc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * ur + lk + 4 * i, c = 16 * uc + lr;
        double* Qp = r < NB ? q.Qaa + r * DS + c : (c < NB ? q.Qba + (r - NB) * DS + c : q.Qbb + (r - NB) * DS + c - NB);
        *Qp -= acc[i];
      }
    };
    auto vrow = [&](int r) {  // vn_r -= X_r y_p
      double s2 = 0.0;
#pragma unroll
      for (int k = 0; k < NB; ++k) s2 += q.S[r * PS + k] * yk[k] + X2[r * PS + k] * yk[NB + k];
      q.vn[r] -= s2;
    };
    // the a quadrant and vn_a first (the first chol32 needs them); the b rows beside that chol32 (chol64's side work)
    if (w < 3) dtile((w + 1) >> 1, w >> 1);
    else if (lane < NB) vrow(lane);
    __syncthreads();
    PH(2)
    chol64(q, kbn, tid, fail, ysol + t.c0 + r0, linv + (size_t)(t.c0 + r0) * (NB * NB),
           linv + (size_t)(t.c0 + r0 + NB) * (NB * NB), linvn + (size_t)(t.c0 + r0) * (NB * NB),
           xinv + t.x_off + (size_t)r0 * ns + r0, ns, L + (size_t)r0 * m + r0 + NB, m, PH_REC, [&] {
             // waves 1..3: the ba quadrant's tiles (2,0) (2,1) (3,0) (3,1), the bb quadrant's (2,2) (3,2) (3,3), vn_b
             const int sw = w - 1;
             for (int tl = sw; tl < 7; tl += 3) {
               const int ur = tl < 4 ? 2 + (tl >> 1) : (tl == 4 ? 2 : 3), uc = tl < 4 ? (tl & 1) : (tl == 6 ? 3 : 2);
               dtile(ur, uc);
             }
             if (sw == 2 && lane < NB) vrow(NB + lane);
           });
    PH(3)
    PH(4)
    return;
  }

  if (t.flags & 16) {
    // ---- inverse task: block column j, block row p (32-blocks) of X = L11^-1. The previous 64-panel is (a, b) =
    // (k0 / 32 - 2, k0 / 32 - 1); W_pj += L_pa X_aj + L_pb X_bj; the current panel's rows (p = k0 / 32, with p + 1)
    // are finalised: X_pj = -A W_pj, X_p+1,j = -(N W_pj + B W_p+1,j).
    const int j = t.tile & 0xffff, p = t.tile >> 16, qa = k0 / NB - 2, qb = qa + 1;
    const bool fin = p * NB == k0;
    const int rows = min(fin ? TT : NB, ns - NB * p);  // output rows (64 when finalising both rows of the panel)
    double* Xf = xinv + t.x_off;
    double* Ls = sm + W64_R;            // 64 x PS: L(rows, q)
    double* Xs = Ls + TT * PS;          // 32 x PS: X_qj (row k, column c)
    double* Wl = Xs + NB * PS;          // 64 x (NB + 1)
    const int lr = lane & 15, lk = lane >> 4;
    // wave w: output rows 16 w .. 16 w + 15 (rows < 64), two 16-column tiles
    dx4 acc[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
    double wv[2][4];  // W so far (the earlier panels' terms), in the MFMA output layout
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * w + lk + 4 * i, c = 16 * h + lr;
        wv[h][i] = ld0(Xf, (NB * j + c) * ns + NB * p + r, j < qa && r < rows);
      }
#pragma unroll
    for (int term = 0; term < 2; ++term) {
      const int qq = term == 0 ? qa : qb;
      if (qq < j) continue;  // X_qj = 0 above the diagonal (uniform)
      double lq[8], xq[4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
        lq[u] = ld0(L, (NB * qq + c) * m + NB * p + r, r < rows);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + 256 * u, k = e & (NB - 1), c = e >> 5;
        xq[u] = Xf[(NB * j + c) * ns + NB * qq + k];
      }
      __syncthreads();  // the previous term's reads of Ls / Xs are done
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
        Ls[r * PS + c] = lq[u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + 256 * u, k = e & (NB - 1), c = e >> 5;
        Xs[k * PS + c] = xq[u];
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        const double a = Ls[(16 * w + lr) * PS + k];
        acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Xs[k * PS + lr], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Xs[k * PS + 16 + lr], acc[1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[h][i] += wv[h][i];
    if (!fin) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * w + lk + 4 * i, c = 16 * h + lr;
          if (r < rows) Xf[(size_t)(NB * j + c) * ns + NB * p + r] = acc[h][i];
        }
      return;
    }
    double lv[3][NB * NB / 256];
    load_li3(la, ln, lb, bh, tid, lv);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) Wl[(16 * w + lk + 4 * i) * (NB + 1) + 16 * h + lr] = acc[h][i];
    store_li3(Li3, tid, lv);
    __syncthreads();
    // wave w: rows 16 w .. of X_p (w < 2: -A W_top) or X_p+1 (w >= 2: -(N W_top + B W_bot))
    dx4 xo[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
    const int wr = 16 * (w & 1);
    const double* L1 = w < 2 ? Li3 : Li3 + NB * PS;
#pragma unroll
    for (int kk = 0; kk < NB / 4; ++kk) {
      const int k = kk * 4 + lk;
      const double a = L1[(wr + lr) * PS + k];
      xo[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Wl[k * (NB + 1) + lr], xo[0], 0, 0, 0);
      xo[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Wl[k * (NB + 1) + 16 + lr], xo[1], 0, 0, 0);
    }
    if (w >= 2) {
#pragma unroll
      for (int kk = 0; kk < NB / 4; ++kk) {
        const int k = kk * 4 + lk;
        const double a = Li3[2 * NB * PS + (wr + lr) * PS + k];
        xo[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Wl[(NB + k) * (NB + 1) + lr], xo[0], 0, 0, 0);
        xo[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Wl[(NB + k) * (NB + 1) + 16 + lr], xo[1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * w + lk + 4 * i, c = 16 * h + lr;
        if (r < rows) Xf[(size_t)(NB * j + c) * ns + NB * p + r] = -xo[h][i];
      }
    return;
  }

  // ---- tile task (I, J): rows I0 = r0 + 64 ti, columns J0 = r0 + 64 tj
  const int ti = t.tile & 0xffff, tj = t.tile >> 16;
  const bool upd = t.flags & 1, writer = tj == 0;
  const int I0 = r0 + ti * TT, J0 = r0 + tj * TT;
  double* Pa = sm + W64_R;
  double* Pb = Pa + TT * PS;
  double* yk = sm + W64_YK;
  const int climit = t.clim;
  double lv[3][NB * NB / 256], pa0[8], pb0[8], pa1[8], pb1[8], cv[16];
  load_li3(la, ln, lb, bh, tid, lv);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
    pa0[u] = ld0(F, (k0 + c) * m + I0 + r, c < kb && I0 + r < m);
    pb0[u] = ld0(F, (k0 + c) * m + J0 + r, upd && c < kb && J0 + r < m);
    pa1[u] = ld0(F, (k0 + NB + c) * m + I0 + r, c < kbb && I0 + r < m);
    pb1[u] = ld0(F, (k0 + NB + c) * m + J0 + r, upd && c < kbb && J0 + r < m);
  }
  const double ykv = ld0(ysol, t.c0 + k0 + tid, tid < kb);
  store_li3(Li3, tid, lv);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
    Pa[r * PS + c] = pa0[u];
    Pb[r * PS + c] = pb0[u];
  }
  if (tid < TT) yk[tid] = ykv;
  if (upd) load_ctile(F, m, I0, J0, climit, tid, cv);
  __syncthreads();
  // X_a = P_a A^T and P_a N^T for the rows of I and J (wave w: rows 16 w ..)
  dx4 xia[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}}, xja[2] = {xia[0], xia[0]}, xib[2] = {xia[0], xia[0]},
      xjb[2] = {xia[0], xia[0]};
  trsm_half(Pa, Li3, lane, w, xia);
  if (upd) trsm_half(Pb, Li3, lane, w, xja);
  if (bh) {
    trsm_half(Pa, Li3 + NB * PS, lane, w, xib);
    if (upd) trsm_half(Pb, Li3 + NB * PS, lane, w, xjb);
  }
  __syncthreads();
  if (bh) {  // X_b = P_a N^T + P_b B^T
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), c = e >> 6;
      Pa[r * PS + c] = pa1[u];
      Pb[r * PS + c] = pb1[u];
    }
    __syncthreads();
    trsm_half(Pa, Li3 + 2 * NB * PS, lane, w, xib);
    if (upd) trsm_half(Pb, Li3 + 2 * NB * PS, lane, w, xjb);
    __syncthreads();
  }
  PH1(2)
  // rows / columns of the next diagonal block [r0, r0 + kbn): its diagonal task applies this panel itself
  const int kbn = max(0, min(TT, ns - r0));
  MfmaTile T;
  T.zero();
  double s2 = 0.0;  // writers: X_I y_p
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !bh) break;
    store_xhalf(Pa, lane, w, h == 0 ? xia : xib);
    if (upd) store_xhalf(Pb, lane, w, h == 0 ? xja : xjb);
    __syncthreads();
    if (writer) {
      if (tid < TT) {
#pragma unroll
        for (int q = 0; q < NB; ++q) s2 += Pa[tid * PS + q] * yk[NB * h + q];
      }
      const int qn = h == 0 ? min(NB, kb) : kbb;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
        if (q < qn && I0 + r < m) L[(size_t)(k0 + NB * h + q) * m + I0 + r] = Pa[r * PS + q];
      }
    }
    if (upd) T.step(Pa, Pb, lane, w);
    __syncthreads();
  }
  if (writer && tid < TT && I0 + tid < m && I0 + tid >= r0 + kbn) v[I0 + tid] -= s2;
  PH1(3)
  if (!upd) { PH1R(7) return; }
  T.store(Pa, lane, w);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = tid + 256 * u, r = idx & (TT - 1), c = idx >> 6;
    const int gi = I0 + r, gj = J0 + c;
    const bool dblk = gi < r0 + kbn && gj < r0 + kbn;
    if (gi < m && gj < climit && gi >= gj && !dblk) F[(size_t)gj * m + gi] = cv[u] - Pa[r * CS + c];
  }
  PH1(4)
  PH1R(7)
}

// ---------------------------------------------------------------------------- contribution block
// U = A22 - L21 L21^T (rows/columns ns..m-1) in one pass with K = ns (gemm_nt.hpp: 64x64 tiles, K in
// double-buffered 16-column LDS chunks). Task: s, b = ti | tj << 16, K = [a, c) (c = 0: [0, ns)).
// The same kernel is the trailing update of a blocked front after each big panel: rows >= kb, columns
// [kb, ns), K = the big panel's columns [ka, kb) of the finished factor.
using SyrkTile = GemmNT<TT, TT>;
__global__ void __launch_bounds__(256) k_syrk(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                              double* __restrict__ fronts, const double* __restrict__ lbuf) {
  __shared__ double sh[SyrkTile::LDS_DOUBLES];
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, ns = me.ns;
  const int ti = t.b & 0xffff, tj = t.b >> 16;
  const int ka = t.a, kb = t.c ? t.c : ns, climit = kb == ns ? m : ns;
  // a childless front's contribution block holds nothing before this pass (its rows and columns are ancestors'
  // variables: no input entries, no children): written, not read
  const bool overwrite = t.c == 0 && me.child_begin == me.child_end;
  SyrkTile::run(lbuf + me.l_off, m, fronts + me.front_off, m, m, climit, kb + ti * TT, kb + tj * TT, ka, kb, sh,
                overwrite);
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
// Per level (descending), two launches, both parallel over columns (no sequential chain):
//   k_bwd_gemv  t_s = y_s - L21^T x_rows for every front of the level; one wave per column, lanes run
//               down the column (coalesced), x_rows gathered from the finished ancestors
//   k_bwd_x     x_s = L11^-T t_s = X^T t_s with the explicit inverse X = L11^-1 built during the
//               factorization (k_step inverse tasks); one wave per column of X
// Task: s, a = first column (4 per workgroup).
__global__ void __launch_bounds__(256) k_bwd_gemv(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                                  const int* __restrict__ rows, const double* __restrict__ lbuf,
                                                  const double* __restrict__ ysol, const double* __restrict__ xsol,
                                                  double* __restrict__ tsol) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, ns = me.ns;
  const int lane = threadIdx.x & 63, j = t.a + (int)(threadIdx.x >> 6);
  if (j >= ns) return;
  const double* col = lbuf + me.l_off + (size_t)j * m + ns;
  const int* rw = rows + me.rows_off;
  double acc = 0.0;
  for (int i = lane; i < me.nr; i += 64) acc += col[i] * xsol[rw[i]];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) tsol[me.c0 + j] = ysol[me.c0 + j] - acc;
}

__global__ void __launch_bounds__(256) k_bwd_x(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                               const double* __restrict__ xinv, const double* __restrict__ tsol,
                                               double* __restrict__ xsol, const int* __restrict__ perm,
                                               double* __restrict__ xout) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int ns = me.ns;
  const int lane = threadIdx.x & 63, j = t.a + (int)(threadIdx.x >> 6);
  if (j >= (t.b ? t.b : ns)) return;
  const double* xc = xinv + me.x_off + (size_t)j * ns;  // column j of X (rows >= j are nonzero)
  const double* tt = tsol + me.c0;
  const int ie = t.c;  // X(j.., j) up to row ie: ns, or the end of a blocked front's big panel (X_bb)
  double a4[4] = {0.0, 0.0, 0.0, 0.0};
  int i = j + lane;
  for (; i + 192 < ie; i += 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a4[u] += xc[i + 64 * u] * tt[i + 64 * u];
  }
  for (; i < ie; i += 64) a4[0] += xc[i] * tt[i];
  double acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) {
    xsol[me.c0 + j] = acc;
    xout[perm[me.c0 + j]] = acc;  // the solution in the caller's order (no separate inverse permutation)
  }
}

// blocked fronts: t_j -= sum_{i in [t.b, ns)} L(i, j) x_i for the columns j of one big panel (the later big
// panels of the supernode are solved already); one wave per column
__global__ void __launch_bounds__(256) k_bwd_inner(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                                   const double* __restrict__ lbuf, const double* __restrict__ xsol,
                                                   double* __restrict__ tsol) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, ns = me.ns;
  const int lane = threadIdx.x & 63, j = t.a + (int)(threadIdx.x >> 6);
  if (j >= t.b) return;
  const double* col = lbuf + me.l_off + (size_t)j * m;
  const double* xx = xsol + me.c0;
  double acc = 0.0;
  for (int i = t.b + lane; i < ns; i += 64) acc += col[i] * xx[i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) tsol[me.c0 + j] -= acc;
}

// ---------------------------------------------------------------------------- persistent tile DAG
// Latency-bound levels (few fronts): the launch-per-panel schedule above pays a kernel boundary, a
// reload of every tile and a reload of L_kk^-1 per 32 columns. Here one launch factors the whole level. Every 64 x 64
// tile of every front of the level is owned by one workgroup (one per CU, all resident), which keeps the tile in
// MFMA accumulators from the first panel to the last, and per panel k (32 columns, k0 = 32 k, in own tile column
// Jp = k0 / 64, half h) plays one role:
//   DIAG   (Jp, Jp): factor the diagonal block (its quadrant (h, h)) with chol32, y_k = L_kk^-1 (v_k - sum L_kq y_q);
//          publish L_kk^-1 and y_k; for h = 0 also the L rows of quadrant (1, 0) (TRSM with the fresh inverse), then
//          update quadrant (1, 1) locally: the next panel's diagonal block needs no hand-off;
//   TRSM   (I, Jp), I > Jp: L_Ik = C_I,half L_kk^-T (the tile's own half-columns), publish it; for h = 0 update the
//          tile's other half with L_Ik and the diagonal tile's quadrant-(1, 0) rows;
//   UPDATE (I, J), J > Jp: C_IJ -= L_Ik L_Jk^T (diagonal tiles also fold L_Ik y_k into their right-hand side).
// Hand-offs (MI355X_MICROARCH.md §visibility, the write-through form): every handed-off double is stored with an
// sc1 (write-through) store, every storing wave drains (vmcnt 0), the workgroup barrier, then one lane stores the
// flag = this call's epoch with an agent-scope atomic; the consumer's lane 0 polls the flag with agent-scope atomic
// loads, the workgroup barrier, then every load of the handed-off bytes is an sc1 load. One workgroup per CU (the
// launch reserves LDS for that). Within a workgroup the roles run per panel in the order DIAG, TRSM, UPDATE and every
// dependency points to an earlier (panel, role): with all workgroups resident the DAG cannot deadlock. A poll that
// spins too long (a bug, never expected) sets the timeout word and the fail flag and stops waiting.
// Outputs are those of the panel-step schedule (lbuf L columns without the 32 x 32 diagonal blocks, linv per panel,
// ysol, the contribution block in the front, the update vector in the front vector) except X = L11^-1: the backward
// solve of these fronts is k_bwd_seq.
using launch::DagFront;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ double ld_wt0(const double* p, long long idx, bool ok) {
  const double v = ld_wt(p + (ok ? idx : 0));
  return ok ? v : 0.0;
}
// every storing wave drains its write-through stores, then one lane raises the flag
__device__ __forceinline__ void dag_signal(unsigned* flag, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr unsigned DAG_SPIN_MAX = 1u << 22;
__device__ __forceinline__ void dag_poll(unsigned* flag, unsigned epoch, unsigned* tmo, int* fail) {
  unsigned spins = 0;
  while (__hip_atomic_load((gu32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0) {
      if (__hip_atomic_load((gu32*)tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch) return;
      if (spins >= DAG_SPIN_MAX) {
        __hip_atomic_store((gu32*)tmo, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *fail = 1;
        return;
      }
    }
  }
}
// lane 0 polls (one or two flags), then the workgroup barrier: every wave's loads come after the match
__device__ __forceinline__ void dag_wait(unsigned* f1, unsigned* f2, unsigned epoch, unsigned* tmo, int* fail) {
  if (threadIdx.x == 0) {
    if (f1) dag_poll(f1, epoch, tmo, fail);
    if (f2 && f2 != f1) dag_poll(f2, epoch, tmo, fail);
  }
  __syncthreads();
}
__device__ __forceinline__ int dag_off(const DagFront& F, int I) { return I < F.nown ? 64 * I : F.ns + 64 * (I - F.nown); }
__device__ __forceinline__ int dag_len(const DagFront& F, int I) {
  return I < F.nown ? min(64, F.ns - 64 * I) : min(64, F.m - F.ns - 64 * (I - F.nown));
}

template <int TPW>
struct DagLds {
  double Li[NB * PS];   // L_kk^-1 row-major (li_tag: which front / panel it holds)
  double Pa[TT * PS];   // staging: a tile's panel columns, or L rows loaded from another workgroup
  double Pb[TT * PS];
  double D[NB * DS];    // diagonal block / its inverse (factor_block)
  __attribute__((aligned(16))) double col[4 * NB];
  double vy[NB], yk[NB];
  double vacc[TPW][TT];       // diagonal tiles: v_rows - sum_q L_rows,q y_q
  double Lout[TPW][TT * PS];  // this panel's L rows produced by each tile slot (TRSM: 64 rows, DIAG: rows 32..63), read
                              // in place by the slot's own later roles of the panel: no hand-off inside a workgroup
};

// acc (a tile's 64 x 64 in the MfmaTile layout of wave w) -> the wave's 32 x 32 quadrant into buf (row-major, stride S,
// at row offset ro); called by the owning wave only
__device__ __forceinline__ void dag_stage(const dx4 (&acc)[2][2], double* buf, int S, int ro, int lane) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[(ro + 16 * x + lk + 4 * i) * S + 16 * y + lr] = acc[x][y][i];
}
// acc -= A B^T over K = 32: A rows ra.. (16 x 2 blocks), B rows rb.., both row-major stride PS
__device__ __forceinline__ void dag_gemm_sub(dx4 (&acc)[2][2], const double* A, int ra, const double* B, int rb, int lane) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int k = kk * 4 + lk;
    const double a0 = -A[(ra + lr) * PS + k], a1 = -A[(ra + 16 + lr) * PS + k];
    const double b0 = B[(rb + lr) * PS + k], b1 = B[(rb + 16 + lr) * PS + k];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
}
// X = P L^-T for 16 rows (r0..r0+15) of P (in `in`) into the same rows of `out` (may alias); columns >= kb zeroed
// (ragged last panel). One wave owns those rows of both buffers.
__device__ __forceinline__ void dag_trsm16(const double* in, double* out, const double* Li, int r0, int kb, int lane) {
  const int lr = lane & 15, lk = lane >> 4;
  dx4 x0 = {0.0, 0.0, 0.0, 0.0}, x1 = x0;
#pragma unroll
  for (int kk = 0; kk < NB / 4; ++kk) {
    const int k = kk * 4 + lk;
    const double a = in[(r0 + lr) * PS + k];
    x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Li[lr * PS + k], x0, 0, 0, 0);
    x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Li[(16 + lr) * PS + k], x1, 0, 0, 0);
  }
  lds_fence();  // this wave's reads of its rows are done before it overwrites them
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + lk + 4 * i;
    out[r * PS + lr] = lr < kb ? x0[i] : 0.0;
    out[r * PS + 16 + lr] = 16 + lr < kb ? x1[i] : 0.0;
  }
}
// slot of this workgroup holding tile (f, I, J), or -1
template <int TPW>
__device__ __forceinline__ int dag_slot(const int4 (&td)[TPW], int f, int I, int J) {
  int s = -1;
#pragma unroll
  for (int q = 0; q < TPW; ++q)
    if (td[q].x == f && td[q].y == I && td[q].z == J) s = q;
  return s;
}

template <int TPW>
__global__ void __launch_bounds__(256, 1) k_dag(const DagFront* __restrict__ frs, const int4* __restrict__ tiles,
                                                double* __restrict__ fronts, double* lbuf, double* __restrict__ vecs,
                                                double* ysol, double* linv, unsigned* flags, unsigned epoch, int* fail,
                                                unsigned* tmo) {
  __shared__ DagLds<TPW> S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int wr = (w & 1) * 32, wc = (w >> 1) * 32;
  int4 td[TPW];
  dx4 acc[TPW][2][2];
  int kmax = 0, li_tag = -1, yk_tag = -1;  // front * 65536 + panel whose L_kk^-1 / y_k S.Li / S.yk hold
  // Signals: a role's write-through stores are drained and its flag raised at once; with `defer` (measured slower, DESIGN
  // §5) the drain and flag wait until this workgroup is about to poll (it must never block while holding a signal: the
  // DAG stays deadlock-free) or until a second diagonal factor has run behind them. pD..pDe / pT: panels of pending
  // DIAG / TRSM signals of slot t, or -1.
  constexpr bool defer = false;
  int pD[TPW], pDe[TPW], pT[TPW];  // pending DIAG signals: panels pD .. pDe (a tile column's two panels)
#pragma unroll
  for (int t = 0; t < TPW; ++t) pD[t] = pDe[t] = pT[t] = -1;
  auto flush = [&]() {
    bool any = false;
#pragma unroll
    for (int t = 0; t < TPW; ++t) any |= pD[t] >= 0 || pT[t] >= 0;
    if (!any) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (tid == 0) {
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        if (pD[t] < 0 && pT[t] < 0) continue;
        const DagFront F = frs[td[t].x];
        for (int q = pD[t]; q >= 0 && q <= pDe[t]; ++q)
          __hip_atomic_store((gu32*)(flags + F.flag_off + q), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pT[t] >= 0)
          __hip_atomic_store((gu32*)(flags + F.flag_off + F.np + td[t].y * F.np + pT[t]), epoch, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t) pD[t] = pDe[t] = pT[t] = -1;
  };
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    td[t] = tiles[(size_t)blockIdx.x * TPW + t];
    if (td[t].x < 0) continue;
    const DagFront F = frs[td[t].x];
    kmax = max(kmax, F.np);
    const int I = td[t].y, J = td[t].z;
    const int ro = dag_off(F, I), rl = dag_len(F, I), co = dag_off(F, J), cl = dag_len(F, J);
    const double* Fp = fronts + F.f_off;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wr + 16 * x + lk + 4 * i, c = wc + 16 * y + lr;
          acc[t][x][y][i] = ld0(Fp, (co + c) * F.m + ro + r, r < rl && c < cl && (I != J || r >= c));
        }
    if (I == J && tid < TT) S.vacc[t][tid] = ld0(vecs + F.v_off, ro + tid, tid < rl);
  }
  __syncthreads();

  for (int k = 0; k < kmax; ++k) {
    const int k0 = NB * k, Jp = k0 >> 6, h = (k0 >> 5) & 1;
    // ---------------- DIAG
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (td[t].x < 0) continue;
      const DagFront F = frs[td[t].x];
      const int I = td[t].y, J = td[t].z;
      if (k >= F.np || J != Jp || I != J) continue;
      const int kb = min(NB, F.ns - k0), ro = dag_off(F, J), rl = dag_len(F, J);
      if (w == 3 * h) {  // quadrant (h, h), lower triangle, row-major into D
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 16 * x + lk + 4 * i, c = 16 * y + lr;
              if (r >= c) S.D[r * DS + c] = acc[t][x][y][i];
            }
      }
      if (tid < NB) S.vy[tid] = S.vacc[t][NB * h + tid];
      __syncthreads();
      if (tid < 64) factor_block(S.D, kb, S.vy, S.col, tid, fail, S.yk);
      __syncthreads();
      double* Lin = linv + (size_t)(F.c0 + k0) * (NB * NB);
#pragma unroll
      for (int u = 0; u < NB * NB / 256; ++u) {
        const int e = tid + 256 * u, i = e >> 5, c = e & (NB - 1);
        const double v = S.D[c * DS + i];  // L^-1(i, c), identity-padded past kb
        S.Li[i * PS + c] = v;
        st_wt(Lin + e, v);
      }
      li_tag = yk_tag = td[t].x * 65536 + k;
      if (tid < kb) st_wt(ysol + F.c0 + k0 + tid, S.yk[tid]);
      if (h == 0 && rl > NB) {
        // quadrant (1, 0): X1 = C10 L_kk^-T (wave 1 holds C10; waves 2 and 3 solve 16 rows each) -> Lout rows 32..
        double* X1 = S.Lout[t];
        if (w == 1) dag_stage(acc[t], S.Pa, PS, NB, lane);
        __syncthreads();
        if (w >= 2) dag_trsm16(S.Pa, X1, S.Li, NB + 16 * (w - 2), kb, lane);
        __syncthreads();
        double* Lf = lbuf + F.l_off;
#pragma unroll
        for (int u = 0; u < NB * NB / 256; ++u) {
          const int e = tid + 256 * u, r = e & (NB - 1), q = e >> 5;
          if (r < rl - NB && q < kb) st_wt(Lf + (size_t)(k0 + q) * F.m + ro + NB + r, X1[(NB + r) * PS + q]);
        }
        if (pD[t] < 0) pD[t] = k;
        pDe[t] = k;
        if (!defer) flush();
        // rows 32.. of the right-hand side, and quadrant (1, 1) of this tile, by panel k (the next panel's diagonal)
        if (tid < NB) {
          double s2 = 0.0;
#pragma unroll
          for (int q = 0; q < NB; ++q) s2 += X1[(NB + tid) * PS + q] * S.yk[q];
          S.vacc[t][NB + tid] -= s2;
        }
        if (w == 3) dag_gemm_sub(acc[t], X1, NB, X1, NB, lane);
        __syncthreads();
        if (k + 1 >= F.np) flush();
      } else {
        if (pD[t] < 0) pD[t] = k;
        pDe[t] = k;
        flush();  // the second factor of the tile column: its drain also covers the first's
      }
    }
    // ---------------- TRSM
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (td[t].x < 0) continue;
      const DagFront F = frs[td[t].x];
      const int I = td[t].y, J = td[t].z;
      if (k >= F.np || J != Jp || I == J) continue;
      const int kb = min(NB, F.ns - k0), ro = dag_off(F, I), rl = dag_len(F, I);
      const int sd = dag_slot(td, td[t].x, Jp, Jp);  // this workgroup factored panel k itself
      const bool li_here = li_tag == td[t].x * 65536 + k;
      if ((w >> 1) == h) dag_stage(acc[t], S.Pa, PS, wr, lane);  // this tile's half-h columns (its panel k)
      if (li_here && yk_tag == li_tag && (sd >= 0 || h == 1)) {
        __syncthreads();
      } else {
        flush();
        dag_wait(flags + F.flag_off + k, nullptr, epoch, tmo, fail);
        const double* Lin = linv + (size_t)(F.c0 + k0) * (NB * NB);
        const double* Lf = lbuf + F.l_off;
        const int dro = dag_off(F, Jp) + NB, drl = dag_len(F, Jp) - NB;  // diagonal tile's quadrant-(1, 0) rows (h = 0)
        double lv[NB * NB / 256], xv[NB * NB / 256];
#pragma unroll
        for (int u = 0; u < NB * NB / 256; ++u) {
          const int e = tid + 256 * u, r = e & (NB - 1), q = e >> 5;
          lv[u] = ld_wt0(Lin, e, !li_here);
          xv[u] = ld_wt0(Lf, (long long)(k0 + q) * F.m + dro + r, h == 0 && sd < 0 && r < drl && q < kb);
        }
        const double yv = ld_wt0(ysol, F.c0 + k0 + tid, tid < kb);  // y_k rides with L_kk^-1 (the diagonal update)
#pragma unroll
        for (int u = 0; u < NB * NB / 256; ++u) {
          const int e = tid + 256 * u, r = e & (NB - 1), q = e >> 5;
          if (!li_here) S.Li[(e >> 5) * PS + (e & (NB - 1))] = lv[u];
          S.Pb[(NB + r) * PS + q] = xv[u];
        }
        if (tid < NB) S.yk[tid] = yv;
        li_tag = yk_tag = td[t].x * 65536 + k;
        __syncthreads();
      }
      double* X = S.Lout[t];
      dag_trsm16(S.Pa, X, S.Li, 16 * w, kb, lane);
      __syncthreads();
      double* Lw = lbuf + F.l_off;
#pragma unroll
      for (int u = 0; u < TT * NB / 256; ++u) {
        const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
        if (r < rl && q < kb) st_wt(Lw + (size_t)(k0 + q) * F.m + ro + r, X[r * PS + q]);
      }
      pT[t] = k;
      if (!defer) flush();
      if (h == 0 && (w >> 1) == 1)  // the other half: -= L_Ik X1^T
        dag_gemm_sub(acc[t], X, wr, sd >= 0 ? S.Lout[sd] : S.Pb, NB, lane);
      __syncthreads();
    }
    // ---------------- UPDATE
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      if (td[t].x < 0) continue;
      const DagFront F = frs[td[t].x];
      const int I = td[t].y, J = td[t].z;
      if (k >= F.np || J <= Jp) continue;
      const int kb = min(NB, F.ns - k0);
      const int roI = dag_off(F, I), rlI = dag_len(F, I), roJ = dag_off(F, J), rlJ = dag_len(F, J);
      const int sI = dag_slot(td, td[t].x, I, Jp), sJ = I == J ? sI : dag_slot(td, td[t].x, J, Jp);
      unsigned* pf = flags + F.flag_off + F.np;
      const bool remote = sI < 0 || (sJ < 0 && I != J);
      const bool yk_here = yk_tag == td[t].x * 65536 + k;
      if (remote) {
        flush();
        dag_wait(sI < 0 ? pf + I * F.np + k : nullptr, sJ < 0 ? pf + J * F.np + k : nullptr, epoch, tmo, fail);
      }
      const double* Lf = lbuf + F.l_off;
      double av[TT * NB / 256], bv[TT * NB / 256];
#pragma unroll
      for (int u = 0; u < TT * NB / 256; ++u) {
        const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
        av[u] = ld_wt0(Lf, (long long)(k0 + q) * F.m + roI + r, sI < 0 && r < rlI && q < kb);
        bv[u] = ld_wt0(Lf, (long long)(k0 + q) * F.m + roJ + r, sJ < 0 && I != J && r < rlJ && q < kb);
      }
      // y_k: from the TRSM / DIAG of this panel on this workgroup, else loaded (published before any flag this
      // tile's operands depend on; a diagonal tile with local operands always has it here)
      const bool yload = I == J && !yk_here;
      const double ykv = ld_wt0(ysol, F.c0 + k0 + tid, yload && tid < kb);
      if (remote) {
#pragma unroll
        for (int u = 0; u < TT * NB / 256; ++u) {
          const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
          if (sI < 0) S.Pa[r * PS + q] = av[u];
          if (sJ < 0 && I != J) S.Pb[r * PS + q] = bv[u];
        }
      }
      if (yload) {
        if (tid < NB) S.yk[tid] = ykv;
        yk_tag = td[t].x * 65536 + k;
      }
      __syncthreads();
      const double* A = sI >= 0 ? S.Lout[sI] : S.Pa;
      const double* B = I == J ? A : (sJ >= 0 ? S.Lout[sJ] : S.Pb);
      if (I == J && tid < TT) {
        double s2 = 0.0;
#pragma unroll
        for (int q = 0; q < NB; ++q) s2 += A[tid * PS + q] * S.yk[q];
        S.vacc[t][tid] -= s2;
      }
      dag_gemm_sub(acc[t], A, wr, B, wc, lane);
      __syncthreads();
    }
    bool dcont = false;  // a diagonal tile factors its second panel next: keep that signal behind its factor
#pragma unroll
    for (int t = 0; t < TPW; ++t) dcont |= pD[t] >= 0;
    if (!dcont) flush();
  }
  flush();
  // ---------------- contribution block and update vector (read by the parent's assembly in the next launch)
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    if (td[t].x < 0) continue;
    const DagFront F = frs[td[t].x];
    const int I = td[t].y, J = td[t].z;
    if (J < F.nown) continue;
    const int ro = dag_off(F, I), rl = dag_len(F, I), co = dag_off(F, J), cl = dag_len(F, J);
    double* Fp = fronts + F.f_off;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wr + 16 * x + lk + 4 * i, c = wc + 16 * y + lr;
          if (r < rl && c < cl && (I != J || r >= c)) Fp[(size_t)(co + c) * F.m + ro + r] = acc[t][x][y][i];
        }
    if (I == J && tid < rl) vecs[F.v_off + ro + tid] = S.vacc[t][tid];
  }
}

// Backward solve of a k_dag front (no explicit X = L11^-1), right-looking: t (= y - L21^T x_rows from k_bwd_gemv) is
// reduced in LDS; from the last block, x_b = L_bb^-T t_b, then t_c -= sum_r L(b0 + r, c) x_b[r] for every column c < b0
// (row block b of L11, 4 threads per column). The sequential chain per block is one 32 x 32 product and one update
// pass over registers; block b-1's rows of L and its L^-1 are loaded while block b is solved.
constexpr int BSQ_C = 6;                 // column passes of 64: ns <= 64 * BSQ_C + 32
constexpr int BSQ_N = 64 * BSQ_C + NB;   // largest ns
__global__ void __launch_bounds__(256) k_bwd_seq(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                                 const double* __restrict__ lbuf, const double* __restrict__ linv,
                                                 const double* __restrict__ tsol, double* __restrict__ xsol,
                                                 const int* __restrict__ perm, double* __restrict__ xout) {
  __shared__ double ts[BSQ_N];
  __shared__ double Lis[2][NB * (NB + 1)];
  __shared__ double xb[NB];
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, ns = me.ns;
  const int tid = threadIdx.x, cq = tid >> 2, rq = tid & 3;
  const double* L = lbuf + me.l_off;
  const int np = (ns + NB - 1) / NB;
  double cur[BSQ_C][8], nxt[BSQ_C][8], li[NB * NB / 256];
  auto load_rows = [&](int b, double (&dst)[BSQ_C][8], double (&lv)[NB * NB / 256]) {
    const int b0 = NB * b;
#pragma unroll
    for (int p = 0; p < BSQ_C; ++p)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int c = 64 * p + cq, i = b0 + 8 * rq + r;
        dst[p][r] = ld0(L, c * m + i, c < b0 && i < ns);
      }
    const double* Li = linv + (size_t)(me.c0 + b0) * (NB * NB);
#pragma unroll
    for (int u = 0; u < NB * NB / 256; ++u) lv[u] = Li[tid + 256 * u];
  };
  for (int i = tid; i < ns; i += 256) ts[i] = tsol[me.c0 + i];
  load_rows(np - 1, cur, li);
  int cb = 0;
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = tid + 256 * u;
    Lis[0][(e >> 5) * (NB + 1) + (e & (NB - 1))] = li[u];
  }
  __syncthreads();
  for (int b = np - 1; b >= 0; --b) {
    const int b0 = NB * b, kb = min(NB, ns - b0);
    if (b > 0) load_rows(b - 1, nxt, li);
    if (tid < NB) {  // x_b = L_bb^-T t_b: x[j] = sum_i L^-1(i, j) t[i]
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int i = 0; i < NB; ++i) a4[i & 3] += (i < kb ? Lis[cb][i * (NB + 1) + tid] * ts[b0 + min(i, kb - 1)] : 0.0);
      const double x = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      xb[tid] = tid < kb ? x : 0.0;
      if (tid < kb) {
        xsol[me.c0 + b0 + tid] = x;
        xout[perm[me.c0 + b0 + tid]] = x;
      }
    }
    __syncthreads();
    if (b > 0) {
#pragma unroll
      for (int p = 0; p < BSQ_C; ++p) {
        const int c = 64 * p + cq;
        double part = 0.0;
#pragma unroll
        for (int r = 0; r < 8; ++r) part += cur[p][r] * xb[8 * rq + r];
        part += __shfl_xor(part, 1, 64);
        part += __shfl_xor(part, 2, 64);
        if (rq == 0 && c < b0) ts[c] -= part;
      }
      cb ^= 1;
#pragma unroll
      for (int u = 0; u < NB * NB / 256; ++u) {
        const int e = tid + 256 * u;
        Lis[cb][(e >> 5) * (NB + 1) + (e & (NB - 1))] = li[u];
      }
#pragma unroll
      for (int p = 0; p < BSQ_C; ++p)
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[p][r] = nxt[p][r];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------- distributed factorization glue
// (landmark-sharded BA) contiguous copies between the front pool / front vectors and an exchange buffer:
// ranges (src, dst, len) in doubles, one workgroup per range
__global__ void __launch_bounds__(256) k_copy_ranges(const long long* __restrict__ rng, const double* __restrict__ src,
                                                     double* __restrict__ dst) {
  const long long so = rng[3 * blockIdx.x], d0 = rng[3 * blockIdx.x + 1], len = rng[3 * blockIdx.x + 2];
  for (long long i = threadIdx.x; i < len; i += 256) dst[d0 + i] = src[so + i];
}
__global__ void __launch_bounds__(256) k_pack_blocks(long long n, int bb, const long long* __restrict__ boff,
                                                     const double* __restrict__ src, double* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long t = i / bb;
  dst[boff[t] + (i - t * bb)] = src[i];
}
// x of the distributed solve: every rank holds its own columns (and rank 0 the shared ones) in xr[0 .. n), zeros
// elsewhere, the not-PD flag of its fronts in xr[n]; after the all-reduce: x = xr, fail |= xr[n] > 0
__global__ void k_dist_fail_in(const int* __restrict__ fail, double* __restrict__ xr, int n) {
  if (threadIdx.x == 0) xr[n] = *fail ? 1.0 : 0.0;
}
__global__ void __launch_bounds__(256) k_dist_x_out(const double* __restrict__ xr, int n, double* __restrict__ x,
                                                    int* __restrict__ fail) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k < n) x[k] = xr[k];
  if (k == 0 && xr[n] > 0.0) *fail = 1;
}
__global__ void __launch_bounds__(256) k_zero_idx(const int* __restrict__ idx, int n, double* __restrict__ x) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k < n) x[idx[k]] = 0.0;
}

namespace launch {

// one workgroup per CU (the validated form of the write-through hand-offs): dynamic LDS tops each instance up to more
// than half of the CU's 160 KB
template <int TPW>
static int dag_reserve() {
  static int r = -1;
  if (r < 0) {
    hipFuncAttributes a;
    HIP_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_dag<TPW>)));
    r = std::max(0, 82 * 1024 - (int)a.sharedSizeBytes);
  }
  return r;
}
void chol_dag(int nworkers, int tpw, const DagFront* fr, const int4* tiles, double* fronts, double* lbuf, double* vecs,
              double* ysol, double* linv, unsigned* flags, unsigned epoch, int* fail, unsigned* tmo, hipStream_t s) {
  if (nworkers <= 0) return;
  if (tpw == 2)
    hipLaunchKernelGGL(k_dag<2>, nworkers, 256, dag_reserve<2>(), s, fr, tiles, fronts, lbuf, vecs, ysol, linv, flags, epoch, fail, tmo);
  else
    hipLaunchKernelGGL(k_dag<4>, nworkers, 256, dag_reserve<4>(), s, fr, tiles, fronts, lbuf, vecs, ysol, linv, flags, epoch, fail, tmo);
  KERNEL_CHECK();
}
int chol_dag_max_workers(int device) {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, device));
  // every worker must be resident at once (they wait on each other): one 256-thread workgroup per CU fits when its
  // LDS (static + the dynamic top-up) is within the CU's and its registers within a SIMD's budget for one wave each.
  // (hipOccupancyMaxActiveBlocksPerMultiprocessor returned "unknown error" for these kernels on the MI355X boxes)
  hipFuncAttributes a2, a4;
  HIP_CHECK(hipFuncGetAttributes(&a2, reinterpret_cast<const void*>(&k_dag<2>)));
  HIP_CHECK(hipFuncGetAttributes(&a4, reinterpret_cast<const void*>(&k_dag<4>)));
  const bool fit = (int)a2.sharedSizeBytes + dag_reserve<2>() <= 160 * 1024 &&
                   (int)a4.sharedSizeBytes + dag_reserve<4>() <= 160 * 1024 && a2.numRegs <= 512 && a4.numRegs <= 512 &&
                   a2.maxThreadsPerBlock >= 256 && a4.maxThreadsPerBlock >= 256;
  return fit ? p.multiProcessorCount : 0;
}
void chol_bwd_seq(int ntasks, const Task* tasks, const FrontDesc* fd, const double* lbuf, const double* linv,
                  const double* tsol, double* xsol, const int* perm, double* xout, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_bwd_seq, ntasks, 256, 0, s, tasks, fd, lbuf, linv, tsol, xsol, perm, xout);
  KERNEL_CHECK();
}

void chol_copy_ranges(int n, const long long* rng, const double* src, double* dst, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy_ranges, n, 256, 0, s, rng, src, dst);
  KERNEL_CHECK();
}
void chol_pack_blocks(long long nblk, int bb, const long long* boff, const double* src, double* dst, hipStream_t s) {
  const long long n = nblk * bb;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_pack_blocks, (unsigned)((n + 255) / 256), 256, 0, s, n, bb, boff, src, dst);
  KERNEL_CHECK();
}
void chol_dist_fail_in(const int* fail, double* xr, int n, hipStream_t s) {
  hipLaunchKernelGGL(k_dist_fail_in, 1, 64, 0, s, fail, xr, n);
  KERNEL_CHECK();
}
void chol_dist_x_out(const double* xr, int n, double* x, int* fail, hipStream_t s) {
  hipLaunchKernelGGL(k_dist_x_out, grid_for(std::max(n, 1), 256), 256, 0, s, xr, n, x, fail);
  KERNEL_CHECK();
}
void chol_zero_idx(const int* idx, int n, double* x, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_zero_idx, grid_for(n, 256), 256, 0, s, idx, n, x);
  KERNEL_CHECK();
}

int debug_phases(unsigned long long* out, int maxrec) {
#ifdef G2OHIP_PHASES
  unsigned n = 0;
  HIP_CHECK(hipDeviceSynchronize());
  HIP_CHECK(hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_phase_n), sizeof n));
  const int cnt = (int)std::min<unsigned>(n, 4096u);
  const int k = std::min(cnt, maxrec);
  if (out && k > 0) HIP_CHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 8 * k));
  const unsigned z = 0;
  HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_n), &z, sizeof z));
  return k;
#else
  (void)out; (void)maxrec;
  return 0;
#endif
}

void chol_prescatter(int nzero, const long long* zr, long long nent, const double* vals, const long long* dst,
                     const int* src, const double* lam, double* fronts, int nfronts, const FrontDesc* fd,
                     const int* perm, const double* rhs, double* vecs, hipStream_t s) {
  if (nzero > 0) {
    hipLaunchKernelGGL(k_zero_ranges, nzero, 256, 0, s, zr, fronts);
    KERNEL_CHECK();
  }
  if (nent > 0) {
    const int nsb = grid_for(nent, 256);
    hipLaunchKernelGGL(k_chol_scatter, nsb + std::max(nfronts, 0), 256, 0, s, nent, nsb, vals, dst, src, lam, fronts,
                       fd, perm, rhs, vecs);
    KERNEL_CHECK();
  } else if (nfronts > 0) {
    hipLaunchKernelGGL(k_vec_init, nfronts, 256, 0, s, fd, perm, rhs, vecs);
    KERNEL_CHECK();
  }
}
void chol_extend_add(int ntasks, const Task* tasks, const FrontDesc* fd, const int* children, const int* relmap,
                     const int* jtab, const int* cmptr, const int2* cment, const int* colptr, const int* ent_row, const int* ent_src, const double* vals, const double* lam,
                     double* fronts, double* vecs, double* lbuf, double* ysol, double* linv, double* linvn, double* xinv,
                     int* fail, int assemble, bool w64, hipStream_t s) {
  if (ntasks <= 0) return;
#define G2OHIP_EA(A_, E_, W_)                                                                                        \
  hipLaunchKernelGGL((k_extend_add<A_, E_, W_>), ntasks, 256, 0, s, tasks, fd, children, relmap, jtab, cmptr, cment, \
                     colptr, ent_row, ent_src, vals, lam, fronts, vecs, lbuf, ysol, linv, linvn, xinv, fail)
  // assemble 2: fronts up to 512 rows (a small column buffer keeps more workgroups per CU)
  if (assemble == 2) { if (w64) G2OHIP_EA(true, 512, true); else G2OHIP_EA(true, 512, false); }
  else if (assemble) { if (w64) G2OHIP_EA(true, 2048, true); else G2OHIP_EA(true, 2048, false); }
  else { if (w64) G2OHIP_EA(false, 1, true); else G2OHIP_EA(false, 1, false); }
#undef G2OHIP_EA
  KERNEL_CHECK();
}
void chol_step(int ntasks, const StepTask* tasks, const StepHead& head, double* fronts, double* lbuf, double* vecs,
               double* ysol, double* linv, double* xinv, int* fail, bool pairs, hipStream_t s) {
  if (ntasks <= 0) return;
  if (pairs)
    hipLaunchKernelGGL(k_step<true>, ntasks, 256, 0, s, tasks, head, fronts, lbuf, vecs, ysol, linv, xinv, fail);
  else
    hipLaunchKernelGGL(k_step<false>, ntasks, 256, 0, s, tasks, head, fronts, lbuf, vecs, ysol, linv, xinv, fail);
  KERNEL_CHECK();
}
void chol_step64(int ntasks, const StepTask* tasks, const StepHead& head, double* fronts, double* lbuf, double* vecs,
                 double* ysol, double* linv, double* linvn, double* xinv, int* fail, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_step64, ntasks, 256, 0, s, tasks, head, fronts, lbuf, vecs, ysol, linv, linvn, xinv, fail);
  KERNEL_CHECK();
}
void chol_syrk(int ntasks, const Task* tasks, const FrontDesc* fd, double* fronts, const double* lbuf, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_syrk, ntasks, 256, 0, s, tasks, fd, fronts, lbuf);
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
void chol_bwd_gemv(int ntasks, const Task* tasks, const FrontDesc* fd, const int* rows, const double* lbuf,
                   const double* ysol, const double* xsol, double* tsol, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_bwd_gemv, ntasks, 256, 0, s, tasks, fd, rows, lbuf, ysol, xsol, tsol);
  KERNEL_CHECK();
}
void chol_bwd_inner(int ntasks, const Task* tasks, const FrontDesc* fd, const double* lbuf, const double* xsol, double* tsol,
                    hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_bwd_inner, ntasks, 256, 0, s, tasks, fd, lbuf, xsol, tsol);
  KERNEL_CHECK();
}
void chol_bwd_x(int ntasks, const Task* tasks, const FrontDesc* fd, const double* xinv, const double* tsol, double* xsol,
                const int* perm, double* xout, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_bwd_x, ntasks, 256, 0, s, tasks, fd, xinv, tsol, xsol, perm, xout);
  KERNEL_CHECK();
}

}  // namespace launch
}  // namespace g2ohip
