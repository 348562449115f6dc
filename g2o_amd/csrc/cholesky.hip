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

using launch::B0Child;
using launch::B0Front;
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
// The block's forward solve is not in this loop (factor_block multiplies by L^-1 afterwards). Entries
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
// (D[c * DS + i] = L^-1(i, c)) for the block's forward solve below, and (linv_out) stored row-major straight from the
// registers: row i of the 32 x 32 block is one coalesced 256-byte store of lanes 32..63, so the caller publishes it
// without a barrier or an LDS pass (r04; X's diagonal blocks, the same values column-major, are copied by k_xdiag
// after the factorization). The diagonal block of L itself is not stored: every consumer of the factor (tile TRSM,
// next-diagonal update, inverse tasks, backward and multi-right-hand-side solves) uses L^-1 for diagonal blocks.
__device__ __forceinline__ void factor_block(double* D, int kb, const double* vy, double* col, int lane, int* fail,
                                             double* ysol, unsigned long long* ph = nullptr, double* ylds = nullptr,
                                             double* linv_out = nullptr) {
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
    if (linv_out) {
#pragma unroll
      for (int i = 0; i < NB; ++i) linv_out[i * NB + (lane - NB)] = row[i];  // L^-1(i, lane - NB), identity-padded
    }
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
template <bool ASM, int EAC>
__global__ void __launch_bounds__(256) k_extend_add(const Task* __restrict__ tasks, const B0Front* __restrict__ b0f,
                                                    const B0Child* __restrict__ b0c, const FrontDesc* __restrict__ fd,
                                                    const int* __restrict__ children, const int* __restrict__ relmap,
                                                    const int* __restrict__ jtab, const int* __restrict__ cmptr,
                                                    const longlong2* __restrict__ cment, const int* __restrict__ colptr, const int* __restrict__ ent_row,
                                                    const int* __restrict__ ent_src, const double* __restrict__ vals,
                                                    const double* __restrict__ lam, double* __restrict__ fronts,
                                                    double* __restrict__ vecs, double* __restrict__ lbuf,
                                                    double* __restrict__ ysol, double* __restrict__ linv,
                                                    double* __restrict__ xinv, int* __restrict__ fail,
                                                    const launch::ScatterJob sj) {
  // a block-0 task's front: the head's by value (clamped index, read with ntask before the scatter branch), past
  // EA_HEAD from b0f
  B0Front bf = sj.b0[min((int)blockIdx.x, launch::EA_HEAD - 1)];
  asm volatile("" ::"s"(bf.front_off), "s"(bf.ce));  // (both halves: the compiler sinks loads used past the branch)
  if ((int)blockIdx.x >= sj.ntask) {  // deferred input scatter of a later level (the launch's chip is mostly idle)
    const long long k = sj.sc0 + (long long)((int)blockIdx.x - sj.ntask) * 256 + threadIdx.x;
    if (k < sj.sc1) {
      const int sr = sj.src[k];
      const double v = vals[sr & 0x7fffffff];
      fronts[sj.dst[k]] = sr < 0 ? v + *lam : v;
    }
    return;
  }
  const int tid = threadIdx.x;
  if ((int)blockIdx.x < sj.nb0) {
    if ((int)blockIdx.x >= launch::EA_HEAD) bf = b0f[blockIdx.x];
    const int m = bf.m, kb0 = bf.kb0;
    double* F = fronts + bf.front_off;
    double* v = vecs + bf.vec_off;
    __shared__ double D[NB * DS];
    __shared__ __attribute__((aligned(16))) double col[4 * NB];  // two 64-lane column buffers
    __shared__ double vy[NB];
    PH_BEGIN(1)
    if constexpr (!ASM) {
      // every store unconditional (zeros outside the block's lower triangle, v past 32 into col's scratch): a
      // predicated store kept its load in the same branch, one dependent round trip per load
      double x[NB * NB / 256];
#pragma unroll
      for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
        const int e = tid + 256 * u_;
        const int r = e & (NB - 1), c = e >> 5;
        x[u_] = ld0(F, c * m + r, r < kb0 && c < kb0 && r >= c);
      }
      const double yv = ld0(v, tid, tid < kb0);
#pragma unroll
      for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
        const int e = tid + 256 * u_;
        D[(e & (NB - 1)) * DS + (e >> 5)] = x[u_];
      }
      *(tid < NB ? &vy[tid] : &col[tid & (4 * NB - 1)]) = yv;
    } else {
      __shared__ int cp[NB + 1];
      for (int i = tid; i < NB * DS; i += 256) D[i] = 0.0;
      if (tid <= kb0) cp[tid] = colptr[bf.c0 + tid];
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
    // children in groups of B0C: every load of a group (records, rel, update entries) is issued before the
    // first add, so a group costs two dependent round trips instead of two per child; the adds then run
    // child by child in the fixed order (bitwise reproducible)
    constexpr int B0C = 4;
    for (int kc = bf.cb; kc < bf.ce; kc += B0C) {
      double val[B0C][NB * NB / 256], vv[B0C];
      int dst[B0C][NB * NB / 256], vdst[B0C];
      B0Child cds[B0C];
#pragma unroll
      for (int c = 0; c < B0C; ++c) cds[c] = b0c[kc + c < bf.ce ? kc + c : kc];
      // the group's records in one round trip (left to itself the compiler interleaved them with the data loads)
      asm volatile("" ::"s"(cds[0].u_off), "s"(cds[1].u_off), "s"(cds[2].u_off), "s"(cds[3].u_off));
      // the update entries first, then the row maps: the destinations computed from the maps then wait for the
      // last loads only (computed in the same loop, they made the compiler wait for the maps before the entries)
      int ri[B0C], rj[B0C][NB * NB / 256], rt[B0C];
#pragma unroll
      for (int c = 0; c < B0C; ++c) {
        const B0Child& cd = cds[c];
#pragma unroll
        for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
          const int e = tid + 256 * u_;
          const int i = e & (NB - 1), j = e >> 5;
          val[c][u_] = ld0(fronts + cd.u_off, j * cd.mc + i, i < cd.nrc && j <= i);
        }
        vv[c] = ld0(vecs + cd.vv_off, tid, tid < cd.nrc && tid < NB);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < B0C; ++c) {
        const B0Child& cd = cds[c];
        const int* rel = relmap + cd.rel_off;
        const int i = tid & (NB - 1);  // (the row of every entry of this thread)
        ri[c] = ld0(rel, i, i < cd.nrc);
#pragma unroll
        for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
          const int j = (tid + 256 * u_) >> 5;
          rj[c][u_] = ld0(rel, j, i < cd.nrc && j <= i);
        }
        rt[c] = ld0(rel, tid, tid < cd.nrc && tid < NB);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < B0C; ++c) {
        const B0Child& cd = cds[c];
        const int n0 = kc + c < bf.ce ? cd.n0 : 0;  // child rows mapping into the block (rel is increasing)
        const int i = tid & (NB - 1);
#pragma unroll
        for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
          const int j = (tid + 256 * u_) >> 5;
          dst[c][u_] = (i < cd.nrc && j <= i && i < n0) ? ri[c] * DS + rj[c][u_] : -1;
        }
        vdst[c] = tid < n0 ? rt[c] : -1;
      }
#pragma unroll
      for (int c = 0; c < B0C; ++c) {
        if (kc + c >= bf.ce) break;
#pragma unroll
        for (int u_ = 0; u_ < NB * NB / 256; ++u_) *(dst[c][u_] >= 0 ? &D[dst[c][u_]] : &col[tid & (4 * NB - 1)]) += val[c][u_];
        // unconditional adds (entries outside the block go into col's scratch, unused until the factor): a
        // predicated add had the compiler sink the entry's load into its branch, a dependent round trip each
        *(vdst[c] >= 0 ? &vy[vdst[c]] : &col[tid & (4 * NB - 1)]) += vv[c];
        __syncthreads();
      }
    }
    PH(2)
    // L_00^-1 straight from wave 0's registers to linv (X's diagonal blocks: k_xdiag after the factorization)
    if (tid < 64) factor_block(D, kb0, vy, col, tid, fail, ysol + bf.c0, PH_REC, nullptr, linv + (size_t)bf.c0 * (NB * NB));
    PH(3)
    PH(4)
    return;
  }
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, kb0 = min(NB, me.ns);
  double* F = fronts + me.front_off;
  double* v = vecs + me.vec_off;
  const int a = t.a, b = t.b;
  const int lane = tid & 63, w = tid >> 6;
  if constexpr (ASM) {
    // In-place assembly: each wave builds its columns in an LDS column buffer (zero, the column's input
    // entries, then every (child, child column) pair mapping to it in child order) and writes each entry
    // of the front once; rows in chunks of EAC. The children's update vectors follow below.
    __shared__ double cbuf[4][EAC];
    // per column its pair range (cmptr), input-entry range (colptr) and first pair record, loaded one column ahead
    // (cment ends with a sentinel record, so cment[q0] is valid for an empty range)
    struct ColMeta { int q0, q1, e0, e1; longlong2 f; };
    auto meta = [&](int jj) {
      ColMeta c;
      c.q0 = cmptr[me.cm_off + jj];
      c.q1 = cmptr[me.cm_off + jj + 1];
      const bool inp = jj < me.ns;
      c.e0 = inp ? colptr[me.c0 + jj] : 0;
      c.e1 = inp ? colptr[me.c0 + jj + 1] : 0;
      c.f = cment[c.q0];
      return c;
    };
    ColMeta cur = a + w < b ? meta(a + w) : ColMeta{0, 0, 0, 0, longlong2{0, 0}};
    for (int j = a + w; j < b; j += 4) {
      const ColMeta nxt = j + 4 < b ? meta(j + 4) : cur;
      const int rlo = j < kb0 ? kb0 : j;  // rows of the first diagonal block: block-0 task
      double* Fj = F + (size_t)j * m;
      const int q0 = cur.q0, q1 = cur.q1;
      for (int rc = rlo; rc < m; rc += EAC) {
        const int rce = min(m, rc + EAC);
        double* cb = cbuf[w] - rc;
        for (int i = rc + lane; i < rce; i += 64) cb[i] = 0.0;
        for (int e = cur.e0 + lane; e < cur.e1; e += 64) {
          int r;
          const double x = input_entry(vals, ent_src, ent_row, e, lam, r);
          if (r >= rc && r < rce) cb[r] = x;
        }
        // one 16-byte record per pair (no dependent descriptor read), the next pair's record in flight while this
        // pair's rows are added; a child's rows map to increasing parent rows, so a batch that starts past the chunk
        // ends the pair
        longlong2 nx = cur.f;
        for (int q = q0; q < q1; ++q) {
          const longlong2 ce = nx;
          if (q + 1 < q1) nx = cment[q + 1];
          const double* Uj = fronts + ce.x;
          const int* rel = relmap + (int)(ce.y & 0x7fffffff);
          const int y = (int)((ce.y >> 32) & 0xffff), nrc = (int)(ce.y >> 48);
          for (int i0 = y + lane; i0 < nrc; i0 += 256) {
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
            if (__builtin_amdgcn_readfirstlane(ri[0]) >= rce) break;  // lane 0 holds the batch's first (smallest) row
          }
        }
        for (int i = rc + lane; i < rce; i += 64) Fj[i] = cb[i];
      }
      cur = nxt;
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
  // 2. children in fixed order, from their block-0 records (the next child's read while this one is added). Every
  // read-modify-write batch reads all its old values (and the entries) before its first store: the rows of one batch
  // are distinct, but the compiler cannot know it and kept each store's load behind the previous store, and it sank
  // the loads of predicated adds into their branches — a dependent round trip per entry (the pins below)
  B0Child nx = b0c[me.child_begin < me.child_end ? me.child_begin : 0];
  for (int k = me.child_begin; k < me.child_end; ++k) {
    const B0Child cd = nx;
    if (k + 1 < me.child_end) nx = b0c[k + 1];
    const int mc = cd.mc, nrc = cd.nrc;
    const double* U = fronts + cd.u_off;  // U(i,j) = U[j*mc + i]
    const double* u = vecs + cd.vv_off;
    const int* rel = relmap + cd.rel_off;
    // child columns whose parent column lies in [a, b) (rel is increasing; precomputed per slab)
    const int j0 = jtab[cd.jt_off + t.c - 1], j1 = jtab[cd.jt_off + t.c];
    for (int j = j0 + tid; j < j1; j += 256) {
      const int rr = rel[j];
      const double uu = u[j];
      const double vo = v[rr >= kb0 ? rr : 0];
      asm volatile("" ::"v"(uu), "v"(vo));
      if (rr >= kb0) v[rr] = vo + uu;
    }
    // lower triangle: one wave per child column, lanes run down the rows (coalesced U reads,
    // mostly-contiguous F writes), 4 entries per lane and batch
    for (int j = j0 + w; j < j1; j += 4) {
      const double* Uj = U + (size_t)j * mc;
      int rj = 0;  // the parent column, rel[j]: lane 0's first row map of the first batch (i = j), no load of its own
      for (int i0 = j + lane; i0 < nrc; i0 += 256) {
        double val[4], old[4];
        int ri[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = i0 + q * 64;
          const bool ok = i < nrc;
          val[q] = Uj[ok ? i : 0];
          ri[q] = rel[ok ? i : 0];
        }
        __builtin_amdgcn_sched_barrier(0);  // the batch's entries and row maps all in flight before the first wait
#pragma unroll
        for (int q = 0; q < 4; ++q) ri[q] = i0 + q * 64 < nrc ? ri[q] : -1;
        if (i0 == j + lane) rj = __builtin_amdgcn_readfirstlane(ri[0]);
        double* Fj = F + (size_t)rj * m;
        const int rlo = rj < kb0 ? kb0 : 0;  // rows of the first diagonal block: block-0 task
#pragma unroll
        for (int q = 0; q < 4; ++q) old[q] = Fj[ri[q] >= rlo ? ri[q] : rj];  // (Fj[rj]: a valid address)
        asm volatile("" ::"v"(val[0]), "v"(val[1]), "v"(val[2]), "v"(val[3]), "v"(old[0]), "v"(old[1]), "v"(old[2]),
                     "v"(old[3]));
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (ri[q] >= rlo) Fj[ri[q]] = old[q] + val[q];
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
__device__ __forceinline__ void load_ctile(const double* F, int m, int rlim, int I0, int J0, int climit, int tid,
                                           double (&cv)[16]) {
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int idx = tid + 256 * u, r = idx & (TT - 1), c = idx >> 6;
    const int gi = I0 + r, gj = J0 + c;
    cv[u] = ld0(F, gj * m + gi, gi < rlim && gj < climit && gi >= gj);
  }
}

// Task flags: 1 update the tile (else TRSM + L21 store only), 4 the step's next-diagonal task,
// 8 the tile may reach into the contribution block (columns >= ns: no separate k_syrk pass),
// 16 an inverse task: block (tj, ti) of X = L11^-1 (see below),
// 64 lagged pair (odd steps of a lagged front, DeviceCholesky::setup): the update also applies the PREVIOUS
//    panel (k0 - 32, whose L rows the strip tiles of the even step stored), so the trailing columns are read and
//    written once per two panels (rank-64); the even steps update only the next panel's strip (clim = r0 + kbn).
// 128 own rows only (deferred L21, DeviceCholesky::setup): the tile's rows stop at ns; L21 and the front vector's
//    rows below come from k_l21 and the contribution pass.
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
  // the task: the chain's tasks ride in the kernel arguments, the rest in a global list; both read with scalar loads
  // (the kernel-argument one at a clamped index, then replaced by VALUE): a select of the two POINTERS made the compiler
  // fetch the task with a flat vector load, a full memory round trip on every step's chain before the first data load
  // could issue. The kernel-argument task is read with ntask, before the scatter branch: read after it, the two were
  // dependent scalar round trips (plus a third for head.n; a task index below ntask is in the head iff < CHOL_HEAD)
  StepTask t = head.t[min((int)blockIdx.x, launch::CHOL_HEAD - 1)];
  asm volatile("" ::"s"(t.m), "s"(t.f_off));  // (both halves: the compiler sinks loads used past the branch)
  if ((int)blockIdx.x >= head.ntask) {  // deferred input scatter of a later level (off this step's chain)
    const long long k = head.sc0 + (long long)((int)blockIdx.x - head.ntask) * 256 + threadIdx.x;
    if (k < head.sc1) {
      const int sr = head.sc_src[k];
      const double v = head.sc_vals[sr & 0x7fffffff];
      fronts[head.sc_dst[k]] = sr < 0 ? v + *head.sc_lam : v;
    }
    return;
  }
  PH_BEGIN(2)
  PH1_BEGIN(3)
  if ((int)blockIdx.x >= launch::CHOL_HEAD) t = tasks[blockIdx.x];  // (the chain's tasks wait for no global load)
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
    // the loads at selected addresses (index 0 when masked: ld0 split in two), the masks applied after a sched_barrier:
    // with ld0's select beside its load the scheduler placed the first select (and its wait) amid the batch, a round
    // trip before the rest of the loads issued
    double lv[NB * NB / 256], pv[NB * NB / 256], cdv[NB * NB / 256], xpv[NB * NB / 256];
#pragma unroll
    for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
      const int e = tid + 256 * u_, r = e & (NB - 1), c = e >> 5;
      lv[u_] = Lin[kb > 0 ? e : 0];  // kb = 0: first block of a big panel, already fully updated
      pv[u_] = F[c < kb ? (k0 + c) * m + r0 + r : 0];
      cdv[u_] = F[r >= c && r < kbn ? (r0 + c) * m + r0 + r : 0];
      xpv[u_] = L[pair ? (k0 - NB + c) * m + r0 + r : 0];  // L rows of the block in the previous panel
    }
    double ykv = ysol[tid < kb ? t.c0 + k0 + tid : 0];
    double vo = v[tid < kbn ? r0 + tid : 0];
    __builtin_amdgcn_sched_barrier(0);
    if (!(tid < kb)) ykv = 0.0;
    if (!(tid < kbn)) vo = 0.0;
#pragma unroll
    for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
      const int e = tid + 256 * u_, r = e & (NB - 1), c = e >> 5;
      Li[c * PS + r] = kb > 0 ? lv[u_] : 0.0;  // e = row * 32 + col of the row-major inverse: (c, r) = (row, col)
      Pa[r * PS + c] = c < kb ? pv[u_] : 0.0;
      Dn[r * DS + c] = r >= c && r < kbn ? cdv[u_] : 0.0;
      Pb[r * PS + c] = pair ? xpv[u_] : 0.0;
    }
    *(tid < NB ? &yk[tid] : &col[tid & (4 * NB - 1)]) = ykv;  // unconditional: keeps the ysol load in the first batch
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
    // L^-1 leaves from wave 0's registers; the block of X = L11^-1 it also is reaches xinv by k_xdiag after the
    // factorization (the inverse tasks read it from linv meanwhile): no barrier and no LDS pass on the chain
    if (tid < 64) factor_block(Dn, kbn, vn, col, tid, fail, ysol + t.c0 + r0, PH_REC, nullptr, linv + (size_t)(t.c0 + r0) * (NB * NB));
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
      // X_{kq,j}(r, c); the diagonal block X_{kq,kq} = L_{kq}^-1 from linv (k_xdiag copies it to X after the factor)
      xq[u] = kq == j ? linv[(size_t)(t.c0 + NB * kq) * (NB * NB) + r * NB + c] : Xf[(NB * j + c) * ns + NB * kq + r];
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
  const int rlim = (t.flags & 128) ? ns : m;  // rows this tile owns
  MfmaTile T;
  T.zero();
  double xpa[8], xpb[8];  // issued with the current panel's loads (one round trip), staged before the C prefetch
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
    xpa[u] = ld0(L, (k0 - NB + q) * m + I0 + r, pair && I0 + r < rlim);
    xpb[u] = ld0(L, (k0 - NB + q) * m + J0 + r, pair && J0 + r < rlim);
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
    pav[u] = ld0(F, (k0 + q) * m + I0 + r, q < kb && I0 + r < rlim);
    pbv[u] = ld0(F, (k0 + q) * m + J0 + r, upd && q < kb && J0 + r < rlim);
  }
  const int climit = t.clim;  // ns; m when the contribution block is fused; the big-panel end when blocked
  // rows/columns of the next diagonal block, [r0, r0 + kbn): this step's diagonal task reads their raw values at its
  // start and applies the panel update itself, so tile tasks never write them
  const int kbn = (t.flags & 32) ? 0 : max(0, min(NB, ns - r0));
  // the writer's forward-solve row of v, read with this first batch (a read at its update, after the TRSM, would be
  // one more memory round trip on the writer tiles)
  const bool vupd = writer && tid < 64 && I0 + tid < rlim && I0 + tid >= r0 + kbn;
  const double vold = ld0(v, I0 + tid, vupd);
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
  if (upd) load_ctile(F, m, rlim, I0, J0, climit, tid, cv);
#pragma unroll
  for (int u_ = 0; u_ < NB * NB / 256; ++u_) {
    const int e = tid + 256 * u_;
    Li[(e >> 5) * PS + (e & (NB - 1))] = lv[u_];
  }
  *(tid < NB ? &yk[tid] : &col[tid & (4 * NB - 1)]) = ykv;  // unconditional: keeps the ysol load in the first batch
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
  if (vupd) {  // forward-solve update: v_i -= x_i y_k
    double s2 = 0.0;
#pragma unroll
    for (int q = 0; q < NB; ++q) s2 += Pa[tid * PS + q] * yk[q];
    v[I0 + tid] = vold - s2;
  }

  // ---- writers store the L21 rows of block I
  if (writer) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, r = e & (TT - 1), q = e >> 6;
      if (q < kb && I0 + r < rlim) L[(k0 + q) * m + I0 + r] = Pa[r * PS + q];
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
    if (gi < rlim && gj < climit && gi >= gj && !dblk) F[(size_t)gj * m + gi] = cv[u] - sh[r * CS + c];
  }
  PH1(4)
  PH1R(7)
}

// ---------------------------------------------------------------------------- contribution block
// U = A22 - L21 L21^T (rows/columns ns..m-1) in one pass with K = ns (gemm_nt.hpp: 64x64 tiles, K in
// double-buffered 16-column LDS chunks). Task: s, b = ti | tj << 16, K = [a, c) (c = 0: [0, ns)).
// The same kernel is the trailing update of a blocked front after each big panel: rows >= kb, columns
// [kb, ns), K = the big panel's columns [ka, kb) of the finished factor.
// Tile: GemmNT (register-staged double buffer) or GemmNTd (LDS-DMA ring, G2OHIP_SYRK_DMA)
// Task bit 31 of b (contribution passes of deferred-L21 fronts, diagonal tiles): the tile also applies the forward
// solve's update to the front vector's rows below the supernode, v_i -= L21(i, :) y1 (the panel steps of such fronts
// update only the supernode's own rows).
template <class SyrkTile>
__global__ void __launch_bounds__(256) k_syrk(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                              double* __restrict__ fronts, const double* __restrict__ lbuf,
                                              const double* __restrict__ ysol, double* __restrict__ vecs) {
  __shared__ __attribute__((aligned(16))) double sh[SyrkTile::LDS_DOUBLES];
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, ns = me.ns;
  const bool vec = t.b < 0;
  const int ti = t.b & 0xffff, tj = (t.b >> 16) & 0x7fff;
  const int ka = t.a, kb = t.c ? t.c : ns, climit = kb == ns ? m : ns;
  // a childless front's contribution block holds nothing before this pass (its rows and columns are ancestors'
  // variables: no input entries, no children): written, not read
  const bool overwrite = t.c == 0 && me.child_begin == me.child_end;
  SyrkTile::run(lbuf + me.l_off, m, fronts + me.front_off, m, m, climit, kb + ti * SyrkTile::ROWS, kb + tj * TT, ka,
                kb, sh, overwrite, vec ? ysol + me.c0 : nullptr, vec ? vecs + me.vec_off : nullptr);
}

// Deferred L21 (wide throughput-bound levels, DeviceCholesky::setup): after a front's panel steps, which factored only
// its own rows, L21 = A21 L11^-T = A21 X^T with the explicit inverse X = L11^-1 the inverse tasks built (diagonal blocks
// copied in by a per-level k_xdiag): one GEMM tile per (row tile ti of the nr rows below, column tile tj), K = [0, 64 tj
// + 64) since X(j, k) = 0 for k > j. A21 is the front's raw rows below the supernode (no panel step touched them).
using L21Tile = GemmNTd<TT, TT, 2, 2, 16, 2>;
__global__ void __launch_bounds__(256) k_l21(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                             const double* __restrict__ fronts, const double* __restrict__ xinv,
                                             double* __restrict__ lbuf) {
  __shared__ __attribute__((aligned(16))) double sh[L21Tile::LDS_DOUBLES];
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int m = me.ns + me.nr, ns = me.ns, nr = me.nr;
  const int ti = t.b & 0xffff, tj = t.b >> 16;
  const int I0 = ti * TT, J0 = tj * TT, kb = min(ns, J0 + TT);
  L21Tile::run_ab(fronts + me.front_off + ns, m, nr, xinv + me.x_off, ns, ns, lbuf + me.l_off + ns, m, nr, ns, I0, J0,
                  0, kb, sh, 2);
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
  // four rows per lane in flight (the column and row-index loads of a batch, then their x gathers), four partial sums
  double a4[4] = {0.0, 0.0, 0.0, 0.0};
  int i = lane;
  for (; i + 192 < me.nr; i += 256) {
    double c[4];
    int r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { c[u] = col[i + 64 * u]; r[u] = rw[i + 64 * u]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) a4[u] += c[u] * xsol[r[u]];
  }
  for (; i < me.nr; i += 64) a4[0] += col[i] * xsol[rw[i]];
  double acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) tsol[me.c0 + j] = ysol[me.c0 + j] - acc;
}

// X's 32 x 32 diagonal blocks are read from linv (L_kk^-1, row-major, as the factorization published them): no copy of
// them into X is needed for the solve (k_xdiag runs only for the deferred-L21 fronts' k_l21)
__global__ void __launch_bounds__(256) k_bwd_x(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                               const double* __restrict__ xinv, const double* __restrict__ linv,
                                               const double* __restrict__ tsol, double* __restrict__ xsol,
                                               const int* __restrict__ perm, double* __restrict__ xout) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int ns = me.ns;
  const int lane = threadIdx.x & 63, j = t.a + (int)(threadIdx.x >> 6);
  if (j >= (t.b ? t.b : ns)) return;
  const double* xc = xinv + me.x_off + (size_t)j * ns;  // column j of X (rows >= j are nonzero)
  const double* tt = tsol + me.c0;
  const int ie = t.c;  // X(j.., j) up to row ie: ns, or the end of a blocked front's big panel (X_bb)
  const int b0 = j & ~(NB - 1), be = min(min(b0 + NB, ns), ie);  // j's diagonal block: rows [j, be) from L_kk^-1
  double a4[4] = {0.0, 0.0, 0.0, 0.0};
  if (j + lane < be) a4[0] = linv[(size_t)(me.c0 + b0) * (NB * NB) + (j + lane - b0) * NB + (j - b0)] * tt[j + lane];
  int i = be + lane;
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
  double a4[4] = {0.0, 0.0, 0.0, 0.0};
  int i = t.b + lane;
  for (; i + 192 < ns; i += 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a4[u] += col[i + 64 * u] * xx[i + 64 * u];
  }
  for (; i < ns; i += 64) a4[0] += col[i] * xx[i];
  double acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) tsol[me.c0 + j] -= acc;
}

// Diagonal 32 x 32 blocks of X = L11^-1 from linv (the panel steps publish L^-1 only there): task (front s, panel
// start a); X column-major with leading dimension ns, rows/columns [a, a + kb)
__global__ void __launch_bounds__(256) k_xdiag(const Task* __restrict__ tasks, const FrontDesc* __restrict__ fd,
                                               const double* __restrict__ linv, double* __restrict__ xinv) {
  const Task t = tasks[blockIdx.x];
  const FrontDesc me = fd[t.s];
  const int a = t.a, kb = min(NB, me.ns - a);
  const double* L = linv + (size_t)(me.c0 + a) * (NB * NB);
  double* X = xinv + me.x_off + (size_t)a * me.ns + a;
  double x[NB * NB / 256];  // (the padded 32 x 32 block is always readable: every load issued before the first store)
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = threadIdx.x + 256 * u, c = e >> 5, i = e & (NB - 1);
    x[u] = L[i * NB + c];
  }
  asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]));  // else each load is sunk into its store's branch
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = threadIdx.x + 256 * u, c = e >> 5, i = e & (NB - 1);  // X(i, c): consecutive threads down a column
    if (c < kb && i < kb) X[(size_t)c * me.ns + i] = x[u];
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
  if (boff[t] >= 0) dst[boff[t] + (i - t * bb)] = src[i];  // -1: a block this rank never reads
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
void chol_extend_add(int ntasks, int nb0, const Task* tasks, const B0Front* b0f, const B0Child* b0c, const FrontDesc* fd,
                     const int* children, const int* relmap,
                     const int* jtab, const int* cmptr, const longlong2* cment, const int* colptr, const int* ent_row, const int* ent_src, const double* vals, const double* lam,
                     double* fronts, double* vecs, double* lbuf, double* ysol, double* linv, double* xinv,
                     int* fail, int assemble, hipStream_t s, const ScatterJob* sj) {
  if (ntasks <= 0) return;
  if (!sj || sj->ntask != ntasks || sj->nb0 != nb0 || nb0 > ntasks)
    throw DeviceError("chol_extend_add: launch arguments do not match the task counts");
  ScatterJob job = *sj;
  if (job.sc1 <= job.sc0) job.sc0 = job.sc1 = 0;
  const int grid = ntasks + (int)((job.sc1 - job.sc0 + 255) / 256);
#define G2OHIP_EA(A_, E_)                                                                                        \
  hipLaunchKernelGGL((k_extend_add<A_, E_>), grid, 256, 0, s, tasks, b0f, b0c, fd, children, relmap, jtab, cmptr, cment, \
                     colptr, ent_row, ent_src, vals, lam, fronts, vecs, lbuf, ysol, linv, xinv, fail, job)
  // assemble 2: fronts up to 512 rows (a small column buffer keeps more workgroups per CU)
  if (assemble == 2) G2OHIP_EA(true, 512);
  else if (assemble == 3) G2OHIP_EA(true, 1024);
  else if (assemble) G2OHIP_EA(true, 2048);
  else G2OHIP_EA(false, 1);
#undef G2OHIP_EA
  KERNEL_CHECK();
}
void chol_step(int ntasks, const StepTask* tasks, const StepHead& head, double* fronts, double* lbuf, double* vecs,
               double* ysol, double* linv, double* xinv, int* fail, bool pairs, hipStream_t s) {
  if (ntasks <= 0) return;
  if (head.ntask != ntasks) throw DeviceError("chol_step: head.ntask does not match the task count");
  const int grid = ntasks + (head.sc1 > head.sc0 ? (int)((head.sc1 - head.sc0 + 255) / 256) : 0);
  if (pairs)
    hipLaunchKernelGGL(k_step<true>, grid, 256, 0, s, tasks, head, fronts, lbuf, vecs, ysol, linv, xinv, fail);
  else
    hipLaunchKernelGGL(k_step<false>, grid, 256, 0, s, tasks, head, fronts, lbuf, vecs, ysol, linv, xinv, fail);
  KERNEL_CHECK();
}
void chol_l21(int ntasks, const Task* tasks, const FrontDesc* fd, const double* fronts, const double* xinv, double* lbuf,
              hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_l21, ntasks, 256, 0, s, tasks, fd, fronts, xinv, lbuf);
  KERNEL_CHECK();
}
// G2OHIP_SYRK_DMA (dev A/B): 1-4 the 64 x 64 LDS-DMA tiles below, 5 / 6 a 128 x 64 tile (K chunks 16 x 2 / 8 x 3
// stages), 0 the register-staged GemmNT; the task lists are built for the variant's row-tile height (syrk_tile_rows)
int syrk_variant() {
  static EnvKnob dma_k{"G2OHIP_SYRK_DMA", 4};
  return dma_k.get();
}
int syrk_tile_rows(int v) { return v == 5 || v == 6 ? 2 * TT : TT; }
// variant: the one DeviceCholesky::setup read and built its row-tile lists for (never re-read here: the knob may change
// between optimizers, and a tile of another height would miss or double-apply rows of those lists)
void chol_syrk(int variant, int ntasks, const Task* tasks, const FrontDesc* fd, double* fronts, const double* lbuf,
               const double* ysol, double* vecs, hipStream_t s) {
  if (ntasks <= 0) return;
  // G2OHIP_SYRK_DMA=k (dev A/B): the LDS-DMA tile GemmNTd with (K chunk, stages) = (32, 2), (16, 3), (8, 4), (16, 2)
  // for k = 1..4. Alone on one 4096^2 SYRK at K = 2048 the (32, 2) ring reaches 47.9 against 41.2 TF/s for the
  // register-staged GemmNT (profiles/r04_ubench_gemm.log), but inside the C3 factorization (contribution passes and
  // big-panel trailing updates of many sizes, next to other launches) it measured slower: factor 29.84 vs 29.18 ms
  // (profiles/r04_ab_c3_syrk.log; 74 KB of LDS leave 2 workgroups per CU against 3). The (16, 2) ring (37 KB, four
  // workgroups per CU) is the one that wins there: C3 factor 29.07 -> 28.54 ms (profiles/r04_ab_c3_knobs.log), the
  // default; G2OHIP_SYRK_DMA=0 is the register-staged GemmNT.
  switch (variant) {
    case 5: hipLaunchKernelGGL((k_syrk<GemmNTd<2 * TT, TT, 2, 2, 16, 2>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs); break;
    case 6: hipLaunchKernelGGL((k_syrk<GemmNTd<2 * TT, TT, 2, 2, 8, 3>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs); break;
    case 1: hipLaunchKernelGGL((k_syrk<GemmNTd<TT, TT, 2, 2, 32, 2>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs); break;
    case 2: hipLaunchKernelGGL((k_syrk<GemmNTd<TT, TT, 2, 2, 16, 3>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs); break;
    case 3: hipLaunchKernelGGL((k_syrk<GemmNTd<TT, TT, 2, 2, 8, 4>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs); break;
    case 4: hipLaunchKernelGGL((k_syrk<GemmNTd<TT, TT, 2, 2, 16, 2>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs); break;
    default: hipLaunchKernelGGL((k_syrk<GemmNT<TT, TT>>), ntasks, 256, 0, s, tasks, fd, fronts, lbuf, ysol, vecs);
  }
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
void chol_xdiag(int ntasks, const Task* tasks, const FrontDesc* fd, const double* linv, double* xinv, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_xdiag, ntasks, 256, 0, s, tasks, fd, linv, xinv);
  KERNEL_CHECK();
}
void chol_bwd_x(int ntasks, const Task* tasks, const FrontDesc* fd, const double* xinv, const double* linv,
                const double* tsol, double* xsol, const int* perm, double* xout, hipStream_t s) {
  if (ntasks <= 0) return;
  hipLaunchKernelGGL(k_bwd_x, ntasks, 256, 0, s, tasks, fd, xinv, linv, tsol, xsol, perm, xout);
  KERNEL_CHECK();
}

}  // namespace launch
}  // namespace g2ohip
