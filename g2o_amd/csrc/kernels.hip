// HIP kernels for the BlockSolver<p,l> hot path on gfx950 (MI355X).
//
//   k_linearize   BlockSolver::buildSystem edge loop (block_solver.hpp:486-506) fused with
//                 BaseBinaryEdge::constructQuadraticForm (base_binary_edge.hpp:61-100):
//                 one lane per edge, J and J^T Omega J in registers, contributions streamed
//                 to per-edge slots (no atomics, no locks).
//   k_vertex_reduce  deterministic segmented reduction of the slots into Hpp/Hll diagonal
//                 blocks and b (replaces the per-vertex omp locks + copyB, :467-517).
//   k_schur_prep  landmark pass of BlockSolver::solve (:342-360): Dinv = (Hll+lambda I)^-1,
//                 and the split Hll+lambda I = U U^T, c = U^-1 b_l.
//   k_schur_diag  Hschur(i,i) = Hpp(i,i) + lambda - sum_l G_il G_il^T, bschur = b - sum G c (:361-400),
//                 G = Hpl U^-T in registers (and stored once per observation), one workgroup per camera.
//   k_schur_rows  Hschur(i,j>i) = Hpp(i,j) - sum_l G_il G_jl^T: one workgroup per camera row (chunk),
//                 the row's G blocks staged into LDS by LDS-DMA in batches; every output has one
//                 owner and a fixed summation order (no atomics).
//   k_backsub     x_l = Dinv (b_l - Hpl^T x_p) (:420-446).
//   k_error/k_oplus  computeActiveErrors (sparse_optimizer.cpp:63-90) and update (:441-454).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.hpp"
#include "device_types.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace g2ohip {
using namespace dev;

// ------------------------------------------------------------------------------ errors / chi2
template <class F>
__global__ void __launch_bounds__(256) k_error(EdgeData d, int ne, double* __restrict__ chi) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  double err[F::D];
  F::error(d, e, err);
  double Om[F::D * F::D];
  load_info<F::D>(info_rec(d, (int)e, F::INFO), Om);
  double s = 0;
#pragma unroll
  for (int i = 0; i < F::D; ++i) {
    double r = 0;
#pragma unroll
    for (int j = 0; j < F::D; ++j) r += Om[i * F::D + j] * err[j];
    s += err[i] * r;
  }
  if (d.rk) {  // activeRobustChi2 (sparse_optimizer.cpp:102-116): rho[0]
    double r0, r1;
    robustify(d.rk, d.rk_delta, s, r0, r1);
    s = r0;
  }
  chi[e] = s;
}

// ------------------------------------------------------------------------------ linearize
// slot layouts (AoS per edge): packed upper col-major H (d(d+1)/2) followed by b (d).
// Stores go through a per-wave LDS image: the wave's 64 consecutive edges own one contiguous run of
// each slot array (and, when their blocks are consecutive, of the off-diagonal blocks), written with
// coalesced 16-byte stores instead of one 16-byte write request per lane and slot chunk.
namespace {
// order one wave's LDS writes before its reads of another lane's words (LDS is in order per wave;
// this stops compiler motion across the point)
__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
// copy n doubles LDS -> global by one wave (dst 8-byte aligned)
__device__ __forceinline__ void wave_copy_out(double* __restrict__ dst, const double* src, int n, int lane) {
  int s = 0;
  if (reinterpret_cast<uintptr_t>(dst) & 15) {  // peel to 16-byte alignment
    if (lane == 0 && n > 0) dst[0] = src[0];
    s = 1;
  }
  const int n2 = (n - s) >> 1;
  double2* d2 = reinterpret_cast<double2*>(dst + s);
  for (int i = lane; i < n2; i += 64) d2[i] = double2{src[s + 2 * i], src[s + 2 * i + 1]};
  if (lane == 0 && ((n - s) & 1)) dst[n - 1] = src[n - 1];
}
}  // namespace

template <class F>
__global__ void __launch_bounds__(256)
    k_linearize(EdgeData d, int ne, const int* __restrict__ h0, const int* __restrict__ h1, double* __restrict__ slot0,
                double* __restrict__ slot1, const long long* __restrict__ off_dst, const unsigned char* __restrict__ off_tr,
                double* __restrict__ off_base, double* __restrict__ off_slot) {
  constexpr int D = F::D, DA = F::DA, DB = F::DB;
  constexpr int SA = DA * (DA + 1) / 2 + DA, SB = DB * (DB + 1) / 2 + DB, SH = DA * DB;
  constexpr int SM = SA > SB ? (SA > SH ? SA : SH) : (SB > SH ? SB : SH);
  __shared__ __attribute__((aligned(16))) double stage[4][64 * SM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int e = blockIdx.x * blockDim.x + tid;
  const int ebase = e - lane, nw = min(64, ne - ebase);  // the wave's edges [ebase, ebase + nw)
  if (nw <= 0) return;                                  // wave-uniform
  double* sw = stage[tid >> 6];
  const bool in = e < ne;
  const bool nfA = in && h0[d.v0[e]] >= 0, nfB = in && h1[d.v1[e]] >= 0;
  double err[D], A[D * DA], B[D * DB], Om[D * D];
  if (nfA || nfB) {
    F::linearize(d, e, err, A, B);
    load_info<D>(info_rec(d, e, F::INFO), Om);
    if (d.rk) {  // robust branch of constructQuadraticForm (base_binary_edge.hpp:104-135): Omega, omega_r scaled by rho'
      double chi = 0;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        double r = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) r += Om[i * D + j] * err[j];
        chi += err[i] * r;
      }
      double r0, r1;
      robustify(d.rk, d.rk_delta, chi, r0, r1);
#pragma unroll
      for (int i = 0; i < D * D; ++i) Om[i] *= r1;
    }
  }
  double wr[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    double s = 0;
#pragma unroll
    for (int c = 0; c < D; ++c) s += Om[r * D + c] * err[c];
    wr[r] = -s;
  }
  double AtO[DA * D];  // A^T Omega
#pragma unroll
  for (int i = 0; i < DA; ++i)
#pragma unroll
    for (int c = 0; c < D; ++c) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < D; ++r) s += A[r * DA + i] * Om[r * D + c];
      AtO[i * D + c] = s;
    }
  // side A slot (edges whose side A is fixed leave garbage in their slot: never read)
  if (nfA) {
    double* o = sw + lane * SA;
    int k = 0;
#pragma unroll
    for (int c = 0; c < DA; ++c)
#pragma unroll
      for (int r = 0; r <= c; ++r) {
        double s = 0;
#pragma unroll
        for (int t = 0; t < D; ++t) s += AtO[r * D + t] * A[t * DA + c];
        o[k++] = s;
      }
#pragma unroll
    for (int i = 0; i < DA; ++i) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < D; ++r) s += A[r * DA + i] * wr[r];
      o[k++] = s;
    }
  }
  wave_sync();
  wave_copy_out(slot0 + (size_t)ebase * SA, sw, nw * SA, lane);
  wave_sync();
  // off-diagonal block: staged when the wave's blocks are consecutive with one orientation. Destinations with
  // bit 62 set are per-edge slots of a block several edges share (summed in order by k_offblock_reduce)
  constexpr long long SLOT_BIT = 1LL << 62;
  const long long od_raw = (nfA && nfB) ? off_dst[e] : -1;
  const bool in_slot = od_raw >= 0 && (od_raw & SLOT_BIT);
  const long long od = od_raw >= 0 ? (od_raw & ~SLOT_BIT) : -1;
  const bool tr = nfA && nfB && off_tr[e];
  const long long od0 = __shfl(od, 0, 64);
  const bool tr0 = __shfl((int)tr, 0, 64) != 0;
  const bool slot0f = __shfl((int)in_slot, 0, 64) != 0;
  const bool run = __all(!in || (od >= 0 && od0 >= 0 && od == od0 + (long long)lane * SH && tr == tr0 && in_slot == slot0f));
  double* const obase = in_slot ? off_slot : off_base;
  if (od >= 0) {
    double* H = run ? sw + lane * SH : obase + od;
    if (tr) {  // DB x DA col-major: (j,i)
#pragma unroll
      for (int i = 0; i < DA; ++i)
#pragma unroll
        for (int j = 0; j < DB; ++j) {
          double s = 0;
#pragma unroll
          for (int r = 0; r < D; ++r) s += AtO[i * D + r] * B[r * DB + j];
          H[i * DB + j] = s;
        }
    } else {  // DA x DB col-major: (i,j)
#pragma unroll
      for (int j = 0; j < DB; ++j)
#pragma unroll
        for (int i = 0; i < DA; ++i) {
          double s = 0;
#pragma unroll
          for (int r = 0; r < D; ++r) s += AtO[i * D + r] * B[r * DB + j];
          H[j * DA + i] = s;
        }
    }
  }
  if (run) {
    wave_sync();
    wave_copy_out((slot0f ? off_slot : off_base) + od0, sw, nw * SH, lane);
    wave_sync();
  }
  if (nfB) {
    double BtO[DB * D];
#pragma unroll
    for (int j = 0; j < DB; ++j)
#pragma unroll
      for (int c = 0; c < D; ++c) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < D; ++r) s += B[r * DB + j] * Om[r * D + c];
        BtO[j * D + c] = s;
      }
    double* o = sw + lane * SB;
    int k = 0;
#pragma unroll
    for (int c = 0; c < DB; ++c)
#pragma unroll
      for (int r = 0; r <= c; ++r) {
        double s = 0;
#pragma unroll
        for (int t = 0; t < D; ++t) s += BtO[r * D + t] * B[t * DB + c];
        o[k++] = s;
      }
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < D; ++r) s += B[r * DB + j] * wr[r];
      o[k++] = s;
    }
  }
  wave_sync();
  wave_copy_out(slot1 + (size_t)ebase * SB, sw, nw * SB, lane);
}

// ------------------------------------------------------------------------------ vertex reduction
// One group of LANES lanes per vertex; lane l sums slots l, l+LANES, ... in order; butterfly
// reduction in a fixed pattern keeps the result bitwise reproducible.
template <int DIM, int LANES>
__global__ void __launch_bounds__(256)
    k_vertex_reduce(int nv, const int* __restrict__ inc_ptr, const int* __restrict__ inc_code,
                    const double* __restrict__ slots, double* __restrict__ Hdiag /* [nv][DIM*DIM] */,
                    double* __restrict__ b /* offset per vertex */, const int* __restrict__ boff) {
  constexpr int SP = DIM * (DIM + 1) / 2, S = SP + DIM;
  // vertices with >= 64 lanes: XCD-contiguous vertex ranges (a landmark's edges, neighbours in the
  // slot arrays, belong to nearby cameras: mostly one L2)
  const int gid = (LANES >= 64 ? xcd_item(blockIdx.x, gridDim.x) : (int)blockIdx.x) * blockDim.x + threadIdx.x;
  const int v = gid / LANES, lane = gid % LANES;
  const bool active = v < nv;
  double acc[S];
#pragma unroll
  for (int k = 0; k < S; ++k) acc[k] = 0;
  if (active) {
    const int p0 = inc_ptr[v], p1 = inc_ptr[v + 1];
    for (int p = p0 + lane; p < p1; p += LANES) {
      const double* s = slots + (size_t)inc_code[p] * S;
#pragma unroll
      for (int k = 0; k < S; ++k) acc[k] += s[k];
    }
  }
  constexpr int WL = LANES > 64 ? 64 : LANES;  // butterfly width (one wave at most)
  if (WL > 1) {
#pragma unroll
    for (int m = WL / 2; m >= 1; m >>= 1)
#pragma unroll
      for (int k = 0; k < S; ++k) acc[k] += __shfl_xor(acc[k], m, WL);
  }
  if constexpr (LANES > 64) {  // LANES == blockDim: the waves' sums combined in wave order
    __shared__ double red[LANES / 64][S];
    if ((lane & 63) == 0) {
#pragma unroll
      for (int k = 0; k < S; ++k) red[lane >> 6][k] = acc[k];
    }
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < S; ++k) {
        double t = red[0][k];
#pragma unroll
        for (int w = 1; w < LANES / 64; ++w) t += red[w][k];
        acc[k] = t;
      }
    }
  }
  if (!active || lane != 0) return;
  double* H = Hdiag + (size_t)v * DIM * DIM;
  int k = 0;
#pragma unroll
  for (int c = 0; c < DIM; ++c)
#pragma unroll
    for (int r = 0; r <= c; ++r) {
      H[c * DIM + r] = acc[k];
      H[r * DIM + c] = acc[k];
      ++k;
    }
  double* bb = b + boff[v];
#pragma unroll
  for (int i = 0; i < DIM; ++i) bb[i] = acc[SP + i];
}

// off-diagonal blocks shared by several edges: sum their per-edge slots (offsets into `slots`) in edge order
__global__ void __launch_bounds__(256) k_offblock_reduce(int nb, int bsz, const int* __restrict__ ptr,
                                                          const long long* __restrict__ soff,
                                                          const double* __restrict__ slots, double* __restrict__ out,
                                                          const long long* __restrict__ dst) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int blk = gid / bsz, k = gid % bsz;
  if (blk >= nb) return;
  double s = 0;
  for (int p = ptr[blk]; p < ptr[blk + 1]; ++p) s += slots[soff[p] + k];
  out[dst[blk] + k] = s;
}

// High-degree vertices (BA cameras, ~1000 incident edges): one workgroup per vertex, 8 slot streams
// (two per wave, one per half-wave); lane k of a half-wave reads entry k of its slot, so every load
// instruction reads two slots' contiguous S-double runs (a few cache lines, not 64 scattered ones), U slots
// per stream in flight. Each lane sums its entry over its stream in slot order; the 8 stream sums are
// added in stream order: a fixed order, bitwise reproducible.
template <int DIM>
__global__ void __launch_bounds__(256)
    k_vertex_reduce_wide(int nv, const int* __restrict__ inc_ptr, const int* __restrict__ inc_code,
                         const double* __restrict__ slots, double* __restrict__ Hdiag, double* __restrict__ b,
                         const int* __restrict__ boff) {
  constexpr int SP = DIM * (DIM + 1) / 2, S = SP + DIM, U = 8, NS = 8;  // U = 16: no change
  static_assert(S <= 32, "one half-wave per slot");
  __shared__ double red[NS][32];
  const int v = xcd_item(blockIdx.x, gridDim.x);
  if (v >= nv) return;  // workgroup-uniform
  const int tid = threadIdx.x, k = tid & 31, q = tid >> 5;  // entry, stream
  const int p0 = inc_ptr[v], p1 = inc_ptr[v + 1];
  double acc = 0.0;
  for (int p = p0 + q; p < p1; p += NS * U) {
    int c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = p + NS * u < p1 ? inc_code[p + NS * u] : -1;
    double d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double* sl = slots + (size_t)(c[u] >= 0 ? c[u] : 0) * S;
      d[u] = (c[u] >= 0 && k < S) ? sl[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += d[u];
  }
  red[q][k] = acc;
  __syncthreads();
  if (tid >= S) return;
  double t = red[0][tid];
#pragma unroll
  for (int j = 1; j < NS; ++j) t += red[j][tid];
  if (tid < SP) {  // packed upper column-major index -> (r, c)
    int c = 0, base = 0;
    while (tid >= base + c + 1) base += ++c;
    const int r = tid - base;
    double* H = Hdiag + (size_t)v * DIM * DIM;
    H[c * DIM + r] = t;
    H[r * DIM + c] = t;
  } else {
    b[boff[v] + tid - SP] = t;
  }
}

// ------------------------------------------------------------------------------ Schur
// Landmark pass (block_solver.hpp:341-360): Dinv = (Hll + lambda I)^-1 (Eigen's fixed-size inverse: cofactors for
// 3x3, the closed form for 2x2; kept for the back-substitution) and the symmetric split
//   Hll + lambda I = U U^T (LD x LD Cholesky),  G_a = Hpl_a U^-T,  c_l = U^-1 b_l,
// so that Hpl Dinv Hpl^T = G G^T and Hpl Dinv b_l = G c_l. k_schur_diag forms G once per observation
// (for its own sums and, stored, for k_schur_rows). Ufac per landmark (UF doubles, r = reciprocal pivots of U):
// LD = 3: r0 r1 r2 u10 u20 u21, LD = 2: r0 r1 u10 0. The Schur kernels are instantiated for the reference's
// BlockSolver_6_3 (PD = 6, LD = 3) and BlockSolver_3_2 (PD = 3, LD = 2) (block_solver.h:188-201).
template <int LD>
struct LmTraits;
template <>
struct LmTraits<3> { static constexpr int UF = 6; };
template <>
struct LmTraits<2> { static constexpr int UF = 4; };

template <int LD>
__global__ void __launch_bounds__(256)
    k_schur_prep(int nl, int lm0, const double* __restrict__ Hll, const double* __restrict__ bl_all,
                 const double* __restrict__ lam, double* __restrict__ Dinv, double* __restrict__ Ufac,
                 double* __restrict__ cl_all, int* __restrict__ fail) {
  constexpr int UF = LmTraits<LD>::UF;
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nl) return;
  const double lambda = *lam;
  const double* Hm = Hll + (size_t)l * LD * LD;
  double a[LD * LD];
#pragma unroll
  for (int k = 0; k < LD * LD; ++k) a[k] = Hm[k];
#pragma unroll
  for (int i = 0; i < LD; ++i) a[i * LD + i] += lambda;
  auto m = [&](int r, int c) { return a[c * LD + r]; };
  double* Do = Dinv + (size_t)l * LD * LD;  // col-major
  double* U = Ufac + (size_t)l * UF;
  const double* bl = bl_all + (size_t)(lm0 + l) * LD;
  double* co = cl_all + (size_t)(lm0 + l) * LD;
  bool bad;
  if constexpr (LD == 3) {
    const double c00 = m(1, 1) * m(2, 2) - m(1, 2) * m(2, 1);
    const double c10 = m(0, 2) * m(2, 1) - m(0, 1) * m(2, 2);
    const double c20 = m(0, 1) * m(1, 2) - m(0, 2) * m(1, 1);
    const double det = c00 * m(0, 0) + c10 * m(1, 0) + c20 * m(2, 0);
    const double inv = 1.0 / det;
    Do[0] = c00 * inv; Do[3] = c10 * inv; Do[6] = c20 * inv;
    Do[1] = (m(1, 2) * m(2, 0) - m(1, 0) * m(2, 2)) * inv;
    Do[4] = (m(0, 0) * m(2, 2) - m(0, 2) * m(2, 0)) * inv;
    Do[7] = (m(0, 2) * m(1, 0) - m(0, 0) * m(1, 2)) * inv;
    Do[2] = (m(1, 0) * m(2, 1) - m(1, 1) * m(2, 0)) * inv;
    Do[5] = (m(0, 1) * m(2, 0) - m(0, 0) * m(2, 1)) * inv;
    Do[8] = (m(0, 0) * m(1, 1) - m(0, 1) * m(1, 0)) * inv;
    bad = !(det != 0.0) || !isfinite(inv);
  } else {  // Eigen compute_inverse_size2: adjugate / (m00 m11 - m10 m01)
    const double det = m(0, 0) * m(1, 1) - m(1, 0) * m(0, 1);
    const double inv = 1.0 / det;
    Do[0] = m(1, 1) * inv; Do[1] = -m(1, 0) * inv; Do[2] = -m(0, 1) * inv; Do[3] = m(0, 0) * inv;
    bad = !(det != 0.0) || !isfinite(inv);
  }
  double Ur[UF], cr[LD];
  if (!lm_ufac<LD>(a, bl, Ur, cr)) bad = true;
#pragma unroll
  for (int k = 0; k < UF; ++k) U[k] = Ur[k];
#pragma unroll
  for (int k = 0; k < LD; ++k) co[k] = cr[k];
  if (bad) *fail = 1;
}

// Diagonal blocks of the reduced system (block_solver.hpp:361-400, the j == i terms):
//   S(i,i) = Hpp(i,i) + lambda I - sum_l G_il G_il^T,   bschur_i = b_i - sum_l G_il c_l,
// one workgroup per camera row, its 256 lanes striding over the row's observations (landmark
// order), G formed in registers from Hpl and U_l (and stored, for k_schur_rows); a fixed butterfly
// per wave and the four wave sums added in wave order (bitwise reproducible).
template <int PD, int LD>
__global__ void __launch_bounds__(256)
    k_schur_diag(int nrows, const int* __restrict__ rptr, const int* __restrict__ robs,
                 const int* __restrict__ obs_lm, int lm0, const double* __restrict__ Hpl,
                 const double* __restrict__ Ufac, const double* __restrict__ cl_all, const int* __restrict__ sdiag,
                 const int* __restrict__ s_hpp, const double* __restrict__ Hpp, const double* __restrict__ b,
                 const double* __restrict__ lam, const unsigned char* __restrict__ lam_own,
                 const double* __restrict__ lam_full, double* __restrict__ S, double* __restrict__ bschur,
                 double* __restrict__ G) {
  constexpr int GB = PD * LD, UF = LmTraits<LD>::UF, NPK = PD * (PD + 1) / 2, NA = NPK + PD;
  static_assert(GB % 2 == 0 && UF % 2 == 0, "16-byte block loads");
  __shared__ double red[4][NA];
  __shared__ __attribute__((aligned(16))) double gst[4][64 * GB];  // per-wave image of 64 G blocks
  // XCD-contiguous camera rows: the observations of one landmark (neighbours in Hpl) are read by
  // rows of nearby cameras, i.e. mostly behind one L2
  const int row = xcd_item(blockIdx.x, nrows), tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double acc[NA];  // packed upper of G G^T (col-major) | G c
#pragma unroll
  for (int k = 0; k < NA; ++k) acc[k] = 0.0;
  const int p1 = rptr[row + 1];
  for (int pb = rptr[row] + w * 64; pb < p1; pb += 256) {  // the wave's blocks [pb, pb + nw)
    const int p = pb + lane, nw = min(64, p1 - pb);
    if (p < p1) {
      const int a = robs[p], l = obs_lm[a];
      const double2* h2 = reinterpret_cast<const double2*>(Hpl + (size_t)a * GB);
      const double2* u2 = reinterpret_cast<const double2*>(Ufac + (size_t)l * UF);
      double g[GB], U[UF], c[LD];
#pragma unroll
      for (int k = 0; k < GB / 2; ++k) { const double2 v = h2[k]; g[2 * k] = v.x; g[2 * k + 1] = v.y; }
#pragma unroll
      for (int k = 0; k < UF / 2; ++k) { const double2 v = u2[k]; U[2 * k] = v.x; U[2 * k + 1] = v.y; }
      const double* cp = cl_all + (size_t)(lm0 + l) * LD;
#pragma unroll
      for (int k = 0; k < LD; ++k) c[k] = cp[k];
      form_G<PD, LD>(g, U);
      {  // every observation lies in exactly one camera row: G is written once, in camera-row order,
         // for k_schur_rows; the wave's blocks leave as one contiguous coalesced run (below)
        double2* go = reinterpret_cast<double2*>(gst[w] + lane * GB);
#pragma unroll
        for (int k = 0; k < GB / 2; ++k) go[k] = double2{g[2 * k], g[2 * k + 1]};
      }
      int k = 0;
#pragma unroll
      for (int cc = 0; cc < PD; ++cc)
#pragma unroll
        for (int r = 0; r <= cc; ++r) {
          double s = g[r] * g[cc];
#pragma unroll
          for (int kk = 1; kk < LD; ++kk) s += g[kk * PD + r] * g[kk * PD + cc];
          acc[k++] += s;
        }
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        double s = g[r] * c[0];
#pragma unroll
        for (int kk = 1; kk < LD; ++kk) s += g[kk * PD + r] * c[kk];
        acc[NPK + r] += s;
      }
    }
    wave_sync();  // converged: the whole wave copies the image out
    wave_copy_out(G + (size_t)pb * GB, gst[w], nw * GB, lane);
    wave_sync();
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < NA; ++k) acc[k] += __shfl_xor(acc[k], m, 64);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NA; ++k) red[w][k] = acc[k];
  }
  __syncthreads();
  if (tid >= NA) return;
  const double v = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
  if (tid >= NPK) {
    const int r = tid - NPK;
    bschur[(size_t)row * PD + r] = b[(size_t)row * PD + r] - v;
    return;
  }
  const int sidx = sdiag[row], hp = s_hpp[sidx];
  const double* Hh = Hpp + (size_t)(hp >= 0 ? hp : 0) * PD * PD;
  double* So = S + (size_t)sidx * PD * PD;
  int cc = 0, r = tid;  // packed upper index tid -> (r, cc), r <= cc
  while (r > cc) { r -= cc + 1; ++cc; }
  const double h0 = hp >= 0 ? Hh[cc * PD + r] : 0.0;
  // lambda on the diagonal: by the rank lam_own names for this row (aligned shards), else lam (rank 0's lambda)
  const double lv = lam_own ? (lam_own[row] ? *lam_full : 0.0) : *lam;
  const double o = (r == cc ? h0 + lv : h0) - v;
  So[cc * PD + r] = o;
  So[r * PD + cc] = o;
}

// The pairs of one staged batch into a Schur row task's accumulators: thread (slot ls, q) owns columns c0 .. c0 + CW - 1
// (c0 = (q & 1) CW) of the slot's block over the slot's pairs of parity q >> 1 (landmark order): acc(j, r) +=
// G_a(r, :) . G_b(c0 + j, :). Gs: the batch's blocks (PD x LD col-major each), sp: pairs (posA | posB << 16) slot-sorted,
// spp: the slot CSR.
template <int PD, int LD>
__device__ __forceinline__ void schur_pairs(const double* Gs, const int* sp, const int* spp, int noff, int ls, int q,
                                            double (&acc)[((PD + 1) / 2) * PD]) {
  constexpr int GB = PD * LD, CW = (PD + 1) / 2;
  const int c0 = (q & 1) * CW, par = q >> 1;
  if (ls >= noff) return;
  const int p1 = spp[ls + 1];
  for (int p = spp[ls] + par; p < p1; p += 2) {
    const int pr = sp[p];
    const double* ga = &Gs[(pr & 0xffff) * GB];
    const double* gb = &Gs[(pr >> 16) * GB + c0];
#pragma unroll
    for (int kk = 0; kk < LD; ++kk) {  // one column of G_a and CW entries of G_b at a time
      double A[PD], Bm[CW];
      if constexpr (PD % 2 == 0) {
#pragma unroll
        for (int k = 0; k < PD / 2; ++k) {
          const double2 x = *reinterpret_cast<const double2*>(ga + kk * PD + 2 * k);
          A[2 * k] = x.x; A[2 * k + 1] = x.y;
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) Bm[j] = gb[kk * PD + j];
      } else {  // odd PD: the second half has CW - 1 columns (the spare one reads column c0 and is zeroed)
#pragma unroll
        for (int r = 0; r < PD; ++r) A[r] = ga[kk * PD + r];
#pragma unroll
        for (int j = 0; j < CW; ++j) {
          const bool in = c0 + j < PD;
          const double v = gb[kk * PD + (in ? j : 0)];
          Bm[j] = in ? v : 0.0;
        }
      }
#pragma unroll
      for (int j = 0; j < CW; ++j)
#pragma unroll
        for (int r = 0; r < PD; ++r) acc[j * PD + r] += A[r] * Bm[j];
    }
  }
}
// The same pairs from the BA split's 10-double records (assembly.hip KXB: Kt = diag(f) Omega A U^-T, 2 x 3 col-major,
// then u = x/z, v = y/z, w = 1/z): G = Bt^T Kt, so G_a G_b^T = Bt_a^T (Kt_a Kt_b^T) Bt_b. Per pair a thread forms the
// 2 x 2 M = Kt_a Kt_b^T, T = M Bt_b(:, c0 .. c0 + 2) and acc(j, r) += Bt_a(:, r) . T(:, j): 18 staged doubles read
// instead of 27, the camera Jacobians rebuilt from three numbers each.
__device__ __forceinline__ void schur_pairs_kx(const double* Gs, const int* sp, const int* spp, int noff, int ls, int q,
                                               double (&acc)[18]) {
  constexpr int GB = 10;
  const int par = q >> 1;
  const bool hi = q & 1;  // columns 3..5 of the block
  if (ls >= noff) return;
  const int p1 = spp[ls + 1];
  for (int p = spp[ls] + par; p < p1; p += 2) {
    const int pr = sp[p];
    const double* ga = &Gs[(pr & 0xffff) * GB];
    const double* gb = &Gs[(pr >> 16) * GB];
    double ka[6], kb[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double2 x = *reinterpret_cast<const double2*>(ga + 2 * k);
      const double2 y = *reinterpret_cast<const double2*>(gb + 2 * k);
      ka[2 * k] = x.x; ka[2 * k + 1] = x.y;
      kb[2 * k] = y.x; kb[2 * k + 1] = y.y;
    }
    const double2 ua2 = *reinterpret_cast<const double2*>(ga + 6), ub2 = *reinterpret_cast<const double2*>(gb + 6);
    const double ua = ua2.x, va = ua2.y, wa = ga[8], ub = ub2.x, vb = ub2.y, wb = gb[8];
    // M = Kt_a Kt_b^T (2 x 2)
    double M[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int s = 0; s < 2; ++s) M[r][s] = ka[r] * kb[s] + ka[2 + r] * kb[2 + s] + ka[4 + r] * kb[4 + s];
    // Bt_b columns c0 .. c0 + 2 (rows 0, 1)
    double b0[3], b1[3];
    if (!hi) {
      b0[0] = ub * vb; b0[1] = -(1.0 + ub * ub); b0[2] = vb;
      b1[0] = 1.0 + vb * vb; b1[1] = -(ub * vb); b1[2] = -ub;
    } else {
      b0[0] = -wb; b0[1] = 0.0; b0[2] = ub * wb;
      b1[0] = 0.0; b1[1] = -wb; b1[2] = vb * wb;
    }
    double T0[3], T1[3];  // T = M Bt_b(:, cols)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      T0[j] = M[0][0] * b0[j] + M[0][1] * b1[j];
      T1[j] = M[1][0] * b0[j] + M[1][1] * b1[j];
    }
    // Bt_a, all six columns
    const double a0[6] = {ua * va, -(1.0 + ua * ua), va, -wa, 0.0, ua * wa};
    const double a1[6] = {1.0 + va * va, -(ua * va), -ua, 0.0, -wa, va * wa};
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        if (r == 4) acc[j * 6 + r] += a1[r] * T1[j];
        else if (r == 3) acc[j * 6 + r] += a0[r] * T0[j];
        else acc[j * 6 + r] += a0[r] * T0[j] + a1[r] * T1[j];
      }
  }
}
// The KX pair loop with a per-task lane map (gmap, built with the batches): lane pair (group) g of the task owns columns
// 3 hi .. 3 hi + 2 of slot gs's block over the slot's pairs p = gk, gk + gn, ... of each batch (gn groups per slot, in
// proportion to the slot's pairs in the task: a batch's pair loop lasts as long as its slowest group)
__device__ __forceinline__ void schur_pairs_kx_g(const double* Gs, const int* sp, const int* spp, int gs, int gk, int gn,
                                                 bool hi, double (&acc)[18]) {
  constexpr int GB = 10;
  const int p1 = spp[gs + 1];
  for (int p = spp[gs] + gk; p < p1; p += gn) {
    const int pr = sp[p];
    const double* ga = &Gs[(pr & 0xffff) * GB];
    const double* gb = &Gs[(pr >> 16) * GB];
    double ka[6], kb[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double2 x = *reinterpret_cast<const double2*>(ga + 2 * k);
      const double2 y = *reinterpret_cast<const double2*>(gb + 2 * k);
      ka[2 * k] = x.x; ka[2 * k + 1] = x.y;
      kb[2 * k] = y.x; kb[2 * k + 1] = y.y;
    }
    const double2 ua2 = *reinterpret_cast<const double2*>(ga + 6), ub2 = *reinterpret_cast<const double2*>(gb + 6);
    const double ua = ua2.x, va = ua2.y, wa = ga[8], ub = ub2.x, vb = ub2.y, wb = gb[8];
    double M[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 2; ++q) M[r][q] = ka[r] * kb[q] + ka[2 + r] * kb[2 + q] + ka[4 + r] * kb[4 + q];
    double b0[3], b1[3];
    if (!hi) {
      b0[0] = ub * vb; b0[1] = -(1.0 + ub * ub); b0[2] = vb;
      b1[0] = 1.0 + vb * vb; b1[1] = -(ub * vb); b1[2] = -ub;
    } else {
      b0[0] = -wb; b0[1] = 0.0; b0[2] = ub * wb;
      b1[0] = 0.0; b1[1] = -wb; b1[2] = vb * wb;
    }
    double T0[3], T1[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      T0[j] = M[0][0] * b0[j] + M[0][1] * b1[j];
      T1[j] = M[1][0] * b0[j] + M[1][1] * b1[j];
    }
    const double a0[6] = {ua * va, -(1.0 + ua * ua), va, -wa, 0.0, ua * wa};
    const double a1[6] = {1.0 + va * va, -(ua * va), -ua, 0.0, -wa, va * wa};
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        if (r == 4) acc[j * 6 + r] += a1[r] * T1[j];
        else if (r == 3) acc[j * 6 + r] += a0[r] * T0[j];
        else acc[j * 6 + r] += a0[r] * T0[j] + a1[r] * T1[j];
      }
  }
}
// The grouped store: the gn groups of a slot add their sums in group order (through LDS, one column half at a time, red:
// >= 128 x 18 doubles of free LDS), the slot's first group stores S(i, j) = Hpp(i, j) - sum (or the part block)
__device__ __forceinline__ void schur_row_store_g(const double (&acc)[18], int gs, int gk, int gn, int noff, int soff,
                                                  const int* s_hpp, const double* Hpp, double* S, int pidx, double* part,
                                                  double* red) {
  const int tid = threadIdx.x, g = tid >> 1, hi = tid & 1;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
    if (hi == h) {
#pragma unroll
      for (int e = 0; e < 18; ++e) red[g * 18 + e] = acc[e];
    }
    __syncthreads();
    if (hi == h && gk == 0 && gs < noff) {
      double sum[18];
#pragma unroll
      for (int e = 0; e < 18; ++e) sum[e] = red[g * 18 + e];
      for (int k = 1; k < gn; ++k)
#pragma unroll
        for (int e = 0; e < 18; ++e) sum[e] += red[(g + k) * 18 + e];
      const int c0 = 3 * h;
      if (pidx > 0) {
        double* Po = part + (size_t)(pidx - 1 + gs) * 36;
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int r = 0; r < 6; ++r) Po[(c0 + j) * 6 + r] = sum[j * 6 + r];
      } else {
        const int sidx = soff + gs;
        const int hp = s_hpp[sidx];
        const double* Hh = Hpp + (size_t)(hp >= 0 ? hp : 0) * 36;
        double* So = S + (size_t)sidx * 36;
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int r = 0; r < 6; ++r) {
            const int k = (c0 + j) * 6 + r;
            So[k] = (hp >= 0 ? Hh[k] : 0.0) - sum[j * 6 + r];
          }
      }
    }
  }
}
// Even + odd pairs (fixed order) and the S block store: thread (h, par) stores rows [0, CW) (par 0) or [CW, PD) (par 1)
// of its columns; S(i, j) = Hpp(i, j) - sum
// pidx > 0 (one part of a split row chunk): the part's sums go to part blocks pidx - 1 + ls, not S (k_schur_part_sum)
template <int PD>
__device__ __forceinline__ void schur_row_store(double (&acc)[((PD + 1) / 2) * PD], int ls, int q, int noff, int soff,
                                                const int* s_hpp, const double* Hpp, double* S, int pidx = 0,
                                                double* part = nullptr) {
  constexpr int CW = (PD + 1) / 2;
  const int c0 = (q & 1) * CW, par = q >> 1;
#pragma unroll
  for (int k = 0; k < CW * PD; ++k) acc[k] += __shfl_xor(acc[k], 2, 4);
  if (ls < noff && pidx > 0) {
    double* Po = part + (size_t)(pidx - 1 + ls) * PD * PD;
#pragma unroll
    for (int j = 0; j < CW; ++j)
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        if ((r >= CW) != (par == 1)) continue;
        if (PD % 2 != 0 && c0 + j >= PD) continue;
        Po[(c0 + j) * PD + r] = acc[j * PD + r];
      }
    return;
  }
  if (ls < noff) {
    const int sidx = soff + ls;
    const int hp = s_hpp[sidx];
    const double* Hh = Hpp + (size_t)(hp >= 0 ? hp : 0) * PD * PD;
    double* So = S + (size_t)sidx * PD * PD;
#pragma unroll
    for (int j = 0; j < CW; ++j)
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        if ((r >= CW) != (par == 1)) continue;
        if (PD % 2 != 0 && c0 + j >= PD) continue;
        const int k = (c0 + j) * PD + r;
        So[k] = (hp >= 0 ? Hh[k] : 0.0) - acc[j * PD + r];
      }
  }
}

// Off-diagonal blocks, row-stationary (block_solver.hpp:361-391, j > i): one workgroup per (camera
// row i, chunk of up to 64 off-diagonal slots of the row's Schur pattern). The row's landmarks are
// walked in landmark order in batches; a batch stages the G blocks (G = Hpl U^-T, written once per
// observation by k_schur_diag, in camera-row order) of the row's own observation a = (l, i) and of
// its partners (l, j), j > i, into LDS by LDS-DMA
// (global_load_lds_dwordx4: 1 KiB lane-linear per wave instruction, no register staging). Two LDS
// buffers: batch k+1 lands while batch k is reduced. Four threads per slot, each half of the block's
// columns over every second pair of the slot's list (landmark order), the two parities combined by
// one fixed shuffle: every output has one owner and a fixed summation order (no atomics, bitwise
// reproducible).
namespace {
constexpr int SCH_SL = launch::SCHUR_SL;  // off-diagonal slots per task
constexpr int SCH_PPB = SCH_SL + 1;       // slot-CSR entries per batch
}  // namespace

// PIPE 1 (default): three index buffers, so a batch's indices are loaded one whole iteration before they are stored to
// LDS, and one raw barrier per batch that waits only for the batch's G blocks (counted vmcnt: the younger index loads
// stay in flight); PIPE 0: two index buffers, the index loads drained by each batch's __syncthreads
// (G2OHIP_SCHUR_PIPE=0, A/B). A variant issuing the next batch's staging right after the barrier and storing the
// indices behind the products (two register sets, the staging as inline assembly) measured the same (C4 142 vs 139 us,
// profiles/r04_ab_schur_pipe2.log) and was dropped.
// SCH_SB: staged blocks per batch (launch::SCHUR_SB for G blocks, launch::SCHUR_SB_KX for the 80-byte Kt records)
template <int PD, int LD, int PIPE, bool KX = false, int SCH_SB = launch::SCHUR_SB, int OCC = 4>
__global__ void __launch_bounds__(256, OCC)
    k_schur_rows(const launch::SchurTask* __restrict__ tasks, const launch::SchurBatch* __restrict__ batches,
                 const int* st_obs, const int* pairs, const int* pp,
                 const double* __restrict__ G, const int* __restrict__ s_hpp, const double* __restrict__ Hpp,
                 double* __restrict__ S, int mode, int ntasks, const long long* __restrict__ zr,
                 double* __restrict__ fronts, double* __restrict__ part, const int* __restrict__ gmap) {
  static_assert(!KX || (PD == 6 && LD == 3), "Kt records: BA blocks");
  constexpr int SCH_NI = (SCH_SB + 255) / 256;
  constexpr int GB = KX ? 10 : PD * LD;              // doubles per staged block: G, PD x LD col-major (or a Kt record)
  constexpr int NPC = GB / 2;                        // 16-B pieces per block
  constexpr int NC = (SCH_SB * NPC + 255) / 256;     // 16-B pieces per thread per batch
  constexpr int CW = (PD + 1) / 2;                   // output columns (and rows) per half
  static_assert(SCH_SB * NPC % 64 == 0, "a wave's LDS-DMA pieces must tile the batch image");
  __shared__ __attribute__((aligned(16))) double Gs[2][SCH_SB * GB];
  constexpr int NIB = PIPE ? 3 : 2;  // index buffers
  __shared__ int so[NIB][SCH_SB];  // staged observation per block
  __shared__ int sp[NIB][SCH_SB];  // pair lists (posA | posB << 16), slot-sorted
  __shared__ int spp[NIB][SCH_PPB];
  if ((int)blockIdx.x >= ntasks) {  // side job: zero one range of the factorization's front pool
    const long long off = zr[2 * (blockIdx.x - ntasks)], len = zr[2 * (blockIdx.x - ntasks) + 1];
    for (long long i = threadIdx.x; i < len; i += 256) fronts[off + i] = 0.0;
    return;
  }
  const int tix = xcd_item(blockIdx.x, ntasks);  // XCD-contiguous rows
  const launch::SchurTask t = tasks[tix];
  // KX: the task's lane map (slot, index among the slot's groups, groups of the slot) for this thread's lane pair
  int gs = 0, gk = 0, gn = 1;
  if constexpr (KX) {
    const int gm = gmap[(size_t)tix * 128 + (threadIdx.x >> 1)];
    gs = gm & 0xff;
    gk = (gm >> 8) & 0xff;
    gn = gm >> 16;
  }
  const int nb = t.b1 - t.b0;
  const int tid = threadIdx.x, w = tid >> 6;
  const int ls = tid >> 2, q = tid & 3;
  double acc[CW * PD];  // columns c0 .. c0 + CW - 1 of the block, all PD rows
#pragma unroll
  for (int k = 0; k < CW * PD; ++k) acc[k] = 0.0;
  // records past the task's end read the next task's (or the trailing dummy) record and go unused
  auto rec = [&](int k) { return batches[t.b0 + min(k, nb)]; };
  int ov[SCH_NI], pv[SCH_NI], ppv = 0;
  auto idx_load = [&](const launch::SchurBatch B, int k) {
#pragma unroll
    for (int u = 0; u < SCH_NI; ++u) {
      const int i = tid + 256 * u;
      ov[u] = ld0(st_obs, B.st0 + i, i < B.nst);
      pv[u] = ld0(pairs, B.pr0 + i, i < B.npr);
    }
    ppv = ld0(pp, (t.b0 + k) * SCH_PPB + tid, tid < SCH_PPB) - B.pr0;
  };
  auto idx_store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < SCH_NI; ++u) {
      const int i = tid + 256 * u;
      if (i < SCH_SB) { so[buf][i] = ov[u]; sp[buf][i] = pv[u]; }
    }
    if (tid < SCH_PPB) spp[buf][tid] = ppv;
  };
  auto stage = [&](const launch::SchurBatch B, int buf, int ib) {  // so[ib] holds B's observations
    const int np = B.nst * NPC;
#pragma unroll
    for (int u = 0; u < NC; ++u) {
      const int i = tid + 256 * u;
      if (i < np) {
        const int item = i / NPC, ch = i - item * NPC;
        __builtin_amdgcn_global_load_lds(
            (const void*)(G + (size_t)so[ib][item] * GB + 2 * ch),
            (__attribute__((address_space(3))) void*)(&Gs[buf][(256 * u + 64 * w) * 2]), 16, 0, 0);
      }
    }
  };
  auto compute = [&](int buf, int ib) {
    if constexpr (KX) schur_pairs_kx_g(Gs[buf], sp[ib], spp[ib], gs, gk, gn, threadIdx.x & 1, acc);
    else schur_pairs<PD, LD>(Gs[buf], sp[ib], spp[ib], t.noff, ls, q, acc);
  };
  // index loads the pipelined passes count with vmcnt. Their pointers are not __restrict__ and every counted wait is
  // an inline-assembly memory clobber, so the compiler can neither sink them below the wait nor hoist them above the
  // staging (read-only restrict loads may move across assembly and barriers).
  auto vld = [](const int* p) { return *p; };

  if constexpr (PIPE == 1) {
    // Invariant at the top of iteration k: Gs[k&1] holds batch k (landed), index buffers k%3 and (k+1)%3 hold batches
    // k and k+1 (visible), ov / pv / ppv hold batch k+2's indices (loads issued during iteration k-1, the youngest
    // vector-memory operations then), B1 / B3 the records k+1 / k+3.
    // The index loads are raw (clamped addresses, no select on the loaded value: a select right behind the load would
    // wait for it); entries past the batch's counts are never read, and the slot CSR is rebased at the store.
    // vector loads of one idx_load3: SCH_NI of st_obs + SCH_NI of pairs + 1 of the slot CSR, all unconditional (clamped
    // addresses). The counted waits below rely on exactly this count: a change to idx_load3 must change NIDX with it
    // (the batch records rec() are uniform scalar loads and do not count). Checked against PIPE 0 bitwise by
    // tests/test_gpu_parity.py::test_schur_rows_pipe_bitwise.
    constexpr int NIDX = 2 * SCH_NI + 1;
    int rpr0 = 0;
    auto idx_load3 = [&](const launch::SchurBatch B, int k) {
#pragma unroll
      for (int u = 0; u < SCH_NI; ++u) {
        const int i = tid + 256 * u;
        ov[u] = vld(st_obs + (i < B.nst ? B.st0 + i : 0));
        pv[u] = vld(pairs + (i < B.npr ? B.pr0 + i : 0));
      }
      ppv = vld(pp + (tid < SCH_PPB ? (t.b0 + k) * SCH_PPB + tid : 0));
      rpr0 = B.pr0;
    };
    auto idx_store3 = [&](int buf) {
#pragma unroll
      for (int u = 0; u < SCH_NI; ++u) {
        const int i = tid + 256 * u;
        if (i < SCH_SB) { so[buf][i] = ov[u]; sp[buf][i] = pv[u]; }
      }
      if (tid < SCH_PPB) spp[buf][tid] = ppv - rpr0;
    };
    launch::SchurBatch B1 = rec(1), B2 = rec(2), B3 = rec(3);
    if (nb > 0) {
      idx_load3(rec(0), 0);
      idx_store3(0);
      if (nb > 1) {
        idx_load3(B1, 1);
        idx_store3(1);
      }
      __syncthreads();  // so[0], so[1] visible
      if (!(mode & 2)) stage(rec(0), 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (nb > 2) {
        idx_load3(B2, 2);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIDX) : "memory");  // batch 0 landed, batch 2's indices in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int k = 0; k < nb; ++k) {
      const int cur = k & 1, i0 = k % 3, i1 = (k + 1) % 3, i2 = (k + 2) % 3;
      // buffer i2 last held batch k-1 (its reads ended before the last barrier); stale values past the task's last
      // batch are never read. The wait (vmcnt(0): the previous iteration's index loads, the only vector-memory
      // operations in flight here) is explicit and compiler-visible so that no wave's path keeps those loads
      // outstanding into the next index loads (which would make the compiler drain the G staging before them).
      __builtin_amdgcn_s_waitcnt(0x0F70);
      idx_store3(i2);
      if (k + 1 < nb && !(mode & 2)) stage(B1, cur ^ 1, i1);
      __builtin_amdgcn_sched_barrier(0);
      const bool more = k + 3 < nb;
      if (more) idx_load3(B3, k + 3);
      __builtin_amdgcn_sched_barrier(0);
      const launch::SchurBatch B4 = rec(k + 4);
      if (!(mode & 1)) compute(cur, i0);
      __builtin_amdgcn_sched_barrier(0);
      if (more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIDX) : "memory");  // batch k+1's G blocks landed
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // batch k+2's indices visible, Gs[cur] / buffer i0 free
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      B1 = B2;
      B2 = B3;
      B3 = B4;
    }
    if constexpr (KX) schur_row_store_g(acc, gs, gk, gn, t.noff, t.soff, s_hpp, Hpp, S, t.pad, part, &Gs[0][0]);
    else schur_row_store<PD>(acc, ls, q, t.noff, t.soff, s_hpp, Hpp, S, t.pad, part);
    return;
  }

  // Invariant at the top of iteration k: Gs[k&1] holds batch k (landed), so/sp/spp[k&1] its indices
  // and pair list, so/sp/spp[(k+1)&1] those of batch k+1; B1, B2 = records k+1, k+2 (already landed:
  // every record is loaded one iteration ahead, before a barrier that drains it).
  launch::SchurBatch B1 = rec(1), B2 = rec(2);
  if (nb > 0) {
    idx_load(rec(0), 0);
    idx_store(0);
    if (nb > 1) idx_load(B1, 1);
    __syncthreads();  // so[0] visible
    if (!(mode & 2)) stage(rec(0), 0, 0);
    if (nb > 1) idx_store(1);
    __syncthreads();  // batch 0 landed (the barrier drains the DMA), so[1] visible
  }
  for (int k = 0; k < nb; ++k) {
    const int cur = k & 1;
    if (k + 1 < nb && !(mode & 2)) stage(B1, cur ^ 1, cur ^ 1);
    if (k + 2 < nb) idx_load(B2, k + 2);
    const launch::SchurBatch B3 = rec(k + 3);
    if (!(mode & 1)) compute(cur, cur);
    __syncthreads();  // batch k+1 landed; Gs, so, sp, spp [cur] free
    if (k + 2 < nb) {
      idx_store(cur);
      __syncthreads();
    }
    B1 = B2;
    B2 = B3;
  }
  if constexpr (KX) schur_row_store_g(acc, gs, gk, gn, t.noff, t.soff, s_hpp, Hpp, S, t.pad, part, &Gs[0][0]);
  else schur_row_store<PD>(acc, ls, q, t.noff, t.soff, s_hpp, Hpp, S, t.pad, part);
}

// back-substitution: x_l = Dinv_l (b_l - sum_a Hpl_a^T x_pose(a)); LANES lanes per landmark stride over
// its observations, combined by a fixed butterfly (bitwise reproducible)
template <int PD, int LD, int LANES>
__global__ void __launch_bounds__(256)
    k_backsub(int nl, const int* __restrict__ lm_ptr, const int* __restrict__ blk_pose, const double* __restrict__ Hpl,
              const double* __restrict__ Dinv, const double* __restrict__ b, int size_poses, int lm0,
              double* __restrict__ x) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = gid / LANES, q = gid % LANES;  // local landmark; global index lm0 + l
  const bool active = l < nl;
  double c[LD];
#pragma unroll
  for (int k = 0; k < LD; ++k) c[k] = 0.0;
  if (active) {
    const int a1 = lm_ptr[l + 1];
    for (int a = lm_ptr[l] + q; a < a1; a += LANES) {
      const double* Bm = Hpl + (size_t)a * PD * LD;
      const double* xp = x + (size_t)blk_pose[a] * PD;
      double s[LD];
#pragma unroll
      for (int k = 0; k < LD; ++k) s[k] = 0.0;
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        const double xr = -xp[r];
#pragma unroll
        for (int k = 0; k < LD; ++k) s[k] += Bm[k * PD + r] * xr;
      }
#pragma unroll
      for (int k = 0; k < LD; ++k) c[k] += s[k];
    }
  }
#pragma unroll
  for (int m = LANES / 2; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < LD; ++k) c[k] += __shfl_xor(c[k], m, LANES);
  if (!active || q != 0) return;
  const double* bl = b + size_poses + (size_t)(lm0 + l) * LD;
#pragma unroll
  for (int k = 0; k < LD; ++k) c[k] += bl[k];
  const double* D = Dinv + (size_t)l * LD * LD;
  double* xl = x + size_poses + (size_t)(lm0 + l) * LD;
#pragma unroll
  for (int r = 0; r < LD; ++r) {
    double s = D[r] * c[0];
#pragma unroll
    for (int k = 1; k < LD; ++k) s += D[k * LD + r] * c[k];
    xl[r] = s;
  }
}

// the same from the symmetric split of a Schur pass whose G blocks were formed at assembly (G = Hpl U^-T stored in
// place of Hpl, same block order): Dinv (b_l - Hpl^T x_p) = U^-T (c_l - G^T x_p), c_l = U^-1 b_l
template <int PD, int LD, int LANES>
__global__ void __launch_bounds__(256)
    k_backsub_g(int nl, const int* __restrict__ lm_ptr, const int* __restrict__ blk_pose, const double* __restrict__ G,
                const double* __restrict__ Ufac, const double* __restrict__ cl_all, int size_poses, int lm0,
                double* __restrict__ x) {
  constexpr int UF = LmTraits<LD>::UF;
  constexpr int GB = PD * LD, GP = GB / 2;  // doubles / 16-B pieces per block
  constexpr int CH = 32;                    // blocks per staged chunk (per wave)
  static_assert(GB % 2 == 0, "blocks are whole 16-B pieces");
  // A wave's landmarks own one contiguous run of G blocks (Hpl order is landmark-major). The run is staged through
  // the wave's LDS slice in lane-linear 16-B pieces (1 KiB per load instruction): a lane reading its own 144-B blocks
  // directly touches a different cache line per lane and piece, and refetches lines from L2 many times (C5 422 -> 362
  // us; prefetching the next chunk into registers measured no faster at half the occupancy).
  __shared__ __attribute__((aligned(16))) double2 gs[4][CH * GP];
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = gid / LANES, q = gid % LANES, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lw0 = (gid - lane) / LANES;  // the wave's first landmark
  if (lw0 >= nl) return;                 // wave-uniform
  const bool active = l < nl;
  const int A0 = lm_ptr[lw0], A1 = lm_ptr[min(lw0 + 64 / LANES, nl)];
  int a = active ? lm_ptr[l] + q : 0;
  const int ae = active ? lm_ptr[l + 1] : 0;
  double c[LD];
#pragma unroll
  for (int k = 0; k < LD; ++k) c[k] = 0.0;
  double2* gw = gs[w];
  for (int c0 = A0; c0 < A1; c0 += CH) {  // wave-uniform chunks; a lane's cursor stays in observation order
    const int n = min(CH, A1 - c0);
    const double2* src = reinterpret_cast<const double2*>(G + (size_t)c0 * GB);
    __builtin_amdgcn_wave_barrier();  // every lane's reads of the previous chunk precede these writes (LDS in order)
    asm volatile("" ::: "memory");
    for (int i = lane; i < n * GP; i += 64) gw[i] = src[i];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    for (; a < ae && a < c0 + n; a += LANES) {
      const double2* Bm = gw + (a - c0) * GP;
      const double* xp = x + (size_t)blk_pose[a] * PD;
      double bv[GB], s[LD];
#pragma unroll
      for (int i = 0; i < GP; ++i) { const double2 v = Bm[i]; bv[2 * i] = v.x; bv[2 * i + 1] = v.y; }
#pragma unroll
      for (int k = 0; k < LD; ++k) s[k] = 0.0;
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        const double xr = -xp[r];
#pragma unroll
        for (int k = 0; k < LD; ++k) s[k] += bv[k * PD + r] * xr;
      }
#pragma unroll
      for (int k = 0; k < LD; ++k) c[k] += s[k];
    }
  }
#pragma unroll
  for (int m = LANES / 2; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < LD; ++k) c[k] += __shfl_xor(c[k], m, LANES);
  if (!active || q != 0) return;
  const double* cl = cl_all + (size_t)(lm0 + l) * LD;
  const double* U = Ufac + (size_t)l * UF;
#pragma unroll
  for (int k = 0; k < LD; ++k) c[k] += cl[k];
  double* xl = x + size_poses + (size_t)(lm0 + l) * LD;
  if constexpr (LD == 3) {  // U^T x = y, U = [[1/r0, 0, 0], [u10, 1/r1, 0], [u20, u21, 1/r2]]
    const double x2 = c[2] * U[2];
    const double x1 = (c[1] - U[5] * x2) * U[1];
    const double x0 = (c[0] - U[3] * x1 - U[4] * x2) * U[0];
    xl[0] = x0; xl[1] = x1; xl[2] = x2;
  } else {
    const double x1 = c[1] * U[1];
    const double x0 = (c[0] - U[2] * x1) * U[0];
    xl[0] = x0; xl[1] = x1;
  }
}

// an edge's chi2 from its error: e^T Omega e, robustified to rho[0] (activeRobustChi2, sparse_optimizer.cpp:102-116)
template <class F>
__device__ __forceinline__ double edge_chi(const EdgeData& d, int e, const double* err) {
  double Om[F::D * F::D];
  load_info<F::D>(info_rec(d, e, F::INFO), Om);
  double c = 0;
#pragma unroll
  for (int i = 0; i < F::D; ++i) {
    double r = 0;
#pragma unroll
    for (int j = 0; j < F::D; ++j) r += Om[i * F::D + j] * err[j];
    c += err[i] * r;
  }
  if (d.rk) {
    double r0, r1;
    robustify(d.rk, d.rk_delta, c, r0, r1);
    c = r0;
  }
  return c;
}

// ------------------------------------------------------------------------------ oplus
__device__ __forceinline__ void d_oplus_se3expmap(int v, const int* __restrict__ xoff, const double* __restrict__ x,
                                            double* __restrict__ st, int* __restrict__ nopl) {
  if (xoff[v] < 0) return;
  const double* u = x + xoff[v];
  double uu[6] = {u[0], u[1], u[2], u[3], u[4], u[5]};
  double qe[4], te[3];
  se3_exp(uu, qe, te);
  double* s = st + (size_t)v * 8;
  const double q[4] = {s[3], s[4], s[5], s[6]};
  const double t[3] = {s[0], s[1], s[2]};
  double rt[3], qn[4];
  qrot(qe, t, rt);  // exp(u) * T : t' = te + qe * t, q' = qe * q
  qmul(qe, q, qn);
  qnormalize_pos(qn);
  s[0] = te[0] + rt[0]; s[1] = te[1] + rt[1]; s[2] = te[2] + rt[2];
  s[3] = qn[0]; s[4] = qn[1]; s[5] = qn[2]; s[6] = qn[3];
}

__device__ __forceinline__ void d_oplus_xyz(int v, const int* __restrict__ xoff, const double* __restrict__ x,
                                            double* __restrict__ st, int* __restrict__ nopl) {
  if (xoff[v] < 0) return;
  const double* u = x + xoff[v];
  double* s = st + (size_t)v * 3;
  s[0] += u[0]; s[1] += u[1]; s[2] += u[2];
}

__device__ __forceinline__ void d_oplus_se3quat(int v, const int* __restrict__ xoff, const double* __restrict__ x,
                                            double* __restrict__ st, int* __restrict__ nopl) {
  if (xoff[v] < 0) return;
  const double* u = x + xoff[v];
  // increment = fromVectorMQT(u) (isometry3d_mappings.cpp:106-111)
  double inc[12];
  const double qx = u[3], qy = u[4], qz = u[5];
  double w = 1 - (qx * qx + qy * qy + qz * qz);
  if (w < 0) {
    inc[0] = 1; inc[1] = 0; inc[2] = 0; inc[3] = 0; inc[4] = 1; inc[5] = 0; inc[6] = 0; inc[7] = 0; inc[8] = 1;
  } else {
    w = sqrt(w);
    quat_to_R(qx, qy, qz, w, inc);
  }
  inc[9] = u[0]; inc[10] = u[1]; inc[11] = u[2];
  double* s = st + (size_t)v * 12;
  double X[12], Y[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) X[k] = s[k];
  iso_mul(X, inc, Y);
  if (++nopl[v] > 1000) {  // vertex_se3.h:110-113 approximateNearestOrthogonalMatrix
    nopl[v] = 0;
    double E[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) E[i * 3 + j] = Y[i] * Y[j] + Y[3 + i] * Y[3 + j] + Y[6 + i] * Y[6 + j] - (i == j ? 1.0 : 0.0);
    double RE[9];
    mat3mul(Y, E, RE);
#pragma unroll
    for (int k = 0; k < 9; ++k) Y[k] = Y[k] - 0.5 * RE[k];
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) s[k] = Y[k];
}

__device__ __forceinline__ void d_oplus_se2(int v, const int* __restrict__ xoff, const double* __restrict__ x,
                                            double* __restrict__ st, int* __restrict__ nopl) {
  if (xoff[v] < 0) return;
  const double* u = x + xoff[v];
  double* s = st + (size_t)v * 3;
  s[0] += u[0];
  s[1] += u[1];
  s[2] = normalize_theta(s[2] + u[2]);
}

__device__ __forceinline__ void d_oplus_xy(int v, const int* __restrict__ xoff, const double* __restrict__ x,
                                            double* __restrict__ st, int* __restrict__ nopl) {  // vertex_point_xy.h:77-81
  if (xoff[v] < 0) return;
  const double* u = x + xoff[v];
  double* s = st + (size_t)v * 2;
  s[0] += u[0];
  s[1] += u[1];
}

// SparseOptimizer::update (sparse_optimizer.cpp:441-454) over every vertex type in one launch: block ranges per type
__global__ void __launch_bounds__(256) k_oplus_multi(launch::OplusList L, const double* __restrict__ x) {
  int t = 0;
  while (t + 1 < L.cnt && (int)blockIdx.x >= L.blk0[t + 1]) ++t;
  const int v = ((int)blockIdx.x - L.blk0[t]) * 256 + threadIdx.x;
  if (v >= L.n[t]) return;
  switch (L.vt[t]) {
    case 1: d_oplus_se3expmap(v, L.xoff[t], x, L.st[t], L.nopl); break;
    case 2: d_oplus_xyz(v, L.xoff[t], x, L.st[t], L.nopl); break;
    case 3: d_oplus_se3quat(v, L.xoff[t], x, L.st[t], L.nopl); break;
    case 4: d_oplus_se2(v, L.xoff[t], x, L.st[t], L.nopl); break;
    case 5: d_oplus_xy(v, L.xoff[t], x, L.st[t], L.nopl); break;
  }
}

// ------------------------------------------------------------------------------ reductions
// Deterministic two-pass sum: fixed chunking, fixed tree.
constexpr int RED_BLOCK = 256;
constexpr int RED_PER_THREAD = 16;

__global__ void __launch_bounds__(RED_BLOCK) k_sum_partial(const double* __restrict__ v, long long n,
                                                           double* __restrict__ partial) {
  __shared__ double sh[RED_BLOCK];
  const long long base = (long long)blockIdx.x * RED_BLOCK * RED_PER_THREAD;
  double s = 0;
#pragma unroll
  for (int k = 0; k < RED_PER_THREAD; ++k) {
    const long long i = base + (long long)k * RED_BLOCK + threadIdx.x;
    if (i < n) s += v[i];
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

__global__ void __launch_bounds__(RED_BLOCK) k_sum_final(const double* __restrict__ partial, int np,
                                                         double* __restrict__ out) {
  __shared__ double sh[RED_BLOCK];
  double s = 0;
  for (int i = threadIdx.x; i < np; i += RED_BLOCK) s += partial[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

// scale terms of OptimizationAlgorithmLevenberg::computeScale (:177-184): x (lambda x + b)
__global__ void k_scale_terms(long long n, const double* __restrict__ x, const double* __restrict__ b,
                              const double* __restrict__ lam, double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double l = *lam;
  out[i] = x[i] * (l * x[i] + b[i]);
}

// one thread's RED_PER_THREAD edges of a chi2 chunk, summed in edge order into s: the edges' errors are formed in groups
// of four with every index and state load of a group in flight together (a guarded edge per iteration cost two dependent
// round trips each, 32 per thread: the whole kernel time at C4); edges past ne read edge 0 and are not added
template <class F>
__device__ __forceinline__ void error_chunk_sum(const EdgeData& d, int ne, long long base, double& s) {
  constexpr int GK = 4;
#pragma unroll 1  // (the group loop stays rolled: unrolled, every family's instance was 4x the code)
  for (int k0 = 0; k0 < RED_PER_THREAD; k0 += GK) {
    double err[GK][F::D];
#pragma unroll
    for (int u = 0; u < GK; ++u) {  // errors first (no branches: the group's loads can interleave)
      const long long e = base + (long long)(k0 + u) * RED_BLOCK + threadIdx.x;
      F::error(d, e < ne ? (int)e : 0, err[u]);
    }
#pragma unroll
    for (int u = 0; u < GK; ++u) {  // then the (robustified) chi2 terms in edge order
      const long long e = base + (long long)(k0 + u) * RED_BLOCK + threadIdx.x;
      const double c = edge_chi<F>(d, e < ne ? (int)e : 0, err[u]);
      if (e < ne) s += c;
    }
  }
}

// computeActiveErrors + activeRobustChi2 fused with the first pass of the deterministic sum: the
// same fixed chunking and tree as k_sum_partial over a chi2 array, without the array
template <class F>
__global__ void __launch_bounds__(RED_BLOCK) k_error_partial(EdgeData d, int ne, double* __restrict__ partial) {
  __shared__ double sh[RED_BLOCK];
  const long long base = (long long)blockIdx.x * RED_BLOCK * RED_PER_THREAD;
  double s = 0;
  error_chunk_sum<F>(d, ne, base, s);
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

// computeActiveErrors (one edge group) and computeScale in one launch: blocks [0, npe) are k_error_partial's
// chunks, the rest k_scale_partial's (same chunking and trees: the same sums bit for bit); k_sum_final2 finishes both
template <class F>
__global__ void __launch_bounds__(RED_BLOCK) k_error_scale_partial(EdgeData d, int ne, int npe, long long n,
                                                                   long long npose, const double* __restrict__ x,
                                                                   const double* __restrict__ b,
                                                                   const double* __restrict__ lam,
                                                                   double* __restrict__ partial) {
  __shared__ double sh[RED_BLOCK];
  double s = 0;
  if ((int)blockIdx.x < npe) {
    error_chunk_sum<F>(d, ne, (long long)blockIdx.x * RED_BLOCK * RED_PER_THREAD, s);
  } else {
    const double lp = lam[4], ll = lam[0];
    const long long base = (long long)(blockIdx.x - npe) * RED_BLOCK * RED_PER_THREAD;
    // every load of the chunk issued before the first term (a guarded load per term was a round trip each)
    double xv[RED_PER_THREAD], bv[RED_PER_THREAD];
#pragma unroll
    for (int k = 0; k < RED_PER_THREAD; ++k) {
      const long long i = base + (long long)k * RED_BLOCK + threadIdx.x;
      xv[k] = x[i < n ? i : 0];
      bv[k] = b[i < n ? i : 0];
    }
#pragma unroll
    for (int k = 0; k < RED_PER_THREAD; ++k) {
      const long long i = base + (long long)k * RED_BLOCK + threadIdx.x;
      if (i < n) {
        const double l = i < npose ? lp : ll;
        s += xv[k] * (l * xv[k] + bv[k]);
      }
    }
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}
// two k_sum_final in one launch: block 0 sums partial[0, n0) into out0, block 1 partial[n0, n0 + n1) into out1
__global__ void __launch_bounds__(RED_BLOCK) k_sum_final2(const double* __restrict__ partial, int n0, int n1,
                                                          double* __restrict__ out0, double* __restrict__ out1) {
  __shared__ double sh[RED_BLOCK];
  const double* p = blockIdx.x == 0 ? partial : partial + n0;
  const int np = blockIdx.x == 0 ? n0 : n1;
  double s = 0;
  for (int i = threadIdx.x; i < np; i += RED_BLOCK) s += p[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) *(blockIdx.x == 0 ? out0 : out1) = sh[0];
}
__device__ __forceinline__ void lm_decide_body(double* __restrict__ p, double current_chi, double ni, int rank0) {
  int f;
  __builtin_memcpy(&f, p + 8, sizeof f);
  const double temp = f == 0 ? p[1] : __DBL_MAX__;
  double rho = current_chi - temp;
  double scale = p[2];
  scale += 1e-3;
  rho /= scale;
  const double lam = p[0];
  double nl, acc;
  if (rho > 0 && isfinite(temp)) {
    nl = lam * lm_scale_factor(rho);
    acc = 1.0;
  } else {
    nl = lam * ni;
    acc = 0.0;
  }
  p[12] = nl;
  p[13] = rank0 ? nl : 0.0;
  p[14] = acc;
  p[15] = rho;
}
__global__ void k_lm_decide(double* __restrict__ p, double current_chi, double ni, int rank0) {
  lm_decide_body(p, current_chi, ni, rank0);
}
// one rank: k_sum_final2's two sums (the same order, one after the other in one workgroup) into p[1] (chi2) and p[2]
// (scale), then the trial decision on them (one launch less per LM trial); an accepted trial also gets the loop's
// closing restoreDiagonal (lambda 0), which the host then skips
__global__ void __launch_bounds__(RED_BLOCK) k_sum_final2_decide(const double* __restrict__ partial, int n0, int n1,
                                                                 double* __restrict__ p, double current_chi, double ni,
                                                                 int rank0, double* host_out) {
  __shared__ double sh[RED_BLOCK];
  for (int q = 0; q < 2; ++q) {
    const double* pp = q == 0 ? partial : partial + n0;
    const int np = q == 0 ? n0 : n1;
    double s = 0;
    for (int i = threadIdx.x; i < np; i += RED_BLOCK) s += pp[i];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
      if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
      __syncthreads();
    }
    if (threadIdx.x == 0) p[1 + q] = sh[0];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    lm_decide_body(p, current_chi, ni, rank0);
    if (p[14] != 0.0) {  // accepted: the trial loop ends here, with restoreDiagonal (the host's set_lambda(0))
      p[0] = 0.0;
      p[4] = 0.0;
      p[5] = 0.0;
    }
    if (host_out)
      for (int k = 0; k < 16; ++k) host_out[k] = p[k];
  }
}

// computeScale (optimization_algorithm_levenberg.cpp:177-184) fused with the first sum pass:
// x (lambda x + b), lambda = lam[4] (rank-0 share) on the pose part, lam[0] on the landmark part
__global__ void __launch_bounds__(RED_BLOCK) k_scale_partial(long long n, long long npose, const double* __restrict__ x,
                                                             const double* __restrict__ b, const double* __restrict__ lam,
                                                             double* __restrict__ partial) {
  __shared__ double sh[RED_BLOCK];
  const double lp = lam[4], ll = lam[0];
  const long long base = (long long)blockIdx.x * RED_BLOCK * RED_PER_THREAD;
  double s = 0;
#pragma unroll
  for (int k = 0; k < RED_PER_THREAD; ++k) {
    const long long i = base + (long long)k * RED_BLOCK + threadIdx.x;
    if (i < n) {
      const double l = i < npose ? lp : ll;
      s += x[i] * (l * x[i] + b[i]);
    }
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int m = RED_BLOCK / 2; m > 0; m >>= 1) {
    if ((int)threadIdx.x < m) sh[threadIdx.x] += sh[threadIdx.x + m];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}

// ------------------------------------------------------------------------------ symmetric block SpMV
// y = (A + lam I) x for A symmetric, stored as its upper blocks (pd x pd col-major): thread per scalar row,
// its block row's entries in a fixed order (rptr/ent: block index, other block row | 0x80000000 when the
// stored block is used transposed), as SparseBlockMatrix::multiplySymmetricUpperTriangle
// (sparse_block_matrix.hpp:289-314). With b: also (y - b)^2 and b^2 per row for the residual norm.
template <int PD>
__global__ void __launch_bounds__(256)
    k_block_symv(int n, const int* __restrict__ rptr, const int2* __restrict__ ent, const int* __restrict__ diag,
                 const double* __restrict__ vals, const double* __restrict__ lam, const double* __restrict__ x,
                 double* __restrict__ y, const double* __restrict__ b, double* __restrict__ r2,
                 double* __restrict__ b2) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  const int i = row / PD, rr = row - i * PD;
  const double* D = vals + (size_t)diag[i] * PD * PD;
  double acc = (lam ? *lam : 0.0) * x[row];
#pragma unroll
  for (int c = 0; c < PD; ++c) acc += D[c * PD + rr] * x[(size_t)i * PD + c];
  for (int e = rptr[i]; e < rptr[i + 1]; ++e) {
    const int2 t = ent[e];
    const int j = t.y & 0x7fffffff;
    const double* B = vals + (size_t)t.x * PD * PD;
    const double* xj = x + (size_t)j * PD;
    if (t.y < 0) {
#pragma unroll
      for (int c = 0; c < PD; ++c) acc += B[rr * PD + c] * xj[c];
    } else {
#pragma unroll
      for (int c = 0; c < PD; ++c) acc += B[c * PD + rr] * xj[c];
    }
  }
  if (y) y[row] = acc;
  if (b) {
    const double d = acc - b[row];
    r2[row] = d * d;
    b2[row] = b[row] * b[row];
  }
}

// ------------------------------------------------------------------------------ launchers
namespace launch {

static EdgeData mk(const EdgeArgs& a) {
  return EdgeData{a.v0, a.v1, a.meas, a.info, a.params, a.s0, a.s1, a.rk, a.rk_delta, a.ue};
}

// host-Jacobian families: runtime (D, DA, DB) -> FamilyHostJ<D, DA, DB> (vertex dims 2, 3 or 6, D = 1..6)
template <int D, int DA, class Fn>
static void hj_b(int DB, Fn& fn) {
  if (DB == 2) fn(FamilyHostJ<D, DA, 2>{});
  else if (DB == 3) fn(FamilyHostJ<D, DA, 3>{});
  else if (DB == 6) fn(FamilyHostJ<D, DA, 6>{});
  else throw std::runtime_error("host-Jacobian edge: vertex dimension must be 2, 3 or 6");
}
template <int D, class Fn>
static void hj_a(int DA, int DB, Fn& fn) {
  if (DA == 2) hj_b<D, 2>(DB, fn);
  else if (DA == 3) hj_b<D, 3>(DB, fn);
  else if (DA == 6) hj_b<D, 6>(DB, fn);
  else throw std::runtime_error("host-Jacobian edge: vertex dimension must be 2, 3 or 6");
}
template <class Fn>
static void family_dispatch(int family, const EdgeArgs& a, Fn&& fn) {
  switch (family) {
    case FAM_BA: fn(FamilyBA{}); break;
    case FAM_SE3: fn(FamilySE3{}); break;
    case FAM_SE2: fn(FamilySE2{}); break;
    case FAM_SE2XY: fn(FamilySE2XY{}); break;
    case FAM_HOSTJ:
      switch (a.D) {
        case 1: hj_a<1>(a.DA, a.DB, fn); break;
        case 2: hj_a<2>(a.DA, a.DB, fn); break;
        case 3: hj_a<3>(a.DA, a.DB, fn); break;
        case 4: hj_a<4>(a.DA, a.DB, fn); break;
        case 5: hj_a<5>(a.DA, a.DB, fn); break;
        case 6: hj_a<6>(a.DA, a.DB, fn); break;
        default: throw std::runtime_error("host-Jacobian edge: error dimension must be 1..6");
      }
      break;
    default: throw std::runtime_error("unknown edge family");
  }
}

void error(int family, const EdgeArgs& a, int ne, double* chi, hipStream_t s) {
  if (ne <= 0) return;
  const unsigned g = grid_for(ne, 256);
  family_dispatch(family, a, [&](auto fam) {
    using F = decltype(fam);
    hipLaunchKernelGGL(k_error<F>, g, 256, 0, s, mk(a), ne, chi);
  });
  KERNEL_CHECK();
}

void linearize(int family, const EdgeArgs& a, int ne, const int* h0, const int* h1, double* slot0, double* slot1,
               const long long* off_dst, const unsigned char* off_tr, double* off_base, double* off_slot, hipStream_t s) {
  if (ne <= 0) return;
  const unsigned g = grid_for(ne, 256);
  family_dispatch(family, a, [&](auto fam) {
    using F = decltype(fam);
    hipLaunchKernelGGL(k_linearize<F>, g, 256, 0, s, mk(a), ne, h0, h1, slot0, slot1, off_dst, off_tr, off_base,
                       off_slot);
  });
  KERNEL_CHECK();
}

static bool vr_wide() {
  static const bool w = !getenv("G2OHIP_VR_WIDE") || atoi(getenv("G2OHIP_VR_WIDE")) != 0;  // dev A/B
  return w;
}
template <int DIM>
static void vreduce_dim(int nv, int lanes, const int* ptr, const int* code, const double* slots, double* H, double* b,
                        const int* boff, hipStream_t s) {
  const unsigned g = grid_for((size_t)nv * lanes, 256);
  switch (lanes) {
    case 1: hipLaunchKernelGGL((k_vertex_reduce<DIM, 1>), g, 256, 0, s, nv, ptr, code, slots, H, b, boff); break;
    case 4: hipLaunchKernelGGL((k_vertex_reduce<DIM, 4>), g, 256, 0, s, nv, ptr, code, slots, H, b, boff); break;
    case 8: hipLaunchKernelGGL((k_vertex_reduce<DIM, 8>), g, 256, 0, s, nv, ptr, code, slots, H, b, boff); break;
    case 64:
      if (vr_wide())
        hipLaunchKernelGGL((k_vertex_reduce_wide<DIM>), nv, 256, 0, s, nv, ptr, code, slots, H, b, boff);
      else
        hipLaunchKernelGGL((k_vertex_reduce<DIM, 64>), g, 256, 0, s, nv, ptr, code, slots, H, b, boff);
      break;
    default: hipLaunchKernelGGL((k_vertex_reduce<DIM, 256>), g, 256, 0, s, nv, ptr, code, slots, H, b, boff); break;
  }
  KERNEL_CHECK();
}

void vertex_reduce(int dim, int nv, int lanes, const int* ptr, const int* code, const double* slots, double* H,
                   double* b, const int* boff, hipStream_t s) {
  if (nv <= 0) return;
  if (dim == 2) vreduce_dim<2>(nv, lanes, ptr, code, slots, H, b, boff, s);
  else if (dim == 3) vreduce_dim<3>(nv, lanes, ptr, code, slots, H, b, boff, s);
  else if (dim == 6) vreduce_dim<6>(nv, lanes, ptr, code, slots, H, b, boff, s);
  else throw std::runtime_error("vertex_reduce: unsupported dim");
}

void offblock_reduce(int nb, int bsz, const int* ptr, const long long* soff, const double* slots, double* out,
                     const long long* dst, hipStream_t s) {
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_offblock_reduce, grid_for((size_t)nb * bsz, 256), 256, 0, s, nb, bsz, ptr, soff, slots, out, dst);
  KERNEL_CHECK();
}

// (pose, landmark) block sizes with Schur kernels: BlockSolver_6_3 and BlockSolver_3_2
template <class Fn>
static void pl_dispatch(int pd, int ld, Fn&& fn) {
  if (pd == 6 && ld == 3) fn(std::integral_constant<int, 6>{}, std::integral_constant<int, 3>{});
  else if (pd == 3 && ld == 2) fn(std::integral_constant<int, 3>{}, std::integral_constant<int, 2>{});
  else throw std::runtime_error("Schur complement: (pose, landmark) dimensions must be (6, 3) or (3, 2)");
}
void schur_prep(int ld, int nl, int lm0, const double* Hll, const double* bl_all, const double* lam, double* Dinv,
                double* Ufac, double* cl_all, int* fail, hipStream_t s) {
  if (nl <= 0) return;
  if (ld == 3)
    hipLaunchKernelGGL(k_schur_prep<3>, grid_for(nl, 256), 256, 0, s, nl, lm0, Hll, bl_all, lam, Dinv, Ufac, cl_all, fail);
  else if (ld == 2)
    hipLaunchKernelGGL(k_schur_prep<2>, grid_for(nl, 256), 256, 0, s, nl, lm0, Hll, bl_all, lam, Dinv, Ufac, cl_all, fail);
  else
    throw std::runtime_error("schur_prep: landmark dimension must be 2 or 3");
  KERNEL_CHECK();
}
int schur_ufac_stride(int ld) { return ld == 3 ? LmTraits<3>::UF : LmTraits<2>::UF; }
void schur_diag(int pd, int ld, int nrows, const int* rptr, const int* robs, const int* obs_lm, int lm0,
                const double* Hpl, const double* Ufac, const double* cl_all, const int* sdiag, const int* s_hpp,
                const double* Hpp, const double* b, const double* lam, const unsigned char* lam_own,
                const double* lam_full, double* S, double* bschur, double* G, hipStream_t s) {
  if (nrows <= 0) return;
  pl_dispatch(pd, ld, [&](auto P, auto L) {
    hipLaunchKernelGGL((k_schur_diag<decltype(P)::value, decltype(L)::value>), nrows, 256, 0, s, nrows, rptr, robs,
                       obs_lm, lm0, Hpl, Ufac, cl_all, sdiag, s_hpp, Hpp, b, lam, lam_own, lam_full, S, bschur, G);
  });
  KERNEL_CHECK();
}
// S(soff + s) = Hpp - sum_p part(xo + p noff + s): one workgroup per group, parts summed in order
template <int PD>
__global__ void __launch_bounds__(256) k_schur_part_sum(const launch::SchurPartGroup* __restrict__ groups,
                                                        const double* __restrict__ part, const int* __restrict__ s_hpp,
                                                        const double* __restrict__ Hpp, double* __restrict__ S) {
  const launch::SchurPartGroup g = groups[blockIdx.x];
  constexpr int BB = PD * PD;
  for (int e = threadIdx.x; e < g.noff * BB; e += 256) {
    const int sl = e / BB, k = e - sl * BB;
    double sum = 0.0;
    for (int p = 0; p < g.np; ++p) sum += part[(size_t)(g.xo + p * g.noff + sl) * BB + k];
    const int sidx = g.soff + sl, hp = s_hpp[sidx];
    S[(size_t)sidx * BB + k] = (hp >= 0 ? Hpp[(size_t)hp * BB + k] : 0.0) - sum;
  }
}
void schur_part_sum(int pd, int ngroups, const SchurPartGroup* groups, const double* part, const int* s_hpp,
                    const double* Hpp, double* S, hipStream_t s) {
  if (ngroups <= 0) return;
  if (pd == 6) hipLaunchKernelGGL(k_schur_part_sum<6>, ngroups, 256, 0, s, groups, part, s_hpp, Hpp, S);
  else if (pd == 3) hipLaunchKernelGGL(k_schur_part_sum<3>, ngroups, 256, 0, s, groups, part, s_hpp, Hpp, S);
  else throw DeviceError("schur_part_sum: pose blocks of 3 or 6");
  KERNEL_CHECK();
}
void schur_rows(int pd, int ld, int ntasks, const SchurTask* tasks, const SchurBatch* batches, const int* st_obs,
                const int* pairs, const int* pp, const double* G, const int* s_hpp, const double* Hpp, double* S,
                int nzero, const long long* zr, double* fronts, hipStream_t s, bool kx, int sb, double* part,
                const int* gmap) {
  if (ntasks <= 0 && nzero <= 0) return;
#ifdef G2OHIP_DEV  // development build only: 1 no pair products, 2 no staging, 3 neither (wrong S, timing splits)
  static const int mode = getenv("G2OHIP_SCHUR_MODE") ? atoi(getenv("G2OHIP_SCHUR_MODE")) : 0;
#else
  constexpr int mode = 0;
#endif
  static EnvKnob pipe_k{"G2OHIP_SCHUR_PIPE", 1};  // 0: two index buffers (A/B; tests/test_gpu_parity.py)
  const int pipe = pipe_k.get();
  const int nz = nzero > 0 ? nzero : 0;
  if (kx) {  // BA split: G rebuilt from the Kt records
    if (pd != 6 || ld != 3) throw DeviceError("schur_rows: Kt records need BlockSolver_6_3 blocks");
    if (!gmap && ntasks > 0) throw DeviceError("schur_rows: Kt records need the tasks' lane map");
    // (108 VGPRs: four workgroups per CU; a register budget for five or six spills 8 / 35 VGPRs at 128-block batches)
    auto go = [&](auto SBc) {
      constexpr int SBK = decltype(SBc)::value;
      if (pipe == 0)
        hipLaunchKernelGGL((k_schur_rows<6, 3, 0, true, SBK>), ntasks + nz, 256, 0, s, tasks, batches, st_obs, pairs,
                           pp, G, s_hpp, Hpp, S, mode, ntasks, zr, fronts, part, gmap);
      else
        hipLaunchKernelGGL((k_schur_rows<6, 3, 1, true, SBK>), ntasks + nz, 256, 0, s, tasks, batches, st_obs, pairs,
                           pp, G, s_hpp, Hpp, S, mode, ntasks, zr, fronts, part, gmap);
    };
    if (sb == 128) go(std::integral_constant<int, 128>{});
    else if (sb == 192) go(std::integral_constant<int, 192>{});
    else if (sb == 256) go(std::integral_constant<int, 256>{});
    else throw DeviceError("schur_rows: unsupported Kt batch size " + std::to_string(sb));
    KERNEL_CHECK();
    return;
  }
  pl_dispatch(pd, ld, [&](auto P, auto L) {
    constexpr int pv = decltype(P)::value, lv = decltype(L)::value;
    if (pipe == 0)
      hipLaunchKernelGGL((k_schur_rows<pv, lv, 0>), ntasks + nz, 256, 0, s, tasks, batches, st_obs, pairs, pp, G, s_hpp,
                         Hpp, S, mode, ntasks, zr, fronts, part, gmap);
    else
      hipLaunchKernelGGL((k_schur_rows<pv, lv, 1>), ntasks + nz, 256, 0, s, tasks, batches, st_obs, pairs, pp, G, s_hpp,
                         Hpp, S, mode, ntasks, zr, fronts, part, gmap);
  });
  KERNEL_CHECK();
}
void backsub(int pd, int ld, int nl, const int* lm_ptr, const int* blk_pose, const double* Hpl, const double* Dinv,
             const double* b, int size_poses, int lm0, double* x, hipStream_t s) {
  if (nl <= 0) return;
  pl_dispatch(pd, ld, [&](auto P, auto L) {
    hipLaunchKernelGGL((k_backsub<decltype(P)::value, decltype(L)::value, 4>), grid_for((size_t)nl * 4, 256), 256, 0,
                       s, nl, lm_ptr, blk_pose, Hpl, Dinv, b, size_poses, lm0, x);
  });
  KERNEL_CHECK();
}
void backsub_g(int pd, int ld, int nl, const int* lm_ptr, const int* blk_pose, const double* G, const double* Ufac,
               const double* cl_all, int size_poses, int lm0, double* x, hipStream_t s) {
  if (nl <= 0) return;
  static EnvKnob lanes_k{"G2OHIP_BACKSUB_LANES", 8};
  const int lanes = lanes_k.get();  // dev A/B (8: C4 48.5 -> 45.3 us)
  pl_dispatch(pd, ld, [&](auto P, auto L) {
    if (lanes == 8)
      hipLaunchKernelGGL((k_backsub_g<decltype(P)::value, decltype(L)::value, 8>), grid_for((size_t)nl * 8, 256), 256,
                         0, s, nl, lm_ptr, blk_pose, G, Ufac, cl_all, size_poses, lm0, x);
    else
      hipLaunchKernelGGL((k_backsub_g<decltype(P)::value, decltype(L)::value, 4>), grid_for((size_t)nl * 4, 256), 256,
                         0, s, nl, lm_ptr, blk_pose, G, Ufac, cl_all, size_poses, lm0, x);
  });
  KERNEL_CHECK();
}

void oplus_multi(const OplusList& L0, const double* x, hipStream_t s) {
  OplusList L = L0;
  int nb = 0;
  for (int t = 0; t < L.cnt; ++t) {
    L.blk0[t] = nb;
    nb += (int)grid_for(L.n[t], 256);
  }
  if (nb <= 0) return;
  hipLaunchKernelGGL(k_oplus_multi, nb, 256, 0, s, L, x);
  KERNEL_CHECK();
}

size_t sum_partials(long long n) { return (size_t)((n + RED_BLOCK * RED_PER_THREAD - 1) / (RED_BLOCK * RED_PER_THREAD)); }

void sum(const double* v, long long n, double* partial, double* out, hipStream_t s) {
  const int np = (int)sum_partials(n);
  if (np > 0) hipLaunchKernelGGL(k_sum_partial, np, RED_BLOCK, 0, s, v, n, partial);
  hipLaunchKernelGGL(k_sum_final, 1, RED_BLOCK, 0, s, partial, np, out);
  KERNEL_CHECK();
}

int error_partials(int family, const EdgeArgs& a, int ne, double* partial, hipStream_t s) {
  const int np = (int)sum_partials(ne);
  if (np <= 0) return 0;
  family_dispatch(family, a, [&](auto fam) {
    using F = decltype(fam);
    hipLaunchKernelGGL(k_error_partial<F>, np, RED_BLOCK, 0, s, mk(a), ne, partial);
  });
  KERNEL_CHECK();
  return np;
}
void error_scale(int family, const EdgeArgs& a, int ne, long long n, long long npose, const double* x, const double* b,
                 const double* lam, double* partial, double* out_chi, double* out_scale, hipStream_t s,
                 const LmDecide* dec) {
  const int npe = (int)sum_partials(ne), nps = (int)sum_partials(n);
  if (npe + nps > 0)
    family_dispatch(family, a, [&](auto fam) {
      using F = decltype(fam);
      hipLaunchKernelGGL(k_error_scale_partial<F>, npe + nps, RED_BLOCK, 0, s, mk(a), ne, npe, n, npose, x, b, lam,
                         partial);
    });
  if (dec)  // out_chi, out_scale = p + 1, p + 2
    hipLaunchKernelGGL(k_sum_final2_decide, 1, RED_BLOCK, 0, s, partial, npe, nps, out_chi - 1, dec->current_chi,
                       dec->ni, dec->rank0 ? 1 : 0, dec->host_out);
  else
    hipLaunchKernelGGL(k_sum_final2, 2, RED_BLOCK, 0, s, partial, npe, nps, out_chi, out_scale);
  KERNEL_CHECK();
}
void sum_final(const double* partial, int np, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_sum_final, 1, RED_BLOCK, 0, s, partial, np, out);
  KERNEL_CHECK();
}
void scale_sum(long long n, long long npose, const double* x, const double* b, const double* lam, double* partial,
               double* out, hipStream_t s) {
  const int np = (int)sum_partials(n);
  if (np > 0) hipLaunchKernelGGL(k_scale_partial, np, RED_BLOCK, 0, s, n, npose, x, b, lam, partial);
  hipLaunchKernelGGL(k_sum_final, 1, RED_BLOCK, 0, s, partial, np, out);
  KERNEL_CHECK();
}
void block_symv(int pd, int n, const int* rptr, const int2* ent, const int* diag, const double* vals, const double* lam,
                const double* x, double* y, const double* b, double* r2, double* b2, hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = grid_for(n, 256);
  if (pd == 6) hipLaunchKernelGGL(k_block_symv<6>, g, 256, 0, s, n, rptr, ent, diag, vals, lam, x, y, b, r2, b2);
  else if (pd == 3) hipLaunchKernelGGL(k_block_symv<3>, g, 256, 0, s, n, rptr, ent, diag, vals, lam, x, y, b, r2, b2);
  else throw std::runtime_error("block_symv: block dimension must be 3 or 6");
  KERNEL_CHECK();
}
void scale_terms(long long n, const double* x, const double* b, const double* lam, double* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scale_terms, grid_for(n, 256), 256, 0, s, n, x, b, lam, out);
  KERNEL_CHECK();
}

}  // namespace launch
}  // namespace g2ohip

// ------------------------------------------------------------------------------ small helpers
namespace g2ohip {
__global__ void k_set_scalars(double* __restrict__ p, double lam, double lam_rank, int reset_fail) {
  p[0] = lam;
  p[4] = lam_rank;
  p[5] = 0.0;
  if (reset_fail) p[8] = 0.0;  // the two int not-PD flags live in p[8]
}
// the LM trial decision, restated from the host loop (Engine::lm_solve, optimization_algorithm_levenberg.cpp:127-141):
// the host reads it back instead of recomputing it, so both sides follow one decision
// max |diag| over nb blocks of dim x dim (col-major), partial per block of threads
__global__ void __launch_bounds__(256) k_diag_absmax(const double* __restrict__ H, int nb, int dim,
                                                     double* __restrict__ out) {
  __shared__ double sh[256];
  double m = 0.0;
  for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < (long long)nb * dim; k += (long long)gridDim.x * 256) {
    const long long blk = k / dim, d = k % dim;
    m = fmax(m, fabs(H[blk * dim * dim + d * dim + d]));
  }
  sh[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}
__global__ void k_max_final(const double* __restrict__ partial, int np, double* __restrict__ out) {
  double m = 0.0;
  for (int i = 0; i < np; ++i) m = fmax(m, partial[i]);
  *out = m;
}
__global__ void __launch_bounds__(256) k_copy_multi(launch::CopyList cl) {
  if (cl.sp && blockIdx.x == 0 && threadIdx.x == 0) {  // k_set_scalars(sp, lam, lam_rank, reset_fail = 1)
    cl.sp[0] = cl.lam;
    cl.sp[4] = cl.lam_rank;
    cl.sp[5] = 0.0;
    cl.sp[8] = 0.0;
  }
  for (int k = 0; k < cl.n; ++k) {  // uniform loop; grid-stride over each buffer
    const double2* src = reinterpret_cast<const double2*>(cl.src[k]);
    double2* dst = reinterpret_cast<double2*>(cl.dst[k]);
    const long long n2 = cl.len[k] / 2;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) dst[i] = src[i];
    if ((cl.len[k] & 1) && blockIdx.x == 0 && threadIdx.x == 0) cl.dst[k][cl.len[k] - 1] = cl.src[k][cl.len[k] - 1];
  }
}
namespace launch {
void copy_multi(const CopyList& cl, hipStream_t s) {
  if (cl.n <= 0 && !cl.sp) return;
  long long mx = 0;
  for (int k = 0; k < cl.n; ++k) mx = std::max(mx, cl.len[k]);
  const unsigned g = (unsigned)std::min<long long>(std::max<long long>((mx / 2 + 255) / 256, 1), 1024);
  hipLaunchKernelGGL(k_copy_multi, g, 256, 0, s, cl);
  KERNEL_CHECK();
}
void set_scalars(double* p, double lam, double lam_rank, hipStream_t s, bool reset_fail) {
  hipLaunchKernelGGL(k_set_scalars, 1, 1, 0, s, p, lam, lam_rank, reset_fail ? 1 : 0);
  KERNEL_CHECK();
}
void lm_decide(double* p, double current_chi, double ni, bool rank0, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_decide, 1, 1, 0, s, p, current_chi, ni, rank0 ? 1 : 0);
  KERNEL_CHECK();
}
// writes max|diag| of two block sets into out (partial needs >= 64 doubles)
void diag_absmax(const double* H1, int nb1, int d1, const double* H2, int nb2, int d2, double* partial, double* out,
                 hipStream_t s) {
  const int g = 32;
  hipLaunchKernelGGL(k_diag_absmax, g, 256, 0, s, H1, nb1, d1, partial);
  if (H2 && nb2 > 0) hipLaunchKernelGGL(k_diag_absmax, g, 256, 0, s, H2, nb2, d2, partial + g);
  else hipLaunchKernelGGL(k_diag_absmax, g, 256, 0, s, H1, 0, d1, partial + g);
  hipLaunchKernelGGL(k_max_final, 1, 1, 0, s, partial, 2 * g, out);
  KERNEL_CHECK();
}
}  // namespace launch
}  // namespace g2ohip
