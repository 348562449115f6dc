// Fused bundle-adjustment assembly (graphs whose only edge type is EdgeSE3ProjectXYZ, BlockSolver_6_3 + Schur):
// BlockSolver::buildSystem (block_solver.hpp:462-521) + BaseBinaryEdge::constructQuadraticForm
// (base_binary_edge.hpp:61-137) without the per-edge slot round trip of the generic path.
//
//   k_linearize_fused  edges sorted landmark-major and cut into wave chunks of whole landmarks (<= 64 edges):
//                      one lane per edge computes J, the Hpl block A^T Omega B (stored, as in the generic path)
//                      and its landmark-side terms A^T Omega A, A^T omega_r; the wave sums each landmark's
//                      terms in edge order (segment heads walk their segment in LDS) and writes Hll and b_l
//                      directly. Landmarks with more than 64 observations span several chunks: each chunk
//                      leaves a partial that k_lm_fixup adds in chunk order.
//   k_cam_assemble     one workgroup per camera over a camera-major copy of its observations: recomputes the
//                      camera Jacobian (cheap) instead of reading per-edge slots, accumulates B^T Omega B and
//                      B^T omega_r per thread in edge order and reduces them in a fixed tree: Hpp(i,i), b_i.
// Every output has one owner and a fixed summation order: bitwise reproducible run to run (no atomics).
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "device_types.hpp"
#include "device_util.hpp"
#include "kernels.hpp"

namespace g2ohip {
using namespace dev;

namespace {
__device__ __forceinline__ void wsync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void copy_out(double* __restrict__ dst, const double* src, int n, int lane) {
  int s = 0;
  if (reinterpret_cast<uintptr_t>(dst) & 15) {
    if (lane == 0 && n > 0) dst[0] = src[0];
    s = 1;
  }
  const int n2 = (n - s) >> 1;
  double2* d2 = reinterpret_cast<double2*>(dst + s);
  for (int i = lane; i < n2; i += 64) d2[i] = double2{src[s + 2 * i], src[s + 2 * i + 1]};
  if (lane == 0 && ((n - s) & 1)) dst[n - 1] = src[n - 1];
}

// copy_out with nontemporal 16-byte stores (no L2 / MALL allocation): streams that outgrow the caches
__device__ __forceinline__ void copy_out_nt(double* __restrict__ dst, const double* src, int n, int lane) {
  typedef double dv2 __attribute__((ext_vector_type(2)));
  int s = 0;
  if (reinterpret_cast<uintptr_t>(dst) & 15) {
    if (lane == 0 && n > 0) __builtin_nontemporal_store(src[0], dst);
    s = 1;
  }
  const int n2 = (n - s) >> 1;
  dv2* d2 = reinterpret_cast<dv2*>(dst + s);
  for (int i = lane; i < n2; i += 64) {
    dv2 v;
    v.x = src[s + 2 * i];
    v.y = src[s + 2 * i + 1];
    __builtin_nontemporal_store(v, d2 + i);
  }
  if (lane == 0 && ((n - s) & 1)) __builtin_nontemporal_store(src[n - 1], dst + n - 1);
}

// error, Jacobians and the (robust-weighted) information of one edge (base_binary_edge.hpp:104-135)
template <class F, bool PC = false>
__device__ __forceinline__ void edge_terms(const EdgeData& d, int e, double* err, double* A, double* B, double* Om,
                                           double* pc = nullptr) {
  constexpr int D = F::D;
  if constexpr (PC) F::linearize(d, e, err, A, B, pc);
  else F::linearize(d, e, err, A, B);
  load_info<D>(info_rec(d, e, F::INFO), Om);
  if (d.rk) {
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
// the same with the edge's vertex indices given: a caller that reads them ahead (software pipeline) starts the state
// loads without a dependent index load (FamilyBA)
template <class F, bool NT = false>
__device__ __forceinline__ void edge_terms_at(const EdgeData& d, int e, int v0, int v1, double* err, double* A, double* B,
                                              double* Om) {
  constexpr int D = F::D;
  double pc[3];
  if constexpr (NT) F::template linearize_at<true>(d, e, v0, v1, err, A, B, pc);
  else F::linearize_at(d, e, v0, v1, err, A, B, pc);
  load_info<D>(info_rec(d, e, F::INFO), Om);
  if (d.rk) {
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
}  // namespace

// KX (with FG, BA only): instead of G = Hpl U^-T (18 doubles) each observation stores the 10-double record the Schur
// row pass rebuilds G from: Kt = diag(fx, fy) Omega A U^-T (2 x 3 col-major), then (u, v, w) = (x/z, y/z, 1/z) of the
// point in the camera frame, then a pad. The camera Jacobian is B = diag(fx, fy) Bt(u, v, w) with
//   Bt = [ u v   -(1 + u^2)   v   -w    0   u w ]
//        [ 1+v^2   -u v      -u    0   -w   v w ]    (types_six_dof_expmap.cpp linearizeOplus, z-scaled)
// so Hpl = B^T Omega A = Bt^T diag(f) Omega A and G = Bt^T Kt. Split landmarks store Kt before U^-T (k_lm_fixup
// applies it).
constexpr int KXB = 10;

template <class F, bool FG, bool KX = false>
// (KX: 20 KB of LDS and 70 VGPRs, seven waves per SIMD; C5 0.51 -> 0.46 ms, C4 53 -> 45 us against five with the U
// records in LDS; eight, forced by __launch_bounds__, spill 20 B per lane and gain nothing: profiles/r06_ab_lin_c{4,5}.log)
__global__ void __launch_bounds__(256)
    k_linearize_fused(EdgeData d, const int4* __restrict__ chunks, int nchunks, const int* __restrict__ h0,
                      const int* __restrict__ h1, const long long* __restrict__ off_dst,
                      const unsigned char* __restrict__ off_tr, double* __restrict__ off_base,
                      double* __restrict__ off_slot, double* __restrict__ Hll, double* __restrict__ bvec,
                      int num_poses, int size_poses, int lm_begin, double* __restrict__ lpart, launch::SchurSplit sp) {
  constexpr int D = F::D, DA = F::DA, DB = F::DB;
  constexpr int UF = 2 * DA;  // U record of a DA = 3 landmark (FG instantiations are BA only)
  // per-lane LDS image: landmark terms (+ U records with a split), or the lane's stored block (G / Hpl, or a Kt record)
  // (the U records reach the segment's lanes from the head lane's registers by __shfl: an LDS image of them behind
  // the landmark terms made the stage 15 doubles per lane and left 5 waves per SIMD, LDS-bound)
  constexpr int SA = DA * (DA + 1) / 2 + DA, SH = DA * DB, SB0 = KX ? 10 : SH;
  constexpr int SM = SA > SB0 ? SA : SB0;
  static_assert(!FG || DA == 3, "U records of DA = 3 landmarks");
  __shared__ __attribute__((aligned(16))) double stage[4][64 * SM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wave = blockIdx.x * 4 + w;
  if (wave >= nchunks) return;  // wave-uniform
  const int4 ch = chunks[wave];
  const int ebase = ch.x, nw = ch.y;
  const int e = ebase + lane;
  const bool in = lane < nw;
  double* sw = stage[w];
  // the edge's terms are formed unconditionally (lanes past the chunk on its first edge), so the state loads issue
  // beside the Hessian-index loads instead of behind them (v0 -> h0 -> states was three dependent round trips); an
  // edge with both vertices fixed is masked below as before
  const int ec = in ? e : ebase;
  const int pv0 = d.v0[ec], pv1 = d.v1[ec];
  const int hA0 = h0[pv0], hB0 = h1[pv1];
  double err[D], A[D * DA], B[D * DB], Om[D * D], pc[3];
  {
    F::linearize_at(d, ec, pv0, pv1, err, A, B, pc);
    load_info<D>(info_rec(d, ec, F::INFO), Om);
    if (d.rk) {
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
  const int pv = in ? pv0 : -1;
  const int hA = in ? hA0 : -1;
  const bool nfA = hA >= 0, nfB = in && hB0 >= 0;
  double wr[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    double s = 0;
#pragma unroll
    for (int c = 0; c < D; ++c) s += Om[r * D + c] * err[c];
    wr[r] = -s;
  }
  double AtO[DA * D];
#pragma unroll
  for (int i = 0; i < DA; ++i)
#pragma unroll
    for (int c = 0; c < D; ++c) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < D; ++r) s += A[r * DA + i] * Om[r * D + c];
      AtO[i * D + c] = s;
    }
  // off-diagonal (Hpl) block, as k_linearize: a coalesced run through LDS when the wave's blocks are consecutive.
  // With a Schur split it is G = Hpl U^-T instead (U of the lane's landmark, known after the landmark sums below;
  // split landmarks store Hpl and k_lm_fixup forms their G)
  auto off_block = [&](const double* U) {
    constexpr long long SLOT_BIT = 1LL << 62;
    const long long od_raw = (nfA && nfB) ? off_dst[e] : -1;
    const bool in_slot = od_raw >= 0 && (od_raw & SLOT_BIT);
    constexpr int BS = KX ? KXB : SH;  // doubles per stored block
    long long od = od_raw >= 0 ? (od_raw & ~SLOT_BIT) - (FG ? sp.hpl_base : 0) : -1;
    if constexpr (KX) {  // no duplicate (landmark, camera) edges in KX mode: no slots
      od = od >= 0 ? od / SH * KXB : -1;
      // an observation of a fixed landmark by a free camera gets a record of its own (Kt = 0) for the camera pass
      if (in && !nfA && nfB) {
        const int x = sp.kx_extra[e];
        od = x >= 0 ? (long long)x * KXB : -1;
      }
    }
    double* base = FG ? sp.G : off_base;
    const bool tr = nfA && nfB && off_tr[e];
    const long long od0 = __shfl(od, 0, 64);
    const bool tr0 = __shfl((int)tr, 0, 64) != 0;
    const bool slot0f = __shfl((int)in_slot, 0, 64) != 0;
    const bool run = __all(!in || (od >= 0 && od0 >= 0 && od == od0 + (long long)lane * BS && tr == tr0 && in_slot == slot0f));
    if (od >= 0) {
      double* H = run ? sw + lane * BS : (in_slot ? off_slot : base) + od;
      if constexpr (KX) {  // Kt = diag(f) Omega A (U^-T unless the landmark is split), then (x/z, y/z, 1/z)
        const double* Kp = param_rec(d, e, 4);
        double W[D * DA];
#pragma unroll
        for (int a2 = 0; a2 < DA; ++a2)
#pragma unroll
          for (int r = 0; r < D; ++r) {
            double s = 0;
#pragma unroll
            for (int c = 0; c < D; ++c) s += Om[r * D + c] * A[c * DA + a2];
            W[a2 * D + r] = nfA ? Kp[r] * s : 0.0;
          }
        if (ch.z < 0 && nfA) form_G<D, DA>(W, U);
#pragma unroll
        for (int k = 0; k < D * DA; ++k) H[k] = W[k];
        H[6] = pc[0] / pc[2];  // as the projection divides (the camera pass rebuilds the error from these)
        H[7] = pc[1] / pc[2];
        H[8] = 1.0 / pc[2];
        H[9] = 0.0;
      } else if (FG || tr) {  // (pose, landmark) block, column-major: H[i * DB + j] = (A^T Omega B)(i, j)
        double g[SH];
#pragma unroll
        for (int i = 0; i < DA; ++i)
#pragma unroll
          for (int j = 0; j < DB; ++j) {
            double s = 0;
#pragma unroll
            for (int r = 0; r < D; ++r) s += AtO[i * D + r] * B[r * DB + j];
            g[i * DB + j] = s;
          }
        if constexpr (FG) {
          if (ch.z < 0) form_G<DB, DA>(g, U);
        }
#pragma unroll
        for (int k = 0; k < SH; ++k) H[k] = g[k];
      } else {
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
      wsync();
      if (KX && sp.kx == 2)
        copy_out_nt((slot0f ? off_slot : base) + od0, sw, nw * BS, lane);
      else
        copy_out((slot0f ? off_slot : base) + od0, sw, nw * BS, lane);
    }
    wsync();
  };
  if constexpr (!FG) off_block(nullptr);
  // landmark-side terms of every lane (zeros when the landmark is fixed), then segment sums in edge order
  {
    double* o = sw + lane * SA;
    int k = 0;
#pragma unroll
    for (int c = 0; c < DA; ++c)
#pragma unroll
      for (int r = 0; r <= c; ++r) {
        double s = 0;
#pragma unroll
        for (int t = 0; t < D; ++t) s += AtO[r * D + t] * A[t * DA + c];
        o[k++] = nfA ? s : 0.0;
      }
#pragma unroll
    for (int i = 0; i < DA; ++i) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < D; ++r) s += A[r * DA + i] * wr[r];
      o[k++] = nfA ? s : 0.0;
    }
  }
  wsync();
  // segment heads by shuffles (no LDS word per lane: the stage alone sets the occupancy, eight waves per SIMD)
  const int pv_prev = __shfl_up(pv, 1, 64);
  const bool head = in && (lane == 0 || pv_prev != pv);
  const unsigned long long heads = __ballot(head);
  const unsigned long long above = lane == 63 ? 0ull : heads & ~((2ull << lane) - 1);  // heads past this lane
  const int seg_end = above ? __builtin_ctzll(above) : nw;
  double Uh[FG ? UF : 1];  // a head lane's U record (split: its landmark's)
#pragma unroll
  for (int k = 0; k < (FG ? UF : 1); ++k) Uh[k] = 0.0;
  if (head && nfA) {
    double acc[SA];
#pragma unroll
    for (int k = 0; k < SA; ++k) acc[k] = sw[lane * SA + k];
    for (int j = lane + 1; j < seg_end; ++j)
#pragma unroll
      for (int k = 0; k < SA; ++k) acc[k] += sw[j * SA + k];
    if (ch.z < 0) {
      double* H = Hll + (size_t)(hA - num_poses - lm_begin) * DA * DA;
      int k = 0;
#pragma unroll
      for (int c = 0; c < DA; ++c)
#pragma unroll
        for (int r = 0; r <= c; ++r) {
          H[c * DA + r] = acc[k];
          H[r * DA + c] = acc[k];
          ++k;
        }
      double* bb = bvec + size_poses + (size_t)(hA - num_poses) * DA;
#pragma unroll
      for (int i = 0; i < DA; ++i) bb[i] = acc[DA * (DA + 1) / 2 + i];
      if constexpr (FG) {  // Hll + lambda I = U U^T, c = U^-1 b_l (k_schur_prep's arithmetic)
        double a[DA * DA];
        int q = 0;
#pragma unroll
        for (int c = 0; c < DA; ++c)
#pragma unroll
          for (int r = 0; r <= c; ++r) {
            a[c * DA + r] = acc[q];
            a[r * DA + c] = acc[q];
            ++q;
          }
#pragma unroll
        for (int i = 0; i < DA; ++i) a[i * DA + i] += sp.lamp ? sp.lamp[0] : sp.lam;
        double U[UF], cl[DA];
        if (!lm_ufac<DA>(a, acc + DA * (DA + 1) / 2, U, cl)) *sp.fail = 1;
        double* Uo = sp.Ufac + (size_t)(hA - num_poses - lm_begin) * UF;
        double* co = sp.cl + (size_t)(hA - num_poses) * DA;
#pragma unroll
        for (int k2 = 0; k2 < UF; ++k2) {
          Uo[k2] = U[k2];
          if constexpr (FG) Uh[k2] = U[k2];
        }
#pragma unroll
        for (int i = 0; i < DA; ++i) co[i] = cl[i];
      }
    } else {  // one landmark of > 64 observations: this chunk's partial
#pragma unroll
      for (int k = 0; k < SA; ++k) lpart[(size_t)ch.z * SA + k] = acc[k];
    }
  }
  if constexpr (FG) {
    wsync();
    // the lane's segment head: the highest head lane at or below it
    const unsigned long long le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const int hl = 63 - __clzll(heads & le);
    double U[UF];
#pragma unroll
    for (int k = 0; k < UF; ++k) U[k] = __shfl(Uh[k], hl & 63, 64);
    wsync();  // every lane's landmark terms read before the run image reuses the stage
    off_block(U);
  }
}

// split landmarks: fix = (hessian index, first partial, count); partials added in chunk order. With a Schur split the
// landmark's U, c follow, and its G blocks (stored as Hpl by the linearize chunks) are formed in place.
template <bool FG, bool KX = false>
__global__ void __launch_bounds__(256) k_lm_fixup(int nfix, const int4* __restrict__ fix, const double* __restrict__ lpart,
                                                  double* __restrict__ Hll, double* __restrict__ bvec, int num_poses,
                                                  int size_poses, int lm_begin, launch::SchurSplit sp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nfix) return;
  const int4 f = fix[i];
  constexpr int SA = 9;
  double acc[SA];
#pragma unroll
  for (int k = 0; k < SA; ++k) acc[k] = 0.0;
  for (int p = f.y; p < f.y + f.z; ++p)
#pragma unroll
    for (int k = 0; k < SA; ++k) acc[k] += lpart[(size_t)p * SA + k];
  const int l = f.x - num_poses - lm_begin;
  double* H = Hll + (size_t)l * 9;
  int k = 0;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r <= c; ++r) {
      H[c * 3 + r] = acc[k];
      H[r * 3 + c] = acc[k];
      ++k;
    }
  double* bb = bvec + size_poses + (size_t)(f.x - num_poses) * 3;
  bb[0] = acc[6]; bb[1] = acc[7]; bb[2] = acc[8];
  if constexpr (FG) {
    double a[9];
    int q = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r <= c; ++r) {
        a[c * 3 + r] = acc[q];
        a[r * 3 + c] = acc[q];
        ++q;
      }
#pragma unroll
    for (int j = 0; j < 3; ++j) a[j * 3 + j] += sp.lamp ? sp.lamp[0] : sp.lam;
    double U[6], cl[3];
    if (!lm_ufac<3>(a, acc + 6, U, cl)) *sp.fail = 1;
#pragma unroll
    for (int j = 0; j < 6; ++j) sp.Ufac[(size_t)l * 6 + j] = U[j];
#pragma unroll
    for (int j = 0; j < 3; ++j) sp.cl[(size_t)(f.x - num_poses) * 3 + j] = cl[j];
    if constexpr (KX) {  // Kt U^-T in place; (u, v, w) as the linearize chunks stored them
      for (int a2 = sp.lm_ptr[l]; a2 < sp.lm_ptr[l + 1]; ++a2) {
        double g[6];
        double* gp = sp.G + (size_t)a2 * KXB;
#pragma unroll
        for (int j = 0; j < 6; ++j) g[j] = gp[j];
        form_G<2, 3>(g, U);
#pragma unroll
        for (int j = 0; j < 6; ++j) gp[j] = g[j];
      }
      return;
    }
    for (int a2 = sp.lm_ptr[l]; a2 < sp.lm_ptr[l + 1]; ++a2) {
      double g[18];
      double* gp = sp.G + (size_t)a2 * 18;
#pragma unroll
      for (int j = 0; j < 18; ++j) g[j] = gp[j];
      form_G<6, 3>(g, U);
#pragma unroll
      for (int j = 0; j < 18; ++j) gp[j] = g[j];
    }
  }
}

// camera-side terms: one workgroup per pose, threads stride over its observations (camera-major copy of the
// edge data, ascending landmark-major edge order), 27 accumulators per thread, fixed-tree reduction: Hpp(i,i), b_i.
// With a Schur split the pass forms the diagonal Schur block directly instead of Hpp(i,i): per observation with a free
// landmark, G G^T = B^T M B and G c_l = B^T W c_l with W = Omega A U^-T (D x LD), M = W W^T = Omega A (Hll + lambda I)^-1
// A^T Omega, so S(i,i) = lambda I + sum B^T (Omega - M) B and bschur_i = sum B^T (omega_r - W c_l), beside b_i
// (block_solver.hpp:361-400's j == i terms in 33 accumulators; Hpp is left to a plain buildSystem).
// KX (with FG): an observation of a free landmark reads the 10-double Kt record the linearize wave left instead of
// re-linearising the edge: with B = diag(f) Bt(u, v, w) and Kt = diag(f) W,
//   B^T (Omega - W W^T) B = Bt^T (F Omega F - Kt Kt^T) Bt,   B^T (omega_r - W c_l) = Bt^T (F omega_r - Kt c_l),
// the error from (u, v) = (x/z, y/z) exactly as the projection computes it (robust weight from its chi2).
// NT (recomputing path): the per-observation streams (vertex indices, measurements) are read nontemporally
// cams (landmark-sharded ranks): the npose cameras of this launch (those with local observations or a diagonal block
// this rank's factorization reads); nullptr: cameras 0 .. npose - 1
template <class F, bool FG, bool KX = false, bool NT = false>
__global__ void __launch_bounds__(256, 3) k_cam_assemble(EdgeData d, const int* __restrict__ cm_ptr,
                                                      const int* __restrict__ cams, int npose,
                                                      double* __restrict__ Hpp, double* __restrict__ bvec,
                                                      int num_poses, int lm_begin, launch::SchurSplit sp) {
  constexpr int D = F::D, DA = F::DA, DB = F::DB;
  constexpr int SP = DB * (DB + 1) / 2, S = SP + DB, NS = FG ? S + DB : S;
  constexpr int UF = 2 * DA;
  __shared__ double red[4][NS];
  int i = xcd_item(blockIdx.x, npose);  // neighbouring cameras share landmarks: one L2
  if (i >= npose) return;  // workgroup-uniform
  if (cams) i = cams[i];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double acc[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) acc[k] = 0.0;
  const int p0 = cm_ptr[i] + tid, p1 = cm_ptr[i + 1];
  // software pipeline over the thread's observations (recomputing path): the vertex indices are read two observations
  // ahead and the landmark's Hessian index one ahead, so an observation's state / U / c loads depend on no load of the
  // same iteration (three dependent round trips per observation before)
  int v0a = 0, v1a = 0, v0b = 0, v1b = 0, hla = -1;
  if constexpr (!KX) {
    v0a = d.v0[p0 < p1 ? p0 : 0];
    v1a = d.v1[p0 < p1 ? p0 : 0];
    v0b = d.v0[p0 + 256 < p1 ? p0 + 256 : 0];
    v1b = d.v1[p0 + 256 < p1 ? p0 + 256 : 0];
    if constexpr (FG) hla = sp.hl[v0a];
  }
  for (int p = p0; p < p1; p += 256) {
    int hl = -1;
    if constexpr (FG && KX) hl = sp.hl[d.v0[p]];
    if constexpr (KX) {  // every camera-major observation has a record (fixed landmarks: Kt = 0)
      const int a = sp.cm_hpl[p];
      {
        const double* rec = sp.G + (size_t)a * KXB;
        double Kt[6];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const double2 x = *reinterpret_cast<const double2*>(rec + 2 * q);
          Kt[2 * q] = x.x; Kt[2 * q + 1] = x.y;
        }
        const double2 uv = *reinterpret_cast<const double2*>(rec + 6);
        const double u = uv.x, v = uv.y, wz = rec[8];
        const double* cp = sp.cl + (size_t)(hl >= 0 ? hl - num_poses : 0) * DA;
        const double c0 = hl >= 0 ? cp[0] : 0.0, c1 = hl >= 0 ? cp[1] : 0.0, c2 = hl >= 0 ? cp[2] : 0.0;
        const double* Kp = param_rec(d, p, 4);
        const double fx = Kp[0], fy = Kp[1];
        const double e0 = d.meas[(size_t)p * 2 + 0] - (u * fx + Kp[2]);
        const double e1 = d.meas[(size_t)p * 2 + 1] - (v * fy + Kp[3]);
        double Om[4];
        load_info<2>(info_rec(d, p, F::INFO), Om);
        if (d.rk) {
          const double chi = e0 * (Om[0] * e0 + Om[1] * e1) + e1 * (Om[2] * e0 + Om[3] * e1);
          double r0, r1;
          robustify(d.rk, d.rk_delta, chi, r0, r1);
#pragma unroll
          for (int q = 0; q < 4; ++q) Om[q] *= r1;
        }
        const double w0 = -(Om[0] * e0 + Om[1] * e1), w1 = -(Om[2] * e0 + Om[3] * e1);
        const double h0 = fx * w0, h1 = fy * w1;  // F omega_r
        const double g0 = h0 - (Kt[0] * c0 + Kt[2] * c1 + Kt[4] * c2);
        const double g1 = h1 - (Kt[1] * c0 + Kt[3] * c1 + Kt[5] * c2);
        const double n00 = fx * Om[0] * fx - (Kt[0] * Kt[0] + Kt[2] * Kt[2] + Kt[4] * Kt[4]);
        const double n01 = fx * Om[1] * fy - (Kt[0] * Kt[1] + Kt[2] * Kt[3] + Kt[4] * Kt[5]);
        const double n11 = fy * Om[3] * fy - (Kt[1] * Kt[1] + Kt[3] * Kt[3] + Kt[5] * Kt[5]);
        const double b0[6] = {u * v, -(1.0 + u * u), v, -wz, 0.0, u * wz};
        const double b1[6] = {1.0 + v * v, -(u * v), -u, 0.0, -wz, v * wz};
        int k = 0;
#pragma unroll
        for (int c = 0; c < DB; ++c) {  // column c of (N Bt): t0, t1
          const double t0 = n00 * b0[c] + n01 * b1[c], t1 = n01 * b0[c] + n11 * b1[c];
#pragma unroll
          for (int r = 0; r <= c; ++r) acc[k++] += b0[r] * t0 + b1[r] * t1;
        }
#pragma unroll
        for (int j = 0; j < DB; ++j) acc[k++] += b0[j] * h0 + b1[j] * h1;
#pragma unroll
        for (int j = 0; j < DB; ++j) acc[k++] += b0[j] * g0 + b1[j] * g1;
      }
    } else {
    const int v0 = v0a, v1 = v1a;
    if constexpr (FG) hl = hla;
    {  // the next observations' indices (two ahead: streaming; one ahead: the Hessian index of a loaded vertex)
      const int pn = p + 512 < p1 ? p + 512 : 0;
      const int v0c = NT ? __builtin_nontemporal_load(d.v0 + pn) : d.v0[pn];
      const int v1c = NT ? __builtin_nontemporal_load(d.v1 + pn) : d.v1[pn];
      if constexpr (FG) hla = sp.hl[v0b];
      v0a = v0b; v1a = v1b;
      v0b = v0c; v1b = v1c;
    }
    double err[D], A[D * DA], B[D * DB], Om[D * D];
    edge_terms_at<F, NT>(d, p, v0, v1, err, A, B, Om);
    double wr[D];
#pragma unroll
    for (int r = 0; r < D; ++r) {
      double s = 0;
#pragma unroll
      for (int c = 0; c < D; ++c) s += Om[r * D + c] * err[c];
      wr[r] = -s;
    }
    double N[D * D];  // Omega, minus M with a Schur split
    double v[D];      // omega_r - W c_l with a Schur split
#pragma unroll
    for (int k = 0; k < D * D; ++k) N[k] = Om[k];
#pragma unroll
    for (int r = 0; r < D; ++r) v[r] = wr[r];
    if constexpr (FG) {
      if (hl >= 0) {
        const double2* u2 = reinterpret_cast<const double2*>(sp.Ufac + (size_t)(hl - num_poses - lm_begin) * UF);
        const double* cp = sp.cl + (size_t)(hl - num_poses) * DA;
        double U[UF], cl[DA];
#pragma unroll
        for (int q = 0; q < UF / 2; ++q) { const double2 x = u2[q]; U[2 * q] = x.x; U[2 * q + 1] = x.y; }
#pragma unroll
        for (int q = 0; q < DA; ++q) cl[q] = cp[q];
        double W[D * DA];  // Omega A, column-major D x DA, then U^-T applied to each row
#pragma unroll
        for (int a = 0; a < DA; ++a)
#pragma unroll
          for (int r = 0; r < D; ++r) {
            double s = 0;
#pragma unroll
            for (int c = 0; c < D; ++c) s += Om[r * D + c] * A[c * DA + a];
            W[a * D + r] = s;
          }
        form_G<D, DA>(W, U);
#pragma unroll
        for (int r = 0; r < D; ++r)
#pragma unroll
          for (int c = 0; c < D; ++c) {
            double s = W[r] * W[c];
#pragma unroll
            for (int a = 1; a < DA; ++a) s += W[a * D + r] * W[a * D + c];
            N[r * D + c] -= s;
          }
#pragma unroll
        for (int r = 0; r < D; ++r) {
          double s = W[r] * cl[0];
#pragma unroll
          for (int a = 1; a < DA; ++a) s += W[a * D + r] * cl[a];
          v[r] -= s;
        }
      }
    }
    double BtN[DB * D];
#pragma unroll
    for (int j = 0; j < DB; ++j)
#pragma unroll
      for (int c = 0; c < D; ++c) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < D; ++r) s += B[r * DB + j] * N[r * D + c];
        BtN[j * D + c] = s;
      }
    int k = 0;
#pragma unroll
    for (int c = 0; c < DB; ++c)
#pragma unroll
      for (int r = 0; r <= c; ++r) {
        double s = 0;
#pragma unroll
        for (int t = 0; t < D; ++t) s += BtN[r * D + t] * B[t * DB + c];
        acc[k++] += s;
      }
#pragma unroll
    for (int j = 0; j < DB; ++j) {
      double s = 0;
#pragma unroll
      for (int r = 0; r < D; ++r) s += B[r * DB + j] * wr[r];
      acc[k++] += s;
    }
    if constexpr (FG) {
#pragma unroll
      for (int j = 0; j < DB; ++j) {
        double s = 0;
#pragma unroll
        for (int r = 0; r < D; ++r) s += B[r * DB + j] * v[r];
        acc[k++] += s;
      }
    }
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < NS; ++k) acc[k] += __shfl_xor(acc[k], m, 64);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NS; ++k) red[w][k] = acc[k];
  __syncthreads();
  if (tid >= NS) return;
  const double t = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
  if (tid < SP) {
    int c = 0, base = 0;
    while (tid >= base + c + 1) base += ++c;
    const int r = tid - base;
    if constexpr (FG) {  // S(i,i) = lambda I + sum B^T (Omega - M) B
      const double lr = sp.lam_own ? (sp.lam_own[i] ? (sp.lamp ? sp.lamp[0] : sp.lam) : 0.0)
                                   : (sp.lamp ? sp.lamp[1] : sp.lam_rank);
      const double o = r == c ? t + lr : t;
      double* So = sp.S + (size_t)sp.sdiag[i] * DB * DB;
      So[c * DB + r] = o;
      So[r * DB + c] = o;
    } else {
      double* H = Hpp + (size_t)i * DB * DB;
      H[c * DB + r] = t;
      H[r * DB + c] = t;
    }
  } else if (tid < S) {
    bvec[(size_t)i * DB + tid - SP] = t;
  } else {
    sp.bschur[(size_t)i * DB + tid - S] = t;
  }
}

// Back-substitution of the Schur split without its G blocks (block_solver.hpp:420-437, x_l = Dinv (b_l - Hpl^T x_p)):
// each observation's Jacobians are recomputed at the state the assembly linearised (the back-substitution precedes the
// update), Hpl_il^T x_i = A^T Omega (B x_i), and x_l = U^-T (c_l - U^-1 sum_i Hpl_il^T x_i) with the landmark's U and
// c = U^-1 b_l from the assembly. LANES lanes per landmark over its edges (landmark-major group order, erng), a fixed
// shuffle tree across them (bitwise reproducible). Reads ~30 bytes per observation instead of a 144-byte G block.
template <class F, int LANES>
__global__ void __launch_bounds__(256)
    k_backsub_j(EdgeData d, int nl, const int2* __restrict__ erng, const int* __restrict__ hcam,
                const double* __restrict__ Ufac, const double* __restrict__ cl_all, int size_poses, int lm0,
                double* __restrict__ x) {
  constexpr int D = F::D, DA = F::DA, DB = F::DB;
  static_assert(DA == 3 && D == 2, "BA landmark blocks");
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int l = gid / LANES, q = gid % LANES;
  const bool active = l < nl;
  double y[DA];
#pragma unroll
  for (int k = 0; k < DA; ++k) y[k] = 0.0;
  if (active) {
    const int2 r = erng[l];
    // software pipeline over the lane's edges: vertex indices two edges ahead, the camera's Hessian index one ahead (an
    // edge's state and x loads then wait for no load of their own iteration)
    const int e0 = r.x + q;
    int v0a = d.v0[e0 < r.y ? e0 : 0], v1a = d.v1[e0 < r.y ? e0 : 0];
    int v0b = d.v0[e0 + LANES < r.y ? e0 + LANES : 0], v1b = d.v1[e0 + LANES < r.y ? e0 + LANES : 0];
    int hca = hcam[v1a];
    for (int e = e0; e < r.y; e += LANES) {
      const int v0 = v0a, v1 = v1a, hc = hca;
      {
        const int en = e + 2 * LANES < r.y ? e + 2 * LANES : 0;
        const int v0c = d.v0[en], v1c = d.v1[en];
        hca = hcam[v1b];
        v0a = v0b; v1a = v1b;
        v0b = v0c; v1b = v1c;
      }
      if (hc < 0) continue;  // fixed camera: no Hpl block
      double err[D], A[D * DA], B[D * DB], Om[D * D];
      edge_terms_at<F>(d, e, v0, v1, err, A, B, Om);
      const double* xp = x + (size_t)hc * DB;
      double u[D];
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        double sacc = 0.0;
#pragma unroll
        for (int j = 0; j < DB; ++j) sacc += B[rr * DB + j] * xp[j];
        u[rr] = sacc;
      }
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        double v = 0.0;
#pragma unroll
        for (int c = 0; c < D; ++c) v += Om[rr * D + c] * u[c];
#pragma unroll
        for (int i = 0; i < DA; ++i) y[i] += A[rr * DA + i] * v;
      }
    }
  }
#pragma unroll
  for (int m = LANES / 2; m >= 1; m >>= 1)
#pragma unroll
    for (int k = 0; k < DA; ++k) y[k] += __shfl_xor(y[k], m, LANES);
  if (!active || q != 0) return;
  const double* U = Ufac + (size_t)l * 6;  // r0 r1 r2 u10 u20 u21: U = [[1/r0,0,0],[u10,1/r1,0],[u20,u21,1/r2]]
  const double* cl = cl_all + (size_t)(lm0 + l) * DA;
  const double z0 = y[0] * U[0];
  const double z1 = (y[1] - U[3] * z0) * U[1];
  const double z2 = (y[2] - U[4] * z0 - U[5] * z1) * U[2];
  const double c0 = cl[0] - z0, c1 = cl[1] - z1, c2 = cl[2] - z2;
  const double x2 = c2 * U[2];
  const double x1 = (c1 - U[5] * x2) * U[1];
  const double x0 = (c0 - U[3] * x1 - U[4] * x2) * U[0];
  double* xl = x + size_poses + (size_t)(lm0 + l) * DA;
  xl[0] = x0; xl[1] = x1; xl[2] = x2;
}

namespace launch {
void linearize_fused(const EdgeArgs& a, const int4* chunks, int nchunks, const int* h0, const int* h1,
                     const long long* off_dst, const unsigned char* off_tr, double* off_base, double* off_slot,
                     double* Hll, double* b, int num_poses, int size_poses, int lm_begin, double* lpart,
                     const SchurSplit* sp, hipStream_t s) {
  if (nchunks <= 0) return;
  const EdgeData d{a.v0, a.v1, a.meas, a.info, a.params, a.s0, a.s1, a.rk, a.rk_delta, a.ue};
  const SchurSplit z = sp ? *sp : SchurSplit{};
  if (sp && sp->kx)
    hipLaunchKernelGGL((k_linearize_fused<FamilyBA, true, true>), grid_for(nchunks, 4), 256, 0, s, d, chunks, nchunks, h0,
                       h1, off_dst, off_tr, off_base, off_slot, Hll, b, num_poses, size_poses, lm_begin, lpart, z);
  else if (sp)
    hipLaunchKernelGGL((k_linearize_fused<FamilyBA, true>), grid_for(nchunks, 4), 256, 0, s, d, chunks, nchunks, h0, h1,
                       off_dst, off_tr, off_base, off_slot, Hll, b, num_poses, size_poses, lm_begin, lpart, z);
  else
    hipLaunchKernelGGL((k_linearize_fused<FamilyBA, false>), grid_for(nchunks, 4), 256, 0, s, d, chunks, nchunks, h0,
                       h1, off_dst, off_tr, off_base, off_slot, Hll, b, num_poses, size_poses, lm_begin, lpart, z);
  KERNEL_CHECK();
}
void lm_fixup(int nfix, const int4* fix, const double* lpart, double* Hll, double* b, int num_poses, int size_poses,
              int lm_begin, const SchurSplit* sp, hipStream_t s) {
  if (nfix <= 0) return;
  const SchurSplit z = sp ? *sp : SchurSplit{};
  if (sp && sp->kx)
    hipLaunchKernelGGL((k_lm_fixup<true, true>), grid_for(nfix, 256), 256, 0, s, nfix, fix, lpart, Hll, b, num_poses,
                       size_poses, lm_begin, z);
  else if (sp)
    hipLaunchKernelGGL(k_lm_fixup<true>, grid_for(nfix, 256), 256, 0, s, nfix, fix, lpart, Hll, b, num_poses,
                       size_poses, lm_begin, z);
  else
    hipLaunchKernelGGL(k_lm_fixup<false>, grid_for(nfix, 256), 256, 0, s, nfix, fix, lpart, Hll, b, num_poses,
                       size_poses, lm_begin, z);
  KERNEL_CHECK();
}
void backsub_j(const EdgeArgs& a, int nl, const int2* erng, const int* hcam, const double* Ufac, const double* cl_all,
               int size_poses, int lm0, double* x, hipStream_t s) {
  if (nl <= 0) return;
  const EdgeData d{a.v0, a.v1, a.meas, a.info, a.params, a.s0, a.s1, a.rk, a.rk_delta, a.ue};
  // lanes per landmark (dev A/B G2OHIP_BACKSUB_J_LANES; profiles/r04_ab_backsub_lanes.log): 4 against 8 / 16, C5
  // 224.7-225.3 -> 227.5-227.6 / 222.6 LM it/s; 2 against 4, C5 225.0-225.1 -> 226.0-226.3, C4 907.5 -> 912.4
  static EnvKnob lanes_k{"G2OHIP_BACKSUB_J_LANES", 2};
  const int lanes = lanes_k.get();
  if (lanes == 2)
    hipLaunchKernelGGL((k_backsub_j<FamilyBA, 2>), grid_for((size_t)nl * 2, 256), 256, 0, s, d, nl, erng, hcam, Ufac,
                       cl_all, size_poses, lm0, x);
  else if (lanes == 4)
    hipLaunchKernelGGL((k_backsub_j<FamilyBA, 4>), grid_for((size_t)nl * 4, 256), 256, 0, s, d, nl, erng, hcam, Ufac,
                       cl_all, size_poses, lm0, x);
  else if (lanes == 16)
    hipLaunchKernelGGL((k_backsub_j<FamilyBA, 16>), grid_for((size_t)nl * 16, 256), 256, 0, s, d, nl, erng, hcam, Ufac,
                       cl_all, size_poses, lm0, x);
  else
    hipLaunchKernelGGL((k_backsub_j<FamilyBA, 8>), grid_for((size_t)nl * 8, 256), 256, 0, s, d, nl, erng, hcam, Ufac,
                       cl_all, size_poses, lm0, x);
  KERNEL_CHECK();
}

// the recomputing camera pass reads its per-observation streams (vertex indices, measurements) nontemporally, so they
// do not push the reused landmark lines (point, U, c) out of L2: C5 camera pass 0.421 / 0.425 -> 0.411 / 0.410 ms
// (profiles/r06_ab_c5_cam_nt.log); G2OHIP_CAM_NT=0 restores plain loads (A/B)
static bool cam_nt() {
  static EnvKnob k{"G2OHIP_CAM_NT", 1};
  return k.get() != 0;
}
void cam_assemble(const EdgeArgs& a, const int* cm_ptr, int npose, double* Hpp, double* b, int num_poses, int lm_begin,
                  const SchurSplit* sp, hipStream_t s, const int* cams) {
  if (npose <= 0) return;
  const EdgeData d{a.v0, a.v1, a.meas, a.info, a.params, a.s0, a.s1, a.rk, a.rk_delta, a.ue};
  const SchurSplit z = sp ? *sp : SchurSplit{};
  if (sp && sp->kx && sp->cm_hpl)
    hipLaunchKernelGGL((k_cam_assemble<FamilyBA, true, true>), npose, 256, 0, s, d, cm_ptr, cams, npose, Hpp, b, num_poses,
                       lm_begin, z);
  else if (sp && cam_nt())
    hipLaunchKernelGGL((k_cam_assemble<FamilyBA, true, false, true>), npose, 256, 0, s, d, cm_ptr, cams, npose, Hpp, b,
                       num_poses, lm_begin, z);
  else if (sp)
    hipLaunchKernelGGL((k_cam_assemble<FamilyBA, true>), npose, 256, 0, s, d, cm_ptr, cams, npose, Hpp, b, num_poses,
                       lm_begin, z);
  else
    hipLaunchKernelGGL((k_cam_assemble<FamilyBA, false>), npose, 256, 0, s, d, cm_ptr, cams, npose, Hpp, b, num_poses,
                       lm_begin, z);
  KERNEL_CHECK();
}
}  // namespace launch
}  // namespace g2ohip
