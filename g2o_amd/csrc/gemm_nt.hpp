// Tile update C(I, J) -= A(I, K) A(J, K)^T on v_mfma_f64_16x16x4f64 — the high-intensity half of the
// supernodal Cholesky (contribution blocks U = A22 - L21 L21^T and the rank-PB trailing updates of
// blocked fronts). A is a finished factor panel in lbuf (column-major, leading dimension m), C a front
// (column-major, leading dimension m), lower triangle only.
//
// One workgroup of WM x WN waves owns a BM x BN tile; each wave a (BM/WM) x (BN/WN) sub-tile of
// MI x NJ 16x16 MFMA blocks, so every A fragment read from LDS feeds NJ MFMAs and every B fragment MI. K runs in chunks of KC columns, double-buffered in LDS (k-major images: the global
// column segments land unchanged, fragment reads are 16 consecutive rows per k), the next chunk's
// global loads in flight under the current chunk's MFMAs: one barrier per chunk.
#pragma once
#include <hip/hip_runtime.h>

#include "device_util.hpp"

namespace g2ohip {

typedef double gdx4 __attribute__((ext_vector_type(4)));

template <int BM, int BN, int WM = 2, int WN = 2, int KC_ = 16>
struct GemmNT {
  static constexpr int ROWS = BM;          // rows of C per tile (k_syrk's row-tile unit)
  static constexpr int NT = 64 * WM * WN;  // threads
  static constexpr int KC = KC_;
  static constexpr int SA = BM + 16;  // k-major LDS strides (doubles), = 16 mod 32: the four k rows of a
  static constexpr int SB = BN + 16;  // fragment read fall on alternating bank halves
  static constexpr int LDS_DOUBLES = 2 * KC * (SA + SB);
  static constexpr int MI = BM / WM / 16, NJ = BN / WN / 16;  // MFMA blocks per wave
  static constexpr int LA = BM * KC / NT, LB = BN * KC / NT;   // global loads per thread per chunk

  // rows [I0, I0+BM) x columns [J0, J0+BN) of C, K = [ka, kb); entries outside rows < mrows,
  // columns < climit or above the diagonal are left untouched. lds: LDS_DOUBLES doubles.
  // overwrite: C is known to be zero (a childless front's contribution block): C = -A A^T without reading it.
  // Short-K tiles (their time is the C traffic) stage the tile in LDS (once it holds no K chunk) and move C a column
  // per wave instruction: 16-lane segments of the MFMA layout would touch 16 columns 32 bytes at a time.
  static constexpr bool LDS_EPILOGUE = (long long)BM * (BN + 1) <= LDS_DOUBLES && NT % BM == 0;
  // yv / vout (diagonal tiles of a contribution pass): also vout[r] -= sum_k A(I0 + r, k) yv[k] for the tile's rows
  __device__ static void run(const double* __restrict__ A, int lda, double* __restrict__ C, int ldc, int mrows,
                             int climit, int I0, int J0, int ka, int kb, double* lds, bool overwrite = false,
                             const double* yv = nullptr, double* vout = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double vdot = 0.0;
    const int wr = w % WM, wc = w / WM;
    const int lr = lane & 15, lk = lane >> 4;
    constexpr int BUF = KC * (SA + SB);  // buffer b: A image at lds + b BUF, B image after it
    // prefetch registers hold the raw loads; the out-of-range mask is applied when they are stashed, so
    // no wait on the loads precedes the chunk's MFMAs (a second register set for a two-chunk distance
    // measured slower: the extra VGPRs cost occupancy)
    double ra[LA], rb[LB];
    unsigned oka = 0, okb = 0;
    auto fetch = [&](int kc) {
      oka = okb = 0;
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int e = tid + NT * u, r = e % BM, k = kc + e / BM;
        const bool ok = k < kb && I0 + r < mrows;
        ra[u] = A[ok ? k * lda + I0 + r : 0];
        oka |= (unsigned)ok << u;
      }
#pragma unroll
      for (int u = 0; u < LB; ++u) {
        const int e = tid + NT * u, r = e % BN, k = kc + e / BN;
        const bool ok = k < kb && J0 + r < mrows;
        rb[u] = A[ok ? k * lda + J0 + r : 0];
        okb |= (unsigned)ok << u;
      }
    };
    auto stash = [&](int b) {
#pragma unroll
      for (int u = 0; u < LA; ++u) {
        const int e = tid + NT * u;
        lds[b * BUF + (e / BM) * SA + e % BM] = (oka >> u) & 1 ? ra[u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < LB; ++u) {
        const int e = tid + NT * u;
        lds[b * BUF + KC * SA + (e / BN) * SB + e % BN] = (okb >> u) & 1 ? rb[u] : 0.0;
      }
    };
    gdx4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = gdx4{0.0, 0.0, 0.0, 0.0};
    fetch(ka);
    stash(0);
    __syncthreads();
    const int nch = (kb - ka + KC - 1) / KC;
    for (int c = 0; c < nch; ++c) {
      const int b = c & 1;
      fetch(ka + (c + 1) * KC);  // past kb: fully masked, stashed into the idle buffer
      const double* pa = lds + b * BUF + wr * (BM / WM) + lr;
      const double* pb = lds + b * BUF + KC * SA + wc * (BN / WN) + lr;
#pragma unroll
      for (int kk = 0; kk < KC / 4; ++kk) {
        const int k = kk * 4 + lk;
        double fa[MI], fb[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = pa[k * SA + 16 * i];
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[j] = pb[k * SB + 16 * j];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
      if (yv && tid < BM) {  // masked entries (k >= kb) were stashed as zeros
        const int k0 = ka + c * KC;
        for (int k = 0; k < KC && k0 + k < kb; ++k) vdot += lds[b * BUF + k * SA + tid] * yv[k0 + k];
      }
      stash(b ^ 1);
      __syncthreads();
    }
    if (yv && tid < BM && I0 + tid < mrows) vout[I0 + tid] -= vdot;
    // (short K only: with a long K loop the tile's own epilogue measured faster, C4 K = 384 pass 48 vs 51 us)
    if (LDS_EPILOGUE && (overwrite || kb - ka <= 2 * KC)) {
      // acc -> LDS tile (row-major, stride BN + 1), then thread t owns row t % BM of columns t / BM, + NT / BM, ...
      constexpr int CS = BN + 1, CPI = NT / BM;  // columns per pass
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            lds[(wr * (BM / WM) + 16 * i + lk + 4 * q) * CS + wc * (BN / WN) + 16 * j + lr] = acc[i][j][q];
      __syncthreads();
      const int r = tid % BM, gi = I0 + r;
      constexpr int NP = BN / CPI;
      double cv[NP];
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const int c = tid / BM + CPI * u, gj = J0 + c;
        cv[u] = overwrite ? 0.0 : ld0(C, gj * ldc + gi, gi < mrows && gj < climit && gi >= gj);
      }
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const int c = tid / BM + CPI * u, gj = J0 + c;
        if (gi < mrows && gj < climit && gi >= gj) C[(size_t)gj * ldc + gi] = cv[u] - lds[r * CS + c];
      }
      return;
    }
    // epilogue: C -= acc, lane holds D[lk + 4q][lr] of each 16x16 block; one block column at a time
    // (all loads of the column in flight, then the stores)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gj = J0 + wc * (BN / WN) + 16 * j + lr;
      double cv[MI][4];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gi = I0 + wr * (BM / WM) + 16 * i + lk + 4 * q;
          cv[i][q] = overwrite ? 0.0 : ld0(C, gj * ldc + gi, gi < mrows && gj < climit && gi >= gj);
        }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gi = I0 + wr * (BM / WM) + 16 * i + lk + 4 * q;
          if (gi < mrows && gj < climit && gi >= gj) C[(size_t)gj * ldc + gi] = cv[i][q] - acc[i][j][q];
        }
    }
  }
};

// The same tile update with the operands staged global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging)
// in an NS-stage ring: chunk c + NS - 1 is issued while chunk c is multiplied, so NS - 1 chunks (KC columns each) are
// in flight across every barrier (counted s_waitcnt vmcnt, raw s_barrier: __syncthreads would drain the DMA).
// The DMA writes lane-linear 1 KiB per wave instruction, so the LDS image of a chunk is CPI = 128 / BM columns per
// instruction (a column = BM contiguous rows of the column-major operand), column groups padded by PAD doubles.
// Out-of-range sources are clamped (rows >= mrows only feed outputs that are never stored; columns >= kb are zeroed at
// the fragment read of the last chunk). A piece is two consecutive rows: the one starting at row mrows - 1 also reads
// the element after the column's last row (the next column's first, or past the operand's end: callers leave one
// 16-byte piece of slack after A).
template <int BM, int BN, int WM = 2, int WN = 2, int KC_ = 16, int NS = 3>
struct GemmNTd {
  static constexpr int ROWS = BM;  // rows of C per tile (k_syrk's row-tile unit)
  static constexpr int NT = 64 * WM * WN, NW = WM * WN;
  static constexpr int KC = KC_;
  static_assert(BM == 64 || BM == 128, "BM: one or two columns per DMA instruction");
  static_assert(BN == 64 || BN == 128, "BN: one or two columns per DMA instruction");
  static constexpr int CPA = 128 / BM, CPB = 128 / BN;      // columns per instruction
  static constexpr int PAD = 16;
  static constexpr int GA = CPA * BM + PAD, GB = CPB * BN + PAD;  // column-group strides (doubles)
  static constexpr int IA = KC / CPA, IB = KC / CPB;           // instructions per chunk and operand
  static_assert(IA % NW == 0 && IB % NW == 0, "every wave issues the same number of DMA instructions");
  static constexpr int JA = IA / NW, JB = IB / NW;             // per wave (= per thread)
  static constexpr int STAGE = IA * GA + IB * GB;              // doubles per stage
  // the LDS epilogue (short K, or a written-only C) needs a BM x (BN + 1) image: 64-row tiles only (a 128-row tile
  // would double its LDS and halve the workgroups per CU; it stores from the MFMA layout instead)
  static constexpr bool LDS_EPI = BM == 64;
  static constexpr int LDS_DOUBLES = LDS_EPI && BM * (BN + 1) > NS * STAGE ? BM * (BN + 1) : NS * STAGE;
  static constexpr int MI = BM / WM / 16, NJ = BN / WN / 16;
  static constexpr int G = JA + JB;                            // DMA instructions per thread per chunk

  __device__ static double* aptr(double* st, int k, int r) { return st + (k / CPA) * GA + (k % CPA) * BM + r; }
  __device__ static double* bptr(double* st, int k, int r) { return st + IA * GA + (k / CPB) * GB + (k % CPB) * BN + r; }

  __device__ __forceinline__ static void run(const double* __restrict__ A, int lda, double* __restrict__ C, int ldc, int mrows,
                             int climit, int I0, int J0, int ka, int kb, double* lds, bool overwrite = false,
                             const double* yv = nullptr, double* vout = nullptr) {
    run_ab(A, lda, mrows, A, lda, mrows, C, ldc, mrows, climit, I0, J0, ka, kb, lds, overwrite ? 1 : 0, yv, vout);
  }
  // General form: C(I, J) op A(I, K) B(J, K)^T with A (rows < arows, leading dimension lda) and B (rows < brows, ldb)
  // column-major. mode 0: C -= A B^T on the lower triangle (rows < mrows, columns < climit); 1: the same with C known
  // to be zero (not read); 2: C = A B^T on the whole tile (no triangle). yv / vout (mode 0 / 1, diagonal tiles): also
  // vout[r] -= sum_k A(I0 + r, k) yv[k] for the tile's rows (the front vector's rows below the supernode).
  __device__ __forceinline__ static void run_ab(const double* __restrict__ A, int lda, int arows, const double* __restrict__ Bm,
                                                int ldb, int brows, double* __restrict__ C, int ldc, int mrows, int climit,
                                                int I0, int J0, int ka, int kb, double* lds, int mode,
                                                const double* yv = nullptr, double* vout = nullptr) {
    const bool overwrite = mode == 1, full = mode == 2;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w % WM, wc = w / WM;
    const int lr = lane & 15, lk = lane >> 4;
    // chunk kc -> stage st: instruction j of wave w covers column group g = j NW + w, lane l the 16-B piece l of it
    auto issue = [&](int kc, double* st) {
#pragma unroll
      for (int j = 0; j < JA; ++j) {
        const int g = j * NW + w, col = g * CPA + lane / (BM / 2), row = 2 * (lane % (BM / 2));
        const int k = min(kc + col, kb - 1), r = min(I0 + row, arows - 1);  // (row arows - 1, arows): see below
        __builtin_amdgcn_global_load_lds((const void*)(A + (size_t)k * lda + r),
                                         (__attribute__((address_space(3))) void*)(st + g * GA), 16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int g = j * NW + w, col = g * CPB + lane / (BN / 2), row = 2 * (lane % (BN / 2));
        const int k = min(kc + col, kb - 1), r = min(J0 + row, brows - 1);
        __builtin_amdgcn_global_load_lds((const void*)(Bm + (size_t)k * ldb + r),
                                         (__attribute__((address_space(3))) void*)(st + IA * GA + g * GB), 16, 0, 0);
      }
    };
    gdx4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = gdx4{0.0, 0.0, 0.0, 0.0};
    const int nch = (kb - ka + KC - 1) / KC;
    double vdot = 0.0;
    // a wave whose output block lies wholly above the diagonal (the upper quadrant of a diagonal tile; lower-triangle
    // modes only) skips its products: nothing of it is stored, and its SIMD serves the other workgroups meanwhile
    const bool upper_w = !full && I0 + wr * (BM / WM) + BM / WM <= J0 + wc * (BN / WN);
    const bool lds_epi = LDS_EPI && !full && (overwrite || kb - ka <= 2 * KC) && NT % BM == 0;
#pragma unroll
    for (int c = 0; c < NS - 1; ++c)
      if (c < nch) issue(ka + c * KC, lds + c * STAGE);
    for (int c = 0; c < nch; ++c) {
      // chunk c landed (the younger chunks issued after it may stay in flight), then every wave's pieces of it are
      // visible and every wave is done with the stage chunk c + NS - 1 overwrites
      const int ahead = min(nch - 1 - c, NS - 2);  // chunks issued after c
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (c + NS - 1 < nch) issue(ka + (c + NS - 1) * KC, lds + ((c + NS - 1) % NS) * STAGE);
      double* st = lds + (c % NS) * STAGE;
      const int kv = min(KC, kb - ka - c * KC);  // valid columns of this chunk
      if (kv < KC) {
        // the tail chunk (uniform): its columns past kv hold clamped copies of column kb - 1; zero them so the
        // full-chunk products below apply unchanged (one path through the chunk loop: a predicated tail path made
        // the compiler carry the accumulators in two register sets and copy them at every chunk's end)
        for (int e = tid; e < (KC - kv) * (BM + BN); e += NT) {
          const int k = kv + e / (BM + BN), r = e % (BM + BN);
          *(r < BM ? aptr(st, k, r) : bptr(st, k, r - BM)) = 0.0;
        }
        __syncthreads();
      }
      // fragments double-buffered in registers: k-step kk + 1's LDS reads are in flight under k-step kk's MFMAs
      double fa[2][MI], fb[2][NJ];
      auto frag = [&](int kk, int s) {
        const int k = kk * 4 + lk;
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[s][i] = *aptr(st, k, wr * (BM / WM) + 16 * i + lr);
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[s][j] = *bptr(st, k, wc * (BN / WN) + 16 * j + lr);
      };
      if (!upper_w) {
        frag(0, 0);
#pragma unroll
        for (int kk = 0; kk < KC / 4; ++kk) {
          if (kk + 1 < KC / 4) frag(kk + 1, (kk + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);  // keep the next reads ahead of these MFMAs (the scheduler sinks them)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[kk & 1][i], fb[kk & 1][j], acc[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (yv && tid < BM) {  // the tile's rows of A times the chunk of y (workgroup-uniform branch per launch task)
        const double* yc = yv + ka + c * KC;
        for (int k = 0; k < kv; ++k) vdot += *aptr(st, k, tid) * yc[k];
      }
    }
    if (yv && tid < BM && I0 + tid < arows) vout[I0 + tid] -= vdot;
    // every DMA retired (the last chunk waited vmcnt(0)); the LDS epilogue reuses the ring after a barrier
    if (lds_epi) {
      __syncthreads();
      constexpr int CS = BN + 1, CPI = NT / BM;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            lds[(wr * (BM / WM) + 16 * i + lk + 4 * q) * CS + wc * (BN / WN) + 16 * j + lr] = acc[i][j][q];
      __syncthreads();
      const int r = tid % BM, gi = I0 + r;
      constexpr int NP = BN / CPI;
      double cv[NP];
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const int c = tid / BM + CPI * u, gj = J0 + c;
        cv[u] = overwrite ? 0.0 : ld0(C, gj * ldc + gi, gi < mrows && gj < climit && gi >= gj);
      }
#pragma unroll
      for (int u = 0; u < NP; ++u) {
        const int c = tid / BM + CPI * u, gj = J0 + c;
        if (gi < mrows && gj < climit && gi >= gj) C[(size_t)gj * ldc + gi] = cv[u] - lds[r * CS + c];
      }
      return;
    }
    if (full) {  // C = A B^T, every entry of the tile in range
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int gj = J0 + wc * (BN / WN) + 16 * j + lr;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int gi = I0 + wr * (BM / WM) + 16 * i + lk + 4 * q;
            if (gi < mrows && gj < climit) C[(size_t)gj * ldc + gi] = acc[i][j][q];
          }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int gj = J0 + wc * (BN / WN) + 16 * j + lr;
      double cv[MI][4];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gi = I0 + wr * (BM / WM) + 16 * i + lk + 4 * q;
          cv[i][q] = overwrite ? 0.0 : ld0(C, gj * ldc + gi, gi < mrows && gj < climit && gi >= gj);
        }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int gi = I0 + wr * (BM / WM) + 16 * i + lk + 4 * q;
          if (gi < mrows && gj < climit && gi >= gj) C[(size_t)gj * ldc + gi] = cv[i][q] - acc[i][j][q];
        }
    }
  }
};

}  // namespace g2ohip

