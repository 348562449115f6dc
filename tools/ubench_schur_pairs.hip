// Dev micro-benchmark (r06): the pair products of the Schur row pass (k_schur_rows with the r05 Kt
// records) on the FP64 VALU against two MFMA formulations, at the C4 row / partner shapes, everything else equal.
//
// Workload (one workgroup per camera row, as k_schur_rows): a row of C4 walks ~1000 landmarks in batches of 192 staged
// 80-byte records [Kt (2 x 3) | u v w | 0]; each staged landmark brings its own observation a and its partners b (camera
// j > i of the same landmark), every partner a pair (a, b) into slot j - i - 1 of the row's <= 64 off-diagonal slots;
// pairs slot-sorted with a per-batch slot CSR. Synthetic C4 geometry: each landmark sees 10 distinct cameras of a
// 64-camera window containing the row. The staged batch is built once per workgroup in LDS, then the pair products of
// NB batches run over it (the pass's 1000 / 35 batches per row), so only the products and their LDS operand reads are
// timed. All variants produce S(i, j) += sum over the slot's pairs of G_a G_b^T with G = Bt^T Kt (checked against each
// other and a host reference).
//   V   the production pair loop (kernels.hip schur_pairs_kx): 4 threads per slot (column half x pair parity), each pair
//       rebuilt from the records (M = Kt_a Kt_b^T, T = M Bt_b, acc += Bt_a^T T)
//   M1  v_mfma_f64_4x4x4f64, one instruction per pair (the 8 x 8 padded G_a G_b^T as four 4 x 4 blocks, K = 3 -> 4),
//       G formed once per staged block into LDS (6 x 3 each); wave w walks slots w, w + 4, ... (16 accumulators)
//   M2  the same with K packed: a slot's pairs concatenated along K (3 per pair), 4 K values per instruction
// Each variant is timed over the same task list; the layout candidate of v_mfma_f64_4x4x4f64 comes from
// tools/ubench_mfma4x4.hip (argv[1]: "ca cb cd", default "0 0 0").
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 tools/ubench_schur_pairs.hip -o tools/ubench_schur_pairs
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

constexpr int SB = 192, SL = 64, GB = 10;

struct Lay {  // per-lane roles of v_mfma_f64_4x4x4f64 (block, x, y) for A (b, i, k), B (b, k, j), D (b, i, j)
  int ab[64], ai[64], ak[64], bb[64], bk[64], bj[64], db[64], di[64], dj[64];
};
__constant__ Lay c_lay;

static void inv_lane(int cand, int lane, int& b, int& x, int& y) {
  switch (cand) {
    case 0: b = lane / 16; x = lane % 4; y = (lane / 4) % 4; break;   // lane = 16 b + x + 4 y
    case 1: b = lane / 16; y = lane % 4; x = (lane / 4) % 4; break;   // lane = 16 b + y + 4 x
    case 2: b = lane % 4; x = (lane / 4) % 4; y = lane / 16; break;   // lane = b + 4 x + 16 y
    case 3: b = lane % 4; y = (lane / 4) % 4; x = lane / 16; break;   // lane = b + 4 y + 16 x
    case 4: x = lane % 4; b = (lane / 4) % 4; y = lane / 16; break;   // lane = x + 4 b + 16 y
    default: y = lane % 4; b = (lane / 4) % 4; x = lane / 16; break;  // lane = y + 4 b + 16 x
  }
}

__device__ __forceinline__ void bt_rows(double u, double v, double w, double (&a0)[6], double (&a1)[6]) {
  a0[0] = u * v; a0[1] = -(1.0 + u * u); a0[2] = v; a0[3] = -w; a0[4] = 0.0; a0[5] = u * w;
  a1[0] = 1.0 + v * v; a1[1] = -(u * v); a1[2] = -u; a1[3] = 0.0; a1[4] = -w; a1[5] = v * w;
}

// ---- V: the production formulation (schur_pairs_kx + the parity combine)
__global__ void __launch_bounds__(256, 4) k_valu(const double* __restrict__ recs, const int* __restrict__ pairs,
                                                 const int* __restrict__ pp, int nbatch, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double Gs[SB * GB];
  __shared__ int sp[SB * 2];
  __shared__ int spp[SL + 1];
  const int row = blockIdx.x, tid = threadIdx.x, ls = tid >> 2, q = tid & 3;
  for (int e = tid; e < SB * GB; e += 256) Gs[e] = recs[(size_t)row * SB * GB + e];
  for (int e = tid; e < SB * 2; e += 256) sp[e] = pairs[(size_t)row * SB * 2 + e];
  if (tid <= SL) spp[tid] = pp[row * (SL + 1) + tid];
  __syncthreads();
  double acc[18];
#pragma unroll
  for (int k = 0; k < 18; ++k) acc[k] = 0.0;
  const int par = q >> 1;
  const bool hi = q & 1;
  for (int it = 0; it < nbatch; ++it) {
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
      double M[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int s = 0; s < 2; ++s) M[r][s] = ka[r] * kb[s] + ka[2 + r] * kb[2 + s] + ka[4 + r] * kb[4 + s];
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
#pragma unroll
  for (int k = 0; k < 18; ++k) acc[k] += __shfl_xor(acc[k], 2, 4);
  if (par == 0) {
    const int c0 = hi ? 3 : 0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 6; ++r) out[((size_t)row * SL + ls) * 36 + (c0 + j) * 6 + r] = acc[j * 6 + r];
  }
}

// G = Bt^T Kt for every staged record, 6 x 3 row-major (18 doubles) into Gm
__device__ __forceinline__ void form_g(const double* Gs, double* Gm, int tid) {
  for (int e = tid; e < SB * 18; e += 256) {
    const int item = e / 18, ik = e - item * 18, i = ik / 3, k = ik - 3 * i;
    const double* r = Gs + item * GB;
    double a0[6], a1[6];
    bt_rows(r[6], r[7], r[8], a0, a1);
    Gm[e] = a0[i] * r[2 * k] + a1[i] * r[2 * k + 1];
  }
}

// ---- M1: one 4x4x4 instruction per pair
__global__ void __launch_bounds__(256, 4) k_mfma1(const double* __restrict__ recs, const int* __restrict__ pairs,
                                                  const int* __restrict__ pp, int nbatch, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double Gs[SB * GB];
  __shared__ double Gm[SB * 18];
  __shared__ int sp[SB * 2];
  __shared__ int spp[SL + 1];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int e = tid; e < SB * GB; e += 256) Gs[e] = recs[(size_t)row * SB * GB + e];
  for (int e = tid; e < SB * 2; e += 256) sp[e] = pairs[(size_t)row * SB * 2 + e];
  if (tid <= SL) spp[tid] = pp[row * (SL + 1) + tid];
  __syncthreads();
  // A (b, i, k): row 4 (b >> 1) + i of G_a, column k; B (b, k, j): row 4 (b & 1) + j of G_b, column k
  const int ra = 4 * (c_lay.ab[lane] >> 1) + c_lay.ai[lane], ka = c_lay.ak[lane];
  const int rb = 4 * (c_lay.bb[lane] & 1) + c_lay.bj[lane], kb = c_lay.bk[lane];
  const bool oka = ra < 6 && ka < 3, okb = rb < 6 && kb < 3;
  const int offa = oka ? ra * 3 + ka : 0, offb = okb ? rb * 3 + kb : 0;
  double acc[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) acc[m] = 0.0;
  for (int it = 0; it < nbatch; ++it) {
    form_g(Gs, Gm, tid);  // (per batch in the real pass)
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int s = w + 4 * m;
      const int p1 = spp[s + 1];
      for (int p = spp[s]; p < p1; ++p) {
        const int pr = sp[p];
        const double a = Gm[(pr & 0xffff) * 18 + offa], b = Gm[(pr >> 16) * 18 + offb];
        acc[m] = __builtin_amdgcn_mfma_f64_4x4x4f64(oka ? a : 0.0, okb ? b : 0.0, acc[m], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  const int r = 4 * (c_lay.db[lane] >> 1) + c_lay.di[lane], c = 4 * (c_lay.db[lane] & 1) + c_lay.dj[lane];
#pragma unroll
  for (int m = 0; m < 16; ++m)
    if (r < 6 && c < 6) out[((size_t)row * SL + w + 4 * m) * 36 + c * 6 + r] = acc[m];
}

// ---- M2: K packed, 4 K values (4/3 pairs) per instruction
__global__ void __launch_bounds__(256, 4) k_mfma2(const double* __restrict__ recs, const int* __restrict__ pairs,
                                                  const int* __restrict__ pp, int nbatch, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double Gs[SB * GB];
  __shared__ double Gm[SB * 18];
  __shared__ int sp[SB * 2];
  __shared__ int spp[SL + 1];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int e = tid; e < SB * GB; e += 256) Gs[e] = recs[(size_t)row * SB * GB + e];
  for (int e = tid; e < SB * 2; e += 256) sp[e] = pairs[(size_t)row * SB * 2 + e];
  if (tid <= SL) spp[tid] = pp[row * (SL + 1) + tid];
  __syncthreads();
  const int ra = 4 * (c_lay.ab[lane] >> 1) + c_lay.ai[lane], ka = c_lay.ak[lane];
  const int rb = 4 * (c_lay.bb[lane] & 1) + c_lay.bj[lane], kb = c_lay.bk[lane];
  const bool oka = ra < 6, okb = rb < 6;
  double acc[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) acc[m] = 0.0;
  for (int it = 0; it < nbatch; ++it) {
    form_g(Gs, Gm, tid);
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int s = w + 4 * m;
      const int p0 = spp[s], kt = 3 * (spp[s + 1] - p0);  // the slot's K extent
      for (int k0 = 0; k0 < kt; k0 += 4) {
        const int xa = k0 + ka, xb = k0 + kb;  // this lane's K position for A and for B
        const bool ia = oka && xa < kt, ib = okb && xb < kt;
        const int pa = sp[p0 + (ia ? xa / 3 : 0)], pb = sp[p0 + (ib ? xb / 3 : 0)];
        const double a = Gm[(pa & 0xffff) * 18 + (ia ? ra * 3 + xa % 3 : 0)];
        const double b = Gm[(pb >> 16) * 18 + (ib ? rb * 3 + xb % 3 : 0)];
        acc[m] = __builtin_amdgcn_mfma_f64_4x4x4f64(ia ? a : 0.0, ib ? b : 0.0, acc[m], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  const int r = 4 * (c_lay.db[lane] >> 1) + c_lay.di[lane], c = 4 * (c_lay.db[lane] & 1) + c_lay.dj[lane];
#pragma unroll
  for (int m = 0; m < 16; ++m)
    if (r < 6 && c < 6) out[((size_t)row * SL + w + 4 * m) * 36 + c * 6 + r] = acc[m];
}

int main(int argc, char** argv) {
  int ca = 0, cb = 0, cd = 0;
  if (argc >= 4) { ca = atoi(argv[1]); cb = atoi(argv[2]); cd = atoi(argv[3]); }
  Lay lay;
  for (int l = 0; l < 64; ++l) {
    inv_lane(ca, l, lay.ab[l], lay.ai[l], lay.ak[l]);
    inv_lane(cb, l, lay.bb[l], lay.bk[l], lay.bj[l]);
    inv_lane(cd, l, lay.db[l], lay.di[l], lay.dj[l]);
  }
  (void)hipMemcpyToSymbol(HIP_SYMBOL(c_lay), &lay, sizeof(Lay));
  const int nrow = 1000, nbatch = 29;  // C4: 1000 rows, ~1000 landmarks each in batches of ~35 landmarks
  std::mt19937 rng(7);
  std::vector<double> recs((size_t)nrow * SB * GB);
  std::vector<int> pairs((size_t)nrow * SB * 2, 0), pp((size_t)nrow * (SL + 1), 0);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  long long npairs = 0;
  for (int row = 0; row < nrow; ++row) {
    // landmarks: 10 distinct cameras of a 64-window containing the row; partners j > row
    std::vector<std::vector<std::pair<int, int>>> slot_pairs(SL);
    int st = 0;
    while (true) {
      const int c0 = row - (int)(rng() % 64);
      std::vector<int> cams{row};
      while ((int)cams.size() < 10) {
        const int c = c0 + (int)(rng() % 64);
        bool dup = false;
        for (int x : cams) dup |= x == c;
        if (!dup) cams.push_back(c);
      }
      int np = 0;
      for (int c : cams) np += c > row;
      if (st + 1 + np > SB) break;
      const int a = st++;
      for (int c : cams)
        if (c > row && c - row - 1 < SL) slot_pairs[c - row - 1].push_back({a, st++});
    }
    for (int e = 0; e < SB; ++e) {
      double* r = &recs[((size_t)row * SB + e) * GB];
      for (int k = 0; k < 6; ++k) r[k] = U(rng);
      r[6] = 0.3 * U(rng); r[7] = 0.3 * U(rng); r[8] = 0.5 + 0.2 * U(rng); r[9] = 0.0;
    }
    int p = 0;
    for (int s = 0; s < SL; ++s) {
      pp[(size_t)row * (SL + 1) + s] = p;
      for (auto& ab : slot_pairs[s]) pairs[(size_t)row * SB * 2 + p++] = ab.first | (ab.second << 16);
    }
    pp[(size_t)row * (SL + 1) + SL] = p;
    npairs += p;
  }
  double *drec, *dout[3];
  int *dpairs, *dpp;
  (void)hipMalloc(&drec, recs.size() * 8);
  (void)hipMalloc(&dpairs, pairs.size() * 4);
  (void)hipMalloc(&dpp, pp.size() * 4);
  for (int v = 0; v < 3; ++v) {
    (void)hipMalloc(&dout[v], (size_t)nrow * SL * 36 * 8);
    (void)hipMemset(dout[v], 0, (size_t)nrow * SL * 36 * 8);
  }
  (void)hipMemcpy(drec, recs.data(), recs.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dpairs, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dpp, pp.data(), pp.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("C4-shaped rows: %d rows x %d batches, %.1f pairs per batch per row (%.2f M pairs per pass)\n", nrow, nbatch,
         (double)npairs / nrow, npairs * nbatch / 1e6);
  auto run = [&](auto kern, int v, const char* name) {
    hipLaunchKernelGGL(kern, nrow, 256, 0, 0, drec, dpairs, dpp, nbatch, dout[v]);
    (void)hipDeviceSynchronize();
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kern, nrow, 256, 0, 0, drec, dpairs, dpp, nbatch, dout[v]);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = std::fmin(best, ms);
    }
    printf("%-44s %8.1f us  (%.2f ns per pair per CU)\n", name, best * 1e3, best * 1e6 * 256 / (npairs * nbatch));
  };
  run(k_valu, 0, "V  VALU pair loop (production)");
  run(k_mfma1, 1, "M1 MFMA 4x4x4, one instruction per pair");
  run(k_mfma2, 2, "M2 MFMA 4x4x4, K packed");
  // check: all three against a host reference (S = nbatch x the batch's sum), relative to the largest entry
  std::vector<double> h[3];
  for (int v = 0; v < 3; ++v) {
    h[v].resize((size_t)nrow * SL * 36);
    (void)hipMemcpy(h[v].data(), dout[v], h[v].size() * 8, hipMemcpyDeviceToHost);
  }
  double maxref = 0, err[3] = {0, 0, 0};
  for (int row = 0; row < nrow; row += 97) {
    for (int s = 0; s < SL; ++s) {
      double ref[36] = {0};
      for (int p = pp[(size_t)row * (SL + 1) + s]; p < pp[(size_t)row * (SL + 1) + s + 1]; ++p) {
        const int pr = pairs[(size_t)row * SB * 2 + p];
        const double* ra = &recs[((size_t)row * SB + (pr & 0xffff)) * GB];
        const double* rb = &recs[((size_t)row * SB + (pr >> 16)) * GB];
        double ga[18], gb[18];
        for (int g = 0; g < 2; ++g) {
          const double* r = g ? rb : ra;
          double* G = g ? gb : ga;
          const double u = r[6], vv = r[7], w = r[8];
          const double a0[6] = {u * vv, -(1.0 + u * u), vv, -w, 0.0, u * w};
          const double a1[6] = {1.0 + vv * vv, -(u * vv), -u, 0.0, -w, vv * w};
          for (int i = 0; i < 6; ++i)
            for (int k = 0; k < 3; ++k) G[i * 3 + k] = a0[i] * r[2 * k] + a1[i] * r[2 * k + 1];
        }
        for (int r = 0; r < 6; ++r)
          for (int c = 0; c < 6; ++c)
            for (int k = 0; k < 3; ++k) ref[c * 6 + r] += nbatch * ga[r * 3 + k] * gb[c * 3 + k];
      }
      for (int e = 0; e < 36; ++e) {
        maxref = std::fmax(maxref, std::fabs(ref[e]));
        for (int v = 0; v < 3; ++v)
          err[v] = std::fmax(err[v], std::fabs(h[v][((size_t)row * SL + s) * 36 + e] - ref[e]));
      }
    }
  }
  printf("check vs host (max abs err / max entry): V %.1e  M1 %.1e  M2 %.1e\n", err[0] / maxref, err[1] / maxref,
         err[2] / maxref);
  return 0;
}
