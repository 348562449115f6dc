// Host orchestration of the MI355X BlockSolver backend.
//
// Mirrors, behind the same contracts:
//   SparseOptimizer::initializeOptimization / buildIndexMapping (sparse_optimizer.cpp:168-279)
//   BlockSolver::buildStructure / buildSystem / setLambda / restoreDiagonal / solve
//       (block_solver.hpp:102-256, 462-565, 314-447)
//   OptimizationAlgorithmLevenberg::solve / computeLambdaInit / computeScale
//       (optimization_algorithm_levenberg.cpp:58-184)
//   SparseOptimizer::optimize (sparse_optimizer.cpp:374-439), G2OBatchStatistics timers
// The graph state lives in HBM during optimize(); the host only reads scalars
// (chi2, scale, the not-PD flag) once per LM trial.
#include "engine.hpp"


#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>
#include <numeric>
#include <sstream>

namespace g2ohip {

static double wall() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int vertex_dim(int t) { return t == G2OHIP_V_SE3_EXPMAP || t == G2OHIP_V_SE3_QUAT ? 6 : (t == G2OHIP_V_XYZ || t == G2OHIP_V_SE2 ? 3 : -1); }
int vertex_est_dim(int t) { return t == G2OHIP_V_SE3_EXPMAP || t == G2OHIP_V_SE3_QUAT ? 7 : 3; }
int vertex_state_stride(int t) {
  switch (t) {
    case G2OHIP_V_SE3_EXPMAP: return 8;
    case G2OHIP_V_XYZ: return 3;
    case G2OHIP_V_SE3_QUAT: return 12;
    case G2OHIP_V_SE2: return 3;
  }
  return 0;
}
int edge_dim(int e) { return e == G2OHIP_E_SE3_PROJECT_XYZ ? 2 : (e == G2OHIP_E_SE3_QUAT ? 6 : (e == G2OHIP_E_SE2 ? 3 : -1)); }
int edge_meas_dim(int e) { return e == G2OHIP_E_SE3_PROJECT_XYZ ? 2 : (e == G2OHIP_E_SE3_QUAT ? 7 : 3); }

// ------------------------------------------------------------------ host-side math for I/O
namespace {
void q2R(double qx, double qy, double qz, double qw, double* R) {
  const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const double twx = tx * qw, twy = ty * qw, twz = tz * qw, txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}
void R2q(const double* R, double* q) {
  double t = R[0] + R[4] + R[8];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (R[7] - R[5]) * t; q[1] = (R[2] - R[6]) * t; q[2] = (R[3] - R[1]) * t;
  } else {
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[i * 4]) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
    double c[3];
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (R[k * 3 + j] - R[j * 3 + k]) * t;
    c[j] = (R[j * 3 + i] + R[i * 3 + j]) * t;
    c[k] = (R[k * 3 + i] + R[i * 3 + k]) * t;
    q[0] = c[0]; q[1] = c[1]; q[2] = c[2];
  }
}
void qnorm_pos(double* q) {
  if (q[3] < 0) for (int k = 0; k < 4; ++k) q[k] = -q[k];
  const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int k = 0; k < 4; ++k) q[k] /= n;
}
void qrot_h(const double* q, const double* v, double* o) {
  double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
  for (double& u : uv) u += u;
  o[0] = v[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
  o[1] = v[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
  o[2] = v[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
}
double norm_theta(double th) {
  const double pi = 3.14159265358979323846;
  if (th >= -pi && th < pi) return th;
  double m = std::floor(th / (2 * pi));
  th -= m * 2 * pi;
  if (th >= pi) th -= 2 * pi;
  if (th < -pi) th += 2 * pi;
  return th;
}
void se3quat_inverse(const double* tq /*t3 q4*/, double* out) {
  double qc[4] = {-tq[3], -tq[4], -tq[5], tq[6]};
  double mt[3] = {-tq[0], -tq[1], -tq[2]}, r[3];
  qrot_h(qc, mt, r);
  out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
  out[3] = qc[0]; out[4] = qc[1]; out[5] = qc[2]; out[6] = qc[3];
}
}  // namespace

void set_state_from_est(int vt, const double* est, double* st) {
  switch (vt) {
    case G2OHIP_V_SE3_EXPMAP: {
      double q[4] = {est[3], est[4], est[5], est[6]};
      qnorm_pos(q);
      st[0] = est[0]; st[1] = est[1]; st[2] = est[2];
      st[3] = q[0]; st[4] = q[1]; st[5] = q[2]; st[6] = q[3]; st[7] = 0;
      break;
    }
    case G2OHIP_V_XYZ: st[0] = est[0]; st[1] = est[1]; st[2] = est[2]; break;
    case G2OHIP_V_SE3_QUAT:  // fromVectorQT (isometry3d_mappings.cpp:126-131): no normalisation
      q2R(est[3], est[4], est[5], est[6], st);
      st[9] = est[0]; st[10] = est[1]; st[11] = est[2];
      break;
    case G2OHIP_V_SE2: st[0] = est[0]; st[1] = est[1]; st[2] = est[2]; break;
  }
}
void est_from_state(int vt, const double* st, double* est) {
  switch (vt) {
    case G2OHIP_V_SE3_EXPMAP:
      for (int k = 0; k < 7; ++k) est[k] = st[k];
      break;
    case G2OHIP_V_SE3_QUAT: {  // toVectorQT
      double q[4];
      R2q(st, q);
      const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      est[0] = st[9]; est[1] = st[10]; est[2] = st[11];
      est[3] = q[0] / n; est[4] = q[1] / n; est[5] = q[2] / n; est[6] = q[3] / n;
      break;
    }
    default: est[0] = st[0]; est[1] = st[1]; est[2] = st[2]; break;
  }
}
void minimal_from_state(int vt, const double* st, double* out) {
  switch (vt) {
    case G2OHIP_V_SE3_EXPMAP:
      for (int k = 0; k < 6; ++k) out[k] = st[k];
      break;
    case G2OHIP_V_SE3_QUAT: {  // toVectorMQT
      double q[4];
      R2q(st, q);
      const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      const double sg = q[3] < 0 ? -1.0 : 1.0;
      out[0] = st[9]; out[1] = st[10]; out[2] = st[11];
      out[3] = sg * q[0] / n; out[4] = sg * q[1] / n; out[5] = sg * q[2] / n;
      break;
    }
    default: out[0] = st[0]; out[1] = st[1]; out[2] = st[2]; break;
  }
}

// ------------------------------------------------------------------ KernelTimer
hipEvent_t KernelTimer::get() {
  if (!pool.empty()) {
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  hipEvent_t e;
  HIP_CHECK(hipEventCreate(&e));
  return e;
}
void KernelTimer::begin(const std::string& name, hipStream_t s) {
  open_ = false;
  if (!enabled || (!only.empty() && name != only)) return;
  open_ = true;
  Rec r;
  r.a = get();
  r.b = nullptr;
  r.name = name;
  HIP_CHECK(hipEventRecord(r.a, s));
  pending.push_back(r);
}
void KernelTimer::end(hipStream_t s) {
  if (!enabled || !open_ || pending.empty()) return;
  open_ = false;
  Rec& r = pending.back();
  r.b = get();
  HIP_CHECK(hipEventRecord(r.b, s));
}
void KernelTimer::collect() {
  for (auto& r : pending) {
    if (r.b) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
      total_ms[r.name] += ms;
      count[r.name] += 1;
      pool.push_back(r.b);
    }
    pool.push_back(r.a);
  }
  pending.clear();
}
KernelTimer::~KernelTimer() {
  for (auto& r : pending) {
    (void)hipEventDestroy(r.a);
    if (r.b) (void)hipEventDestroy(r.b);
  }
  for (auto e : pool) (void)hipEventDestroy(e);
}

// ------------------------------------------------------------------ DeviceCholesky
void DeviceCholesky::setup(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj,
                           hipStream_t s) {
  pd = bdim;
  BlockPattern P;
  P.nb = nblocks;
  P.dim.assign(nblocks, bdim);
  P.offset.resize(nblocks + 1);
  for (int k = 0; k <= nblocks; ++k) P.offset[k] = k * bdim;
  std::vector<int> deg(nblocks, 0);
  for (size_t t = 0; t < bi.size(); ++t)
    if (bi[t] != bj[t]) { deg[bi[t]]++; deg[bj[t]]++; }
  P.adjp.assign(nblocks + 1, 0);
  for (int k = 0; k < nblocks; ++k) P.adjp[k + 1] = P.adjp[k] + deg[k];
  P.adji.assign(P.adjp[nblocks], 0);
  std::vector<int> fill(P.adjp.begin(), P.adjp.end() - 1);
  for (size_t t = 0; t < bi.size(); ++t)
    if (bi[t] != bj[t]) { P.adji[fill[bi[t]]++] = bj[t]; P.adji[fill[bj[t]]++] = bi[t]; }
  sym = analyze(P);
  if ((long long)sym.max_front * sym.max_front >= (1LL << 31))
    throw DeviceError("front too large for 32-bit in-front indexing");
  // input entries per (permuted) scalar column: input block t (bi, bj) col-major bdim x bdim, value index
  // k = t bdim^2 + c bdim + r; the entry lands at front row rpos of its column (assembled per level by
  // k_extend_add, lambda added on the diagonal)
  nent = (long long)bi.size() * bdim * bdim;
  if (nent >= (1LL << 31)) throw DeviceError("reduced system too large for 32-bit entry indexing");
  std::vector<int> ecol, erow, esrc, cpv, ent_rowv, ent_srcv;
  std::vector<long long> edst, edsts;
  ecol.reserve(nent);
  erow.reserve(nent);
  esrc.reserve(nent);
  for (size_t t = 0; t < bi.size(); ++t)
    for (int c = 0; c < bdim; ++c)
      for (int r = 0; r < bdim; ++r) {
        const long long k = (long long)t * bdim * bdim + (long long)c * bdim + r;
        if (bi[t] == bj[t] && r > c) continue;
        const int gi = bi[t] * bdim + r, gj = bj[t] * bdim + c;
        const int a = sym.pinv[gi], b = sym.pinv[gj];
        const int row = std::max(a, b), col = std::min(a, b);
        const int sn = sym.block_sn[col / bdim];
        const Supernode& q = sym.sn[sn];
        int rpos;
        if (row < q.c0 + q.ns) rpos = row - q.c0;
        else {
          const int* rb = sym.rows.data() + q.rows_off;
          const int* it = std::lower_bound(rb, rb + q.nr, row);
          if (it == rb + q.nr || *it != row) throw std::runtime_error("cholesky setup: entry outside the symbolic pattern");
          rpos = q.ns + (int)(it - rb);
        }
        ecol.push_back(col);
        erow.push_back(rpos | (gi == gj ? (1 << 30) : 0));
        esrc.push_back((int)k);
        edst.push_back(q.front_off + (long long)(col - q.c0) * (q.ns + q.nr) + rpos);
      }
  {
    std::vector<int> cp(sym.n + 1, 0);
    for (int c : ecol) cp[c + 1]++;
    for (int c = 0; c < sym.n; ++c) cp[c + 1] += cp[c];
    std::vector<int> fillp(cp.begin(), cp.end() - 1), hr(ecol.size()), hs(ecol.size());
    for (size_t e = 0; e < ecol.size(); ++e) {
      const int d = fillp[ecol[e]]++;
      hr[d] = erow[e];
      hs[d] = esrc[e];
    }
    std::vector<long long> hd(ecol.size());
    fillp.assign(cp.begin(), cp.end() - 1);
    for (size_t e = 0; e < ecol.size(); ++e) hd[fillp[ecol[e]]++] = edst[e];
    colptr.upload(cp, s);
    ent_row.upload(hr.empty() ? std::vector<int>{0} : hr, s);
    ent_src.upload(hs.empty() ? std::vector<int>{0} : hs, s);
    cpv.swap(cp);
    ent_rowv.swap(hr);
    ent_srcv.swap(hs);
    edsts.swap(hd);
  }
  // extend-add slab width per level: EA columns where the level has enough of them to fill the chip
  // several times over, else 4 (latency-bound upper levels)
  std::vector<int> level_slab(sym.levels.size(), 4), sn_level(sym.sn.size(), 0);
  for (size_t l = 0; l < sym.levels.size(); ++l) {
    long long lcols = 0;
    for (int sn : sym.levels[l]) { lcols += sym.sn[sn].ns + sym.sn[sn].nr; sn_level[sn] = (int)l; }
    level_slab[l] = lcols >= 16LL * launch::CHOL_EA * 256 ? launch::CHOL_EA : 4;
  }
  // per child: [#rows mapping into the parent's first diagonal block | first child row of every parent
  // slab] (rel is increasing), so the extend-add tasks need no search on the chain
  std::vector<int> hjt, hcmp;
  std::vector<int2> hcme;
  std::vector<launch::FrontDesc> hfd(sym.sn.size());
  long long loff = 0, xoff = 0;
  for (size_t k = 0; k < sym.sn.size(); ++k) {
    const Supernode& q = sym.sn[k];
    int jt = 0;
    if (q.parent >= 0) {
      const Supernode& pq = sym.sn[q.parent];
      const int mp = pq.ns + pq.nr, slab = level_slab[sn_level[q.parent]], kb0 = std::min(launch::CHOL_NB, pq.ns);
      const int* rel = sym.relmap.data() + q.rows_off;
      jt = (int)hjt.size();
      hjt.push_back((int)(std::lower_bound(rel, rel + q.nr, kb0) - rel));
      for (int a = 0; a < mp + slab; a += slab) hjt.push_back((int)(std::lower_bound(rel, rel + q.nr, std::min(a, mp)) - rel));
    }
    // (child, child column) pairs of every column of this front, children in fixed order
    const int m = q.ns + q.nr, cm = (int)hcmp.size();
    {
      std::vector<int> cnt(m + 1, 0);
      for (int ci = sym.children_ptr[k]; ci < sym.children_ptr[k + 1]; ++ci) {
        const Supernode& cq = sym.sn[sym.children[ci]];
        for (int jc = 0; jc < cq.nr; ++jc) cnt[sym.relmap[cq.rows_off + jc] + 1]++;
      }
      for (int j = 0; j < m; ++j) cnt[j + 1] += cnt[j];
      const int base = (int)hcme.size();
      hcme.resize(base + cnt[m]);
      std::vector<int> fillc(cnt.begin(), cnt.end() - 1);
      for (int ci = sym.children_ptr[k]; ci < sym.children_ptr[k + 1]; ++ci) {
        const int c = sym.children[ci];
        const Supernode& cq = sym.sn[c];
        for (int jc = 0; jc < cq.nr; ++jc) hcme[base + fillc[sym.relmap[cq.rows_off + jc]]++] = int2{c, jc};
      }
      for (int j = 0; j <= m; ++j) hcmp.push_back(base + cnt[j]);
    }
    hfd[k] = launch::FrontDesc{q.front_off, q.vec_off, loff, q.rows_off, xoff, q.c0, q.ns, q.nr, q.parent,
                               sym.children_ptr[k], sym.children_ptr[k + 1], jt, cm};
    loff += (long long)(q.ns + q.nr) * q.ns;
    xoff += (long long)q.ns * q.ns;  // X = L11^-1, column-major
  }
  lpool = loff;
  fd.upload(hfd, s);
  jtab.upload(hjt.empty() ? std::vector<int>{0} : hjt, s);
  cmptr.upload(hcmp.empty() ? std::vector<int>{0} : hcmp, s);
  cment.upload(hcme.empty() ? std::vector<int2>{int2{0, 0}} : hcme, s);
  std::vector<int> ll;
  level_off.assign(1, 0);
  for (auto& lv : sym.levels) {
    ll.insert(ll.end(), lv.begin(), lv.end());
    level_off.push_back((int)ll.size());
  }
  // work lists per level: extend-add, first diagonal block, one step per 32-wide panel,
  // contribution blocks
  {
    using launch::Task;
    const int NB = launch::CHOL_NB, TT = launch::CHOL_TT, EA = launch::CHOL_EA;
    std::vector<Task> tk;
    std::vector<launch::StepTask> stk;
    std::vector<int> sn_pb(sym.sn.size(), 0);  // big-panel width of blocked fronts (0: unblocked)
    ops.clear();
    // contribution blocks: fused into the panel steps (each step's rank-32 update also reaches the
    // contribution block) where the steps are latency-bound on the diagonal chain and the extra tiles
    // run in its shadow; a separate K = ns k_syrk pass where a level's first step already has more
    // tiles than one round of the chip (re-reading the contribution block every step costs more)
    const char* fe = getenv("G2OHIP_CHOL_FUSED_MAX");  // dev A/B: fused-tile threshold per step
    const long long fused_max = fe ? atoll(fe) : 2LL * 256;
    const char* bm = getenv("G2OHIP_CHOL_BLOCK_MIN");  // dev A/B: widest supernode factored unblocked
    const int block_min = bm ? atoi(bm) : 512;
    const char* bp = getenv("G2OHIP_CHOL_PB");  // dev A/B: big-panel width (multiple of 64)
    const int block_pb = bp ? std::max(64, atoi(bp) / 64 * 64) : 256;
    const char* wf = getenv("G2OHIP_CHOL_WIDE_FRONTS");  // dev A/B: fronts per level that make it "wide"
    const int wide_fronts = wf ? atoi(wf) : 64;
    const char* wp = getenv("G2OHIP_CHOL_WIDE_PB");
    const int wide_pb = wp ? std::max(64, atoi(wp) / 64 * 64) : 128;
    const bool dev_noinv = getenv("G2OHIP_DEV_NOINV") != nullptr;  // timing experiments only (wrong solve)
    const bool dev_diagonly = getenv("G2OHIP_DEV_DIAGONLY") != nullptr;  // timing experiments only (wrong factor)
    const char* pm = getenv("G2OHIP_CHOL_PRE_MAX");  // dev A/B: largest level (bytes) pre-scattered
    const long long pre_max = pm ? atoll(pm) : (256LL << 20);
    std::vector<long long> zr, pdst;
    std::vector<int> psrc;
    for (size_t l = 0; l < sym.levels.size(); ++l) {
      const auto& lv = sym.levels[l];
      long long tiles0 = 0;  // fused tiles of the level's first step
      for (int sn : lv) {
        const Supernode& q = sym.sn[sn];
        const int r0 = std::min(NB, q.ns), T = (q.ns + q.nr - r0 + TT - 1) / TT;
        tiles0 += (long long)T * (T + 1) / 2;
      }
      const bool fused_contrib = tiles0 <= fused_max;
      // k_extend_add: every front's first-diagonal-block task first, then the slabs
      // small levels (all fronts <= pre_max bytes together) are zeroed + scattered before the first level
      // (two massively parallel passes off the critical chain); large ones are assembled in place
      long long lbytes = 0;
      for (int sn : lv) lbytes += 8LL * (sym.sn[sn].ns + sym.sn[sn].nr) * (sym.sn[sn].ns + sym.sn[sn].nr);
      const bool pre = lbytes <= pre_max;
      if (pre)
        for (int sn : lv) {
          const Supernode& q = sym.sn[sn];
          const long long len = (long long)(q.ns + q.nr) * (q.ns + q.nr);
          for (long long o = 0; o < len; o += 65536) { zr.push_back(q.front_off + o); zr.push_back(std::min(65536LL, len - o)); }
          for (int c = q.c0; c < q.c0 + q.ns; ++c)
            for (int e = cpv[c]; e < cpv[c + 1]; ++e) {
              pdst.push_back(edsts[e]);
              psrc.push_back(ent_srcv[e] | ((ent_rowv[e] >> 30) ? (int)0x80000000 : 0));
            }
        }
      int lmaxm = 0;
      for (int sn : lv) lmaxm = std::max(lmaxm, sym.sn[sn].ns + sym.sn[sn].nr);
      Op ea{pre ? 0 : (lmaxm <= 512 ? 5 : 4), (int)tk.size(), 0};
      for (int sn : lv) tk.push_back(Task{sn, 0, 0, 1});
      // every front is assembled here (input entries, zeros, children); slabs of EA columns where the level
      // has enough of them to fill the chip several times over, else 4 (latency-bound upper levels)
      const int slab = level_slab[l];
      for (int sn : lv) {
        const Supernode& q = sym.sn[sn];
        const int m = q.ns + q.nr;
        if (pre && sym.children_ptr[sn + 1] == sym.children_ptr[sn]) continue;  // nothing left to assemble
        for (int a = 0; a < m; a += slab) tk.push_back(Task{sn, a, std::min(a + slab, m), 2 + a / slab});
      }
      ea.count = (int)tk.size() - ea.off;
      ops.push_back(ea);
      int maxp = 0;
      for (int sn : lv) maxp = std::max(maxp, (sym.sn[sn].ns + NB - 1) / NB);
      // blocked fronts (wide supernodes on levels with a separate contribution pass): the rank-32 tile
      // updates of the panel steps stop at the end of the current big panel of PB columns; after each big
      // panel one high-intensity k_syrk launch applies its rank-PB update to the rest of the supernode's
      // columns, and a next-diagonal task (kb = 0) factors the first block of the next big panel
      // throughput-bound levels (many fronts: the panel steps' rank-32 tile traffic, not the diagonal
      // chain, sets their time) block every front wider than one small big panel
      const bool wide = (int)lv.size() >= wide_fronts;
      const int lpb = wide ? wide_pb : block_pb, lmin = wide ? wide_pb : block_min;
      auto blocked = [&](const Supernode& q) { return !fused_contrib && q.ns > lmin; };
      for (int p = 0; p < maxp; ++p) {
        Op st{2, (int)stk.size(), 0};
        // task order inside the launch (= dispatch order): every front's next-diagonal task first (the
        // critical chain must start at once, on a CU of its own), then the tile tasks, then the
        // inverse tasks (X = L11^-1 for the backward solve), which have the most slack
        std::vector<launch::StepTask> diag_t, tile_t, inv_t;
        for (int sn : lv) {
          const Supernode& q = sym.sn[sn];
          const int k0 = p * NB;
          if (k0 >= q.ns) continue;
          const int kb = std::min(NB, q.ns - k0), r0 = k0 + kb, m = q.ns + q.nr;
          const bool blk = blocked(q);
          const int pend = blk ? std::min((k0 / lpb + 1) * lpb, q.ns) : q.ns;  // big-panel end
          const bool bnd = blk && r0 == pend && r0 < q.ns;  // next block starts a big panel: no diag task
          // fused: every panel step also applies its rank-kb update to the contribution block (the
          // step is latency-bound on the diagonal chain, the extra tiles run in its shadow)
          const int clim = fused_contrib ? m : pend;
          const int T = (m - r0 + TT - 1) / TT, TJ = (clim - r0 + TT - 1) / TT;
          const int fl = (fused_contrib ? 8 : 0) | (bnd ? 32 : 0);
          auto mk = [&](int tile, int flags) {
            return launch::StepTask{hfd[sn].front_off, hfd[sn].l_off, hfd[sn].vec_off, hfd[sn].x_off, m, q.ns, q.c0,
                                    k0 | (kb << 16), tile, flags, clim};
          };
          if (r0 < q.ns && !bnd) diag_t.push_back(mk(0, 4));
          for (int tj = 0; tj < std::max(TJ, 1); ++tj)
            for (int ti = tj; ti < T; ++ti) tile_t.push_back(mk(ti | (tj << 16), (tj < TJ ? 1 : 0) | fl));
          // inverse tasks: block row p-1's term into every pending block (bp, j), bp >= p, j < p;
          // block row p is final after this step. Blocked fronts build only the diagonal big-panel
          // blocks of X (their backward solve substitutes big panel by big panel)
          const int nblk = (q.ns + NB - 1) / NB;
          const bool bsolve = blk && q.ns > block_min;  // narrower blocked fronts keep the full X
          const int ib0 = bsolve ? (k0 / lpb) * (lpb / NB) : 0;
          const int ib1 = bsolve ? std::min(nblk, ib0 + lpb / NB) : nblk;
          if (bsolve) sn_pb[sn] = lpb;
          for (int bp = p; bp < ib1 && p - 1 >= ib0 && !dev_noinv; ++bp)
            for (int j = ib0; j < p; ++j) inv_t.push_back(mk(j | (bp << 16), 16));
        }
        stk.insert(stk.end(), diag_t.begin(), diag_t.end());
        if (!dev_diagonly) stk.insert(stk.end(), tile_t.begin(), tile_t.end());
        if (!dev_diagonly) stk.insert(stk.end(), inv_t.begin(), inv_t.end());
        st.count = (int)stk.size() - st.off;
        if (st.count) ops.push_back(st);
        if ((p + 1) * NB % lpb) continue;
        // end of a big panel: trailing update of the blocked fronts, then their next first blocks
        Op gm{3, (int)tk.size(), 0};
        Op d0{2, (int)stk.size(), 0};
        for (int sn : lv) {
          const Supernode& q = sym.sn[sn];
          const int kb = (p + 1) * NB, ka = kb - lpb, m = q.ns + q.nr;
          if (!blocked(q) || kb >= q.ns) continue;
          const int T = (m - kb + TT - 1) / TT, TJ = (q.ns - kb + TT - 1) / TT;
          for (int tj = 0; tj < TJ; ++tj)
            for (int ti = tj; ti < T; ++ti) tk.push_back(Task{sn, ka, ti | (tj << 16), kb});
          stk.push_back(launch::StepTask{hfd[sn].front_off, hfd[sn].l_off, hfd[sn].vec_off, hfd[sn].x_off, m, q.ns,
                                         q.c0, kb, 0, 4, q.ns});
        }
        gm.count = (int)tk.size() - gm.off;
        d0.count = (int)stk.size() - d0.off;
        if (gm.count) ops.push_back(gm);
        if (d0.count) ops.push_back(d0);
      }
      Op sy{3, (int)tk.size(), 0};
      for (int sn : lv) {
        if (fused_contrib) break;
        const Supernode& q = sym.sn[sn];
        const int T = (q.nr + TT - 1) / TT;
        for (int tj = 0; tj < T; ++tj)
          for (int ti = tj; ti < T; ++ti) tk.push_back(Task{sn, 0, ti | (tj << 16), 0});
      }
      sy.count = (int)tk.size() - sy.off;
      if (sy.count) ops.push_back(sy);
    }
    nzero = (int)(zr.size() / 2);
    npre = (long long)pdst.size();
    zero_rng.upload(zr.empty() ? std::vector<long long>{0, 0} : zr, s);
    pre_dst.upload(pdst.empty() ? std::vector<long long>{0} : pdst, s);
    pre_src.upload(psrc.empty() ? std::vector<int>{0} : psrc, s);
    // backward solve per level: gemv tasks (front, 4 columns) for every front, then x = X^T t for the
    // unblocked fronts (one launch) and, for blocked fronts, rounds over their big panels from the last:
    // t_b -= L(later rows of the supernode, b)^T x, x_b = X_bb^T t_b
    bwd_off.assign(1, (int)tk.size());
    bwd_ops.clear();
    max_ns = 1;
    for (size_t l = 0; l < sym.levels.size(); ++l) {
      const auto& lv = sym.levels[l];
      BwdLevel bl;
      bl.gemv = {(int)tk.size(), 0};
      for (int sn : lv) {
        const int ns = sym.sn[sn].ns;
        max_ns = std::max(max_ns, ns);
        for (int a = 0; a < ns; a += launch::CHOL_BW) tk.push_back(Task{sn, a, 0, 0});
      }
      bl.gemv.second = (int)tk.size() - bl.gemv.first;
      bl.xall = {(int)tk.size(), 0};
      int rounds = 0;
      for (int sn : lv) {
        const int ns = sym.sn[sn].ns;
        if (sn_pb[sn]) { rounds = std::max(rounds, (ns + sn_pb[sn] - 1) / sn_pb[sn]); continue; }
        for (int a = 0; a < ns; a += launch::CHOL_BW) tk.push_back(Task{sn, a, 0, ns});
      }
      bl.xall.second = (int)tk.size() - bl.xall.first;
      for (int r = 0; r < rounds; ++r) {
        std::pair<int, int> g{(int)tk.size(), 0}, x{0, 0};
        for (int sn : lv) {  // inner gemv: t_b -= L([be, ns), b)^T x([be, ns))
          const int ns = sym.sn[sn].ns, pb = sn_pb[sn];
          if (!pb) continue;
          const int nbp = (ns + pb - 1) / pb, b = nbp - 1 - r;
          if (b < 0 || r == 0) continue;
          const int bs = b * pb, be = std::min(ns, bs + pb);
          for (int a = bs; a < be; a += launch::CHOL_BW) tk.push_back(Task{sn, a, be, 0});
        }
        g.second = (int)tk.size() - g.first;
        x.first = (int)tk.size();
        for (int sn : lv) {  // x_b = X_bb^T t_b
          const int ns = sym.sn[sn].ns, pb = sn_pb[sn];
          if (!pb) continue;
          const int nbp = (ns + pb - 1) / pb, b = nbp - 1 - r;
          if (b < 0) continue;
          const int bs = b * pb, be = std::min(ns, bs + pb);
          for (int a = bs; a < be; a += launch::CHOL_BW) tk.push_back(Task{sn, a, be, be});
        }
        x.second = (int)tk.size() - x.first;
        bl.rounds.push_back({g, x});
      }
      bwd_ops.push_back(bl);
      bwd_off.push_back((int)tk.size());
    }
    tasks.upload(tk.empty() ? std::vector<Task>{Task{0, 0, 0, 0}} : tk, s);
    step_tasks.upload(stk.empty() ? std::vector<launch::StepTask>(1) : stk, s);
  }
  children.upload(sym.children.empty() ? std::vector<int>{0} : sym.children, s);
  relmap.upload(sym.relmap.empty() ? std::vector<int>{0} : sym.relmap, s);
  rows.upload(sym.rows.empty() ? std::vector<int>{0} : sym.rows, s);
  perm.upload(sym.perm, s);
  fronts.resize(std::max<int64_t>(sym.front_pool, 1));
  vecs.resize(std::max<int64_t>(sym.vec_pool, 1));
  rhs_p.resize(std::max(sym.n, 1));
  y_p.resize(std::max(sym.n, 1));
  lbuf.resize(std::max<long long>(lpool, 1));
  linv.resize((size_t)(sym.n + launch::CHOL_NB) * launch::CHOL_NB * launch::CHOL_NB);  // one 32x32 L_kk^-1 per panel start
  xinv.resize(std::max<long long>(xoff, 1));
  t_p.resize(std::max(sym.n, 1));
  x_p.resize(std::max(sym.n, 1));
}

void DeviceCholesky::factor(const double* vals, const double* lam, const double* rhs, int* fail, hipStream_t s) {
  launch::chol_permute(sym.n, perm.get(), rhs, rhs_p.get(), s);
  launch::chol_vec_init((int)sym.sn.size(), fd.get(), rhs_p.get(), vecs.get(), s);
  launch::chol_prescatter(nzero, zero_rng.get(), npre, vals, pre_dst.get(), pre_src.get(), lam, fronts.get(), s);
  for (const Op& op : ops) {
    const launch::Task* t = tasks.get() + op.off;
    switch (op.kind) {
      case 0:
      case 4:
      case 5: launch::chol_extend_add(op.count, t, fd.get(), children.get(), relmap.get(), jtab.get(), cmptr.get(),
                                      cment.get(), colptr.get(),
                                      ent_row.get(),
                                      ent_src.get(), vals, lam, fronts.get(), vecs.get(),
                                      lbuf.get(), y_p.get(), linv.get(), xinv.get(), fail, op.kind == 0 ? 0 : (op.kind == 5 ? 2 : 1), s); break;
      case 2: launch::chol_step(op.count, step_tasks.get() + op.off, fronts.get(), lbuf.get(), vecs.get(), y_p.get(),
                                linv.get(), xinv.get(), fail, s);
        break;
      default: launch::chol_syrk(op.count, t, fd.get(), fronts.get(), lbuf.get(), s); break;
    }
  }
}

void DeviceCholesky::solve(double* x, hipStream_t s) {
  for (size_t l = level_off.size() - 1; l-- > 0;) {  // root level first
    const BwdLevel& bl = bwd_ops[l];
    launch::chol_bwd_gemv(bl.gemv.second, tasks.get() + bl.gemv.first, fd.get(), rows.get(), lbuf.get(), y_p.get(),
                          x_p.get(), t_p.get(), s);
    launch::chol_bwd_x(bl.xall.second, tasks.get() + bl.xall.first, fd.get(), xinv.get(), t_p.get(), x_p.get(), s);
    for (const auto& rd : bl.rounds) {
      launch::chol_bwd_inner(rd.first.second, tasks.get() + rd.first.first, fd.get(), lbuf.get(), x_p.get(), t_p.get(), s);
      launch::chol_bwd_x(rd.second.second, tasks.get() + rd.second.first, fd.get(), xinv.get(), t_p.get(), x_p.get(), s);
    }
  }
  launch::chol_ipermute(sym.n, perm.get(), x_p.get(), x, s);
}

// ------------------------------------------------------------------ Engine: graph
Engine::Engine(int dev) : device(dev) {
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  dscal.resize(12);  // [0] lambda [1] chi2 [2] scale [3] maxdiag [4] lambda (rank 0) [5] 0 | [8..9] fail flags (int)
  dscal.zero(stream);
  for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
  for (auto& e : lm_ev_) HIP_CHECK(hipEventCreate(&e));
}
Engine::~Engine() {
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
  for (auto& e : lm_ev_) if (e) (void)hipEventDestroy(e);
  comm.reset();
  if (stream) (void)hipStreamDestroy(stream);
}

int Engine::add_vertices(int type, int n, const int* ids, const double* est, const int* fixed, const int* marg) {
  if (vertex_dim(type) < 0 || n < 0) return G2OHIP_ERR_ARG;
  const int ed = vertex_est_dim(type), sd = vertex_state_stride(type);
  for (int k = 0; k < n; ++k) {
    if (hg.idmap.count(ids[k])) return G2OHIP_ERR_ARG;
    HVertex v{ids[k], type, vertex_dim(type), fixed ? fixed[k] != 0 : false, marg ? marg[k] != 0 : false,
              (int)hg.by_type[type].size()};
    hg.idmap[v.id] = (int)hg.verts.size();
    hg.by_type[type].push_back((int)hg.verts.size());
    hg.verts.push_back(v);
    const size_t o = hg.st[type].size();
    hg.st[type].resize(o + sd, 0.0);
    set_state_from_est(type, est + (size_t)k * ed, hg.st[type].data() + o);
    if (type == G2OHIP_V_SE3_QUAT) hg.nopl.push_back(0);
  }
  initialized = false;
  device_state_dirty = true;
  return G2OHIP_OK;
}

int Engine::add_edges(int type, int n, const int* v0, const int* v1, const double* meas, const double* info,
                      const double* params) {
  const int D = edge_dim(type);
  if (D < 0 || n < 0) return G2OHIP_ERR_ARG;
  if (hg.etype && hg.etype != type) return G2OHIP_ERR_UNSUPPORTED;  // one edge family per graph
  if (type == G2OHIP_E_SE3_PROJECT_XYZ && !params) return G2OHIP_ERR_ARG;
  hg.etype = type;
  const int nm = edge_meas_dim(type);
  for (int k = 0; k < n; ++k) {
    auto a = hg.idmap.find(v0[k]), b = hg.idmap.find(v1[k]);
    if (a == hg.idmap.end() || b == hg.idmap.end()) return G2OHIP_ERR_ARG;
    hg.ev0.push_back(a->second);
    hg.ev1.push_back(b->second);
  }
  hg.emeas.insert(hg.emeas.end(), meas, meas + (size_t)n * nm);
  hg.einfo.insert(hg.einfo.end(), info, info + (size_t)n * D * D);
  if (type == G2OHIP_E_SE3_PROJECT_XYZ) hg.eparams.insert(hg.eparams.end(), params, params + (size_t)n * 4);
  initialized = false;
  return G2OHIP_OK;
}

// optimizable_graph.cpp:397-661 for the tags on this path
int Engine::load(const char* path, int marginalize_xyz) {
  std::ifstream in(path);
  if (!in) return G2OHIP_ERR_ARG;
  std::string line, tag;
  std::vector<int> fix;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    if (!(ss >> tag) || tag[0] == '#') continue;
    int r = 0;
    if (tag == "VERTEX_SE3:EXPMAP") {  // file holds cam2world (types_six_dof_expmap.cpp:93-101)
      int id; double v[7], w[7];
      ss >> id; for (double& d : v) ss >> d;
      double q[4] = {v[3], v[4], v[5], v[6]};
      double tq[7] = {v[0], v[1], v[2], q[0], q[1], q[2], q[3]};
      se3quat_inverse(tq, w);
      int z = 0;
      r = add_vertices(G2OHIP_V_SE3_EXPMAP, 1, &id, w, &z, &z);
    } else if (tag == "VERTEX_XYZ") {
      int id; double v[3];
      ss >> id >> v[0] >> v[1] >> v[2];
      int z = 0, m = marginalize_xyz ? 1 : 0;
      r = add_vertices(G2OHIP_V_XYZ, 1, &id, v, &z, &m);
    } else if (tag == "VERTEX_SE3:QUAT") {
      int id; double v[7];
      ss >> id; for (double& d : v) ss >> d;
      int z = 0;
      r = add_vertices(G2OHIP_V_SE3_QUAT, 1, &id, v, &z, &z);
    } else if (tag == "VERTEX_SE2") {
      int id; double v[3];
      ss >> id >> v[0] >> v[1] >> v[2];
      int z = 0;
      r = add_vertices(G2OHIP_V_SE2, 1, &id, v, &z, &z);
    } else if (tag == "FIX") {
      int id;
      while (ss >> id) fix.push_back(id);
    } else if (tag == "EDGE_SE3_PROJECT_XYZ:EXPMAP") {
      int a, b; double m[2], o[3], p[4];
      ss >> a >> b >> m[0] >> m[1] >> o[0] >> o[1] >> o[2] >> p[0] >> p[1] >> p[2] >> p[3];
      double info[4] = {o[0], o[1], o[1], o[2]};
      r = add_edges(G2OHIP_E_SE3_PROJECT_XYZ, 1, &a, &b, m, info, p);
    } else if (tag == "EDGE_SE3:QUAT") {
      int a, b; double m[7], info[36];
      ss >> a >> b; for (double& d : m) ss >> d;
      for (int i = 0; i < 6; ++i) for (int j = i; j < 6; ++j) { ss >> info[i * 6 + j]; info[j * 6 + i] = info[i * 6 + j]; }
      r = add_edges(G2OHIP_E_SE3_QUAT, 1, &a, &b, m, info, nullptr);
    } else if (tag == "EDGE_SE2") {
      int a, b; double m[3], info[9];
      ss >> a >> b >> m[0] >> m[1] >> m[2];
      for (int i = 0; i < 3; ++i) for (int j = i; j < 3; ++j) { ss >> info[i * 3 + j]; info[j * 3 + i] = info[i * 3 + j]; }
      r = add_edges(G2OHIP_E_SE2, 1, &a, &b, m, info, nullptr);
    } else {
      return G2OHIP_ERR_UNSUPPORTED;
    }
    if (r) return r;
  }
  for (int id : fix) {
    auto it = hg.idmap.find(id);
    if (it != hg.idmap.end()) hg.verts[it->second].fixed = true;
  }
  return G2OHIP_OK;
}

int Engine::save(const char* path) {
  sync_host_state();
  FILE* f = fopen(path, "w");
  if (!f) return G2OHIP_ERR_ARG;
  for (auto& v : hg.verts) {
    const double* st = hg.st[v.type].data() + (size_t)v.local * vertex_state_stride(v.type);
    double e[7];
    est_from_state(v.type, st, e);
    switch (v.type) {
      case G2OHIP_V_SE3_EXPMAP: {
        double c[7];
        se3quat_inverse(e, c);
        fprintf(f, "VERTEX_SE3:EXPMAP %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", v.id, c[0], c[1], c[2], c[3], c[4], c[5], c[6]);
        break;
      }
      case G2OHIP_V_XYZ: fprintf(f, "VERTEX_XYZ %d %.17g %.17g %.17g\n", v.id, e[0], e[1], e[2]); break;
      case G2OHIP_V_SE3_QUAT:
        fprintf(f, "VERTEX_SE3:QUAT %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", v.id, e[0], e[1], e[2], e[3], e[4], e[5], e[6]);
        break;
      case G2OHIP_V_SE2: fprintf(f, "VERTEX_SE2 %d %.17g %.17g %.17g\n", v.id, e[0], e[1], e[2]); break;
    }
    if (v.fixed) fprintf(f, "FIX %d\n", v.id);
  }
  const int D = edge_dim(hg.etype), nm = edge_meas_dim(hg.etype);
  for (size_t k = 0; k < hg.ev0.size(); ++k) {
    const int a = hg.verts[hg.ev0[k]].id, b = hg.verts[hg.ev1[k]].id;
    const double* m = hg.emeas.data() + k * nm;
    const double* I = hg.einfo.data() + k * D * D;
    if (hg.etype == G2OHIP_E_SE3_PROJECT_XYZ) {
      const double* p = hg.eparams.data() + k * 4;
      fprintf(f, "EDGE_SE3_PROJECT_XYZ:EXPMAP %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", a, b, m[0], m[1],
              I[0], I[1], I[3], p[0], p[1], p[2], p[3]);
    } else {
      fprintf(f, "%s %d %d", hg.etype == G2OHIP_E_SE3_QUAT ? "EDGE_SE3:QUAT" : "EDGE_SE2", a, b);
      for (int i = 0; i < nm; ++i) fprintf(f, " %.17g", m[i]);
      for (int i = 0; i < D; ++i) for (int j = i; j < D; ++j) fprintf(f, " %.17g", I[i * D + j]);
      fprintf(f, "\n");
    }
  }
  fclose(f);
  return G2OHIP_OK;
}

void Engine::ensure_device_state() {
  if (!device_state_dirty) return;
  for (int t = 1; t <= 4; ++t)
    if (!hg.st[t].empty()) dstate[t].upload(hg.st[t], stream);
  if (!hg.nopl.empty()) dnopl.upload(hg.nopl, stream);
  device_state_dirty = false;
  ++state_ver;
  host_state_stale = false;
}

void Engine::sync_host_state() {
  if (!host_state_stale) return;
  for (int t = 1; t <= 4; ++t)
    if (!hg.st[t].empty()) dstate[t].download(hg.st[t].data(), hg.st[t].size(), stream);
  if (!hg.nopl.empty()) dnopl.download(hg.nopl.data(), hg.nopl.size(), stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  host_state_stale = false;
}

int Engine::get_estimates(int type, double* out, int* ids) {
  if (type < 1 || type > 4) return G2OHIP_ERR_ARG;
  sync_host_state();
  const int ed = vertex_est_dim(type), sd = vertex_state_stride(type);
  const auto& lst = hg.by_type[type];
  for (size_t k = 0; k < lst.size(); ++k) {
    if (out) est_from_state(type, hg.st[type].data() + k * sd, out + k * ed);
    if (ids) ids[k] = hg.verts[lst[k]].id;
  }
  return (int)lst.size();
}

int Engine::set_estimates(int type, const double* est) {
  if (type < 1 || type > 4) return G2OHIP_ERR_ARG;
  sync_host_state();
  const int ed = vertex_est_dim(type), sd = vertex_state_stride(type);
  for (size_t k = 0; k < hg.by_type[type].size(); ++k) set_state_from_est(type, est + k * ed, hg.st[type].data() + k * sd);
  device_state_dirty = true;
  return G2OHIP_OK;
}

int Engine::minimal_state(double* out) {
  sync_host_state();
  std::vector<int> order(hg.verts.size());
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return hg.verts[a].id < hg.verts[b].id; });
  int n = 0;
  for (int k : order) {
    const HVertex& v = hg.verts[k];
    if (out) minimal_from_state(v.type, hg.st[v.type].data() + (size_t)v.local * vertex_state_stride(v.type), out + n);
    n += v.dim;
  }
  return n;
}

// ------------------------------------------------------------------ Engine: structure
int Engine::initialize() {  // sparse_optimizer.cpp:201-279 + buildIndexMapping :168-192
  if (hg.ev0.empty()) return G2OHIP_ERR_STATE;
  switch (hg.etype) {
    case G2OHIP_E_SE3_PROJECT_XYZ: family = FAM_BA; vt0 = G2OHIP_V_XYZ; vt1 = G2OHIP_V_SE3_EXPMAP; break;
    case G2OHIP_E_SE3_QUAT: family = FAM_SE3; vt0 = vt1 = G2OHIP_V_SE3_QUAT; break;
    case G2OHIP_E_SE2: family = FAM_SE2; vt0 = vt1 = G2OHIP_V_SE2; break;
    default: return G2OHIP_ERR_UNSUPPORTED;
  }
  for (size_t k = 0; k < hg.ev0.size(); ++k)
    if (hg.verts[hg.ev0[k]].type != vt0 || hg.verts[hg.ev1[k]].type != vt1) return G2OHIP_ERR_UNSUPPORTED;
  std::vector<char> has(hg.verts.size(), 0);
  for (size_t k = 0; k < hg.ev0.size(); ++k) has[hg.ev0[k]] = has[hg.ev1[k]] = 1;
  active.clear();
  for (size_t k = 0; k < hg.verts.size(); ++k)
    if (has[k]) active.push_back((int)k);
  std::sort(active.begin(), active.end(), [&](int a, int b) { return hg.verts[a].id < hg.verts[b].id; });
  ivmap.clear();
  hidx.assign(hg.verts.size(), -1);
  for (int k = 0; k < 2; ++k)
    for (int vi : active) {
      const HVertex& v = hg.verts[vi];
      if (!v.fixed && (int)v.marg == k) {
        hidx[vi] = (int)ivmap.size();
        ivmap.push_back(vi);
      }
    }
  pd = ld = 0;
  num_poses = num_landmarks = 0;
  for (int vi : ivmap) {
    const HVertex& v = hg.verts[vi];
    if (!v.marg) {
      if (pd && pd != v.dim) return G2OHIP_ERR_UNSUPPORTED;
      pd = v.dim;
      ++num_poses;
    } else {
      if (v.dim != 3) return G2OHIP_ERR_UNSUPPORTED;
      ld = 3;
      ++num_landmarks;
    }
  }
  if (num_poses == 0) return G2OHIP_ERR_UNSUPPORTED;
  size_poses = num_poses * pd;
  size_landmarks = num_landmarks * ld;
  do_schur = num_landmarks > 0;  // optimization_algorithm_with_hessian.cpp:48-73
  if (do_schur && (family != FAM_BA || pd != 6)) return G2OHIP_ERR_UNSUPPORTED;
  initialized = true;
  structure_built = false;
  edges_ready = false;
  return G2OHIP_OK;
}

void Engine::setup_edges_device() {
  const int nall = (int)hg.ev0.size();
  local_edges.clear();
  int lm_begin = 0, lm_end = num_landmarks;
  if (do_schur && nranks > 1) {
    lm_begin = (int)((long long)num_landmarks * rank / nranks);
    lm_end = (int)((long long)num_landmarks * (rank + 1) / nranks);
  }
  local_lm.clear();
  for (int l = lm_begin; l < lm_end; ++l) local_lm.push_back(l);
  for (int k = 0; k < nall; ++k) {
    int owner = 0;
    if (do_schur && nranks > 1) {
      const int h = hidx[hg.ev0[k]];  // BA: vertex 0 is the point
      if (h >= num_poses) {
        const int l = h - num_poses;
        for (int r = 0; r < nranks; ++r)
          if (l >= (int)((long long)num_landmarks * r / nranks) && l < (int)((long long)num_landmarks * (r + 1) / nranks))
            owner = r;
      }
    } else if (nranks > 1) {
      owner = rank;  // pose graphs: replicas
    }
    if (owner == rank) local_edges.push_back(k);
  }
  ne = (int)local_edges.size();
  const int D = edge_dim(hg.etype), nm = edge_meas_dim(hg.etype);
  std::vector<int> v0(ne), v1(ne);
  int minfo = D * (D + 1) / 2, mmeas = family == FAM_BA ? 2 : (family == FAM_SE3 ? 12 : 3);
  std::vector<double> meas((size_t)ne * mmeas), info((size_t)ne * minfo), params(family == FAM_BA ? (size_t)ne * 4 : 1);
  for (int k = 0; k < ne; ++k) {
    const int e = local_edges[k];
    v0[k] = hg.verts[hg.ev0[e]].local;
    v1[k] = hg.verts[hg.ev1[e]].local;
    const double* m = hg.emeas.data() + (size_t)e * nm;
    double* mo = meas.data() + (size_t)k * mmeas;
    if (family == FAM_BA) {
      mo[0] = m[0]; mo[1] = m[1];
      for (int j = 0; j < 4; ++j) params[(size_t)k * 4 + j] = hg.eparams[(size_t)e * 4 + j];
    } else if (family == FAM_SE3) {  // edge_se3.cpp:42-50: normalise q, Z = fromVectorQT, store Z^-1
      double q[4] = {m[3], m[4], m[5], m[6]};
      const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      for (double& x : q) x /= n;
      double Z[9];
      q2R(q[0], q[1], q[2], q[3], Z);
      double Rt[9] = {Z[0], Z[3], Z[6], Z[1], Z[4], Z[7], Z[2], Z[5], Z[8]};
      for (int j = 0; j < 9; ++j) mo[j] = Rt[j];
      for (int i = 0; i < 3; ++i) mo[9 + i] = -(Rt[i * 3] * m[0] + Rt[i * 3 + 1] * m[1] + Rt[i * 3 + 2] * m[2]);
    } else {  // edge_se2.cpp:41-47: inverse measurement
      const double th = norm_theta(-m[2]);
      const double c = std::cos(th), s = std::sin(th);
      mo[0] = c * (-m[0]) - s * (-m[1]);
      mo[1] = s * (-m[0]) + c * (-m[1]);
      mo[2] = th;
    }
    const double* I = hg.einfo.data() + (size_t)e * D * D;
    double* io = info.data() + (size_t)k * minfo;
    int q = 0;
    for (int c = 0; c < D; ++c)
      for (int r = 0; r <= c; ++r) io[q++] = I[r * D + c];
  }
  dv0.upload(v0, stream);
  dv1.upload(v1, stream);
  dmeas.upload(meas, stream);
  dinfo.upload(info, stream);
  dparams.upload(params, stream);
  dpartial.resize(std::max<size_t>(launch::sum_partials(std::max<long long>(std::max<long long>(ne, vector_size()), 1)) + 64, 128));
  edges_ready = true;
  ++state_ver;  // the edge set (and so chi2) changed
}

int Engine::build_structure() {  // block_solver.hpp:102-256
  if (!initialized) {
    int r = initialize();
    if (r) return r;
  }
  ensure_device_state();
  setup_edges_device();
  // per-type hessian index and x offsets
  const int lm_begin = local_lm.empty() ? 0 : local_lm.front();
  const int lm_end = local_lm.empty() ? 0 : local_lm.back() + 1;
  for (int t = 1; t <= 4; ++t) {
    const auto& lst = hg.by_type[t];
    std::vector<int> hx(std::max<size_t>(lst.size(), 1), -1), xo(std::max<size_t>(lst.size(), 1), -1);
    for (size_t k = 0; k < lst.size(); ++k) {
      const int h = hidx[lst[k]];
      hx[k] = h;
      if (h < 0) continue;
      if (h < num_poses) xo[k] = h * pd;
      else if (h - num_poses >= lm_begin && h - num_poses < lm_end) xo[k] = size_poses + (h - num_poses) * ld;
    }
    d_hidx[t].upload(hx, stream);
    d_xoff[t].upload(xo, stream);
  }
  // off-diagonal blocks (mapHessianMemory)
  const int DA = vertex_dim(vt0), DB = vertex_dim(vt1);
  std::map<std::pair<int, int>, int> hppmap;  // (i<j) -> block id
  hpp_bi.assign(num_poses, 0);
  hpp_bj.assign(num_poses, 0);
  for (int i = 0; i < num_poses; ++i) hpp_bi[i] = hpp_bj[i] = i;
  struct OffRef { int kind; int a, b; bool tr; };
  std::vector<OffRef> offref(ne, OffRef{0, 0, 0, false});
  std::vector<std::pair<int, int>> plpairs;  // (lm, pose)
  for (int k = 0; k < ne; ++k) {
    const int e = local_edges[k];
    int i1 = hidx[hg.ev0[e]], i2 = hidx[hg.ev1[e]];
    if (i1 < 0 || i2 < 0) continue;
    const bool m1 = i1 >= num_poses, m2 = i2 >= num_poses;
    if (!m1 && !m2) {
      bool tr = i1 > i2;
      if (tr) std::swap(i1, i2);
      auto it = hppmap.find({i1, i2});
      if (it == hppmap.end()) {
        it = hppmap.emplace(std::make_pair(i1, i2), (int)hpp_bi.size()).first;
        hpp_bi.push_back(i1);
        hpp_bj.push_back(i2);
      }
      offref[k] = OffRef{1, it->second, 0, tr};
    } else if (m1 && !m2) {
      offref[k] = OffRef{2, i2, i1 - num_poses, true};
      plpairs.push_back({i1 - num_poses, i2});
    } else if (!m1 && m2) {
      offref[k] = OffRef{2, i1, i2 - num_poses, false};
      plpairs.push_back({i2 - num_poses, i1});
    } else {
      return G2OHIP_ERR_UNSUPPORTED;  // landmark-landmark edges
    }
  }
  nHpp = (int)hpp_bi.size();
  std::sort(plpairs.begin(), plpairs.end());
  plpairs.erase(std::unique(plpairs.begin(), plpairs.end()), plpairs.end());
  nHpl = (int)plpairs.size();
  const long long hpl_base = (long long)nHpp * pd * pd;
  std::vector<long long> offdst(std::max(ne, 1), -1);
  std::vector<unsigned char> offtr(std::max(ne, 1), 0);
  std::vector<long long> blkdst;  // per distinct off block id (global index over hpp offdiag + hpl)
  std::vector<int> blk_count;
  auto blk_key = [&](const OffRef& r) -> long long {
    if (r.kind == 1) return r.a;  // hpp block id
    auto it = std::lower_bound(plpairs.begin(), plpairs.end(), std::make_pair(r.b, r.a));
    return nHpp + (long long)(it - plpairs.begin());
  };
  blk_count.assign(nHpp + nHpl, 0);
  std::vector<long long> ekey(ne, -1);
  for (int k = 0; k < ne; ++k) {
    if (!offref[k].kind) continue;
    ekey[k] = blk_key(offref[k]);
    blk_count[ekey[k]]++;
    offtr[k] = offref[k].tr ? 1 : 0;
    offdst[k] = ekey[k] < nHpp ? ekey[k] * pd * pd : hpl_base + (ekey[k] - nHpp) * pd * ld;
  }
  off_dup = false;
  for (int c : blk_count) if (c > 1) off_dup = true;
  off_bsz = DA * DB;
  if (off_dup) {  // per-edge slots + ordered reduction into the blocks
    std::vector<int> ptr(nHpp + nHpl + 1, 0), edges;
    for (int k = 0; k < ne; ++k) if (ekey[k] >= 0) ptr[ekey[k] + 1]++;
    for (size_t b = 0; b + 1 < ptr.size(); ++b) ptr[b + 1] += ptr[b];
    edges.assign(ptr.back(), 0);
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    for (int k = 0; k < ne; ++k) if (ekey[k] >= 0) edges[fill[ekey[k]]++] = k;
    std::vector<long long> dstb(nHpp + nHpl, -1);
    for (int b = 0; b < nHpp + nHpl; ++b) dstb[b] = b < nHpp ? (long long)b * pd * pd : hpl_base + (long long)(b - nHpp) * pd * ld;
    // blocks without off-diagonal contributions (pose diagonal blocks) keep an empty list
    for (int k = 0; k < ne; ++k) if (ekey[k] >= 0) offdst[k] = (long long)k * off_bsz;
    noffb = nHpp + nHpl;
    doffb_ptr.upload(ptr, stream);
    doffb_edges.upload(edges.empty() ? std::vector<int>{0} : edges, stream);
    std::vector<long long> dstb2;
    std::vector<int> ptr2{0}, edges2;
    // only keep blocks with >= 1 contribution (diagonal Hpp blocks are reduced elsewhere)
    for (int b = 0; b < nHpp + nHpl; ++b) {
      if (ptr[b + 1] == ptr[b]) continue;
      for (int p = ptr[b]; p < ptr[b + 1]; ++p) edges2.push_back(edges[p]);
      ptr2.push_back((int)edges2.size());
      dstb2.push_back(dstb[b]);
    }
    noffb = (int)dstb2.size();
    doffb_ptr.upload(ptr2, stream);
    doffb_edges.upload(edges2.empty() ? std::vector<int>{0} : edges2, stream);
    doffb_dst.upload(dstb2.empty() ? std::vector<long long>{0} : dstb2, stream);
    doffslot.resize((size_t)std::max(ne, 1) * off_bsz);
  }
  doff_dst.upload(offdst, stream);
  doff_tr.upload(offtr, stream);
  // storage
  dH.resize(std::max<long long>((long long)nHpp * pd * pd + (long long)nHpl * pd * ld, 1));
  dH.zero(stream);
  const int nLloc = (int)local_lm.size();
  dHll.resize(std::max(nLloc * 9, 1));
  dHll.zero(stream);
  const long long n = vector_size();
  db.resize(std::max<long long>(n, 1));
  db.zero(stream);
  dx.resize(std::max<long long>(n, 1));
  dx.zero(stream);
  slot_stride0 = DA * (DA + 1) / 2 + DA;
  slot_stride1 = DB * (DB + 1) / 2 + DB;
  dslot0.resize((size_t)std::max(ne, 1) * slot_stride0);
  dslot1.resize((size_t)std::max(ne, 1) * slot_stride1);
  // vertex incidence lists (hessian order), slot code = local_edge * 2 + side
  {
    std::vector<std::vector<int>> incp(num_poses), incl(nLloc);
    for (int k = 0; k < ne; ++k) {
      const int e = local_edges[k];
      const int hs[2] = {hidx[hg.ev0[e]], hidx[hg.ev1[e]]};
      for (int s = 0; s < 2; ++s) {
        const int h = hs[s];
        if (h < 0) continue;
        if (h < num_poses) incp[h].push_back(k * 2 + s);
        else incl[h - num_poses - lm_begin].push_back(k * 2 + s);
      }
    }
    auto build = [&](VRed& vr, std::vector<std::vector<int>>& inc, int dim, int boff0) {
      vr.dim = dim;
      vr.nv = (int)inc.size();
      std::vector<int> ptr(vr.nv + 1, 0), code, bo(std::max(vr.nv, 1), 0);
      for (int v = 0; v < vr.nv; ++v) {
        ptr[v + 1] = ptr[v] + (int)inc[v].size();
        code.insert(code.end(), inc[v].begin(), inc[v].end());
        bo[v] = boff0 + v * dim;
      }
      const double avg = vr.nv ? (double)code.size() / vr.nv : 0;
      vr.lanes = avg >= 128 ? 64 : (avg >= 16 ? 8 : (avg >= 6 ? 4 : 1));
      vr.ptr.upload(ptr, stream);
      vr.code.upload(code.empty() ? std::vector<int>{0} : code, stream);
      vr.boff.upload(bo, stream);
    };
    build(vr_pose, incp, pd, 0);
    vr_pose.H = dH.get();
    if (do_schur) {
      build(vr_lm, incl, ld, size_poses + lm_begin * ld);
      vr_lm.H = dHll.get();
    } else {
      vr_lm.nv = 0;
    }
  }
  // Schur structures
  if (do_schur) {
    // Hpl blocks are ordered (landmark, pose): lm_ptr over local landmarks
    std::vector<int> lm_ptr(nLloc + 1, 0), blk_pose(std::max(nHpl, 1), 0), blk_lm(std::max(nHpl, 1), 0);
    for (int a = 0; a < nHpl; ++a) {
      lm_ptr[plpairs[a].first - lm_begin + 1]++;
      blk_pose[a] = plpairs[a].second;
      blk_lm[a] = plpairs[a].first;  // global landmark index
    }
    for (int l = 0; l < nLloc; ++l) lm_ptr[l + 1] += lm_ptr[l];
    d_lm_ptr.upload(lm_ptr, stream);
    d_blk_pose.upload(blk_pose, stream);
    d_blk_lm.upload(blk_lm, stream);
    // global Schur pattern from ALL edges (identical on every rank)
    std::vector<std::vector<int>> lmposes(num_landmarks);
    for (size_t e = 0; e < hg.ev0.size(); ++e) {
      const int hp = hidx[hg.ev1[e]], hl = hidx[hg.ev0[e]];
      if (hp < 0 || hl < num_poses) continue;
      lmposes[hl - num_poses].push_back(hp);
    }
    std::vector<std::vector<int>> rowcols(num_poses);
    for (int i = 0; i < num_poses; ++i) rowcols[i].push_back(i);
    for (int b = num_poses; b < nHpp; ++b) rowcols[hpp_bi[b]].push_back(hpp_bj[b]);
    // pose-pose edges owned by other ranks must also be in the global pattern
    for (size_t e = 0; e < hg.ev0.size(); ++e) {
      int i1 = hidx[hg.ev0[e]], i2 = hidx[hg.ev1[e]];
      if (i1 < 0 || i2 < 0 || i1 >= num_poses || i2 >= num_poses) continue;
      rowcols[std::min(i1, i2)].push_back(std::max(i1, i2));
    }
    for (auto& ps : lmposes) {
      std::sort(ps.begin(), ps.end());
      ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
      for (size_t u = 0; u < ps.size(); ++u)
        for (size_t v = u; v < ps.size(); ++v) rowcols[ps[u]].push_back(ps[v]);
    }
    std::vector<int> srow_ptr(num_poses + 1, 0);
    s_bi.clear();
    s_bj.clear();
    for (int i = 0; i < num_poses; ++i) {
      auto& rc = rowcols[i];
      std::sort(rc.begin(), rc.end());
      rc.erase(std::unique(rc.begin(), rc.end()), rc.end());
      for (int j : rc) { s_bi.push_back(i); s_bj.push_back(j); }
      srow_ptr[i + 1] = (int)s_bi.size();
    }
    nS = (int)s_bi.size();
    // Schur tasks. Diagonal blocks (k_schur_diag): per camera row its observations in landmark order.
    // Off-diagonal blocks (k_schur_rows): per camera row, chunks of <= SCHUR_SL off-diagonal slots;
    // per chunk the row's observations (l, i) in landmark order that have partners (l, j) in the
    // chunk, each staging its own block and those partners; batches of <= SCHUR_SB staged blocks.
    {
      constexpr int SB = launch::SCHUR_SB, SL = launch::SCHUR_SL;
      std::vector<int> rptr(num_poses + 1, 0), robs(std::max(nHpl, 1), 0);
      for (int a = 0; a < nHpl; ++a) rptr[blk_pose[a] + 1]++;
      for (int i = 0; i < num_poses; ++i) rptr[i + 1] += rptr[i];
      {
        std::vector<int> fill(rptr.begin(), rptr.end() - 1);
        for (int a = 0; a < nHpl; ++a) robs[fill[blk_pose[a]]++] = a;  // ascending a = landmark order
      }
      std::vector<int> gpos(std::max(nHpl, 1), 0);  // observation -> its G block (camera-row order)
      for (int r = 0; r < nHpl; ++r) gpos[robs[r]] = r;
      std::vector<int> obs_lm(std::max(nHpl, 1), 0), sdiag(num_poses);
      for (int l = 0; l < nLloc; ++l)
        for (int a = lm_ptr[l]; a < lm_ptr[l + 1]; ++a) obs_lm[a] = l;
      for (int i = 0; i < num_poses; ++i) sdiag[i] = srow_ptr[i];  // (i, i) is the first block of row i
      sch_rptr.upload(rptr, stream);
      sch_robs.upload(robs, stream);
      sch_obs_lm.upload(obs_lm, stream);
      sch_sdiag.upload(sdiag, stream);

      std::vector<launch::SchurTask> tasks;
      std::vector<launch::SchurBatch> batches;
      std::vector<int> st_obs, prs, pp;
      std::vector<int> camslot(num_poses, -1);
      struct P3 { int ls, a, b; };
      std::vector<P3> cur;
      std::vector<std::pair<int, int>> tmp;
      npairs = 0;
      for (int i = 0; i < num_poses; ++i) {
        const int s_lo = srow_ptr[i], s_hi = srow_ptr[i + 1];
        for (int k = s_lo; k < s_hi; ++k) camslot[s_bj[k]] = k - s_lo;  // slot 0 = the diagonal block
        const int noff_total = s_hi - s_lo - 1;
        for (int ch = 0; ch * SL < noff_total; ++ch) {
          launch::SchurTask T{};
          T.row = i;
          const int off_lo = 1 + ch * SL;
          T.noff = std::min(SL, noff_total - ch * SL);
          T.soff = s_lo + off_lo;
          T.b0 = (int)batches.size();
          int bst0 = (int)st_obs.size();
          cur.clear();
          auto flush = [&]() {
            const int nst = (int)st_obs.size() - bst0;
            if (nst == 0) return;
            launch::SchurBatch B{};
            B.st0 = bst0;
            B.nst = nst;
            B.pr0 = (int)prs.size();
            std::vector<int> cnt(SL + 1, 0);
            for (const P3& p : cur) cnt[p.ls + 1]++;
            for (int k = 0; k < SL; ++k) cnt[k + 1] += cnt[k];
            for (int k = 0; k <= SL; ++k) pp.push_back(B.pr0 + cnt[k]);
            std::vector<int> fillp(cnt.begin(), cnt.end() - 1), out(cur.size());
            for (const P3& p : cur) out[fillp[p.ls]++] = p.a | (p.b << 16);  // stable: landmark order per slot
            prs.insert(prs.end(), out.begin(), out.end());
            B.npr = (int)cur.size();
            npairs += B.npr;
            batches.push_back(B);
            cur.clear();
            bst0 = (int)st_obs.size();
          };
          for (int r = rptr[i]; r < rptr[i + 1]; ++r) {
            const int a = robs[r], l = obs_lm[a];
            tmp.clear();
            for (int a2 = a + 1; a2 < lm_ptr[l + 1]; ++a2) {
              const int sl = camslot[blk_pose[a2]] - off_lo;
              if (sl >= 0 && sl < T.noff) tmp.push_back({a2, sl});
            }
            if (tmp.empty()) continue;
            const int need = 1 + (int)tmp.size();
            if ((int)st_obs.size() - bst0 + need > SB) flush();
            const int posA = (int)st_obs.size() - bst0;
            st_obs.push_back(gpos[a]);
            for (auto& [a2, sl] : tmp) {
              const int posB = (int)st_obs.size() - bst0;
              st_obs.push_back(gpos[a2]);
              cur.push_back(P3{sl, posA, posB});
            }
          }
          flush();
          T.b1 = (int)batches.size();
          tasks.push_back(T);
        }
        for (int k = s_lo; k < s_hi; ++k) camslot[s_bj[k]] = -1;
      }
      nsch_tasks = (int)tasks.size();
      nstaged = (long long)st_obs.size();
      auto nz = [](std::vector<int>& v) -> std::vector<int>& { if (v.empty()) v.push_back(0); return v; };
      sch_tasks.upload(tasks.empty() ? std::vector<launch::SchurTask>(1) : tasks, stream);
      batches.push_back(launch::SchurBatch{});  // trailing dummy: k_schur_rows reads one record ahead
      sch_batches.upload(batches, stream);
      sch_st_obs.upload(nz(st_obs), stream);
      sch_pairs.upload(nz(prs), stream);
      sch_pp.upload(nz(pp), stream);
    }
    std::vector<int> shpp(nS, -1);
    nHppUsed = 0;
    for (int t = 0; t < nS; ++t) {
      if (s_bi[t] == s_bj[t]) shpp[t] = s_bi[t];
      else {
        auto it = hppmap.find({s_bi[t], s_bj[t]});
        if (it != hppmap.end()) shpp[t] = it->second;
      }
      nHppUsed += shpp[t] >= 0;
    }
    ds_hpp.upload(shpp, stream);
    dDinv.resize(std::max(nLloc * 9, 1));
    dUfac.resize(std::max(nLloc * 6, 1));
    dG.resize(std::max<long long>((long long)nHpl * 18, 1));  // G = Hpl U^-T per observation (6x3)
    dCl.resize(std::max<long long>((long long)num_landmarks * ld, 1));  // c = U^-1 b_l (global landmark index)
    dS.resize((size_t)nS * pd * pd + size_poses);  // [S blocks | bschur] contiguous for one all-reduce
    if (use_pcg()) pcg.setup(num_poses, pd, s_bi, s_bj, stream);
    else chol.setup(num_poses, pd, s_bi, s_bj, stream);
  } else if (use_pcg()) {
    pcg.setup(num_poses, pd, hpp_bi, hpp_bj, stream);
  } else {
    chol.setup(num_poses, pd, hpp_bi, hpp_bj, stream);
  }
  HIP_CHECK(hipStreamSynchronize(stream));
  structure_built = true;
  return G2OHIP_OK;
}

// ------------------------------------------------------------------ Engine: numeric steps
static EdgeArgs edge_args(const DevBuf<int>& v0, const DevBuf<int>& v1, const DevBuf<double>& meas,
                          const DevBuf<double>& info, const DevBuf<double>& params, const double* s0, const double* s1) {
  return EdgeArgs{v0.get(), v1.get(), meas.get(), info.get(), params.get(), s0, s1};
}

void Engine::allreduce_sum(double* p, size_t n) {
  if (nranks <= 1 || !comm) return;
  comm->allreduce_sum(p, n, stream);
}

void Engine::compute_errors_async() {
  ensure_device_state();
  EdgeArgs a = edge_args(dv0, dv1, dmeas, dinfo, dparams, dstate[vt0].get(), dstate[vt1].get());
  timer.begin("error", stream);
  launch::error_sum(family, a, ne, dpartial.get(), dscal.get() + 1, stream);
  timer.end(stream);
  if (do_schur) allreduce_sum(dscal.get() + 1, 1);
}

double Engine::chi2_sync() {
  ensure_device_state();
  if (chi_ver == state_ver) return chi_cache;  // same device state: computeActiveErrors is deterministic
  compute_errors_async();
  double c = 0;
  HIP_CHECK(hipMemcpyAsync(&c, dscal.get() + 1, sizeof(double), hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  timer.collect();
  chi_cache = c;
  chi_ver = state_ver;
  return c;
}

double Engine::chi2() {
  if (!initialized && initialize()) return std::nan("");
  ensure_device_state();
  if (!edges_ready) setup_edges_device();
  return chi2_sync();
}

int Engine::build_system() {  // block_solver.hpp:462-521
  if (!structure_built) {
    int r = build_structure();
    if (r) return r;
  }
  ensure_device_state();
  EdgeArgs a = edge_args(dv0, dv1, dmeas, dinfo, dparams, dstate[vt0].get(), dstate[vt1].get());
  timer.begin("linearize", stream);
  launch::linearize(family, a, ne, d_hidx[vt0].get(), d_hidx[vt1].get(), dslot0.get(), dslot1.get(), doff_dst.get(),
                    doff_tr.get(), off_dup ? doffslot.get() : dH.get(), stream);
  timer.end(stream);
  if (off_dup) launch::offblock_reduce(noffb, off_bsz, doffb_ptr.get(), doffb_edges.get(), doffslot.get(), dH.get(),
                                       doffb_dst.get(), stream);
  timer.begin("vreduce", stream);
  launch::vertex_reduce(pd, vr_pose.nv, vr_pose.lanes, vr_pose.ptr.get(), vr_pose.code.get(), dslot0.get(), dslot1.get(),
                        slot_stride0, slot_stride1, vr_pose.H, db.get(), vr_pose.boff.get(), stream);
  if (do_schur)
    launch::vertex_reduce(ld, vr_lm.nv, vr_lm.lanes, vr_lm.ptr.get(), vr_lm.code.get(), dslot0.get(), dslot1.get(),
                          slot_stride0, slot_stride1, vr_lm.H, db.get(), vr_lm.boff.get(), stream);
  timer.end(stream);
  return G2OHIP_OK;
}

void Engine::set_lambda_device(double l, bool reset_fail) {
  lambda_host = l;
  launch::set_scalars(dscal.get(), l, rank == 0 ? l : 0.0, stream, reset_fail);
}

int Engine::set_lambda(double lambda, int /*backup*/) {  // block_solver.hpp:524-550 (lambda kept virtual)
  set_lambda_device(lambda);
  lambda_set = true;
  return G2OHIP_OK;
}
int Engine::restore_diagonal() {  // :552-565
  set_lambda_device(0.0);
  lambda_set = false;
  return G2OHIP_OK;
}

void Engine::solve_async(bool reset_fail) {  // block_solver.hpp:314-447
  if (reset_fail) HIP_CHECK(hipMemsetAsync(failp(), 0, sizeof(int) * 2, stream));
  const bool sev = stats_level >= 2;  // stage events for G2OBatchStatistics
  if (sev) HIP_CHECK(hipEventRecord(ev_[0], stream));
  ev_valid_ = sev;
  if (!do_schur) {
    if (sev) HIP_CHECK(hipEventRecord(ev_[1], stream));
    if (use_pcg()) {
      timer.begin("pcg", stream);
      pcg.solve(dH.get(), dscal.get(), db.get(), dx.get(), stream);
      timer.end(stream);
      if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
      if (sev) HIP_CHECK(hipEventRecord(ev_[3], stream));
      return;
    }
    timer.begin("chol_factor", stream);
    chol.factor(dH.get(), dscal.get(), db.get(), failp(), stream);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
    timer.begin("chol_solve", stream);
    chol.solve(dx.get(), stream);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[3], stream));
    return;
  }
  const int lm_begin = local_lm.empty() ? 0 : local_lm.front();
  const int nLloc = (int)local_lm.size();
  const double* Hpl = dH.get() + (long long)nHpp * pd * pd;
  double* S = dS.get();
  double* bschur = dS.get() + (size_t)nS * pd * pd;
  timer.begin("schur_dinv", stream);
  launch::schur_prep(nLloc, lm_begin, dHll.get(), db.get() + size_poses, dscal.get(), dDinv.get(), dUfac.get(),
                     dCl.get(), failp() + 1, stream);
  timer.end(stream);
  timer.begin("schur_diag", stream);
  launch::schur_diag(num_poses, sch_rptr.get(), sch_robs.get(), sch_obs_lm.get(), lm_begin, Hpl, dUfac.get(), dCl.get(),
                     sch_sdiag.get(), ds_hpp.get(), dH.get(), db.get(), dscal.get() + 4, S, bschur, dG.get(), stream);
  timer.end(stream);
  timer.begin("schur_rows", stream);
  launch::schur_rows(nsch_tasks, sch_tasks.get(), sch_batches.get(), sch_st_obs.get(), sch_pairs.get(), sch_pp.get(),
                     dG.get(), ds_hpp.get(), dH.get(), S, stream);
  timer.end(stream);
  allreduce_sum(S, (size_t)nS * pd * pd + size_poses);
  if (sev) HIP_CHECK(hipEventRecord(ev_[1], stream));
  if (use_pcg()) {
    timer.begin("pcg", stream);
    pcg.solve(S, dscal.get() + 5, bschur, dx.get(), stream);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
  } else {
    timer.begin("chol_factor", stream);
    chol.factor(S, dscal.get() + 5, bschur, failp(), stream);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
    timer.begin("chol_solve", stream);
    chol.solve(dx.get(), stream);
    timer.end(stream);
  }
  if (sev) HIP_CHECK(hipEventRecord(ev_[3], stream));
  timer.begin("backsub", stream);
  launch::backsub(nLloc, d_lm_ptr.get(), d_blk_pose.get(), Hpl, dDinv.get(), db.get(), size_poses, lm_begin, dx.get(),
                  stream);
  timer.end(stream);
}

int Engine::solve_sync() {
  if (!structure_built) return G2OHIP_ERR_STATE;
  solve_async(true);
  int f[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(f, failp(), sizeof f, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  timer.collect();
  return f[0] ? 0 : 1;
}

void Engine::update_async() {  // sparse_optimizer.cpp:441-454
  timer.begin("oplus", stream);
  for (int t = 1; t <= 4; ++t) {
    const int n = (int)hg.by_type[t].size();
    if (!n) continue;
    launch::oplus(t, n, d_xoff[t].get(), dx.get(), dstate[t].get(), t == G2OHIP_V_SE3_QUAT ? dnopl.get() : nullptr, stream);
  }
  timer.end(stream);
  host_state_stale = true;
  ++state_ver;
}

int Engine::update_from(const double* xh) {
  if (!structure_built) return G2OHIP_ERR_STATE;
  ensure_device_state();
  if (xh) HIP_CHECK(hipMemcpyAsync(dx.get(), xh, sizeof(double) * vector_size(), hipMemcpyHostToDevice, stream));
  update_async();
  HIP_CHECK(hipStreamSynchronize(stream));
  timer.collect();
  return G2OHIP_OK;
}

int Engine::get_x(double* x) {
  if (!structure_built) return G2OHIP_ERR_STATE;
  dx.download(x, vector_size(), stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  return G2OHIP_OK;
}
int Engine::get_b(double* b) {
  if (!structure_built) return G2OHIP_ERR_STATE;
  db.download(b, vector_size(), stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  return G2OHIP_OK;
}

int Engine::push() {  // base_vertex.h:93-95 for all active vertices (stream-ordered device copy)
  ensure_device_state();
  if ((int)stack_.size() <= stack_depth_) stack_.emplace_back(5);
  auto& lvl = stack_[stack_depth_++];
  launch::CopyList cl{};
  for (int t = 1; t <= 4; ++t) {
    if (!dstate[t].size()) continue;
    lvl[t].resize(dstate[t].size());
    cl.src[cl.n] = dstate[t].get();
    cl.dst[cl.n] = lvl[t].get();
    cl.len[cl.n++] = (long long)dstate[t].size();
  }
  launch::copy_multi(cl, stream);  // one launch for every vertex type
  return G2OHIP_OK;
}
int Engine::pop() {
  if (stack_depth_ == 0) return G2OHIP_ERR_STATE;
  auto& lvl = stack_[--stack_depth_];
  launch::CopyList cl{};
  for (int t = 1; t <= 4; ++t)
    if (lvl[t].size()) {
      cl.src[cl.n] = lvl[t].get();
      cl.dst[cl.n] = dstate[t].get();
      cl.len[cl.n++] = (long long)lvl[t].size();
    }
  launch::copy_multi(cl, stream);
  host_state_stale = true;
  ++state_ver;
  return G2OHIP_OK;
}
int Engine::discard_top() {
  if (stack_depth_ == 0) return G2OHIP_ERR_STATE;
  --stack_depth_;
  return G2OHIP_OK;
}

double Engine::lambda_init() {  // optimization_algorithm_levenberg.cpp:152-175
  // Hpp diagonal blocks are partial per rank when sharded: reduce them first (copy)
  const double* Hp = dH.get();
  DevBuf<double> tmp;
  if (do_schur && nranks > 1) {
    tmp.resize((size_t)num_poses * pd * pd);
    HIP_CHECK(hipMemcpyAsync(tmp.get(), dH.get(), tmp.bytes(), hipMemcpyDeviceToDevice, stream));
    allreduce_sum(tmp.get(), tmp.size());
    Hp = tmp.get();
  }
  launch::diag_absmax(Hp, num_poses, pd, do_schur ? dHll.get() : nullptr, do_schur ? (int)local_lm.size() : 0, ld,
                      dpartial.get(), dscal.get() + 3, stream);
  if (nranks > 1 && comm) {
    comm->allreduce_max(dscal.get() + 3, 1, stream);
  }
  double m = 0;
  HIP_CHECK(hipMemcpyAsync(&m, dscal.get() + 3, sizeof(double), hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  return 1e-5 * m;
}

// OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:58-150)
int Engine::lm_solve(int iteration, const g2ohip_config& cfg, g2ohip_batch_stats* st) {
  if (iteration == 0) {
    if (!structure_built) {
      double t0 = wall();
      int r = build_structure();
      if (r) return 2;  // Fail
      if (st) st->timeSymbolicDecomposition = wall() - t0;
    }
  }
  double t = wall();
  const double currentChi0 = chi2_sync();
  if (st) { st->timeResiduals = wall() - t; t = wall(); }
  double currentChi = currentChi0;
  double tempChi = currentChi;
  hipEvent_t e0 = lm_ev_[0], e1 = lm_ev_[1], e2 = lm_ev_[2], e3 = lm_ev_[3], q0 = lm_ev_[4], q1 = lm_ev_[5];
  if (st && stats_level >= 2) HIP_CHECK(hipEventRecord(q0, stream));
  if (built_ver != state_ver || iteration == 0) build_system();  // else enqueued by the previous iteration
  if (st && stats_level >= 2) HIP_CHECK(hipEventRecord(q1, stream));  // timeQuadraticForm from events
  built_ver = 0;
  if (iteration == 0) {
    current_lambda = cfg.user_lambda_init > 0 ? cfg.user_lambda_init : lambda_init();
    ni = 2;
  }
  const int maxTrials = cfg.max_trials_after_failure > 0 ? cfg.max_trials_after_failure : 10;
  double rho = 0;
  int& qmax = levenberg_iterations;
  qmax = 0;
  bool first_trial = true;
  do {
    push();
    if (st) st->levenbergIterations++;
    const bool ev1 = st && stats_level >= 1, ev2 = st && stats_level >= 2;
    set_lambda_device(current_lambda, true);  // also clears the not-PD flags
    if (ev1) HIP_CHECK(hipEventRecord(e0, stream));
    solve_async(false);
    if (ev1) HIP_CHECK(hipEventRecord(e1, stream));
    update_async();
    if (ev2) HIP_CHECK(hipEventRecord(e2, stream));
    // computeScale (:177-184) on the device, sum x (lambda x + b), while lambda is still set; the
    // restoreDiagonal that follows (:113) is the next setLambda (lambda is virtual, never in H)
    launch::scale_sum(vector_size(), size_poses, dx.get(), db.get(), dscal.get(), dpartial.get(), dscal.get() + 2,
                      stream);
    allreduce_sum(dscal.get() + 2, 1);
    compute_errors_async();
    if (ev2) HIP_CHECK(hipEventRecord(e3, stream));
    double hs[12];  // lambda, chi2, scale, ... | fail flags (one readback per trial)
    HIP_CHECK(hipMemcpyAsync(hs, dscal.get(), sizeof hs, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    timer.collect();
    tempChi = hs[1];
    int f[2];
    std::memcpy(f, hs + 8, sizeof f);
    const bool ok2 = f[0] == 0;
    if (ev2 && first_trial) {
      float mq = 0;
      HIP_CHECK(hipEventElapsedTime(&mq, q0, q1));
      st->timeQuadraticForm = mq * 1e-3;
    }
    first_trial = false;
    if (ev1) {
      float ms01 = 0;
      HIP_CHECK(hipEventElapsedTime(&ms01, e0, e1));
      st->timeLinearSolution += ms01 * 1e-3;
    }
    if (ev2) {
      float ms12 = 0, a = 0, b = 0, c = 0;
      HIP_CHECK(hipEventElapsedTime(&ms12, e1, e2));
      HIP_CHECK(hipEventElapsedTime(&a, ev_[0], ev_[1]));
      HIP_CHECK(hipEventElapsedTime(&b, ev_[1], ev_[2]));
      HIP_CHECK(hipEventElapsedTime(&c, ev_[1], ev_[3]));
      st->timeUpdate = ms12 * 1e-3;
      st->timeSchurComplement = do_schur ? a * 1e-3 : 0.0;
      st->timeNumericDecomposition = b * 1e-3;
      st->timeLinearSolver = c * 1e-3;
    }
    if (!ok2) tempChi = std::numeric_limits<double>::max();
    rho = currentChi - tempChi;
    double scale = hs[2];
    scale += 1e-3;
    rho /= scale;
    if (rho > 0 && std::isfinite(tempChi)) {
      double alpha = 1. - std::pow((2 * rho - 1), 3);
      alpha = std::min(alpha, 2. / 3.);
      const double scaleFactor = std::max(1. / 3., alpha);
      current_lambda *= scaleFactor;
      ni = 2;
      currentChi = tempChi;
      discard_top();
    } else {
      current_lambda *= ni;
      ni *= 2;
      pop();
      if (!std::isfinite(current_lambda)) break;
    }
    qmax++;
  } while (rho < 0 && qmax < maxTrials);
  set_lambda_device(0.0);  // restoreDiagonal of the last trial (block_solver.hpp:552-565)
  // the state left behind has chi2 currentChi (accepted: the last tempChi; rejected: popped back)
  chi_cache = currentChi;
  chi_ver = state_ver;
  // the next iteration starts with buildSystem on exactly this state: enqueue it now so the GPU works
  // while the host returns to the caller (skipped when the loop is about to stop)
  const bool more = !(qmax == maxTrials || rho == 0 || !std::isfinite(current_lambda));
  if (more) {
    build_system();
    built_ver = state_ver;
  }
  if (qmax == maxTrials || rho == 0 || !std::isfinite(current_lambda)) return 1;  // Terminate
  return 0;                                                                       // OK
}

int Engine::optimize_step(const g2ohip_config* cfgp, int i, g2ohip_batch_stats* st) {
  g2ohip_config cfg{10, 0.0, 0};
  if (cfgp) cfg = *cfgp;
  if (!initialized) {
    int r = initialize();
    if (r) return r;
  }
  if (ivmap.empty()) return -1;
  if (i == 0) structure_built = false;  // algorithm init: symbolic rebuilt on iteration 0 (linear_solver init())
  if (st) {
    std::memset(st, 0, sizeof *st);
    st->iteration = i;
    st->numEdges = (int)hg.ev0.size();
    st->numVertices = (int)active.size();
  }
  const double ts = wall();
  const int result = lm_solve(i, cfg, st);
  if (st || cfg.verbose) {
    const double c = chi2_sync();
    if (st) {
      st->chi2 = c;
      st->lambda = current_lambda;
      st->timeIteration = wall() - ts;
      st->hessianPoseDimension = size_poses;
      st->hessianLandmarkDimension = size_landmarks;
      st->hessianDimension = size_poses + size_landmarks;
      st->choleskyNNZ = (long long)chol.sym.nnzL;
    }
    if (cfg.verbose && rank == 0)
      fprintf(stderr, "iteration= %d\t chi2= %.6f\t time= %g\t edges= %zu\t lambda= %.6f\t levenbergIter= %d\n", i, c,
              wall() - ts, hg.ev0.size(), current_lambda, levenberg_iterations);
  }
  return result;
}

int Engine::optimize(const g2ohip_config* cfgp, int iterations, g2ohip_batch_stats* stats) {
  if (!initialized) {
    int r = initialize();
    if (r) return r;
  }
  if (ivmap.empty()) return -1;
  int cj = 0, result = 0;
  bool ok = true;
  for (int i = 0; i < iterations && ok; ++i) {
    result = optimize_step(cfgp, i, stats ? stats + i : nullptr);
    if (result < 0) return result;
    ok = result == 0;
    ++cj;
  }
  if (result == 2) return 0;
  return cj;
}

int Engine::stage(double lambda, double* b, double* x, double* Hs, double* bs, long long* dims) {
  if (!initialized) {
    int r = initialize();
    if (r) return r;
  }
  if (!structure_built) {
    int r = build_structure();
    if (r) return r;
  }
  const long long n = vector_size();
  if (dims) { dims[0] = n; dims[1] = size_poses; dims[2] = size_landmarks; }
  if (!b && !x && !Hs && !bs) return 1;
  build_system();
  set_lambda(lambda, 1);
  const int ok = solve_sync();
  if (b) db.download(b, n, stream);
  if (x) dx.download(x, n, stream);
  if (Hs || bs) {
    const int np = size_poses;
    std::vector<double> blocks;
    const std::vector<int>& bi = do_schur ? s_bi : hpp_bi;
    const std::vector<int>& bj = do_schur ? s_bj : hpp_bj;
    blocks.resize(bi.size() * pd * pd);
    if (do_schur) dS.download(blocks.data(), blocks.size(), stream);
    else dH.download(blocks.data(), blocks.size(), stream);
    std::vector<double> bsv(np);
    if (do_schur) HIP_CHECK(hipMemcpyAsync(bsv.data(), dS.get() + (size_t)nS * pd * pd, sizeof(double) * np, hipMemcpyDeviceToHost, stream));
    else db.download(bsv.data(), np, stream);
    HIP_CHECK(hipStreamSynchronize(stream));
    if (Hs) {
      std::fill(Hs, Hs + (size_t)np * np, 0.0);
      for (size_t t = 0; t < bi.size(); ++t)
        for (int c = 0; c < pd; ++c)
          for (int r = 0; r < pd; ++r) {
            double v = blocks[t * pd * pd + c * pd + r];
            if (!do_schur && bi[t] == bj[t] && r == c) v += lambda;
            const int gi = bi[t] * pd + r, gj = bj[t] * pd + c;
            Hs[(size_t)gi * np + gj] = v;
            Hs[(size_t)gj * np + gi] = v;
          }
    }
    if (bs) std::memcpy(bs, bsv.data(), sizeof(double) * np);
  }
  HIP_CHECK(hipStreamSynchronize(stream));
  restore_diagonal();
  return ok;
}

int Engine::set_comm(const unsigned char* uid, int r, int nr) {
  if (nr <= 1) { rank = 0; nranks = 1; comm.reset(); return G2OHIP_OK; }
  HIP_CHECK(hipSetDevice(device));
  std::string err;
  Comm* c = make_rccl_comm(uid, r, nr, err);
  if (!c) throw DeviceError(err);
  comm.reset(c);
  rank = r;
  nranks = nr;
  structure_built = false;
  edges_ready = false;
  return G2OHIP_OK;
}

int Engine::set_comm_local(const std::string& key, int r, int nr) {
  if (nr <= 1) { rank = 0; nranks = 1; comm.reset(); return G2OHIP_OK; }
  comm.reset(make_local_comm(key, r, nr));
  rank = r;
  nranks = nr;
  structure_built = false;
  edges_ready = false;
  return G2OHIP_OK;
}

double Engine::kernel_bytes(const std::string& name) const {
  // algorithmic bytes per launch (SURVEY.md §8d formulas)
  const double npl = nHpl, pb = (double)pd * ld * 8;
  // Schur row pass (off-diagonal blocks): G of every observation once, the off-diagonal Hpp blocks
  // present in S, the off-diagonal S blocks written once
  if (name == "schur_rows") return npl * pb + (double)(nHppUsed - num_poses) * pd * pd * 8 +
                                   (double)(nS - num_poses) * pd * pd * 8;
  // diagonal blocks: Hpl, U and c per observation's landmark, G written, Hpp diagonal, S diagonal + bschur
  if (name == "schur_diag") return 2 * npl * pb + local_lm.size() * 9 * 8.0 + (double)num_poses * pd * pd * 8 * 2 +
                                   size_poses * 16.0;
  if (name == "schur_dinv") return local_lm.size() * ((9 + 3) * 8.0 + (9 + 6 + 3) * 8.0);
  if (name == "linearize") return ne * (family == FAM_BA ? (2 + 3 + 4) * 8.0 + 8 + (double)(slot_stride0 + slot_stride1 + pd * ld) * 8 : 0.0);
  if (name == "backsub") return local_lm.size() * (3 * 8.0 * 2 + 72) + npl * (pb + 4) + size_poses * 8.0;
  if (name == "chol_factor") return (double)chol.sym.front_pool * 8 * 2;
  return 0;
}
double Engine::kernel_flops(const std::string& name) const {
  if (name == "chol_factor") return chol.sym.flops;
  if (name == "schur_rows") return (double)npairs * (108 * 2);
  return 0;
}

}  // namespace g2ohip
