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
#include <charconv>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>
#include <numeric>
#include <sstream>
#include <thread>

namespace g2ohip {

static double wall() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int vertex_dim(int t) {
  return t == G2OHIP_V_SE3_EXPMAP || t == G2OHIP_V_SE3_QUAT ? 6
         : (t == G2OHIP_V_XYZ || t == G2OHIP_V_SE2 ? 3 : (t == G2OHIP_V_XY ? 2 : -1));
}
int vertex_est_dim(int t) { return t == G2OHIP_V_SE3_EXPMAP || t == G2OHIP_V_SE3_QUAT ? 7 : (t == G2OHIP_V_XY ? 2 : 3); }
int vertex_state_stride(int t) {
  switch (t) {
    case G2OHIP_V_SE3_EXPMAP: return 8;
    case G2OHIP_V_XYZ: return 3;
    case G2OHIP_V_SE3_QUAT: return 12;
    case G2OHIP_V_SE2: return 3;
    case G2OHIP_V_XY: return 2;
  }
  return 0;
}
static bool is_hostj(int e) { return e > G2OHIP_E_HOSTJ(0) && e <= G2OHIP_E_HOSTJ(6); }
int edge_dim(int e) {
  if (is_hostj(e)) return e - G2OHIP_E_HOSTJ(0);
  return e == G2OHIP_E_SE3_PROJECT_XYZ || e == G2OHIP_E_SE2_XY ? 2 : (e == G2OHIP_E_SE3_QUAT ? 6 : (e == G2OHIP_E_SE2 ? 3 : -1));
}
int edge_meas_dim(int e) {
  if (is_hostj(e)) return 0;
  return e == G2OHIP_E_SE3_PROJECT_XYZ || e == G2OHIP_E_SE2_XY ? 2 : (e == G2OHIP_E_SE3_QUAT ? 7 : 3);
}

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
    case G2OHIP_V_XY: st[0] = est[0]; st[1] = est[1]; break;
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
    default:
      for (int k = 0; k < vertex_est_dim(vt); ++k) est[k] = st[k];
      break;
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
    default:
      for (int k = 0; k < vertex_dim(vt); ++k) out[k] = st[k];
      break;
  }
}

// ------------------------------------------------------------------ KernelTimer
// Events that only time work (read after a stream synchronisation, never waited on for data): without the system-scope
// fence an event record costs no L2 writeback / invalidate between the kernels it brackets (the default record added
// ~4 us of idle GPU per record to the LM iteration). G2OHIP_EVENT_FENCE=1 restores default events (A/B).
static unsigned timing_event_flags() {
  static const unsigned f = [] {
    const char* v = getenv("G2OHIP_EVENT_FENCE");
    return (v && atoi(v) != 0) ? (unsigned)hipEventDefault : (unsigned)hipEventDisableSystemFence;
  }();
  return f;
}
hipEvent_t KernelTimer::get() {
  if (!pool.empty()) {
    hipEvent_t e = pool.back();
    pool.pop_back();
    return e;
  }
  hipEvent_t e;
  HIP_CHECK(hipEventCreateWithFlags(&e, timing_event_flags()));
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
  if (pre_sym) sym = *pre_sym;
  else sym = analyze(block_pattern(nblocks, bdim, bi, bj));
  pre_sym.reset();
  const std::shared_ptr<const DistPlan> plan_given = std::move(pre_plan);
  pre_plan.reset();
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
  // ---- distribution over ranks (landmark-sharded BA): cut the elimination tree into a shared top and whole subtrees,
  // each subtree owned by one rank. Candidate cuts: starting from the tree's roots, the candidate subtree with the
  // largest serial work is split (its root joins the shared top), one cut per split, up to 4 candidates per rank; each
  // cut's subtrees go to ranks largest first (longest-processing-time rule). Every cut is priced with the level-
  // synchronous model (plan_distribution, symbolic.cpp: a rank's fronts of one tree level run in the same launches, as
  // do the shared ones) plus the exchanges it adds (root all-gather, x all-reduce) and its input (reduce-scatter +
  // tail all-reduce), and kept only if it beats the replicated factorization's model:
  // a tree whose top is all chain (C4 at 8 ranks: one-bandwidth separators) gains less from distribution than its
  // exchange costs. dist_force (G2OHIP_DIST_FACTOR=1, the simulation mode) takes the best cut regardless.
  sn_owner.assign(sym.sn.size(), -1);
  n_owned_fronts = n_shared_fronts = n_roots = 0;
  dist_on = false;
  std::fill(dist_model, dist_model + 5, 0.0);
  if (dist_nranks > 1) {
    const DistPlan P = plan_given ? *plan_given
                                  : plan_distribution(sym, bi, bj, bdim, nblocks, dist_nranks, dist_rank,
                                                      rs_enable && (bool)reduce_scatter, dist_force, aligned,
                                                      pose_work.empty() ? nullptr : &pose_work);
    rs_model[0] = P.input_s;
    rs_model[1] = P.input_repl_s;
    dist_on = P.on;
    dist_model[0] = P.rank_s;
    dist_model[1] = P.shared_s;
    dist_model[2] = P.repl_s;
    dist_model[3] = P.xch_s;
    dist_model[4] = dist_on ? 1.0 : 0.0;
    shard_model = dist_on ? P.shard_s : P.shard_repl_s;
    if (dist_on) {
      sn_owner = P.owner;
      for (int k = 0; k < (int)sym.sn.size(); ++k) {
        if (sn_owner[k] < 0) ++n_shared_fronts;
        else if (sn_owner[k] == dist_rank) ++n_owned_fronts;
      }
    }
  }
  // reduce-scatter layout of the input (see engine.hpp): block t -> rs_buf offset; the entry sources remapped into it
  rs_on = dist_on && rs_enable && reduce_scatter;
  rs_seg = rs_tail_len = rs_rhs_off = rs_local = 0;
  rs_nblk = (long long)bi.size();
  if (rs_on) {
    // block classes: 0..N-1 reduce-scattered to that rank, N shared (tail all-reduce), N+1 complete on this rank
    // (aligned shards: read from its own partial S), N+2 another rank's complete block (never read here)
    const int N = dist_nranks, B = bdim * bdim;
    const bool al = aligned && blk_local.size() == bi.size();
    std::vector<long long> cnt(N + 3, 0), boff(bi.size());
    std::vector<int> own(bi.size());
    for (size_t t = 0; t < bi.size(); ++t) {
      const int o = sn_owner[sym.block_sn[std::min(sym.bpinv[bi[t]], sym.bpinv[bj[t]])]];
      own[t] = o < 0 ? N : (al && blk_local[t]) ? (o == dist_rank ? N + 1 : N + 2) : o;
      cnt[own[t]]++;
    }
    rs_seg = *std::max_element(cnt.begin(), cnt.begin() + N) * B;
    rs_rhs_off = (long long)N * rs_seg + cnt[N] * B;
    rs_tail_len = cnt[N] * B + (long long)nblocks * bdim;
    rs_local = cnt[N + 1] * B;
    const long long loc0 = rs_rhs_off + (long long)nblocks * bdim;
    std::vector<long long> fillc(N + 3, 0);
    for (size_t t = 0; t < bi.size(); ++t) {
      const int o = own[t];
      const long long k = fillc[o]++ * B;
      boff[t] = o < N ? (long long)o * rs_seg + k : o == N ? (long long)N * rs_seg + k : o == N + 1 ? loc0 + k : -1;
    }
    if (loc0 + rs_local >= (1LL << 31)) throw DeviceError("reduce-scatter layout too large for 32-bit entry indexing");
    // another rank's complete blocks feed only that rank's fronts: their entries are never assembled here
    for (int& k : ent_srcv) k = boff[k / B] < 0 ? 0 : (int)(boff[k / B] + k % B);
    ent_src.upload(ent_srcv.empty() ? std::vector<int>{0} : ent_srcv, s);
    rs_bmap.upload(boff.empty() ? std::vector<long long>{0} : boff, s);
    rs_rhs_rng.upload(std::vector<long long>{(long long)bi.size() * B, rs_rhs_off, (long long)nblocks * bdim}, s);
    rs_buf.resize(std::max<long long>(loc0 + rs_local, 1));
    rs_buf.zero(s);  // segment padding is never written: zeros go into the reduce-scatter
  }
  // forward plan: the level front lists in execution order (distributed: this rank's fronts level by level, the root
  // exchange, then the shared fronts level by level); the backward solve walks the same plan in reverse
  std::vector<std::vector<int>> fplan;
  int xch_at = -1;
  if (distributed()) {
    for (const auto& lv : sym.levels) {
      std::vector<int> o;
      for (int sn : lv) if (sn_owner[sn] == dist_rank) o.push_back(sn);
      if (!o.empty()) fplan.push_back(o);
    }
    xch_at = (int)fplan.size();
    for (const auto& lv : sym.levels) {
      std::vector<int> o;
      for (int sn : lv) if (sn_owner[sn] < 0) o.push_back(sn);
      if (!o.empty()) fplan.push_back(o);
    }
  } else {
    fplan = sym.levels;
  }
  // per child: [#rows mapping into the parent's first diagonal block | first child row of every parent
  // slab] (rel is increasing), so the extend-add tasks need no search on the chain
  std::vector<int> hjt, hcmp;
  std::vector<longlong2> hcme;
  std::vector<launch::FrontDesc> hfd(sym.sn.size());
  long long loff = 0, xoff = 0;
  for (size_t k = 0; k < sym.sn.size(); ++k) {
    const Supernode& q = sym.sn[k];
    int jt = 0;
    if (q.parent >= 0) {
      const Supernode& pq = sym.sn[q.parent];
      const int mp = pq.ns + pq.nr, slab = level_slab[sn_level[q.parent]];
      const int kb0 = std::min(launch::CHOL_NB, pq.ns);
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
        // per pair: its update-matrix column (child rows jc .. nr-1 at U + i), the child's relmap, jc and nr
        const long long mc = cq.ns + cq.nr, u0 = cq.front_off + (cq.ns + 0) * mc + cq.ns;
        if (cq.rows_off >= (1LL << 31) || cq.nr >= (1 << 16)) throw DeviceError("extend-add record overflow");
        for (int jc = 0; jc < cq.nr; ++jc)
          hcme[base + fillc[sym.relmap[cq.rows_off + jc]]++] =
              longlong2{u0 + (long long)jc * mc, cq.rows_off | ((long long)jc << 32) | ((long long)cq.nr << 48)};
      }
      for (int j = 0; j <= m; ++j) hcmp.push_back(base + cnt[j]);
    }
    hfd[k] = launch::FrontDesc{q.front_off, q.vec_off, loff, q.rows_off, xoff, q.c0, q.ns, q.nr, q.parent,
                               sym.children_ptr[k], sym.children_ptr[k + 1], jt, cm};
    loff += (long long)(q.ns + q.nr) * q.ns;
    xoff += (long long)q.ns * q.ns;  // X = L11^-1, column-major
  }
  lpool = loff;
  {  // block-0 child records, in the children array's order (k_extend_add's block-0 tasks)
    std::vector<launch::B0Child> hb0c;
    for (int c : sym.children) {
      const Supernode& cq = sym.sn[c];
      const long long mc = cq.ns + cq.nr;
      if (cq.rows_off >= (1LL << 31)) throw DeviceError("block-0 record overflow");
      hb0c.push_back(launch::B0Child{cq.front_off + cq.ns * mc + cq.ns, cq.vec_off + cq.ns, (int)mc, cq.nr,
                                     (int)cq.rows_off, hjt[hfd[c].jt_off], hfd[c].jt_off});
    }
    b0child.upload(hb0c.empty() ? std::vector<launch::B0Child>(1) : hb0c, s);
  }
  fd.upload(hfd, s);
  jtab.upload(hjt.empty() ? std::vector<int>{0} : hjt, s);
  cmptr.upload(hcmp.empty() ? std::vector<int>{0} : hcmp, s);
  hcme.push_back(longlong2{0, 0});  // sentinel: k_extend_add reads a column's first record even for an empty range
  cment.upload(hcme, s);
  std::vector<int> ll;
  level_off.assign(1, 0);
  for (auto& lv : sym.levels) {
    ll.insert(ll.end(), lv.begin(), lv.end());
    level_off.push_back((int)ll.size());
  }
  lfronts.upload(ll.empty() ? std::vector<int>{0} : ll, s);
  {
    std::vector<long long> wo(std::max<size_t>(sym.sn.size(), 1), 0);
    long long w = 0;
    for (size_t k = 0; k < sym.sn.size(); ++k) { wo[k] = w; w += (long long)sym.sn[k].nr * 64; }
    wpool = std::max(w, 1LL);
    woff.upload(wo, s);
  }
  // work lists per level: extend-add, first diagonal block, one step per 32-wide panel,
  // contribution blocks
  {
    using launch::Task;
    const int NB = launch::CHOL_NB, TT = launch::CHOL_TT, EA = launch::CHOL_EA;
    // envelope of a band supernode (Supernode::env_off): the first own column with a structural nonzero among the
    // front rows [r, r + 64); dense supernodes: 0
    auto tile_fnz = [&](int sn, int r) {
      const Supernode& q = sym.sn[sn];
      if (q.env_off < 0) return 0;
      const int m = q.ns + q.nr;
      int f = 1 << 30;
      for (int i = r; i < std::min(r + TT, m); ++i) f = std::min(f, sym.fnz[q.env_off + i]);
      return f;
    };
    auto tile_nz = [&](int sn, int r, int kend) { return tile_fnz(sn, r) < kend; };
    // k_syrk's row tiles: SR rows (64, or 128 for the 128 x 64 tile variants)
    syrk_var = launch::syrk_variant();  // pinned: chol_syrk launches this tile for these row-tile lists
    const int SR = launch::syrk_tile_rows(syrk_var);
    auto rows_fnz = [&](int sn, int r) { return SR == TT ? tile_fnz(sn, r) : std::min(tile_fnz(sn, r), tile_fnz(sn, r + TT)); };
    auto rows_nz = [&](int sn, int r, int kend) { return rows_fnz(sn, r) < kend; };
    std::vector<Task> tk;
    std::vector<launch::StepTask> stk;
    std::vector<launch::B0Front> hb0;
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
    // wide levels block only supernodes wider than 512 columns (r06: C3 factor 26.04 -> 25.22 ms against 128, its
    // levels of >= 64 fronts, all <= 384 columns wide, then take the deferred-L21 path — panel steps over the own rows,
    // the rows below in one k_l21 GEMM — instead of 128-column big panels whose steps re-read the rows below;
    // profiles/r06_ab_defer_widepb.log, r06_ab_c3_blocking.log)
    const char* wp = getenv("G2OHIP_CHOL_WIDE_PB");
    const int wide_pb = wp ? std::max(64, atoi(wp) / 64 * 64) : 512;
#ifdef G2OHIP_DEV  // development build only (make dev): timing experiments that give a wrong result on purpose
    const bool dev_noinv = getenv("G2OHIP_DEV_NOINV") != nullptr;  // no inverse tasks (wrong solve)
    const bool dev_diagonly = getenv("G2OHIP_DEV_DIAGONLY") != nullptr;  // diagonal tasks only (wrong factor)
#else
    constexpr bool dev_noinv = false, dev_diagonly = false;
#endif
    // lagged trailing updates on levels with a separate contribution pass (their steps are bound by the rank-32
    // tile traffic, not the diagonal chain): even steps update only the next panel's column strip, odd steps
    // apply two panels at once (rank 64) to the rest of the supernode's columns (G2OHIP_CHOL_LAG=0: every step
    // updates every trailing column, A/B)
    const char* lg = getenv("G2OHIP_CHOL_LAG");
    const int lag_mode = lg ? atoi(lg) : 1;  // 0 off, 1 throughput-bound levels, 2 every unblocked level
    const bool lag_on = lag_mode != 0;
    // fused-contribution levels are lagged when their first step has more tiles than one per CU (C4: the 4-front
    // level, 183 -> 161 us; the 1- and 2-front levels are bound by the diagonal chain and lose ~6 us each)
    const char* lfm = getenv("G2OHIP_CHOL_LAG_FUSED_MIN");
    const long long lag_fused_min = lag_mode >= 2 ? 0 : (lfm ? atoll(lfm) : 256);
    // deferred L21 on wide throughput-bound levels: the panel steps factor only each front's own rows (the trailing tiles
    // below the supernode are most of a lagged step's load burst), then L21 = A21 X^T in one GEMM launch (k_l21, with
    // the explicit X = L11^-1 the inverse tasks build) and the contribution pass updates the front vector's lower rows
    // (G2OHIP_CHOL_DEFER_L21: 0 off, 1 levels of >= G2OHIP_CHOL_DEFER_MIN fronts (default 16), 2 every eligible level)
    const char* dlv = getenv("G2OHIP_CHOL_DEFER_L21");
    const int dl_mode = dlv ? atoi(dlv) : 1;
    const char* dlm = getenv("G2OHIP_CHOL_DEFER_MIN");
    const int dl_min = dlm ? atoi(dlm) : 16;
    std::vector<unsigned char> sn_dl(sym.sn.size(), 0);
    n_deferred_l21 = 0;
    const char* cbk = getenv("G2OHIP_EA_CB_ZERO");  // dev A/B: 1 = in-place assembly also zeroes childless fronts' CBs
    const bool cb_keep = cbk && atoi(cbk) == 1;
    const char* eb = getenv("G2OHIP_EA_BIG");
    const int ea_big = eb ? atoi(eb) : 1024;  // C3 factor 28.29 (2048) -> 27.71 ms (1024), 28.31 (512)
    const char* pm = getenv("G2OHIP_CHOL_PRE_MAX");  // dev A/B: largest level (bytes) pre-scattered
    const long long pre_max = pm ? atoll(pm) : (256LL << 20);
    std::vector<long long> zr, pdst;
    std::vector<int> psrc;
    std::vector<long long> pre_lev_off;  // per level: its first entry in pdst / psrc (level-major)
    for (size_t l = 0; l < fplan.size(); ++l) {
      pre_lev_off.push_back((long long)pdst.size());
      if ((int)l == xch_at) {  // subtree roots -> every rank (before the first shared front is assembled)
        ops.push_back(Op{8, 0, 0});
       
      }
      const auto& lv = fplan[l];
      long long tiles0 = 0;  // fused tiles of the level's first step
      if (l == 0) n_blocked = n_inplace_levels = n_pre_levels = n_syrk_ops = n_bwd_rounds = 0;
      for (int sn : lv) {
        const Supernode& q = sym.sn[sn];
        const int r0 = std::min(NB, q.ns), T = (q.ns + q.nr - r0 + TT - 1) / TT;
        tiles0 += (long long)T * (T + 1) / 2;
      }
      const bool fused_contrib = tiles0 <= fused_max;
      // k_extend_add: every front's first-diagonal-block task first, then the slabs
      // small levels (all fronts <= pre_max bytes together) are zeroed + scattered before the first level
      // (two massively parallel passes off the critical chain); large ones are assembled in place
      // levels whose fronts are mostly input entries (a dense reduced system: few children) are pre-scattered
      // too, whatever their size: one thread per entry instead of a dependent gather chain per front column
      long long lbytes = 0, lent = 0, ltri = 0;
      for (int sn : lv) {
        const Supernode& q = sym.sn[sn];
        const long long m = q.ns + q.nr;
        lbytes += 8LL * m * m;
        lent += cpv[q.c0 + q.ns] - cpv[q.c0];
        ltri += (long long)q.ns * (2 * m - q.ns + 1) / 2;
      }
      const bool pre = lbytes <= pre_max || 2 * lent >= ltri;
      (pre ? n_pre_levels : n_inplace_levels)++;
      if (pre)
        for (int sn : lv) {
          const Supernode& q = sym.sn[sn];
          // only the lower triangle is ever read (tiles, contribution passes and extend-add touch rows >= columns):
          // zero column j's rows [j, m), whole small fronts in one range
          const long long m = q.ns + q.nr, len = m * m;
          // a childless front whose contribution block comes from a separate k_syrk pass gets it written, not added
          // (k_syrk's overwrite): its columns >= ns need no zeros
          const bool cb_written = !fused_contrib && sym.children_ptr[sn + 1] == sym.children_ptr[sn];
          const long long zcols = cb_written ? q.ns : m;
          if (m <= 64)
            for (long long o = 0; o < len; o += 65536) { zr.push_back(q.front_off + o); zr.push_back(std::min(65536LL, len - o)); }
          else
            for (long long j = 0; j < zcols; ++j) { zr.push_back(q.front_off + j * m + j); zr.push_back(m - j); }
          for (int c = q.c0; c < q.c0 + q.ns; ++c)
            for (int e = cpv[c]; e < cpv[c + 1]; ++e) {
              pdst.push_back(edsts[e]);
              psrc.push_back(ent_srcv[e] | ((ent_rowv[e] >> 30) ? (int)0x80000000 : 0));
            }
        }
      int lmaxm = 0;
      for (int sn : lv) lmaxm = std::max(lmaxm, sym.sn[sn].ns + sym.sn[sn].nr);
      // column buffer of the in-place assembly: 512 rows (five workgroups per CU) up to m = 512, else ea_big rows
      // (G2OHIP_EA_BIG, dev A/B: 512 / 1024 / 2048; profiles/r04_ab_c3_ea.log)
      Op ea{pre ? 0 : (lmaxm <= 512 || ea_big == 512 ? 5 : ea_big == 1024 ? 9 : 4), (int)tk.size(), 0};
      // first diagonal blocks: assembled and factored beside the slabs (the launch's first nb0 workgroups, records
      // in b0front from ea.b0)
      ea.b0 = (int)hb0.size();
      ea.nb0 = (int)lv.size();
      for (int sn : lv) {
        tk.push_back(Task{sn, 0, 0, 1});
        const Supernode& q = sym.sn[sn];
        hb0.push_back(launch::B0Front{q.front_off, q.vec_off, q.ns + q.nr, std::min(NB, q.ns), q.c0,
                                      sym.children_ptr[sn], sym.children_ptr[sn + 1]});
      }
      // every front is assembled here (input entries, zeros, children); slabs of EA columns where the level
      // has enough of them to fill the chip several times over, else 4 (latency-bound upper levels)
      const int slab = level_slab[sn_level[lv[0]]];
      for (int sn : lv) {
        const Supernode& q = sym.sn[sn];
        const int m = q.ns + q.nr;
        const bool childless = sym.children_ptr[sn + 1] == sym.children_ptr[sn];
        if (pre && childless) continue;  // nothing left to assemble
        // a childless front's contribution block is written (not read) by its level's separate k_syrk pass
        // (overwrite): its own columns only (the pre-scattered levels skip those zeros the same way)
        const int mcols = childless && !fused_contrib && !cb_keep ? q.ns : m;
        for (int a = 0; a < mcols; a += slab) tk.push_back(Task{sn, a, std::min(a + slab, mcols), 2 + a / slab});
      }
      ea.count = (int)tk.size() - ea.off;
      ops.push_back(ea);
      if (getenv("G2OHIP_PRINT_LEVELS")) {  // diagnostics (stderr): the level's shape and its extend-add launch
        int mm = 0, mns = 0, nch = 0, mnrc = 0;
        long long cb = 0;
        for (int sn : lv) {
          const Supernode& q = sym.sn[sn];
          mm = std::max(mm, q.ns + q.nr);
          mns = std::max(mns, q.ns);
          for (int ci = sym.children_ptr[sn]; ci < sym.children_ptr[sn + 1]; ++ci) {
            const Supernode& cq = sym.sn[sym.children[ci]];
            ++nch;
            mnrc = std::max(mnrc, cq.nr);
            cb += (long long)cq.nr * (cq.nr + 1) / 2;
          }
        }
        fprintf(stderr, "level %zu: fronts %zu max_m %d max_ns %d children %d max_child_nr %d child_cb_MB %.1f slab %d %s ea_tasks %d\n",
                l, lv.size(), mm, mns, nch, mnrc, cb * 8e-6, slab, pre ? "pre" : "inplace", ea.count);
      }
     
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
      const bool dl_level = dl_mode != 0 && !fused_contrib && !distributed() && (dl_mode == 2 || (int)lv.size() >= dl_min);
      for (int sn : lv) {
        const Supernode& q = sym.sn[sn];
        sn_dl[sn] = dl_level && !blocked(q) && q.nr > 0 && q.env_off < 0 ? 1 : 0;
        n_deferred_l21 += sn_dl[sn];
      }
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
          // fused contribution (lag mode 2): the contribution columns ride with the pairs; an even LAST step updates
          // every trailing column with its own panel (nothing may stay behind for the parent)
          const bool lagged = lag_on && !blk && (!fused_contrib || tiles0 > lag_fused_min);
          const bool last = r0 >= q.ns;
          const bool strip = lagged && (p % 2 == 0) && !(fused_contrib && last), pair = lagged && (p % 2 == 1);
          // fused: every panel step also applies its rank-kb update to the contribution block (the
          // step is latency-bound on the diagonal chain, the extra tiles run in its shadow); lagged even steps
          // stop at the next panel's strip
          const int clim = strip ? std::min(q.ns, r0 + NB) : (fused_contrib ? m : pend);
          const int rows = sn_dl[sn] ? q.ns : m;  // deferred L21: the supernode's own rows only
          const int T = (rows - r0 + TT - 1) / TT, TJ = (clim - r0 + TT - 1) / TT;
          const int fl = (fused_contrib ? 8 : 0) | (bnd ? 32 : 0) | (pair ? 64 : 0) | (sn_dl[sn] ? 128 : 0);
          auto mk = [&](int tile, int flags) {
            return launch::StepTask{hfd[sn].front_off, hfd[sn].l_off, hfd[sn].vec_off, hfd[sn].x_off, m, q.ns, q.c0,
                                    k0 | (kb << 16), tile, flags, clim};
          };
          if (r0 < q.ns && !bnd) diag_t.push_back(mk(0, 4 | (pair ? 64 : 0)));
          // band supernodes: a tile whose rows carry no structural nonzero in the panel (or, for the update, whose
          // column rows carry none) would only move exact zeros: no task (its L rows stay zero in the pre-zeroed lbuf)
          for (int tj = 0; tj < std::max(TJ, 1); ++tj) {
            const bool nzj = tile_nz(sn, r0 + TT * tj, k0 + kb);
            if (tj > 0 && !nzj) continue;
            for (int ti = tj; ti < T; ++ti) {
              if (!tile_nz(sn, r0 + TT * ti, k0 + kb)) continue;
              tile_t.push_back(mk(ti | (tj << 16), (tj < TJ && nzj ? 1 : 0) | fl));
            }
          }
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
        for (int k = st.off; k < st.off + st.count; ++k)
          if (stk[k].flags & 64) st.kind = 6;
        if (st.count) { ops.push_back(st); }
        if ((p + 1) * NB % lpb) continue;
        // end of a big panel: trailing update of the blocked fronts, then their next first blocks
        Op gm{3, (int)tk.size(), 0};
        Op d0{2, (int)stk.size(), 0};
        for (int sn : lv) {
          const Supernode& q = sym.sn[sn];
          const int kb = (p + 1) * NB, ka = kb - lpb, m = q.ns + q.nr;
          if (!blocked(q) || kb >= q.ns) continue;
          const int T = (m - kb + SR - 1) / SR, TJ = (q.ns - kb + TT - 1) / TT;
          for (int tj = 0; tj < TJ; ++tj) {
            if (!tile_nz(sn, kb + TT * tj, kb)) continue;
            for (int ti = TT * tj / SR; ti < T; ++ti)
              if (rows_nz(sn, kb + SR * ti, kb)) tk.push_back(Task{sn, ka, ti | (tj << 16), kb});
          }
          stk.push_back(launch::StepTask{hfd[sn].front_off, hfd[sn].l_off, hfd[sn].vec_off, hfd[sn].x_off, m, q.ns,
                                         q.c0, kb, 0, 4, q.ns});
        }
        gm.count = (int)tk.size() - gm.off;
        d0.count = (int)stk.size() - d0.off;
        if (gm.count) { ops.push_back(gm); ++n_syrk_ops; }
        if (d0.count) { ops.push_back(d0); }
      }
      {  // deferred L21: X's diagonal blocks for the level's fronts, then L21 = A21 X^T
        Op xd{11, (int)tk.size(), 0};
        for (int sn : lv)
          if (sn_dl[sn])
            for (int a = 0; a < sym.sn[sn].ns; a += NB) tk.push_back(Task{sn, a, 0, 0});
        xd.count = (int)tk.size() - xd.off;
        if (xd.count) ops.push_back(xd);
        Op gl{12, (int)tk.size(), 0};
        for (int sn : lv) {
          if (!sn_dl[sn]) continue;
          const Supernode& q = sym.sn[sn];
          for (int ti = 0; ti < (q.nr + TT - 1) / TT; ++ti)
            for (int tj = 0; tj < (q.ns + TT - 1) / TT; ++tj) tk.push_back(Task{sn, 0, ti | (tj << 16), 0});
        }
        gl.count = (int)tk.size() - gl.off;
        if (gl.count) ops.push_back(gl);
      }
      Op sy{3, (int)tk.size(), 0};
      for (int sn : lv) {
        if (fused_contrib) break;
        const Supernode& q = sym.sn[sn];
        const int T = (q.nr + SR - 1) / SR, TJ = (q.nr + TT - 1) / TT;
        const bool childless = sym.children_ptr[sn + 1] == sym.children_ptr[sn];
        for (int tj = 0; tj < TJ; ++tj)
          for (int ti = TT * tj / SR; ti < T; ++ti) {
            // band supernodes: K starts where both tile row sets have structural nonzeros; a tile with none only keeps
            // its entries (childless fronts' contribution blocks are written, not read: an empty K writes the zeros)
            const int ka = std::max(rows_fnz(sn, q.ns + SR * ti), tile_fnz(sn, q.ns + TT * tj));
            if (ka >= q.ns && !childless) continue;
            // deferred L21: the first tile of each row tile (its diagonal) also applies the forward solve to the
            // vector's rows below
            const int vb = sn_dl[sn] && ti == TT * tj / SR && (TT * tj) % SR == 0 ? (int)0x80000000 : 0;
            tk.push_back(Task{sn, std::min(ka, q.ns), ti | (tj << 16) | vb, 0});
          }
      }
      sy.count = (int)tk.size() - sy.off;
      if (sy.count) { ops.push_back(sy); ++n_syrk_ops; }
      for (int sn : lv) n_blocked += blocked(sym.sn[sn]) ? 1 : 0;
    }
    // root exchange (distributed): per subtree root, the lower triangle of its contribution block column by column
    // and its update vector, packed into the owning rank's segment of one buffer (segments of xch_seg doubles, the
    // largest rank's roots); one all-gather hands every segment to every rank, which unpacks the others' roots into its
    // front pool / front vectors
    if (distributed()) {
      std::vector<long long> pf, pv, uf, uv, zi, roff(dist_nranks, 0);
      n_roots = 0;
      auto add = [](std::vector<long long>& v, long long a, long long b, long long n) { v.push_back(a); v.push_back(b); v.push_back(n); };
      for (size_t k = 0; k < sym.sn.size(); ++k) {  // segment sizes first
        const int par = sym.sn[k].parent;
        if (sn_owner[k] < 0 || par < 0 || sn_owner[par] >= 0) continue;
        const long long nr = sym.sn[k].nr;
        roff[sn_owner[k]] += nr * (nr + 1) / 2 + nr;
      }
      xch_seg = std::max<long long>(*std::max_element(roff.begin(), roff.end()), 1);
      std::fill(roff.begin(), roff.end(), 0);
      for (size_t k = 0; k < sym.sn.size(); ++k) {
        const int par = sym.sn[k].parent;
        if (sn_owner[k] < 0 || par < 0 || sn_owner[par] >= 0) continue;
        ++n_roots;
        const Supernode& q = sym.sn[k];
        const long long m = q.ns + q.nr;
        const int o = sn_owner[k];
        const bool mine = o == dist_rank;
        long long off = (long long)o * xch_seg + roff[o];
        for (int j = 0; j < q.nr; ++j) {
          const long long fo = q.front_off + (long long)(q.ns + j) * m + q.ns + j, len = q.nr - j;
          if (mine) add(pf, fo, off, len); else add(uf, off, fo, len);
          off += len;
        }
        if (q.nr > 0) {
          if (mine) add(pv, q.vec_off + q.ns, off, q.nr); else add(uv, off, q.vec_off + q.ns, q.nr);
          off += q.nr;
        }
        roff[o] = off - (long long)o * xch_seg;
      }
      xch_len = (long long)dist_nranks * xch_seg;
      xch_pack_f = (int)pf.size() / 3; xch_pack_v = (int)pv.size() / 3;
      xch_unpack_f = (int)uf.size() / 3; xch_unpack_v = (int)uv.size() / 3;
      std::vector<long long> all;
      for (auto* v : {&pf, &pv, &uf, &uv}) all.insert(all.end(), v->begin(), v->end());
      xch_ranges.upload(all.empty() ? std::vector<long long>{0, 0, 0} : all, s);
      xch_buf.resize(std::max<long long>(xch_len, 1));
      std::vector<int> zx;
      for (size_t k = 0; k < sym.sn.size(); ++k)
        if (sn_owner[k] < 0)
          for (int c = sym.sn[k].c0; c < sym.sn[k].c0 + sym.sn[k].ns; ++c) zx.push_back(sym.perm[c]);
      nxzero = (int)zx.size();
      xzero_idx.upload(zx.empty() ? std::vector<int>{0} : zx, s);
      xred.resize((size_t)sym.n + 1);
    }
    nzero = (int)(zr.size() / 2);
    npre = (long long)pdst.size();
    pre_lev_off.push_back(npre);
    zero_rng.upload(zr.empty() ? std::vector<long long>{0, 0} : zr, s);
    pre_dst.upload(pdst.empty() ? std::vector<long long>{0} : pdst, s);
    pre_src.upload(psrc.empty() ? std::vector<int>{0} : psrc, s);
    // backward solve per level: gemv tasks (front, 4 columns) for every front, then x = X^T t for the
    // unblocked fronts (one launch) and, for blocked fronts, rounds over their big panels from the last:
    // t_b -= L(later rows of the supernode, b)^T x, x_b = X_bb^T t_b
    bwd_off.assign(1, (int)tk.size());
    bwd_ops.clear();
    max_ns = 1;
    for (size_t l = 0; l < fplan.size(); ++l) {
      const auto& lv = fplan[l];
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
        if (g.second) ++n_bwd_rounds;
      }
      // a level of roots only (no rows below: t = y - 0) skips its gemv launch; k_bwd_x reads y itself
      bool roots = bl.rounds.empty();
      for (int sn : lv) roots = roots && sym.sn[sn].nr == 0;
      if (roots) {
        bl.t_is_y = true;
        bl.gemv.second = 0;
      }
      bwd_ops.push_back(bl);
      bwd_off.push_back((int)tk.size());
    }
    // X's diagonal blocks stay in linv (the factorization publishes every L_kk^-1 there only): k_bwd_x reads them from
    // it, so no copy runs after the factorization (the deferred-L21 fronts' level k_xdiag launches remain: k_l21 reads X
    // whole)
    if (getenv("G2OHIP_PRINT_OPS")) {  // diagnostics (stderr): the factor's launch list in order, k_syrk with its flops
      for (size_t k = 0; k < ops.size(); ++k) {
        const Op& op = ops[k];
        double fma = 0;
        int kmin = 1 << 30, kmax = 0;
        if (op.kind == 3)
          for (int i = op.off; i < op.off + op.count; ++i) {
            const Task& t = tk[i];
            const int K = t.c ? t.c - t.a : sym.sn[t.s].ns - t.a;
            kmin = std::min(kmin, K);
            kmax = std::max(kmax, K);
            fma += (double)SR * TT * std::max(K, 0);
          }
        fprintf(stderr, "op %zu kind %d count %d%s", k, op.kind, op.count, op.kind == 3 ? "" : "\n");
        if (op.kind == 3) fprintf(stderr, " K %d..%d tile_gflop %.4f\n", kmin, kmax, 2 * fma * 1e-9);
      }
    }
    tasks.upload(tk.empty() ? std::vector<Task>{Task{0, 0, 0, 0}} : tk, s);
    step_tasks.upload(stk.empty() ? std::vector<launch::StepTask>(1) : stk, s);
    b0front.upload(hb0.empty() ? std::vector<launch::B0Front>(1) : hb0, s);
    ea_jobs.assign(ops.size(), launch::ScatterJob{});
    for (size_t k = 0; k < ops.size(); ++k) {
      const int kd = ops[k].kind;
      if (kd != 0 && kd != 4 && kd != 5 && kd != 9) continue;
      launch::ScatterJob& j = ea_jobs[k];
      j.ntask = ops[k].count;
      j.nb0 = ops[k].nb0;
      for (int i = 0; i < launch::EA_HEAD && i < ops[k].nb0; ++i) j.b0[i] = hb0[ops[k].b0 + i];
    }
    heads.assign(ops.size(), launch::StepHead{});
    for (size_t k = 0; k < ops.size(); ++k) {
      if (ops[k].kind != 2 && ops[k].kind != 6) continue;
      launch::StepHead& h = heads[k];
      h.ntask = ops[k].count;
      for (int i = 0; i < launch::CHOL_HEAD && i < ops[k].count; ++i)  // the first workgroups (diagonal tasks among them)
        h.t[i] = stk[ops[k].off + i];
    }
    // Deferred input scatter: a pre-scattered level's entries are needed only from its own extend-add on, so they ride
    // as extra workgroups in the previous level's first panel-step launch (chain-bound: the chip is mostly idle beside
    // its diagonal task) instead of all in one scatter launch before the first level. Its fronts were zeroed before the
    // factorization and no earlier level touches them. Levels up to the last one without a preceding step launch keep
    // the up-front scatter. Single-process factorizations only (G2OHIP_SCATTER_DEFER=0: all up front, A/B).
    {
      const char* dv = getenv("G2OHIP_SCATTER_DEFER");
      const bool defer = !distributed() && !(dv && atoi(dv) == 0);
      const int nlev = (int)fplan.size();
      std::vector<int> first_step(nlev, -1), ea_op(nlev, -1);
      int lev = -1;
      for (size_t k = 0; k < ops.size(); ++k) {
        const int kd = ops[k].kind;
        if (kd == 0 || kd == 4 || kd == 5 || kd == 9) {  // every level opens with its extend-add op
          if (++lev < nlev) ea_op[lev] = (int)k;
        } else if ((kd == 2 || kd == 6) && lev >= 0 && lev < nlev && first_step[lev] < 0) {
          first_step[lev] = (int)k;
        }
      }
      auto ents = [&](int l) { return pre_lev_off[l + 1] - pre_lev_off[l]; };
      // host launch of level l's entries: the previous level's extend-add, else its first panel step, whichever has
      // at most 256 workgroups of its own (latency-bound: the chip idle beside it); none: the entries stay up front
      auto host = [&](int l) {
        const int e = ea_op[l - 1], f = first_step[l - 1];
        if (e >= 0 && ops[e].count > 0 && ops[e].count <= 256) return e;
        if (f >= 0 && ops[f].count <= 256) return f;
        return -1;
      };
      int P = 0;  // levels 0 .. P scattered up front
      for (int l = 1; l < nlev; ++l)
        if (ents(l) > 0 && (!defer || lev != nlev - 1 || host(l) < 0)) P = l;
      npre_first = npre > 0 ? pre_lev_off[P + 1] : 0;
      n_deferred_levels = 0;
      for (int l = P + 1; l < nlev; ++l) {
        if (ents(l) == 0) continue;
        const int k = host(l);
        if (ops[k].kind == 2 || ops[k].kind == 6) {
          heads[k].sc0 = pre_lev_off[l];
          heads[k].sc1 = pre_lev_off[l + 1];
        } else {
          ops[k].sc0 = pre_lev_off[l];
          ops[k].sc1 = pre_lev_off[l + 1];
        }
        ++n_deferred_levels;
      }
    }
  }
  children.upload(sym.children.empty() ? std::vector<int>{0} : sym.children, s);
  relmap.upload(sym.relmap.empty() ? std::vector<int>{0} : sym.relmap, s);
  rows.upload(sym.rows.empty() ? std::vector<int>{0} : sym.rows, s);
  perm.upload(sym.perm, s);
  fronts.resize(std::max<int64_t>(sym.front_pool, 1) + 2);  // + a 16-byte piece of slack (k_l21 reads A21 by GemmNTd)
  vecs.resize(std::max<int64_t>(sym.vec_pool, 1));
  rhs_p.resize(std::max(sym.n, 1));
  y_p.resize(std::max(sym.n, 1));
  lbuf.resize(std::max<long long>(lpool, 1) + 2);  // + one 16-byte piece of slack after the last front (GemmNTd)
  if (!sym.fnz.empty()) lbuf.zero(s);  // band supernodes: the L rows of skipped tiles are read as zeros
  linv.resize((size_t)(sym.n + launch::CHOL_NB) * launch::CHOL_NB * launch::CHOL_NB);  // one 32x32 L_kk^-1 per panel start
  xinv.resize(std::max<long long>(xoff, 1) + 2);  // + slack: k_l21 stages X by GemmNTd
  // X's blocks above the diagonal are never written (the inverse tasks and k_xdiag fill the lower part, the diagonal
  // blocks with their zeros above): zero once, so a full-tile read of X (k_l21's B operand) sees an exact triangle
  xinv.zero(s);
  t_p.resize(std::max(sym.n, 1));
  x_p.resize(std::max(sym.n, 1));
}

void DeviceCholesky::factor(const double* vals, const double* lam, const double* rhs, int* fail, hipStream_t s,
                            bool prezeroed) {
  last_fail = fail;
  launch::chol_prescatter(prezeroed ? 0 : nzero, zero_rng.get(), npre_first, vals, pre_dst.get(), pre_src.get(), lam,
                          fronts.get(), (int)sym.sn.size(), fd.get(), perm.get(), rhs, vecs.get(), s);
  for (const Op& op : ops) {
    const launch::Task* t = tasks.get() + op.off;
    switch (op.kind) {
      case 0:
      case 4:
      case 5:
      case 9: {
        launch::ScatterJob sj = ea_jobs[&op - ops.data()];
        sj.sc0 = op.sc0;
        sj.sc1 = op.sc1;
        sj.dst = pre_dst.get();
        sj.src = pre_src.get();
        launch::chol_extend_add(op.count, op.nb0, t, b0front.get() + op.b0, b0child.get(), fd.get(), children.get(),
                                relmap.get(), jtab.get(), cmptr.get(),
                                cment.get(), colptr.get(), ent_row.get(), ent_src.get(), vals, lam, fronts.get(),
                                vecs.get(), lbuf.get(), y_p.get(), linv.get(), xinv.get(), fail,
                                op.kind == 0 ? 0 : op.kind == 5 ? 2 : op.kind == 9 ? 3 : 1, s, &sj);
        break;
      }
      case 2:
      case 6: {
        launch::StepHead h = heads[&op - ops.data()];
        if (h.sc1 > h.sc0) {  // this launch also scatters a later level's input entries (setup: deferred scatter)
          h.sc_vals = vals;
          h.sc_dst = pre_dst.get();
          h.sc_src = pre_src.get();
          h.sc_lam = lam;
        }
        launch::chol_step(op.count, step_tasks.get() + op.off, h, fronts.get(), lbuf.get(), vecs.get(), y_p.get(),
                          linv.get(), xinv.get(), fail, op.kind == 6, s);
        break;
      }
      case 8: {  // subtree roots -> every rank
        const long long* R = xch_ranges.get();
        launch::chol_copy_ranges(xch_pack_f, R, fronts.get(), xch_buf.get(), s);
        launch::chol_copy_ranges(xch_pack_v, R + 3LL * xch_pack_f, vecs.get(), xch_buf.get(), s);
        allgather(xch_buf.get(), (size_t)xch_seg);
        launch::chol_copy_ranges(xch_unpack_f, R + 3LL * (xch_pack_f + xch_pack_v), xch_buf.get(), fronts.get(), s);
        launch::chol_copy_ranges(xch_unpack_v, R + 3LL * (xch_pack_f + xch_pack_v + xch_unpack_f), xch_buf.get(),
                                 vecs.get(), s);
        break;
      }
      case 11: launch::chol_xdiag(op.count, t, fd.get(), linv.get(), xinv.get(), s); break;
      case 12: launch::chol_l21(op.count, t, fd.get(), fronts.get(), xinv.get(), lbuf.get(), s); break;
      default: launch::chol_syrk(syrk_var, op.count, t, fd.get(), fronts.get(), lbuf.get(), y_p.get(), vecs.get(), s); break;
    }
  }
}

void DeviceCholesky::reduce_input(const double* vals, hipStream_t s) {
  launch::chol_pack_blocks(rs_nblk, pd * pd, rs_bmap.get(), vals, rs_buf.get(), s);
  launch::chol_copy_ranges(1, rs_rhs_rng.get(), vals, rs_buf.get(), s);
  if (rs_seg > 0) reduce_scatter(rs_buf.get(), (size_t)rs_seg);  // rs_seg is the same on every rank
  allreduce(rs_buf.get() + (size_t)dist_nranks * rs_seg, (size_t)rs_tail_len);
}

void DeviceCholesky::solve(double* x, hipStream_t s) {
  // distributed: every rank solves the shared top and its own subtrees into a zeroed buffer, rank 0 alone keeps the
  // shared columns, and one all-reduce (with the not-PD flag in its last entry) gives every rank the whole x
  double* xo = x;
  if (distributed()) {
    xo = xred.get();
    xred.zero(s);
  }
  for (size_t l = bwd_ops.size(); l-- > 0;) {  // the forward plan in reverse (root level first)
    const BwdLevel& bl = bwd_ops[l];
    launch::chol_bwd_gemv(bl.gemv.second, tasks.get() + bl.gemv.first, fd.get(), rows.get(), lbuf.get(), y_p.get(),
                          x_p.get(), t_p.get(), s);
    launch::chol_bwd_x(bl.xall.second, tasks.get() + bl.xall.first, fd.get(), xinv.get(), linv.get(), bl.t_is_y ? y_p.get() : t_p.get(),
                       x_p.get(), perm.get(), xo, s);
    for (const auto& rd : bl.rounds) {
      launch::chol_bwd_inner(rd.first.second, tasks.get() + rd.first.first, fd.get(), lbuf.get(), x_p.get(), t_p.get(), s);
      launch::chol_bwd_x(rd.second.second, tasks.get() + rd.second.first, fd.get(), xinv.get(), linv.get(), t_p.get(), x_p.get(),
                         perm.get(), xo, s);
    }
  }
  if (distributed()) {
    if (dist_rank != 0) launch::chol_zero_idx(xzero_idx.get(), nxzero, xo, s);
    launch::chol_dist_fail_in(last_fail, xo, sym.n, s);
    allreduce(xo, (size_t)sym.n + 1);
    launch::chol_dist_x_out(xo, sym.n, x, last_fail, s);
  }
}

void DeviceCholesky::solve_multi(double* Y, double* W, double* T, int K, hipStream_t s) {
  if (K < 1 || K > 64) throw std::runtime_error("solve_multi: K must be in [1, 64]");
  for (size_t l = 0; l + 1 < level_off.size(); ++l)
    launch::marg_forward(level_off[l + 1] - level_off[l], lfronts.get() + level_off[l], fd.get(), children.get(),
                         relmap.get(), lbuf.get(), linv.get(), woff.get(), W, Y, T, sym.n, K, s);
  for (size_t l = level_off.size() - 1; l-- > 0;)
    launch::marg_backward(level_off[l + 1] - level_off[l], lfronts.get() + level_off[l], fd.get(), rows.get(),
                          lbuf.get(), linv.get(), Y, T, sym.n, K, s);
}

// ------------------------------------------------------------------ Engine: graph
Engine::Engine(int dev) : device(dev) {
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  // [0] lambda [1] chi2 [2] scale [3] maxdiag [4] lambda (rank 0) [5] 0 | [8] fail flags (two ints) | [12] next lambda
  // [13] next lambda (rank 0) [14] accepted [15] rho (lm_decide)
  dscal.resize(16);
  dscal.zero(stream);
  for (auto& e : ev_) HIP_CHECK(hipEventCreateWithFlags(&e, timing_event_flags()));
  for (auto& e : lm_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, timing_event_flags()));
  HIP_CHECK(hipEventCreateWithFlags(&rb_ev_, hipEventDisableTiming));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hscal_), 16 * sizeof(double), hipHostMallocDefault));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hdec_), 16 * sizeof(double),
                          hipHostMallocMapped | hipHostMallocCoherent));
  HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hdec_dev_), hdec_, 0));
}
Engine::~Engine() {
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
  for (auto& e : lm_ev_) if (e) (void)hipEventDestroy(e);
  if (rb_ev_) (void)hipEventDestroy(rb_ev_);
  if (hscal_) (void)hipHostFree(hscal_);
  if (hdec_) (void)hipHostFree(hdec_);
  comm.reset();
  if (stream) (void)hipStreamDestroy(stream);
}

int Engine::add_vertices(int type, int n, const int* ids, const double* est, const int* fixed, const int* marg) {
  if (vertex_dim(type) < 0 || n < 0) return G2OHIP_ERR_ARG;
  sync_host_state();  // the appended states are uploaded with the rest: the optimized ones must be current here
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
  if (type == G2OHIP_E_SE3_PROJECT_XYZ && !params) return G2OHIP_ERR_ARG;
  const int nm = edge_meas_dim(type);
  if (nm > 0 && !meas && n > 0) return G2OHIP_ERR_ARG;
  for (int k = 0; k < n; ++k)
    if (!hg.idmap.count(v0[k]) || !hg.idmap.count(v1[k])) return G2OHIP_ERR_ARG;
  HEdgeSet* es = hg.set_of(type);
  if (!es) {
    hg.esets.emplace_back();
    es = &hg.esets.back();
    es->type = type;
    es->D = D;
    es->nm = nm;
  }
  for (int k = 0; k < n; ++k) {
    es->ev0.push_back(hg.idmap[v0[k]]);
    es->ev1.push_back(hg.idmap[v1[k]]);
  }
  if (nm > 0) es->meas.insert(es->meas.end(), meas, meas + (size_t)n * nm);
  es->info.insert(es->info.end(), info, info + (size_t)n * D * D);
  if (type == G2OHIP_E_SE3_PROJECT_XYZ) es->params.insert(es->params.end(), params, params + (size_t)n * 4);
  es->payload.clear();
  initialized = false;
  return G2OHIP_OK;
}

int Engine::set_robust_kernel(int type, int kind, double delta) {
  HEdgeSet* es = hg.set_of(type);
  if (!es || kind < G2OHIP_RK_NONE || kind > G2OHIP_RK_DCS || !(delta > 0)) return G2OHIP_ERR_ARG;
  es->rk = kind;
  es->rk_delta = delta;
  ++state_ver;  // the robust chi2 of the same state changes
  return G2OHIP_OK;
}

int Engine::set_host_payload(int type, const double* payload) {
  HEdgeSet* es = hg.set_of(type);
  if (!es || !is_hostj(type) || !payload) return G2OHIP_ERR_ARG;
  std::vector<int> dims(es->ev0.size() * 2);
  size_t len = 0;
  for (size_t k = 0; k < es->ev0.size(); ++k)
    len += (size_t)es->D * (1 + hg.verts[es->ev0[k]].dim + hg.verts[es->ev1[k]].dim);
  es->payload.assign(payload, payload + len);
  es->payload_ver = 0;  // caller-provided: used as is
  if (initialized && edges_ready) {
    for (auto& g : groups)
      if (g.set == (int)(es - hg.esets.data())) {
        // gather the group's edges (the host payload has per-edge strides of the edge's own dims; a group has
        // one (DA, DB), so offsets come from a prefix over the set)
        std::vector<size_t> off(es->ev0.size() + 1, 0);
        for (size_t k = 0; k < es->ev0.size(); ++k)
          off[k + 1] = off[k] + (size_t)es->D * (1 + hg.verts[es->ev0[k]].dim + hg.verts[es->ev1[k]].dim);
        const int P = g.payload_stride();
        std::vector<double> buf((size_t)std::max(g.ne, 1) * P);
        for (int k = 0; k < g.ne; ++k)
          std::memcpy(buf.data() + (size_t)k * P, es->payload.data() + off[g.edges[k]], sizeof(double) * P);
        g.meas.upload(buf, stream);
      }
    ++state_ver;  // errors (chi2) of the host-J edges changed
  }
  return G2OHIP_OK;
}

int Engine::set_host_callback(g2ohip_host_edge_fn fn, void* user) {
  host_fn = fn;
  host_user = user;
  return G2OHIP_OK;
}

// OptimizableGraph::load (optimizable_graph.cpp:397-661) for the tags on this path, parsed in parallel: the file
// is read once, cut into line-aligned chunks, each chunk parsed by its own thread (strtod/strtol, no streams)
// into typed records, and the records added in file order with batched add_vertices / add_edges. Unknown tags
// are skipped with one warning per tag (:455-460); FIX lines fix vertices after loading (:409-417).
namespace {
struct ParsedVertex { int type, id; double est[7]; };
struct ParsedEdge { int type, a, b; double m[7], info[36], p[4]; };
struct ParsedChunk {
  std::vector<ParsedVertex> verts;
  std::vector<ParsedEdge> edges;
  std::vector<int> fix;
  std::vector<std::string> unknown;
  bool bad = false;
};
struct Cursor {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p; }
  double d() {
    ws();
    char* end = nullptr;
    const double v = std::strtod(p, &end);
    if (end == p || end > e) { ok = false; return 0; }
    p = end;
    return v;
  }
  int i() {
    ws();
    char* end = nullptr;
    const long v = std::strtol(p, &end, 10);
    if (end == p || end > e) { ok = false; return 0; }
    p = end;
    return (int)v;
  }
  bool more() { ws(); return p < e; }
};
void parse_chunk(const char* b, const char* e, ParsedChunk& out) {
  while (b < e) {
    const char* nl = static_cast<const char*>(std::memchr(b, '\n', (size_t)(e - b)));
    const char* le = nl ? nl : e;
    Cursor c{b, le};
    c.ws();
    const char* t0 = c.p;
    while (c.p < le && *c.p != ' ' && *c.p != '\t' && *c.p != '\r') ++c.p;
    const std::string tag(t0, c.p);
    b = nl ? nl + 1 : e;
    if (tag.empty() || tag[0] == '#') continue;
    if (tag == "VERTEX_SE3:EXPMAP" || tag == "VERTEX_SE3:QUAT") {
      ParsedVertex v{tag == "VERTEX_SE3:EXPMAP" ? G2OHIP_V_SE3_EXPMAP : G2OHIP_V_SE3_QUAT, c.i(), {}};
      for (double& x : v.est) x = c.d();
      if (v.type == G2OHIP_V_SE3_EXPMAP) {  // the file holds cam2world (types_six_dof_expmap.cpp:93-101)
        double w[7];
        se3quat_inverse(v.est, w);
        std::memcpy(v.est, w, sizeof w);
      }
      out.verts.push_back(v);
    } else if (tag == "VERTEX_XYZ" || tag == "VERTEX_SE2") {
      ParsedVertex v{tag == "VERTEX_XYZ" ? G2OHIP_V_XYZ : G2OHIP_V_SE2, c.i(), {}};
      for (int k = 0; k < 3; ++k) v.est[k] = c.d();
      out.verts.push_back(v);
    } else if (tag == "VERTEX_XY") {  // vertex_point_xy.cpp:46-50
      ParsedVertex v{G2OHIP_V_XY, c.i(), {}};
      for (int k = 0; k < 2; ++k) v.est[k] = c.d();
      out.verts.push_back(v);
    } else if (tag == "FIX") {
      while (c.more()) {
        const int id = c.i();
        if (!c.ok) break;
        out.fix.push_back(id);
      }
      c.ok = true;
    } else if (tag == "EDGE_SE3_PROJECT_XYZ:EXPMAP") {  // types_six_dof_expmap.cpp:363-378
      ParsedEdge ed{G2OHIP_E_SE3_PROJECT_XYZ, c.i(), c.i(), {}, {}, {}};
      ed.m[0] = c.d(); ed.m[1] = c.d();
      const double o0 = c.d(), o1 = c.d(), o2 = c.d();
      ed.info[0] = o0; ed.info[1] = o1; ed.info[2] = o1; ed.info[3] = o2;
      for (double& x : ed.p) x = c.d();
      out.edges.push_back(ed);
    } else if (tag == "EDGE_SE2_XY") {  // edge_se2_pointxy.cpp:46-52
      ParsedEdge ed{G2OHIP_E_SE2_XY, c.i(), c.i(), {}, {}, {}};
      ed.m[0] = c.d(); ed.m[1] = c.d();
      const double o0 = c.d(), o1 = c.d(), o2 = c.d();
      ed.info[0] = o0; ed.info[1] = o1; ed.info[2] = o1; ed.info[3] = o2;
      out.edges.push_back(ed);
    } else if (tag == "EDGE_SE3:QUAT" || tag == "EDGE_SE2") {  // edge_se3.cpp:42-65, edge_se2.cpp:41-53
      const bool se3 = tag == "EDGE_SE3:QUAT";
      const int D = se3 ? 6 : 3, nm = se3 ? 7 : 3;
      ParsedEdge ed{se3 ? G2OHIP_E_SE3_QUAT : G2OHIP_E_SE2, c.i(), c.i(), {}, {}, {}};
      for (int k = 0; k < nm; ++k) ed.m[k] = c.d();
      for (int r = 0; r < D; ++r)
        for (int q = r; q < D; ++q) ed.info[r * D + q] = ed.info[q * D + r] = c.d();
      out.edges.push_back(ed);
    } else {
      if (std::find(out.unknown.begin(), out.unknown.end(), tag) == out.unknown.end()) out.unknown.push_back(tag);
      continue;
    }
    if (!c.ok) { out.bad = true; return; }
  }
}
}  // namespace

int Engine::load(const char* path, int marginalize_xyz) {
  FILE* f = fopen(path, "rb");
  if (!f) return G2OHIP_ERR_ARG;
  std::vector<char> buf;
  {
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    // one byte more than the file, NUL: strtod / strtol stop there even on a last line without its newline
    buf.assign(sz > 0 ? (size_t)sz + 1 : 1, '\0');
    const size_t got = sz > 0 ? std::fread(buf.data(), 1, (size_t)sz, f) : 0;
    fclose(f);
    if (got + 1 != buf.size()) return G2OHIP_ERR_ARG;
  }
  const char* base = buf.data();
  const size_t n = buf.size() - 1;
  const int nthreads = (int)std::max<size_t>(1, std::min<size_t>(16, n / (1 << 20)));
  std::vector<size_t> cut(nthreads + 1, n);
  cut[0] = 0;
  for (int t = 1; t < nthreads; ++t) {
    size_t c = std::max(cut[t - 1], n * t / nthreads);
    while (c < n && base[c - 1] != '\n') ++c;
    cut[t] = c;
  }
  std::vector<ParsedChunk> chunks(nthreads);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
      th.emplace_back([&, t] { parse_chunk(base + cut[t], base + cut[t + 1], chunks[t]); });
    for (auto& x : th) x.join();
  }
  std::vector<std::string> warned;
  for (auto& c : chunks) {
    if (c.bad) return G2OHIP_ERR_ARG;
    for (auto& u : c.unknown)
      if (std::find(warned.begin(), warned.end(), u) == warned.end()) {
        warned.push_back(u);
        fprintf(stderr, "g2o_hip load: unknown type %s (lines skipped)\n", u.c_str());
      }
  }
  // vertices in file order, batched per run of one type
  std::vector<int> ids, fx, mg;
  std::vector<double> est;
  auto flush_v = [&](int type) -> int {
    if (ids.empty()) return G2OHIP_OK;
    const int r = add_vertices(type, (int)ids.size(), ids.data(), est.data(), fx.data(), mg.data());
    ids.clear(); est.clear(); fx.clear(); mg.clear();
    return r;
  };
  int cur = 0;
  for (auto& c : chunks)
    for (auto& v : c.verts) {
      if (v.type != cur) {
        if (int r = flush_v(cur)) return r;
        cur = v.type;
      }
      ids.push_back(v.id);
      est.insert(est.end(), v.est, v.est + vertex_est_dim(v.type));
      fx.push_back(0);
      mg.push_back((v.type == G2OHIP_V_XYZ || v.type == G2OHIP_V_XY) && marginalize_xyz ? 1 : 0);
    }
  if (int r = flush_v(cur)) return r;
  // edges in file order, batched per run of one type
  std::vector<int> ea, eb;
  std::vector<double> em, ei, ep;
  auto flush_e = [&](int type) -> int {
    if (ea.empty()) return G2OHIP_OK;
    const int r = add_edges(type, (int)ea.size(), ea.data(), eb.data(), em.data(), ei.data(),
                            type == G2OHIP_E_SE3_PROJECT_XYZ ? ep.data() : nullptr);
    ea.clear(); eb.clear(); em.clear(); ei.clear(); ep.clear();
    return r;
  };
  cur = 0;
  for (auto& c : chunks)
    for (auto& ed : c.edges) {
      if (ed.type != cur) {
        if (int r = flush_e(cur)) return r;
        cur = ed.type;
      }
      const int D = edge_dim(ed.type), nm = edge_meas_dim(ed.type);
      ea.push_back(ed.a);
      eb.push_back(ed.b);
      em.insert(em.end(), ed.m, ed.m + nm);
      ei.insert(ei.end(), ed.info, ed.info + D * D);
      if (ed.type == G2OHIP_E_SE3_PROJECT_XYZ) ep.insert(ep.end(), ed.p, ed.p + 4);
    }
  if (int r = flush_e(cur)) return r;
  for (auto& c : chunks)
    for (int id : c.fix) {
      auto it = hg.idmap.find(id);
      if (it != hg.idmap.end()) hg.verts[it->second].fixed = true;
    }
  return G2OHIP_OK;
}

// OptimizableGraph::save (optimizable_graph.cpp:663-679): vertices in insertion order (each followed by its FIX line),
// then the edges of every type. The lines are formatted in parallel — contiguous ranges of vertices / edges per thread,
// std::to_chars shortest round-trip decimals (the value read back is bit-identical) — and written in order.
namespace {
struct LineBuf {
  std::string s;
  char tmp[64];
  void tag(const char* t) { s += t; }
  void i(int v) {
    s += ' ';
    const auto r = std::to_chars(tmp, tmp + sizeof tmp, v);
    s.append(tmp, r.ptr);
  }
  void d(double v) {
    s += ' ';
    const auto r = std::to_chars(tmp, tmp + sizeof tmp, v);
    s.append(tmp, r.ptr);
  }
  void nl() { s += '\n'; }
};
template <class F>
void parallel_ranges(size_t n, int nthreads, F&& f) {
  if (nthreads <= 1 || n < 4096) { f(0, 0, n); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back([&, t] { f(t, n * t / nthreads, n * (t + 1) / nthreads); });
  for (auto& x : th) x.join();
}
}  // namespace

int Engine::save(const char* path) {
  sync_host_state();
  FILE* f = fopen(path, "wb");
  if (!f) return G2OHIP_ERR_ARG;
  const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<LineBuf> out(nt);
  bool ok = true;
  auto flush = [&] {
    for (auto& o : out) {
      if (!o.s.empty() && std::fwrite(o.s.data(), 1, o.s.size(), f) != o.s.size()) ok = false;
      o.s.clear();
    }
  };
  parallel_ranges(hg.verts.size(), nt, [&](int t, size_t lo, size_t hi) {
    LineBuf& L = out[t];
    L.s.reserve((hi - lo) * 96);
    for (size_t k = lo; k < hi; ++k) {
      const HVertex& v = hg.verts[k];
      const double* st = hg.st[v.type].data() + (size_t)v.local * vertex_state_stride(v.type);
      double e[7], c[7];
      est_from_state(v.type, st, e);
      int ne = 3;
      switch (v.type) {
        case G2OHIP_V_SE3_EXPMAP: L.tag("VERTEX_SE3:EXPMAP"); se3quat_inverse(e, c); std::memcpy(e, c, sizeof c); ne = 7; break;
        case G2OHIP_V_XYZ: L.tag("VERTEX_XYZ"); break;
        case G2OHIP_V_SE3_QUAT: L.tag("VERTEX_SE3:QUAT"); ne = 7; break;
        case G2OHIP_V_SE2: L.tag("VERTEX_SE2"); break;
        case G2OHIP_V_XY: L.tag("VERTEX_XY"); ne = 2; break;
      }
      L.i(v.id);
      for (int q = 0; q < ne; ++q) L.d(e[q]);
      L.nl();
      if (v.fixed) { L.tag("FIX"); L.i(v.id); L.nl(); }
    }
  });
  flush();
  for (const HEdgeSet& es : hg.esets) {
    if (is_hostj(es.type)) {  // the device does not know the host type's tag: the host saves those edges
      fprintf(stderr, "g2o_hip save: %zu host-Jacobian edges (type %d) not written\n", es.ev0.size(), es.type);
      continue;
    }
    const int D = es.D, nm = es.nm;
    parallel_ranges(es.ev0.size(), nt, [&](int t, size_t lo, size_t hi) {
      LineBuf& L = out[t];
      L.s.reserve((hi - lo) * 200);
      for (size_t k = lo; k < hi; ++k) {
        const int a = hg.verts[es.ev0[k]].id, b = hg.verts[es.ev1[k]].id;
        const double* m = es.meas.data() + k * nm;
        const double* I = es.info.data() + k * D * D;
        if (es.type == G2OHIP_E_SE2_XY) {  // edge_se2_pointxy.cpp:54-61
          L.tag("EDGE_SE2_XY"); L.i(a); L.i(b);
          L.d(m[0]); L.d(m[1]); L.d(I[0]); L.d(I[1]); L.d(I[3]);
        } else if (es.type == G2OHIP_E_SE3_PROJECT_XYZ) {  // types_six_dof_expmap.cpp:380-393
          const double* p = es.params.data() + k * 4;
          L.tag("EDGE_SE3_PROJECT_XYZ:EXPMAP"); L.i(a); L.i(b);
          L.d(m[0]); L.d(m[1]); L.d(I[0]); L.d(I[1]); L.d(I[3]);
          for (int q = 0; q < 4; ++q) L.d(p[q]);
        } else {  // edge_se3.cpp:67-75, edge_se2.cpp:55-63: measurement, upper triangle of the information row-wise
          L.tag(es.type == G2OHIP_E_SE3_QUAT ? "EDGE_SE3:QUAT" : "EDGE_SE2"); L.i(a); L.i(b);
          for (int q = 0; q < nm; ++q) L.d(m[q]);
          for (int r = 0; r < D; ++r) for (int q = r; q < D; ++q) L.d(I[r * D + q]);
        }
        L.nl();
      }
    });
    flush();
  }
  if (std::fclose(f) != 0) ok = false;
  return ok ? G2OHIP_OK : G2OHIP_ERR_ARG;
}

long long Engine::host_payload_len(int type) {
  HEdgeSet* es = hg.set_of(type);
  if (!es || !is_hostj(type)) return G2OHIP_ERR_ARG;
  long long len = 0;
  for (size_t k = 0; k < es->ev0.size(); ++k)
    len += (long long)es->D * (1 + hg.verts[es->ev0[k]].dim + hg.verts[es->ev1[k]].dim);
  return len;
}

// Octave sparse-matrix text of a symmetric matrix held as upper blocks (bi <= bj, pd x pd column-major): every entry of
// every stored block and the mirror of the off-diagonal ones, sorted by (column, row), 1-based
// (SparseBlockMatrix::writeOctave sparse_block_matrix.hpp:579-617; csparse_helper.cpp:62-111 for the debug dump,
// whose input is the upper CCS of fillCCS: diagonal blocks contribute their upper triangle, mirrored).
static bool write_octave_blocks(const char* path, const std::vector<int>& bi, const std::vector<int>& bj, int pd,
                                const double* blocks, int nb, double diag_add, bool upper_diag_only, bool fixed9) {
  struct Tr { int r, c; double x; };
  std::vector<Tr> ent;
  ent.reserve(bi.size() * pd * pd * 2);
  for (size_t t = 0; t < bi.size(); ++t) {
    const double* B = blocks + t * pd * pd;
    const bool dg = bi[t] == bj[t];
    for (int c = 0; c < pd; ++c)
      for (int r = 0; r < pd; ++r) {
        const int gr = bi[t] * pd + r, gc = bj[t] * pd + c;
        if (dg) {
          // symmetric diagonal block: the upper entry (min, max) as stored, both positions written
          const double x = B[std::max(r, c) * pd + std::min(r, c)] + (r == c ? diag_add : 0.0);
          if (upper_diag_only && r > c) continue;
          ent.push_back({gr, gc, x});
          if (upper_diag_only && r != c) ent.push_back({gc, gr, x});
        } else {
          ent.push_back({gr, gc, B[c * pd + r]});
          ent.push_back({gc, gr, B[c * pd + r]});
        }
      }
  }
  std::sort(ent.begin(), ent.end(), [](const Tr& a, const Tr& b) { return a.c < b.c || (a.c == b.c && a.r < b.r); });
  std::string name = path;
  const size_t dot = name.find_last_of('.');
  if (dot != std::string::npos) name = name.substr(0, dot);
  FILE* f = std::fopen(path, "w");
  if (!f) return false;
  const int n = nb * pd;
  std::fprintf(f, "# name: %s\n# type: sparse matrix\n# nnz: %zu\n# rows: %d\n# columns: %d\n\n", name.c_str(),
               ent.size(), n, n);
  for (const Tr& e : ent) std::fprintf(f, fixed9 ? "%d %d %.9f\n" : "%d %d %.9g\n", e.r + 1, e.c + 1, e.x);
  return std::fclose(f) == 0;
}

int Engine::save_hessian(const char* path) {
  if (!structure_built) return G2OHIP_ERR_STATE;
  if (nranks > 1) return G2OHIP_ERR_UNSUPPORTED;  // Hpp diagonal blocks are partial per landmark shard
  if (use_cgls()) return G2OHIP_ERR_UNSUPPORTED;  // JacobiSolver never assembles Hpp
  ensure_hpp();
  std::vector<double> blocks(hpp_bi.size() * pd * pd);
  dH.download(blocks.data(), blocks.size(), stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  // the reference's Hpp holds lambda between setLambda and restoreDiagonal; here lambda is virtual
  return write_octave_blocks(path, hpp_bi, hpp_bj, pd, blocks.data(), num_poses, lambda_set ? lambda_host : 0.0, false,
                             true)
             ? 1
             : 0;
}

void Engine::write_debug_dump() {
  // the matrix the failed factorization saw: S (lambda already on its diagonal) or Hpp + lambda
  const std::vector<int>& bi = do_schur ? s_bi : hpp_bi;
  const std::vector<int>& bj = do_schur ? s_bj : hpp_bj;
  std::vector<double> blocks(bi.size() * pd * pd);
  if (do_schur) dS.download(blocks.data(), blocks.size(), stream);
  else dH.download(blocks.data(), blocks.size(), stream);
  HIP_CHECK(hipStreamSynchronize(stream));
  fprintf(stderr, "Cholesky failure, writing %s (Hessian loadable by Octave)%s\n", debug_path.c_str(),
          chol.rs_on ? " — rank 0's partial sums (reduce-scattered S; set writeDebug before initializeOptimization)" : "");
  write_octave_blocks(debug_path.c_str(), bi, bj, pd, blocks.data(), num_poses, do_schur ? 0.0 : lambda_host, true,
                      false);
}

void Engine::ensure_device_state() {
  if (!device_state_dirty) return;
  for (int t = 1; t < NVT; ++t)
    if (!hg.st[t].empty()) dstate[t].upload(hg.st[t], stream);
  if (!hg.nopl.empty()) dnopl.upload(hg.nopl, stream);
  device_state_dirty = false;
  ++state_ver;
  host_state_stale = false;
}

void Engine::sync_host_state() {
  if (!host_state_stale) return;
  for (int t = 1; t < NVT; ++t)
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
// device family of an edge type (host-J types: any endpoint vertex types)
static int family_of(int etype, int& vtA, int& vtB) {
  switch (etype) {
    case G2OHIP_E_SE3_PROJECT_XYZ: vtA = G2OHIP_V_XYZ; vtB = G2OHIP_V_SE3_EXPMAP; return FAM_BA;
    case G2OHIP_E_SE3_QUAT: vtA = vtB = G2OHIP_V_SE3_QUAT; return FAM_SE3;
    case G2OHIP_E_SE2: vtA = vtB = G2OHIP_V_SE2; return FAM_SE2;
    case G2OHIP_E_SE2_XY: vtA = G2OHIP_V_SE2; vtB = G2OHIP_V_XY; return FAM_SE2XY;
  }
  vtA = vtB = 0;
  return is_hostj(etype) ? FAM_HOSTJ : FAM_NONE;
}

int Engine::initialize() {  // sparse_optimizer.cpp:201-279 + buildIndexMapping :168-192
  if (hg.num_edges() == 0) return G2OHIP_ERR_STATE;
  has_hostj = false;
  std::vector<char> has(hg.verts.size(), 0);
  for (const HEdgeSet& es : hg.esets) {
    int vtA, vtB;
    const int fam = family_of(es.type, vtA, vtB);
    if (fam == FAM_NONE) return G2OHIP_ERR_UNSUPPORTED;
    has_hostj |= fam == FAM_HOSTJ;
    for (size_t k = 0; k < es.ev0.size(); ++k) {
      const HVertex &a = hg.verts[es.ev0[k]], &b = hg.verts[es.ev1[k]];
      if (fam != FAM_HOSTJ && (a.type != vtA || b.type != vtB)) return G2OHIP_ERR_UNSUPPORTED;
      has[es.ev0[k]] = has[es.ev1[k]] = 1;
    }
  }
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
      if (pd && pd != v.dim) return G2OHIP_ERR_UNSUPPORTED;  // BlockSolver<p, l>: one pose block size
      pd = v.dim;
      ++num_poses;
    } else {
      if (ld && ld != v.dim) return G2OHIP_ERR_UNSUPPORTED;  // one landmark block size
      ld = v.dim;
      ++num_landmarks;
    }
  }
  if (num_poses == 0) return G2OHIP_ERR_UNSUPPORTED;
  size_poses = num_poses * pd;
  size_landmarks = num_landmarks * ld;
  do_schur = num_landmarks > 0;  // optimization_algorithm_with_hessian.cpp:48-73
  // the Schur kernels are instantiated for BlockSolver_6_3 and BlockSolver_3_2 (block_solver.h:188-201)
  if (do_schur && !((pd == 6 && ld == 3) || (pd == 3 && ld == 2))) return G2OHIP_ERR_UNSUPPORTED;
  // landmark-landmark edges have no place in BlockSolver's Schur layout here
  for (const HEdgeSet& es : hg.esets)
    for (size_t k = 0; k < es.ev0.size(); ++k) {
      const int a = hidx[es.ev0[k]], b = hidx[es.ev1[k]];
      if (a >= num_poses && b >= num_poses) return G2OHIP_ERR_UNSUPPORTED;
    }
  initialized = true;
  structure_built = false;
  edges_ready = false;
  return G2OHIP_OK;
}

// SparseOptimizer::updateInitialization (sparse_optimizer.cpp:465-502) + BlockSolver::updateStructure
// (block_solver.hpp:258-312). The vertices that gained edges since the last initialization join the running
// optimization behind the existing ones: each free one takes the next hessian index (the reference numbers the
// caller's vertex set in its iteration order; here the new vertices in id order), so the blocks of x, b, Hpp and the
// marginals of the vertices already there keep their places. The structure (pattern, symbolic factorization) is
// rebuilt on the next build, as the reference's updateStructure + LinearSolver::init do. Non-Schur only: the
// reference refuses marginalized vertices here ("Schur not supported", block_solver.hpp:274-277; abort in
// sparse_optimizer.cpp:491-492), this returns G2OHIP_ERR_UNSUPPORTED and leaves the graph's indexing unchanged.
int Engine::update_initialization() {
  if (ivmap.empty()) return G2OHIP_ERR_STATE;  // initializeOptimization first
  if (do_schur) return G2OHIP_ERR_UNSUPPORTED;
  std::vector<char> was(hg.verts.size(), 0), has(hg.verts.size(), 0);
  for (int vi : active) was[vi] = 1;
  bool hj = false;
  for (const HEdgeSet& es : hg.esets) {
    int vtA, vtB;
    const int fam = family_of(es.type, vtA, vtB);
    if (fam == FAM_NONE) return G2OHIP_ERR_UNSUPPORTED;
    hj |= fam == FAM_HOSTJ;
    for (size_t k = 0; k < es.ev0.size(); ++k) {
      const HVertex &a = hg.verts[es.ev0[k]], &b = hg.verts[es.ev1[k]];
      if (fam != FAM_HOSTJ && (a.type != vtA || b.type != vtB)) return G2OHIP_ERR_UNSUPPORTED;
      has[es.ev0[k]] = has[es.ev1[k]] = 1;
    }
  }
  std::vector<int> fresh;
  for (size_t k = 0; k < hg.verts.size(); ++k)
    if (has[k] && !was[k]) fresh.push_back((int)k);
  std::sort(fresh.begin(), fresh.end(), [&](int a, int b) { return hg.verts[a].id < hg.verts[b].id; });
  for (int vi : fresh) {
    const HVertex& v = hg.verts[vi];
    if (!v.fixed && (v.marg || v.dim != pd)) return G2OHIP_ERR_UNSUPPORTED;  // BlockSolver<p, l>: one pose size
  }
  hidx.resize(hg.verts.size(), -1);
  for (int vi : fresh) {
    active.push_back(vi);
    if (hg.verts[vi].fixed) continue;
    hidx[vi] = (int)ivmap.size();
    ivmap.push_back(vi);
    ++num_poses;
  }
  size_poses = num_poses * pd;
  has_hostj = hj;
  initialized = true;
  structure_built = false;
  edges_ready = false;
  return G2OHIP_OK;
}

EdgeArgs Engine::group_args(const EGroup& g) const {
  EdgeArgs a{g.v0.get(), g.v1.get(), g.meas.get(), g.info.get(), g.params.get(),
             g.vtA ? dstate[g.vtA].get() : nullptr, g.vtB ? dstate[g.vtB].get() : nullptr};
  a.rk = hg.esets[g.set].rk;
  a.rk_delta = hg.esets[g.set].rk_delta;
  a.D = g.D;
  a.DA = g.DA;
  a.DB = g.DB;
  a.ue = g.ue;
  return a;
}

// upload the host-J payload of one group (its local edges, gathered from the set's insertion-order payload)
static void upload_group_payload(const HostGraph& hg, EGroup& g, hipStream_t s) {
  const HEdgeSet& es = hg.esets[g.set];
  const int P = g.payload_stride();
  std::vector<double> buf((size_t)std::max(g.ne, 1) * P, 0.0);
  if (!es.payload.empty()) {
    std::vector<size_t> off(es.ev0.size() + 1, 0);
    for (size_t k = 0; k < es.ev0.size(); ++k)
      off[k + 1] = off[k] + (size_t)es.D * (1 + hg.verts[es.ev0[k]].dim + hg.verts[es.ev1[k]].dim);
    if (off.back() != es.payload.size()) throw std::runtime_error("host-J payload size does not match the edges");
    for (int k = 0; k < g.ne; ++k)
      std::memcpy(buf.data() + (size_t)k * P, es.payload.data() + off[g.edges[k]], sizeof(double) * P);
  }
  g.meas.upload(buf, s);
}

void Engine::refresh_host_payload(bool jacobians) {
  if (!has_hostj) return;
  for (size_t si = 0; si < hg.esets.size(); ++si) {
    HEdgeSet& es = hg.esets[si];
    if (!is_hostj(es.type)) continue;
    if (host_fn) {
      if (!jacobians && es.payload_ver == state_ver) continue;  // errors of this state already there
      sync_host_state();  // the callback reads the estimates the device holds
      size_t len = 0;
      for (size_t k = 0; k < es.ev0.size(); ++k)
        len += (size_t)es.D * (1 + hg.verts[es.ev0[k]].dim + hg.verts[es.ev1[k]].dim);
      es.payload.assign(len, 0.0);
      if (host_fn(host_user, es.type, jacobians ? 1 : 0, es.payload.data()) != 0)
        throw std::runtime_error("host edge callback failed for edge type " + std::to_string(es.type));
      es.payload_ver = state_ver;
    } else if (es.payload.empty()) {
      throw std::runtime_error("host-Jacobian edges (type " + std::to_string(es.type) +
                               ") need g2ohip_set_host_jacobians or a host edge callback");
    }
    for (auto& g : groups)
      if (g.set == (int)si) upload_group_payload(hg, g, stream);
  }
}

// the Kt records of nrec observations stay cache-resident between the linearize and camera passes (MALL)
static bool kx_records_cached(double nrec) { return nrec * 80.0 <= 192.0 * (1 << 20); }

void Engine::setup_edges_device() {
  // landmark shards: contiguous ranges of the hessian order, aligned with the factorization's cut (align_shards) or
  // the uniform split
  std::vector<int> bnd(nranks + 1);
  for (int r = 0; r <= nranks; ++r) bnd[r] = lm_bnd.empty() ? (int)((long long)num_landmarks * r / nranks) : lm_bnd[r];
  int lm_begin = 0, lm_end = num_landmarks;
  if (do_schur && nranks > 1) {
    lm_begin = bnd[rank];
    lm_end = bnd[rank + 1];
  }
  local_lm.clear();
  for (int l = lm_begin; l < lm_end; ++l) local_lm.push_back(l);
  // an edge belongs to the rank owning its landmark endpoint; edges without a (free) landmark are assembled by rank 0
  // once. Pose graphs run replicas: every rank assembles every edge.
  auto owner_of = [&](int va, int vb) {
    if (!(do_schur && nranks > 1)) return rank;
    const int h = hidx[va] >= num_poses ? hidx[va] : (hidx[vb] >= num_poses ? hidx[vb] : -1);
    if (h < 0) return 0;
    return (int)(std::upper_bound(bnd.begin(), bnd.end(), h - num_poses) - bnd.begin()) - 1;
  };
  groups.clear();
  ne = 0;
  for (size_t si = 0; si < hg.esets.size(); ++si) {
    const HEdgeSet& es = hg.esets[si];
    int vtA, vtB;
    const int fam = family_of(es.type, vtA, vtB);
    // groups: one per (endpoint vertex type pair) in first-seen order; device families have exactly one
    std::vector<std::pair<int, int>> keys;
    std::vector<std::vector<int>> lists;
    for (size_t k = 0; k < es.ev0.size(); ++k) {
      const int va = es.ev0[k], vb = es.ev1[k];
      if (owner_of(va, vb) != rank) continue;
      const std::pair<int, int> key{hg.verts[va].type, hg.verts[vb].type};
      size_t gi = std::find(keys.begin(), keys.end(), key) - keys.begin();
      if (gi == keys.size()) { keys.push_back(key); lists.emplace_back(); }
      lists[gi].push_back((int)k);
    }
    for (size_t gi = 0; gi < keys.size(); ++gi) {
      groups.emplace_back();
      EGroup& g = groups.back();
      g.set = (int)si;
      g.family = fam;
      g.vtA = keys[gi].first;
      g.vtB = keys[gi].second;
      g.D = es.D;
      g.DA = vertex_dim(g.vtA);
      g.DB = vertex_dim(g.vtB);
      g.edges = std::move(lists[gi]);
      g.ne = (int)g.edges.size();
      ne += g.ne;
    }
  }
  // fused BA assembly: the only edge group is BA and the Schur complement is formed (G2OHIP_ASM_FUSED=0 keeps the
  // generic slot path, for A/B checks)
  {
    const char* fz = getenv("G2OHIP_ASM_FUSED");
    ba_fused = do_schur && groups.size() == 1 && groups[0].family == FAM_BA && !(fz && atoi(fz) == 0);
  }
  if (ba_fused) {  // landmark-major edge order (stable: per landmark, the given order)
    EGroup& g = groups[0];
    const HEdgeSet& es = hg.esets[g.set];
    std::stable_sort(g.edges.begin(), g.edges.end(), [&](int a, int b) { return hidx[es.ev0[a]] < hidx[es.ev0[b]]; });
  }
  for (EGroup& g : groups) {
    const HEdgeSet& es = hg.esets[g.set];
    const int D = g.D, nm = es.nm, gne = g.ne;
    std::vector<int> v0(std::max(gne, 1), 0), v1(std::max(gne, 1), 0);
    const int minfo = D * (D + 1) / 2;
    const int mmeas = g.family == FAM_BA || g.family == FAM_SE2XY ? 2 : (g.family == FAM_SE3 ? 12 : (g.family == FAM_SE2 ? 3 : 0));
    std::vector<double> meas((size_t)std::max(gne, 1) * std::max(mmeas, 1)), info((size_t)std::max(gne, 1) * minfo),
        params(g.family == FAM_BA ? (size_t)gne * 4 : 1);
    for (int k = 0; k < gne; ++k) {
      const int e = g.edges[k];
      v0[k] = hg.verts[es.ev0[e]].local;
      v1[k] = hg.verts[es.ev1[e]].local;
      const double* m = es.meas.data() + (size_t)e * nm;
      double* mo = meas.data() + (size_t)k * mmeas;
      if (g.family == FAM_BA) {
        mo[0] = m[0]; mo[1] = m[1];
        for (int j = 0; j < 4; ++j) params[(size_t)k * 4 + j] = es.params[(size_t)e * 4 + j];
      } else if (g.family == FAM_SE3) {  // edge_se3.cpp:42-50: normalise q, Z = fromVectorQT, store Z^-1
        double q[4] = {m[3], m[4], m[5], m[6]};
        const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (double& x : q) x /= n;
        double Z[9];
        q2R(q[0], q[1], q[2], q[3], Z);
        double Rt[9] = {Z[0], Z[3], Z[6], Z[1], Z[4], Z[7], Z[2], Z[5], Z[8]};
        for (int j = 0; j < 9; ++j) mo[j] = Rt[j];
        for (int i = 0; i < 3; ++i) mo[9 + i] = -(Rt[i * 3] * m[0] + Rt[i * 3 + 1] * m[1] + Rt[i * 3 + 2] * m[2]);
      } else if (g.family == FAM_SE2) {  // edge_se2.cpp:41-47: inverse measurement
        const double th = norm_theta(-m[2]);
        const double c = std::cos(th), s = std::sin(th);
        mo[0] = c * (-m[0]) - s * (-m[1]);
        mo[1] = s * (-m[0]) + c * (-m[1]);
        mo[2] = th;
      } else if (g.family == FAM_SE2XY) {
        mo[0] = m[0]; mo[1] = m[1];
      }
      const double* I = es.info.data() + (size_t)e * D * D;
      double* io = info.data() + (size_t)k * minfo;
      int q = 0;
      for (int c = 0; c < D; ++c)
        for (int r = 0; r <= c; ++r) io[q++] = I[r * D + c];
    }
    g.v0.upload(v0, stream);
    g.v1.upload(v1, stream);
    {  // BA: edges sharing one information matrix / one set of intrinsics (the usual monocular case) read a single
       // record instead of 24 + 32 bytes per edge (G2OHIP_UNIFORM_RECORDS=0 keeps per-edge records, A/B)
      const char* ev = getenv("G2OHIP_UNIFORM_RECORDS");
      g.ue = 0;
      if (g.family == FAM_BA && gne > 1 && !(ev && atoi(ev) == 0)) {
        auto uniform = [&](const std::vector<double>& v, int st) {
          for (int k = 1; k < gne; ++k)
            if (std::memcmp(v.data() + (size_t)k * st, v.data(), sizeof(double) * st) != 0) return false;
          return true;
        };
        if (uniform(info, minfo)) { g.ue |= 1; info.resize(minfo); }
        if (uniform(params, 4)) { g.ue |= 2; params.resize(4); }
      }
    }
    g.info.upload(info, stream);
    g.params.upload(params, stream);
    if (g.family == FAM_HOSTJ) upload_group_payload(hg, g, stream);
    else g.meas.upload(meas, stream);
  }
  if (ba_fused) {
    const EGroup& g = groups[0];
    const HEdgeSet& es = hg.esets[g.set];
    // wave chunks of whole landmarks (<= 64 edges); a landmark with more observations gets chunks of its own
    // whose partial sums k_lm_fixup adds
    std::vector<int4> chunks, fix;
    int npart = 0;
    int cb = 0, cn = 0;
    auto close = [&]() {
      if (cn) chunks.push_back(int4{cb, cn, -1, 0});
      cn = 0;
    };
    for (int k = 0; k < g.ne;) {
      int k2 = k + 1;
      while (k2 < g.ne && es.ev0[g.edges[k2]] == es.ev0[g.edges[k]]) ++k2;
      const int len = k2 - k;
      if (len <= 64) {
        if (cn + len > 64) close();
        if (!cn) cb = k;
        cn += len;
      } else {
        close();
        const int h = hidx[es.ev0[g.edges[k]]];
        const int p0 = npart;
        for (int a = k; a < k2; a += 64) chunks.push_back(int4{a, std::min(64, k2 - a), npart++, 0});
        if (h >= 0) fix.push_back(int4{h, p0, npart - p0, 0});
      }
      k = k2;
    }
    close();
    fz_nchunks = (int)chunks.size();
    fz_nfix = (int)fix.size();
    fz_chunks.upload(chunks.empty() ? std::vector<int4>{int4{0, 0, -1, 0}} : chunks, stream);
    fz_fix.upload(fix.empty() ? std::vector<int4>{int4{0, 0, 0, 0}} : fix, stream);
    fz_lpart.resize((size_t)std::max(npart, 1) * 9);
    // camera-major copy of the observations of every free camera. Edge order within a camera (G2OHIP_CAM_ORDER, dev
    // A/B): 1 (default for the re-linearising camera pass) by the landmark's first observing camera, then landmark-major — neighbouring cameras, which run
    // side by side on one XCD, then sweep their landmarks in step and re-read them from that L2 (a landmark's observers
    // lie in one window of cameras, its id anywhere); 0 landmark-major (the gathers of U, c and the point then land
    // on lines no other in-flight camera touches soon; C5 camera pass 0.407-0.409 -> 0.374-0.376 ms, L2 hit rate 62 %
    // before, profiles/r06_ab_camorder_c5.log, r06_pmc_c5_l2.csv)
    std::vector<std::vector<int>> lists(num_poses);
    for (int k = 0; k < g.ne; ++k) {
      const int h = hidx[es.ev1[g.edges[k]]];
      if (h >= 0 && h < num_poses) lists[h].push_back(k);
    }
    {
      // (only where the camera pass re-linearises from the per-landmark data: the records path gathers the 80-byte
      // records in camera order, which the landmark-major order keeps ascending; C4 0.047 vs 0.048-0.049 ms)
      const char* co = getenv("G2OHIP_CAM_ORDER");
      const int cam_order = co ? atoi(co) : (kx_records_cached((double)g.ne) ? 0 : 1);
      if (cam_order != 0) {
        std::vector<int> first(g.ne, INT_MAX);  // per edge: its landmark's first free observing camera
        for (int k = 0; k < g.ne;) {           // the group is landmark-major: one run of edges per landmark
          int k2 = k, mc = INT_MAX;
          const int v = es.ev0[g.edges[k]];
          while (k2 < g.ne && es.ev0[g.edges[k2]] == v) {
            const int h = hidx[es.ev1[g.edges[k2]]];
            if (h >= 0 && h < num_poses) mc = std::min(mc, h);
            ++k2;
          }
          for (int j = k; j < k2; ++j) first[j] = mc;
          k = k2;
        }
        for (auto& L : lists)
          std::stable_sort(L.begin(), L.end(), [&](int x, int y) { return first[x] < first[y]; });
      }
    }
    std::vector<int> ptr(num_poses + 1, 0), cv0, cv1;
    std::vector<double> cmeas, cinfo, cpar;
    cm_e_h.clear();
    for (int i = 0; i < num_poses; ++i) {
      ptr[i + 1] = ptr[i] + (int)lists[i].size();
      for (int k : lists[i]) {
        cm_e_h.push_back(k);
        const int e = g.edges[k];
        cv0.push_back(hg.verts[es.ev0[e]].local);
        cv1.push_back(hg.verts[es.ev1[e]].local);
        cmeas.push_back(es.meas[(size_t)e * 2]);
        cmeas.push_back(es.meas[(size_t)e * 2 + 1]);
        const double* I = es.info.data() + (size_t)e * 4;
        cinfo.push_back(I[0]);  // packed upper, column-major: (0,0) (0,1) (1,1)
        cinfo.push_back(I[1]);
        cinfo.push_back(I[3]);
        for (int j = 0; j < 4; ++j) cpar.push_back(es.params[(size_t)e * 4 + j]);
      }
    }
    auto nz_i = [](std::vector<int>& v) -> std::vector<int>& { if (v.empty()) v.push_back(0); return v; };
    auto nz_d = [](std::vector<double>& v) -> std::vector<double>& { if (v.empty()) v.assign(4, 0.0); return v; };
    cm_ptr_h = ptr;
    {  // per local landmark its edge range in the (landmark-major) group order
      const int lm_b = local_lm.empty() ? 0 : local_lm.front();
      lm_eptr_h.assign(local_lm.size() + 1, 0);
      std::vector<int2> erng(std::max<size_t>(local_lm.size(), 1), int2{0, 0});
      std::vector<char> seen(local_lm.size(), 0);
      for (int k = 0; k < g.ne; ++k) {
        const int h = hidx[es.ev0[g.edges[k]]];
        if (h < num_poses) continue;
        const int l = h - num_poses - lm_b;
        lm_eptr_h[l + 1]++;
        if (!seen[l]) { seen[l] = 1; erng[l].x = k; }
        erng[l].y = k + 1;  // contiguous: the group is sorted landmark-major
      }
      for (size_t l = 0; l < local_lm.size(); ++l) lm_eptr_h[l + 1] += lm_eptr_h[l];
      d_bs_erng.upload(erng, stream);
    }
    cm_ptr.upload(ptr, stream);
    cm_v0.upload(nz_i(cv0), stream);
    cm_v1.upload(nz_i(cv1), stream);
    cm_meas.upload(nz_d(cmeas), stream);
    if ((g.ue & 1) && cinfo.size() > 3) cinfo.resize(3);  // the shared record (see the group's upload)
    if ((g.ue & 2) && cpar.size() > 4) cpar.resize(4);
    cm_info.upload(nz_d(cinfo), stream);
    cm_params.upload(nz_d(cpar), stream);
  }
  long long maxp = std::max<long long>(vector_size(), 1);
  long long ptot = 0;
  for (auto& g : groups) ptot += (long long)launch::sum_partials(std::max(g.ne, 1));
  dpartial.resize(std::max<size_t>(launch::sum_partials(maxp) + (size_t)ptot + 64, 128));  // chi2 + scale partials
  edges_ready = true;
  ++state_ver;  // the edge set (and so chi2) changed
}

// Upper block pattern (i <= j, row-major, sorted) of the reduced camera system from ALL edges (identical on every
// rank whatever its shard): the diagonal, pose-pose edges and the pose clique of every free landmark
// (block_solver.hpp:216-251).
void Engine::schur_pattern(std::vector<int>& sbi, std::vector<int>& sbj, std::vector<int>& srow_ptr) const {
  std::vector<std::vector<int>> lmposes(num_landmarks);
  std::vector<std::vector<int>> rowcols(num_poses);
  for (int i = 0; i < num_poses; ++i) rowcols[i].push_back(i);
  for (const HEdgeSet& es : hg.esets)
    for (size_t e = 0; e < es.ev0.size(); ++e) {
      const int i1 = hidx[es.ev0[e]], i2 = hidx[es.ev1[e]];
      if (i1 < 0 || i2 < 0) continue;
      if (i1 >= num_poses && i2 < num_poses) lmposes[i1 - num_poses].push_back(i2);
      else if (i2 >= num_poses && i1 < num_poses) lmposes[i2 - num_poses].push_back(i1);
      else if (i1 < num_poses && i2 < num_poses) rowcols[std::min(i1, i2)].push_back(std::max(i1, i2));
    }
  for (auto& ps : lmposes) {
    std::sort(ps.begin(), ps.end());
    ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
    for (size_t u = 0; u < ps.size(); ++u)
      for (size_t v = u; v < ps.size(); ++v) rowcols[ps[u]].push_back(ps[v]);
  }
  srow_ptr.assign(num_poses + 1, 0);
  sbi.clear();
  sbj.clear();
  for (int i = 0; i < num_poses; ++i) {
    auto& rc = rowcols[i];
    std::sort(rc.begin(), rc.end());
    rc.erase(std::unique(rc.begin(), rc.end()), rc.end());
    for (int j : rc) { sbi.push_back(i); sbj.push_back(j); }
    srow_ptr[i + 1] = (int)sbi.size();
  }
}

// Per pose: the landmark-sharded work that follows it in the cut's model (its observations of free landmarks).
std::vector<double> Engine::pose_work() const {
  std::vector<double> w(num_poses, 0.0);
  for (const HEdgeSet& es : hg.esets)
    for (size_t e = 0; e < es.ev0.size(); ++e) {
      const int i1 = hidx[es.ev0[e]], i2 = hidx[es.ev1[e]];
      if (i1 >= num_poses && i2 >= 0 && i2 < num_poses) w[i2] += dist_cost::OBS_S;
      else if (i2 >= num_poses && i1 >= 0 && i1 < num_poses) w[i1] += dist_cost::OBS_S;
    }
  return w;
}

// Landmark shards aligned with the distributed factorization's cut. With landmark sharding and a cut
// the model takes (plan_distribution with aligned input: the same plan DeviceCholesky::setup will make), every
// landmark goes to the rank whose subtrees its Schur blocks land in (align_landmarks), and the landmarks' hessian order
// is regrouped by rank (stable within a rank), so every shard is one contiguous range [lm_bnd[r], lm_bnd[r+1]). A
// rank's subtree blocks of S are then complete on that rank (lambda on their diagonal included: lam_own); only the
// shared blocks and the rhs are exchanged. G2OHIP_DIST_ALIGN=0 keeps the uniform split of the landmark order.
void Engine::align_shards() {
  lm_bnd.clear();
  dist_aligned = false;
  al_bpinv.clear();
  al_bowner.clear();
  al_sym.reset();
  al_plan.reset();
  al_sbi.clear();
  al_sbj.clear();
  // the hessian order buildIndexMapping gives (initialize): poses, then the free landmarks in id order
  ivmap.resize(num_poses);
  for (int vi : active) {
    const HVertex& v = hg.verts[vi];
    if (!v.fixed && v.marg) {
      hidx[vi] = (int)ivmap.size();
      ivmap.push_back(vi);
    }
  }
  if (!(do_schur && nranks > 1 && comm) || use_pcg() || use_cgls() || write_debug) return;
  auto env0 = [](const char* n) { const char* e = getenv(n); return e && atoi(e) == 0; };
  if (env0("G2OHIP_DIST_FACTOR") || env0("G2OHIP_DIST_ALIGN")) return;
  std::vector<int> sbi, sbj, srp;
  schur_pattern(sbi, sbj, srp);
  auto symp = std::make_shared<const Symbolic>(analyze(block_pattern(num_poses, pd, sbi, sbj)));
  const Symbolic& sym = *symp;
  const char* df = getenv("G2OHIP_DIST_FACTOR");
  // the flags and weights build_structure gives DeviceCholesky::setup (which takes this analysis and plan instead of
  // making them again: al_sym / al_plan)
  const bool rs = !env0("G2OHIP_DIST_RS");
  const std::vector<double> pw = pose_work();
  auto planp = std::make_shared<const DistPlan>(
      plan_distribution(sym, sbi, sbj, pd, num_poses, nranks, rank, rs, df && atoi(df) == 1, true, &pw));
  const DistPlan& D = *planp;
  al_sym = symp;
  al_sbi = sbi;
  al_sbj = sbj;
  if (!D.on) return;
  al_plan = planp;
  // per landmark its free poses (all edges)
  std::vector<std::vector<int>> lp(num_landmarks);
  for (const HEdgeSet& es : hg.esets)
    for (size_t e = 0; e < es.ev0.size(); ++e) {
      const int i1 = hidx[es.ev0[e]], i2 = hidx[es.ev1[e]];
      if (i1 >= num_poses && i2 >= 0 && i2 < num_poses) lp[i1 - num_poses].push_back(i2);
      else if (i2 >= num_poses && i1 >= 0 && i1 < num_poses) lp[i2 - num_poses].push_back(i1);
    }
  std::vector<int> lm_ptr(num_landmarks + 1, 0), lm_cams;
  for (int l = 0; l < num_landmarks; ++l) {
    lm_cams.insert(lm_cams.end(), lp[l].begin(), lp[l].end());
    lm_ptr[l + 1] = (int)lm_cams.size();
  }
  const std::vector<int> own = align_landmarks(sym, D.owner, nranks, lm_ptr, lm_cams);
  std::vector<int> order(num_landmarks);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return own[a] < own[b]; });
  const std::vector<int> lmv(ivmap.begin() + num_poses, ivmap.end());
  ivmap.resize(num_poses);
  lm_bnd.assign(nranks + 1, 0);
  for (int l : order) {
    hidx[lmv[l]] = (int)ivmap.size();
    ivmap.push_back(lmv[l]);
    lm_bnd[own[l] + 1]++;
  }
  for (int r = 0; r < nranks; ++r) lm_bnd[r + 1] += lm_bnd[r];
  al_bpinv = sym.bpinv;
  al_bowner.resize(sym.nb);
  for (int k = 0; k < sym.nb; ++k) al_bowner[k] = D.owner[sym.block_sn[k]];
  lam_own_h.assign(num_poses, 0);
  for (int i = 0; i < num_poses; ++i) {
    const int o = al_bowner[al_bpinv[i]];
    lam_own_h[i] = (o == rank || (o < 0 && rank == 0)) ? 1 : 0;
  }
  d_lam_own.upload(lam_own_h, stream);
  dist_aligned = true;
}

// Lane groups (pairs of lanes, 128 per k_schur_rows workgroup) per slot of a Kt-record Schur task, in proportion to the
// slots' pairs in the task (T): every slot one, the rest one at a time to the slot with the most pairs per group (ties:
// the lower slot). A batch's pair loop lasts as long as its slowest group.
static void slot_groups(const long long* T, int noff, int* g) {
  for (int s = 0; s < noff; ++s) g[s] = 1;
  for (int extra = 128 - noff; extra > 0; --extra) {
    int bs = 0;
    double bv = -1.0;
    for (int s = 0; s < noff; ++s) {
      const double v = (double)T[s] / g[s];
      if (v > bv) { bv = v; bs = s; }
    }
    ++g[bs];
  }
}

// Slot-balanced batches of one Schur row chunk (Engine::build_structure): items = (observation, first partner in part,
// partners), part = (partner observation, slot). A batch's pair loop lasts as long as its busiest slot's pair list (four
// lanes per slot, one barrier per batch), so the observations are dealt greedily — most partners first, each to the
// batch, among a rotating window of WIN batches with room, where its busiest slot stays lowest (ties: the emptier one) —
// within batches of at most sb staged records. asg[k] = item k's batch; returns the batch count.
static int balance_batches(const std::vector<int3>& items, const std::vector<std::pair<int, int>>& part, int sb, int sl,
                           int noff, bool prop, bool local, int* asg, std::vector<int>& cap, std::vector<int>& cnt, std::vector<int>& ord,
                           std::vector<int>& opn) {
  constexpr int WIN = 8;  // a model of C4's rows: 8 candidates and all open batches balance alike, 4 worse
  // local: +-6 batches (C5 Schur rows 0.80 -> 0.73 ms against the rotating window; +-4..16 alike, +-1 0.81)
  constexpr int LOCAL_HW = 6;
  long long stt = 0;
  for (const int3& it : items) stt += 1 + it.z;
  // the slots' lane groups (prop: slot_groups, as the Kt-record pass's lane map will have them; else two pair streams per
  // slot): a batch's time on slot s is ceil(pairs / groups)
  std::vector<long long> T(sl, 0);
  for (const auto& pr : part) T[pr.second]++;
  std::vector<int> gw(sl, 2);  // (the G-block pass: four lanes per slot, two pair streams)
  if (prop) slot_groups(T.data(), noff, gw.data());
  int nbt = (int)std::max<long long>(1, (stt + sb - 1) / sb);
  cap.assign(nbt, 0);
  cnt.assign((size_t)nbt * sl, 0);
  ord.resize(items.size());
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return items[x].z > items[y].z; });
  opn.resize(nbt);
  std::iota(opn.begin(), opn.end(), 0);
  for (size_t q = 0; q < ord.size(); ++q) {
    const int3 it = items[ord[q]];
    const int need = 1 + it.z;
    int best = -1, bv = INT_MAX, bc = INT_MAX;
    auto consider = [&](int b) {
      if (cap[b] + need > sb) return;
      int v = 0;
      for (int k = 0; k < it.z; ++k) {
        const int q = part[it.y + k].second;
        v = std::max(v, (cnt[(size_t)b * sl + q] + gw[q]) / gw[q]);  // ceil((count + 1) / groups)
      }
      if (v < bv || (v == bv && cap[b] < bc)) { bv = v; bc = cap[b]; best = b; }
    };
    // candidates: local — the batches around the item's place in landmark order (neighbouring rows, which share
    // landmarks, then stage them at about the same time: L2 hits); else a rotating window over the batches that still
    // have room for the smallest observation
    const int no = (int)opn.size(), w = std::min(WIN, no);
    if (local) {
      const int nat = (int)((long long)ord[q] * nbt / std::max<size_t>(items.size(), 1));
      for (int b = std::max(0, nat - LOCAL_HW); b <= std::min(nbt - 1, nat + LOCAL_HW); ++b) consider(b);
    } else {
      for (int k = 0; k < w; ++k) consider(opn[(q + k) % no]);
    }
    if (best < 0)
      for (int k = 0; k < no; ++k) consider(opn[k]);
    if (best < 0) {  // no batch has room: a new one
      best = nbt++;
      cap.push_back(0);
      cnt.resize((size_t)nbt * sl, 0);
      opn.push_back(best);
    }
    asg[ord[q]] = best;
    cap[best] += need;
    for (int k = 0; k < it.z; ++k) cnt[(size_t)best * sl + part[it.y + k].second]++;
    if (cap[best] + 2 > sb)  // full for every observation (each stages itself and a partner at least)
      for (int k = 0; k < (int)opn.size(); ++k)
        if (opn[k] == best) { opn[k] = opn.back(); opn.pop_back(); break; }
  }
  return nbt;
}

// staged Kt records per Schur row batch (G2OHIP_SCHUR_SB_KX: 128, 192 or 256; A/B)
int Engine::kx_batch_size() {
  const char* v = getenv("G2OHIP_SCHUR_SB_KX");
  const int sb = v ? atoi(v) : launch::SCHUR_SB_KX;
  return sb == 128 || sb == 192 || sb == 256 ? sb : launch::SCHUR_SB_KX;
}

int Engine::build_structure() {  // block_solver.hpp:102-256
  knob_epoch().fetch_add(1, std::memory_order_acq_rel);  // launch-time knobs re-read from here on
  if (!initialized) {
    int r = initialize();
    if (r) return r;
  }
  ensure_device_state();
  if (comm) comm->rearm();  // a new collective sequence: RCCL's call-sequence check covers its first calls again
  align_shards();
  setup_edges_device();
  ++structure_ver;  // every cache keyed on the block pattern (marginals factor, BlockSymv) is stale from here
  // per-type hessian index and x offsets
  const int lm_begin = local_lm.empty() ? 0 : local_lm.front();
  const int lm_end = local_lm.empty() ? 0 : local_lm.back() + 1;
  for (int t = 1; t < NVT; ++t) {
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
  // off-diagonal blocks (mapHessianMemory, block_solver.hpp:142-210) over every local edge of every group
  std::vector<long long> gfirst(groups.size() + 1, 0);  // flat local edge index of each group's first edge
  for (size_t gi = 0; gi < groups.size(); ++gi) gfirst[gi + 1] = gfirst[gi] + groups[gi].ne;
  auto verts_of = [&](size_t gi, int k, int& va, int& vb) {
    const HEdgeSet& es = hg.esets[groups[gi].set];
    const int e = groups[gi].edges[k];
    va = es.ev0[e];
    vb = es.ev1[e];
  };
  std::map<std::pair<int, int>, int> hppmap;  // (i<j) -> block id
  hpp_bi.assign(num_poses, 0);
  hpp_bj.assign(num_poses, 0);
  for (int i = 0; i < num_poses; ++i) hpp_bi[i] = hpp_bj[i] = i;
  struct OffRef { int kind; int a, b; bool tr; };
  std::vector<OffRef> offref(std::max(ne, 1), OffRef{0, 0, 0, false});
  std::vector<std::pair<int, int>> plpairs;  // (lm, pose)
  for (size_t gi = 0; gi < groups.size(); ++gi)
    for (int k = 0; k < groups[gi].ne; ++k) {
      int va, vb;
      verts_of(gi, k, va, vb);
      const long long f = gfirst[gi] + k;
      int i1 = hidx[va], i2 = hidx[vb];
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
        offref[f] = OffRef{1, it->second, 0, tr};
      } else if (m1 && !m2) {
        offref[f] = OffRef{2, i2, i1 - num_poses, true};
        plpairs.push_back({i1 - num_poses, i2});
      } else if (!m1 && m2) {
        offref[f] = OffRef{2, i1, i2 - num_poses, false};
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
  auto blk_key = [&](const OffRef& r) -> long long {
    if (r.kind == 1) return r.a;  // hpp block id
    auto it = std::lower_bound(plpairs.begin(), plpairs.end(), std::make_pair(r.b, r.a));
    return nHpp + (long long)(it - plpairs.begin());
  };
  auto blk_off = [&](long long key) { return key < nHpp ? key * pd * pd : hpl_base + (key - nHpp) * pd * ld; };
  std::vector<int> blk_count(nHpp + nHpl, 0);
  std::vector<long long> ekey(std::max(ne, 1), -1);
  for (int f = 0; f < ne; ++f) {
    if (!offref[f].kind) continue;
    ekey[f] = blk_key(offref[f]);
    blk_count[ekey[f]]++;
  }
  // a block written by one local edge is stored directly by it; a block several edges share (two edges between
  // the same vertex pair, e.g. duplicate observations or an odometry edge beside another type) gets one slot per
  // edge, summed in edge order afterwards (deterministic; the reference's unlocked += races here, §2.3)
  constexpr long long SLOT_BIT = 1LL << 62;
  std::vector<long long> offdst(std::max(ne, 1), -1), slotoff(std::max(ne, 1), -1);
  long long nslotd = 0;
  for (int f = 0; f < ne; ++f) {
    if (ekey[f] < 0) continue;
    const long long bsz = ekey[f] < nHpp ? (long long)pd * pd : (long long)pd * ld;
    if (blk_count[ekey[f]] == 1) {
      offdst[f] = blk_off(ekey[f]);
    } else {
      slotoff[f] = nslotd;
      offdst[f] = SLOT_BIT | nslotd;
      nslotd += bsz;
    }
  }
  for (int c = 0; c < 2; ++c) {
    OffRed& R = offred[c];
    std::vector<int> ptr{0};
    std::vector<long long> so, dst;
    std::vector<std::vector<long long>> lists;
    std::map<long long, int> bl;  // block key -> list (ascending block key: a fixed launch order)
    for (int f = 0; f < ne; ++f)
      if (slotoff[f] >= 0 && ((ekey[f] < nHpp) == (c == 0))) {
        auto it = bl.find(ekey[f]);
        if (it == bl.end()) { it = bl.emplace(ekey[f], (int)lists.size()).first; lists.emplace_back(); }
        lists[it->second].push_back(slotoff[f]);
      }
    for (auto& kv : bl) {
      so.insert(so.end(), lists[kv.second].begin(), lists[kv.second].end());
      ptr.push_back((int)so.size());
      dst.push_back(blk_off(kv.first));
    }
    R.nb = (int)dst.size();
    R.bsz = c == 0 ? pd * pd : pd * ld;
    R.ptr.upload(ptr, stream);
    R.soff.upload(so.empty() ? std::vector<long long>{0} : so, stream);
    R.dst.upload(dst.empty() ? std::vector<long long>{0} : dst, stream);
  }
  doffslot.resize((size_t)std::max<long long>(nslotd, 1));
  // per-vertex-side slots: arena by vertex dimension, each group's sides contiguous
  for (long long& c : nslot) c = 0;
  for (EGroup& g : groups) {
    long long& ca = nslot[g.DA];
    g.slotA = ca;
    ca += g.ne;
    long long& cb = nslot[g.DB];
    g.slotB = cb;
    cb += g.ne;
  }
  for (size_t gi = 0; gi < groups.size(); ++gi) {
    EGroup& g = groups[gi];
    std::vector<long long> od(offdst.begin() + gfirst[gi], offdst.begin() + gfirst[gi + 1]);
    std::vector<unsigned char> tr(g.ne);
    for (int k = 0; k < g.ne; ++k) tr[k] = offref[gfirst[gi] + k].tr ? 1 : 0;
    if (od.empty()) { od.push_back(-1); tr.push_back(0); }
    g.off_dst.upload(od, stream);
    g.off_tr.upload(tr, stream);
    if (gi == 0 && ba_fused) {
      // the split's Kt records: one per Hpl block, plus one per observation of a fixed landmark by a free camera (Kt = 0)
      // behind them; camera-major observation -> its record
      std::vector<int> xe(std::max(g.ne, 1), -1), ch(std::max<size_t>(cm_e_h.size(), 1), -1);
      n_kx_extra = 0;
      for (int k = 0; k < g.ne; ++k) {
        const int e2 = g.edges[k];
        if (hidx[hg.esets[g.set].ev0[e2]] < 0 && hidx[hg.esets[g.set].ev1[e2]] >= 0) xe[k] = nHpl + n_kx_extra++;
      }
      for (size_t p = 0; p < cm_e_h.size(); ++p) {
        const long long o = od[cm_e_h[p]];
        if (o >= 0 && !(o & SLOT_BIT)) ch[p] = (int)((o - hpl_base) / ((long long)pd * ld));
        else ch[p] = xe[cm_e_h[p]];
      }
      cm_hpl.upload(ch, stream);
      kx_extra.upload(xe, stream);
    }
  }
  // storage
  dH.resize(std::max<long long>((long long)nHpp * pd * pd + (long long)nHpl * pd * ld, 1));
  dH.zero(stream);
  const int nLloc = (int)local_lm.size();
  dHll.resize(std::max(nLloc * ld * ld, 1));
  dHll.zero(stream);
  const long long n = vector_size();
  db.resize(std::max<long long>(n, 1));
  db.zero(stream);
  dx.resize(std::max<long long>(n, 1));
  dx.zero(stream);
  for (int d : {2, 3, 6})  // the fused BA path needs no slots
    dslot[d].resize((size_t)std::max<long long>(ba_fused ? 1 : nslot[d], 1) * (d * (d + 1) / 2 + d));
  // vertex incidence lists (hessian order): code = slot index in the arena of the vertex's dimension, in
  // group / edge order (a fixed summation order)
  {
    std::vector<std::vector<int>> incp(num_poses), incl(nLloc);
    for (size_t gi = 0; gi < groups.size(); ++gi) {
      const EGroup& g = groups[gi];
      for (int k = 0; k < g.ne; ++k) {
        int va, vb;
        verts_of(gi, k, va, vb);
        const int hs[2] = {hidx[va], hidx[vb]};
        const long long code[2] = {g.slotA + k, g.slotB + k};
        for (int sd = 0; sd < 2; ++sd) {
          const int h = hs[sd];
          if (h < 0) continue;
          if (code[sd] >= (1LL << 31)) throw DeviceError("too many edge slots for 32-bit slot codes");
          if (h < num_poses) incp[h].push_back((int)code[sd]);
          else incl[h - num_poses - lm_begin].push_back((int)code[sd]);
        }
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
    std::vector<int> srow_ptr;
    schur_pattern(s_bi, s_bj, srow_ptr);
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

      // one batch set per staged-block size: SB blocks per batch (G blocks: launch::SCHUR_SB; the split's 80-byte Kt
      // records: G2OHIP_SCHUR_SB_KX, default launch::SCHUR_SB_KX)
      struct BatchSet {
        std::vector<launch::SchurTask> tasks;
        std::vector<launch::SchurBatch> batches;
        std::vector<int> st_obs, st_obs_h, prs, pp;
        std::vector<launch::SchurPartGroup> groups;  // row chunks split into parts (their partial sums' reduction)
        std::vector<int> gmap;  // per task 128 lane-group entries: slot | index << 8 | groups << 16 (Kt-record pass)
        long long npairs = 0, nparts_blocks = 0;
      };
      // Per-rank task lists of the landmark-sharded BA (aligned shards + the distributed factorization reading only its
      // own subtrees' and the shared blocks): a row chunk with no local pair whose slots all land in another rank's
      // subtrees writes nothing anyone reads here, and is skipped (dS is zeroed once, so a skipped block reads 0).
      // Chunks are split into parts (partial sums reduced by k_schur_part_sum) when the row tasks would not fill the
      // chip twice: a task's batches are a serial chain, and a rank with an eighth of the rows would otherwise be
      // bound by its longest row (G2OHIP_SCHUR_SPLIT_TASKS: the target task count, 0 off; default 2048 in the sharded
      // path, off on one GPU).
      const char* dvr = getenv("G2OHIP_DIST_RS");
      const char* ssk = getenv("G2OHIP_SCHUR_SKIP");  // dev A/B: 0 = every rank runs every row chunk and camera
      const bool sch_skip = dist_aligned && nranks > 1 && comm && !write_debug && !(dvr && atoi(dvr) == 0) &&
                            !(ssk && atoi(ssk) == 0);
      // G2OHIP_SCHUR_BALANCE (dev A/B): 0 batches in landmark order; else slot-balanced batches (build_batches) whose
      // candidates are the batches near the observation's landmark-order place or a rotating window over the open ones
      const char* sbal = getenv("G2OHIP_SCHUR_BALANCE");
      const bool sch_balance = !(sbal && atoi(sbal) == 0);
      const bool sch_bal_local = !(sbal && atoi(sbal) == 2);  // 2 = the rotating window
      const char* sst = getenv("G2OHIP_SCHUR_SPLIT_TASKS");
      const int split_target = sst ? atoi(sst) : (nranks > 1 && comm ? 2048 : 0);
      auto blk_owner = [&](int i, int j) { return al_bowner[std::min(al_bpinv[i], al_bpinv[j])]; };
      // kx_lanes: the set the Kt-record pass (per-task lane map) walks — balanced for its lanes, else for the G-block pass's
      auto build_batches = [&](int SB, BatchSet& bs, bool kx_lanes) {
      auto& tasks = bs.tasks;
      auto& batches = bs.batches;
      auto& st_obs = bs.st_obs;
      auto& st_obs_h = bs.st_obs_h;
      auto& prs = bs.prs;
      auto& pp = bs.pp;
      long long& npairs = bs.npairs;
      // a task and its lane map (slot_groups over the pairs of its batches [b0, b1))
      std::vector<long long> tslot(SL);
      auto push_task = [&](const launch::SchurTask& T) {
        std::fill(tslot.begin(), tslot.end(), 0);
        for (int b = T.b0; b < T.b1; ++b)
          for (int q = 0; q < SL; ++q) tslot[q] += pp[(size_t)b * (SL + 1) + q + 1] - pp[(size_t)b * (SL + 1) + q];
        int g[SL];
        slot_groups(tslot.data(), T.noff, g);
        for (int q = 0; q < T.noff; ++q)
          for (int k = 0; k < g[q]; ++k) bs.gmap.push_back(q | (k << 8) | (g[q] << 16));
        tasks.push_back(T);
      };
      std::vector<int> camslot(num_poses, -1);
      struct P3 { int ls, a, b; };
      std::vector<P3> cur;
      std::vector<std::pair<int, int>> tmp;
      std::vector<int3> bal_items;                   // (observation, first partner in bal_part, partners)
      std::vector<std::pair<int, int>> bal_part;     // (partner observation, slot)
      std::vector<int> bal_bptr, bal_seq, bal_fill;  // (reused across rows)
      npairs = 0;
      // pass 1: per row chunk its staged blocks (0: no local pair) and whether it must run at all
      std::vector<long long> ch_staged;
      std::vector<int> ch_items;
      std::vector<unsigned char> ch_live;
      for (int i = 0; i < num_poses; ++i) {
        const int s_lo = srow_ptr[i], s_hi = srow_ptr[i + 1];
        for (int k = s_lo; k < s_hi; ++k) camslot[s_bj[k]] = k - s_lo;
        const int noff_total = s_hi - s_lo - 1;
        for (int ch = 0; ch * SL < noff_total; ++ch) {
          const int off_lo = 1 + ch * SL, noff = std::min(SL, noff_total - ch * SL);
          long long st = 0;
          int nit = 0;  // observations with a partner in the chunk
          for (int r = rptr[i]; r < rptr[i + 1]; ++r) {
            const int a = robs[r], l = obs_lm[a];
            int np = 0;
            for (int a2 = a + 1; a2 < lm_ptr[l + 1]; ++a2) {
              const int sl = camslot[blk_pose[a2]] - off_lo;
              np += sl >= 0 && sl < noff;
            }
            if (np) { st += 1 + np; ++nit; }
          }
          bool live = st > 0 || !sch_skip;
          for (int k = 0; k < noff && !live; ++k) {
            const int o = blk_owner(i, s_bj[s_lo + off_lo + k]);
            live = o < 0 || o == rank;
          }
          ch_staged.push_back(st);
          ch_items.push_back(nit);
          ch_live.push_back(live ? 1 : 0);
        }
        for (int k = s_lo; k < s_hi; ++k) camslot[s_bj[k]] = -1;
      }
      long long nlive = 0;
      for (size_t c = 0; c < ch_live.size(); ++c) nlive += ch_live[c];
      const int P = split_target > 0 && nlive > 0 ? (int)std::min<long long>(8, std::max<long long>(1, (split_target + nlive - 1) / nlive)) : 1;
      // slot-balanced batches (see the emission below): every balanced chunk's observation -> batch assignment, rows in
      // parallel (host threads; the greedy is the structure build's largest host step at C5), stored per chunk item
      std::vector<long long> bal_off(ch_items.size() + 1, 0);
      for (size_t c = 0; c < ch_items.size(); ++c) bal_off[c + 1] = bal_off[c] + ch_items[c];
      std::vector<int> bal_asg_all(sch_balance ? (size_t)std::max<long long>(bal_off.back(), 1) : 1, -1);
      std::vector<int> bal_nb_all(sch_balance ? ch_items.size() : 0, 0);
      if (sch_balance) {
        std::vector<long long> row_c0(num_poses + 1, 0);  // first chunk index of each row
        for (int i = 0; i < num_poses; ++i) {
          const int noff_total = srow_ptr[i + 1] - srow_ptr[i] - 1;
          row_c0[i + 1] = row_c0[i] + (noff_total > 0 ? (noff_total + SL - 1) / SL : 0);
        }
        const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::atomic<int> next_row{0};
        auto work = [&]() {
          std::vector<int> cs(num_poses, -1), cap, cnt, ord, opn;
          std::vector<int3> items;
          std::vector<std::pair<int, int>> part;
          for (int i; (i = next_row.fetch_add(1)) < num_poses;) {
            const int s_lo = srow_ptr[i], s_hi = srow_ptr[i + 1];
            for (int k = s_lo; k < s_hi; ++k) cs[s_bj[k]] = k - s_lo;
            const int noff_total = s_hi - s_lo - 1;
            for (int ch = 0; ch * SL < noff_total; ++ch) {
              const size_t cidx = (size_t)row_c0[i] + ch;
              if (!ch_live[cidx]) continue;
              const long long tot = ch_staged[cidx];
              const int npart = (int)std::max<long long>(1, std::min<long long>(P, tot / (2LL * SB)));
              if (npart != 1) continue;
              const int off_lo = 1 + ch * SL, noff = std::min(SL, noff_total - ch * SL);
              items.clear();
              part.clear();
              for (int r = rptr[i]; r < rptr[i + 1]; ++r) {
                const int a = robs[r], l = obs_lm[a];
                const int o0 = (int)part.size();
                for (int a2 = a + 1; a2 < lm_ptr[l + 1]; ++a2) {
                  const int sl = cs[blk_pose[a2]] - off_lo;
                  if (sl >= 0 && sl < noff) part.push_back({a2, sl});
                }
                const int n = (int)part.size() - o0;
                if (n) items.push_back(int3{a, o0, n});
              }
              int* asg = bal_asg_all.data() + bal_off[cidx];
              bal_nb_all[cidx] = balance_batches(items, part, SB, SL, noff, kx_lanes, sch_bal_local, asg, cap, cnt, ord, opn);
            }
            for (int k = s_lo; k < s_hi; ++k) cs[s_bj[k]] = -1;
          }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nth; ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
      }
      size_t cidx = 0;
      for (int i = 0; i < num_poses; ++i) {
        const int s_lo = srow_ptr[i], s_hi = srow_ptr[i + 1];
        for (int k = s_lo; k < s_hi; ++k) camslot[s_bj[k]] = k - s_lo;  // slot 0 = the diagonal block
        const int noff_total = s_hi - s_lo - 1;
        for (int ch = 0; ch * SL < noff_total; ++ch, ++cidx) {
          if (!ch_live[cidx]) continue;
          const long long tot = ch_staged[cidx];
          // parts of at least two batches each
          const int np = (int)std::max<long long>(1, std::min<long long>(P, tot / (2LL * SB)));
          launch::SchurTask T{};
          T.row = i;
          const int off_lo = 1 + ch * SL;
          T.noff = std::min(SL, noff_total - ch * SL);
          T.soff = s_lo + off_lo;
          T.b0 = (int)batches.size();
          long long xo = 0;
          if (np > 1) {
            xo = bs.nparts_blocks;
            bs.nparts_blocks += (long long)np * T.noff;
            bs.groups.push_back(launch::SchurPartGroup{T.soff, T.noff, (int)xo, np});
            T.pad = (int)xo + 1;  // part 0's partial blocks (k_schur_rows stores acc there, not Hpp - acc)
          }
          int part = 0;
          long long cum = 0;
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
          if (np == 1 && sch_balance) {
            // slot-balanced batches: a batch's pair loop lasts as long as its busiest slot's pair list (four lanes per
            // slot, one barrier per batch), so the row's observations are dealt to the batches greedily — most partners
            // first, each to the batch (of those with room, among a window of candidates) where its busiest slot stays
            // lowest — instead of in landmark order; each batch keeps its observations in landmark order
            bal_items.clear();
            bal_part.clear();
            for (int r = rptr[i]; r < rptr[i + 1]; ++r) {
              const int a = robs[r], l = obs_lm[a];
              const int o0 = (int)bal_part.size();
              for (int a2 = a + 1; a2 < lm_ptr[l + 1]; ++a2) {
                const int sl = camslot[blk_pose[a2]] - off_lo;
                if (sl >= 0 && sl < T.noff) bal_part.push_back({a2, sl});
              }
              const int n = (int)bal_part.size() - o0;
              if (n) bal_items.push_back(int3{a, o0, n});
            }
            const int nbt = bal_nb_all[cidx];
            const int* asg = bal_asg_all.data() + bal_off[cidx];
            // each batch's observations in landmark order: a counting sort of the items by batch (stable)
            bal_bptr.assign(nbt + 1, 0);
            for (size_t k = 0; k < bal_items.size(); ++k) bal_bptr[asg[k] + 1]++;
            for (int b = 0; b < nbt; ++b) bal_bptr[b + 1] += bal_bptr[b];
            bal_seq.resize(bal_items.size());
            {
              std::vector<int>& fillb = bal_fill;
              fillb.assign(bal_bptr.begin(), bal_bptr.end() - 1);
              for (size_t k = 0; k < bal_items.size(); ++k) bal_seq[fillb[asg[k]]++] = (int)k;
            }
            for (int b = 0; b < nbt; ++b) {
              for (int kk = bal_bptr[b]; kk < bal_bptr[b + 1]; ++kk) {
                const int3 it = bal_items[bal_seq[kk]];
                const int posA = (int)st_obs.size() - bst0;
                st_obs.push_back(gpos[it.x]);
                st_obs_h.push_back(it.x);
                for (int m = 0; m < it.z; ++m) {
                  const auto& pr = bal_part[it.y + m];
                  const int posB = (int)st_obs.size() - bst0;
                  st_obs.push_back(gpos[pr.first]);
                  st_obs_h.push_back(pr.first);
                  cur.push_back(P3{pr.second, posA, posB});
                }
              }
              flush();
            }
          } else
          for (int r = rptr[i]; r < rptr[i + 1]; ++r) {
            const int a = robs[r], l = obs_lm[a];
            tmp.clear();
            for (int a2 = a + 1; a2 < lm_ptr[l + 1]; ++a2) {
              const int sl = camslot[blk_pose[a2]] - off_lo;
              if (sl >= 0 && sl < T.noff) tmp.push_back({a2, sl});
            }
            if (tmp.empty()) continue;
            const int need = 1 + (int)tmp.size();
            const int want = np > 1 ? (int)std::min<long long>(np - 1, cum * np / tot) : 0;
            while (part < want) {  // the next part: a task of its own (the same slots, its own partial blocks)
              flush();
              T.b1 = (int)batches.size();
              push_task(T);
              ++part;
              T.b0 = (int)batches.size();
              T.pad = (int)xo + part * T.noff + 1;
            }
            cum += need;
            if ((int)st_obs.size() - bst0 + need > SB) flush();
            const int posA = (int)st_obs.size() - bst0;
            st_obs.push_back(gpos[a]);
            st_obs_h.push_back(a);
            for (auto& [a2, sl] : tmp) {
              const int posB = (int)st_obs.size() - bst0;
              st_obs.push_back(gpos[a2]);
              st_obs_h.push_back(a2);
              cur.push_back(P3{sl, posA, posB});
            }
          }
          flush();
          T.b1 = (int)batches.size();
          push_task(T);
          if (np > 1 && part != np - 1) {  // trailing parts without observations: their partial blocks are zeros
            for (int q = part + 1; q < np; ++q) {
              T.b0 = T.b1 = (int)batches.size();
              T.pad = (int)xo + q * T.noff + 1;
              push_task(T);
            }
          }
        }
        for (int k = s_lo; k < s_hi; ++k) camslot[s_bj[k]] = -1;
      }
      batches.push_back(launch::SchurBatch{});  // trailing dummy: k_schur_rows reads one record ahead
      };
      auto nz = [](std::vector<int>& v) -> std::vector<int>& { if (v.empty()) v.push_back(0); return v; };
      // the split camera pass of a sharded rank: cameras with local observations or a diagonal block this rank reads
      {
        std::vector<int> cl;
        if (sch_skip && (int)cm_ptr_h.size() == num_poses + 1)
          for (int i = 0; i < num_poses; ++i) {
            const int o = blk_owner(i, i);
            if (cm_ptr_h[i + 1] > cm_ptr_h[i] || o < 0 || o == rank) cl.push_back(i);
          }
        ncam_list = (int)cl.size();
        d_cam_list.upload(cl.empty() ? std::vector<int>{0} : cl, stream);
      }
      sch_part_blocks = 0;
      {
        BatchSet bs;
        build_batches(SB, bs, kx_batch_size() == SB);
        npairs = bs.npairs;
        nsch_tasks = (int)bs.tasks.size();
        nstaged = (long long)bs.st_obs.size();
        nsch_groups = (int)bs.groups.size();
        sch_groups.upload(bs.groups.empty() ? std::vector<launch::SchurPartGroup>(1) : bs.groups, stream);
        sch_part_blocks = bs.nparts_blocks;
        sch_tasks.upload(bs.tasks.empty() ? std::vector<launch::SchurTask>(1) : bs.tasks, stream);
        sch_batches.upload(bs.batches, stream);
        sch_st_obs.upload(nz(bs.st_obs), stream);
        sch_st_obs_h.upload(nz(bs.st_obs_h), stream);
        sch_pairs.upload(nz(bs.prs), stream);
        sch_pp.upload(nz(bs.pp), stream);
        sch_gmap.upload(nz(bs.gmap), stream);
      }
      // the Kt-record set (BA split; decided with the split below): another block size needs its own batches
      kx_sb = kx_batch_size();
      nsch_tasks_kx = nsch_groups_kx = 0;
      if (kx_sb != SB && ba_fused && pd == 6 && ld == 3) {
        BatchSet bs;
        build_batches(kx_sb, bs, true);
        nsch_tasks_kx = (int)bs.tasks.size();
        nsch_groups_kx = (int)bs.groups.size();
        sch_groups_kx.upload(bs.groups.empty() ? std::vector<launch::SchurPartGroup>(1) : bs.groups, stream);
        sch_part_blocks = std::max(sch_part_blocks, bs.nparts_blocks);
        sch_tasks_kx.upload(bs.tasks.empty() ? std::vector<launch::SchurTask>(1) : bs.tasks, stream);
        sch_batches_kx.upload(bs.batches, stream);
        sch_st_obs_kx.upload(nz(bs.st_obs_h), stream);
        sch_pairs_kx.upload(nz(bs.prs), stream);
        sch_pp_kx.upload(nz(bs.pp), stream);
        sch_gmap_kx.upload(nz(bs.gmap), stream);
      }
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
    dDinv.resize(std::max(nLloc * ld * ld, 1));
    dUfac.resize(std::max(nLloc * launch::schur_ufac_stride(ld), 1));
    // G = Hpl U^-T per observation (pd x ld), or the split's 10-double Kt records (+ the fixed-landmark ones)
    dG.resize(std::max<long long>(std::max((long long)nHpl * pd * ld, ((long long)nHpl + n_kx_extra) * 10), 1));
    dCl.resize(std::max<long long>((long long)num_landmarks * ld, 1));  // c = U^-1 b_l (global landmark index)
    dS.resize((size_t)nS * pd * pd + size_poses);  // [S blocks | bschur] contiguous for one all-reduce
    // blocks and rhs rows the per-rank task lists never write (sch_skip) must read as zeros in the whole-dS all-reduce of
    // stage(): zero once per structure
    dS.zero(stream);
    dSchurPart.resize(std::max<long long>(sch_part_blocks * pd * pd, 1));
    {  // landmark side of the Schur complement formed during assembly (G2OHIP_SCHUR_SPLIT=0: the plain passes, A/B)
      const char* ev = getenv("G2OHIP_SCHUR_SPLIT");
      fz_split_ok = ba_fused && nslotd == 0 && pd == 6 && ld == 3 && !use_cgls() && !(ev && atoi(ev) == 0);
      // the split stores 10-double Kt records instead of G (assembly.hip KXB): 80 instead of 144 bytes written per
      // observation and staged by the Schur row pass (G2OHIP_SCHUR_KX=0: G, A/B). The stored-G back-substitution
      // (G2OHIP_BACKSUB_RECOMPUTE=0) needs G.
      const char* kx = getenv("G2OHIP_SCHUR_KX");
      const char* bsr = getenv("G2OHIP_BACKSUB_RECOMPUTE");
      fz_kx = fz_split_ok && !(kx && atoi(kx) == 0) && !(bsr && atoi(bsr) == 0);
      fz_lambda = std::numeric_limits<double>::quiet_NaN();
    }
    if (use_cgls()) {  // the fork's JacobiSolver_6_3: CGLS on J, no reduced system to factor
      if (!ba_fused || nranks > 1) throw DeviceError("lm_pcg6_3_eigen needs a single-GPU graph of BA edges only");
      const EGroup& g = groups[0];
      const HEdgeSet& es = hg.esets[g.set];
      std::vector<int> ecam(g.ne), ept(g.ne);
      for (int k = 0; k < g.ne; ++k) {
        const int hc = hidx[es.ev1[g.edges[k]]], hl = hidx[es.ev0[g.edges[k]]];
        ecam[k] = hc >= 0 && hc < num_poses ? hc : -1;
        ept[k] = hl >= num_poses ? hl - num_poses - lm_begin : -1;
      }
      cgls.setup(num_poses, nLloc, g.ne, lm_eptr_h, cm_ptr_h, cm_e_h, ecam, ept, stream);
    } else if (use_pcg()) {
      pcg.setup(num_poses, pd, s_bi, s_bj, stream);
    } else {
      // landmark shards: the factorization is distributed too (subtrees of the elimination tree per rank, DESIGN.md
      // §6); G2OHIP_DIST_FACTOR=0 keeps the replicated factorization (every rank factors all of S)
      const char* df = getenv("G2OHIP_DIST_FACTOR");
      const bool dist = nranks > 1 && comm && !(df && atoi(df) == 0);
      chol.dist_rank = dist ? rank : 0;
      chol.dist_nranks = dist ? nranks : 1;
      chol.dist_force = df && atoi(df) == 1;
      chol.allreduce = [this](double* p, size_t n) { allreduce_sum(p, n); };
      chol.allgather = [this](double* p, size_t n) { comm->allgather(p, n, stream); };
      // the reduced system itself reduce-scattered by subtree ownership (G2OHIP_DIST_RS=0: all-reduced whole, A/B);
      // not with the not-PD dump, which writes the whole S from rank 0
      const char* drs = getenv("G2OHIP_DIST_RS");
      chol.rs_enable = dist && !write_debug && !(drs && atoi(drs) == 0);
      chol.reduce_scatter = [this](double* p, size_t n) { comm->reduce_scatter_sum(p, n, stream); };
      // timing only (tools/dist_factor_time.py): one process plays rank r of N of the distributed factorization with
      // no-op exchanges — the kernel chain rank r would run, on this GPU; the solution is not meaningful
      const char* sim = getenv("G2OHIP_DIST_SIMULATE");
      int sr = 0, sn = 0;
      bool sim_on = false;
      if (!dist && sim && sscanf(sim, "%d/%d", &sr, &sn) == 2 && sn > 1 && sr >= 0 && sr < sn) {
        sim_on = true;
        chol.dist_rank = sr;
        chol.dist_nranks = sn;
        chol.dist_force = true;
        chol.allreduce = [](double*, size_t) {};
        chol.allgather = [](double*, size_t) {};
        chol.reduce_scatter = [](double*, size_t) {};
        chol.rs_enable = !(drs && atoi(drs) == 0);
      }
      chol.aligned = dist_aligned && dist;
      chol.blk_local.clear();
      // the simulated rank plays the aligned cut the product would take (landmark shards follow the cut: every block of
      // its subtrees is complete locally, only the shared blocks are exchanged); G2OHIP_DIST_SIMULATE_ALIGNED=0: the
      // uniform-shard cut
      const char* sal = getenv("G2OHIP_DIST_SIMULATE_ALIGNED");
      if (sim_on && !(sal && atoi(sal) == 0) && do_schur) {
        chol.aligned = true;
        chol.blk_local.assign(nS, 1);
      }
      if (chol.aligned && !sim_on) {
        // blocks written by a rank other than the one whose subtrees read them: those of edges without a free
        // landmark (assembled by rank 0: pose-pose edges, edges to fixed landmarks) — both endpoints' diagonal blocks
        // and their off-diagonal block — where the reading rank is not rank 0. Landmark blocks and lambda (lam_own)
        // are written by the reading rank itself.
        std::vector<unsigned char> by0(nS, 0);
        auto blk = [&](int i, int j) {
          const int* b = s_bj.data() + srow_ptr[i];
          const int* e = s_bj.data() + srow_ptr[i + 1];
          const int* it = std::lower_bound(b, e, j);
          return it != e && *it == j ? (int)(it - s_bj.data()) : -1;
        };
        for (const HEdgeSet& es : hg.esets)
          for (size_t e = 0; e < es.ev0.size(); ++e) {
            const int i1 = hidx[es.ev0[e]], i2 = hidx[es.ev1[e]];
            if (i1 >= num_poses || i2 >= num_poses) continue;  // a free landmark endpoint: its owner's
            for (int h : {i1, i2})
              if (h >= 0) { const int t = blk(h, h); if (t >= 0) by0[t] = 1; }
            if (i1 >= 0 && i2 >= 0 && i1 != i2) { const int t = blk(std::min(i1, i2), std::max(i1, i2)); if (t >= 0) by0[t] = 1; }
          }
        chol.blk_local.assign(nS, 1);
        for (int t = 0; t < nS; ++t) {
          const int o = al_bowner[std::min(al_bpinv[s_bi[t]], al_bpinv[s_bj[t]])];
          if (by0[t] && o != 0) chol.blk_local[t] = 0;
        }
      }
      chol.pose_work = pose_work();
      if (al_sym && s_bi == al_sbi && s_bj == al_sbj) {  // the pattern align_shards analysed: reuse its work
        chol.pre_sym = al_sym;
        if (chol.aligned && al_plan) chol.pre_plan = al_plan;
      }
      al_sym.reset();
      al_plan.reset();
      chol.setup(num_poses, pd, s_bi, s_bj, stream);
      if (chol.aligned && !chol.distributed())
        throw DeviceError("aligned landmark shards without the distributed factorization they were cut for");
    }
  } else if (use_pcg()) {
    pcg.setup(num_poses, pd, hpp_bi, hpp_bj, stream);
  } else {
    chol.set_replicated();
    chol.setup(num_poses, pd, hpp_bi, hpp_bj, stream);
  }
  HIP_CHECK(hipStreamSynchronize(stream));
  structure_built = true;
  return G2OHIP_OK;
}

// ------------------------------------------------------------------ Engine: numeric steps
void Engine::allreduce_sum(double* p, size_t n) {
  if (nranks <= 1 || !comm) return;
  comm->allreduce_sum(p, n, stream);
}

void Engine::compute_errors_async(bool reduce) {  // computeActiveErrors + activeRobustChi2 (sparse_optimizer.cpp:63-116)
  ensure_device_state();
  refresh_host_payload(false);
  timer.begin("error", stream);
  int np = 0;  // every group's partials back to back, summed in one fixed tree
  for (const EGroup& g : groups) np += launch::error_partials(g.family, group_args(g), g.ne, dpartial.get() + np, stream);
  launch::sum_final(dpartial.get(), np, dscal.get() + 1, stream);
  timer.end(stream);
  if (do_schur && reduce) allreduce_sum(dscal.get() + 1, 1);
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

int Engine::build_system() { return build_system_split(std::numeric_limits<double>::quiet_NaN()); }

// a Schur-split assembly leaves Hpp's diagonal blocks unwritten (S(i,i) is formed directly): the entry points that
// read Hpp get a plain buildSystem of the same state first
void Engine::ensure_hpp() {
  if (!std::isnan(fz_lambda)) build_system();
}

int Engine::build_system_split(double lambda, const double* lamp) {  // block_solver.hpp:462-521
  if (!structure_built) {
    int r = build_structure();
    if (r) return r;
  }
  ensure_device_state();
  refresh_host_payload(true);
  fz_lambda = std::numeric_limits<double>::quiet_NaN();
  if (ba_fused) {  // assembly.hip: landmark side reduced inside the linearize waves, camera side recomputed per camera
    const EGroup& g = groups[0];
    const int lm_begin = local_lm.empty() ? 0 : local_lm.front();
    launch::SchurSplit sp{};
    const bool split = fz_split_ok && (std::isfinite(lambda) || lamp);
    if (split) {  // block_solver.hpp:341-400 (the landmark pass and the diagonal terms) at lambda, during assembly
      sp.lam = lambda;
      sp.lam_rank = rank == 0 ? lambda : 0.0;
      sp.lamp = lamp;
      sp.lam_own = dist_aligned ? d_lam_own.get() : nullptr;
      sp.Ufac = dUfac.get();
      sp.cl = dCl.get();
      sp.G = dG.get();
      sp.kx = fz_kx ? 1 : 0;
      {  // Kt records that outgrow the caches are stored nontemporally (C5's 800 MB: linearize 0.458 -> 0.43 ms; C4's 80 MB
         // stay cached for the camera pass, which NT stores slow 47 -> 53 us: profiles/r06_ab_lin_nts.log);
         // G2OHIP_LIN_NTS (dev A/B): 0 never, 1 always
        const char* nts = getenv("G2OHIP_LIN_NTS");
        const int nt = nts ? atoi(nts) : (kx_records_cached((double)nHpl + n_kx_extra) ? 0 : 1);
        if (fz_kx && nt == 1) sp.kx = 2;
      }
      // the camera pass from the Kt records while they stay cache-resident (the pass gathers them in camera order; C4's
      // 80 MB: 52 -> 48 us), else re-linearising every observation from the per-landmark point, U and c (C5's 800 MB of
      // records: 0.42 -> 0.49 ms, where the per-landmark gathers are 96 MB; profiles/r05_ab_c5_dl_camkx.log).
      // G2OHIP_CAM_KX=0 / 1 forces either (A/B)
      static EnvKnob cam_kx{"G2OHIP_CAM_KX", -1};
      const int ck = cam_kx.get();
      const bool use_ck = ck == 1 || (ck < 0 && kx_records_cached((double)nHpl + n_kx_extra));
      sp.cm_hpl = fz_kx && use_ck ? cm_hpl.get() : nullptr;
      sp.kx_extra = fz_kx ? kx_extra.get() : nullptr;
      sp.hpl_base = (long long)nHpp * pd * pd;
      sp.lm_ptr = d_lm_ptr.get();
      sp.hl = d_hidx[g.vtA].get();
      sp.sdiag = sch_sdiag.get();
      sp.S = dS.get();
      sp.bschur = dS.get() + (size_t)nS * pd * pd;
      sp.fail = failp() + 1;
      // a device lambda is not known here: +inf never equals a trial's lambda, so solve_async re-assembles unless the
      // host, having read the decision, confirms the value (lm_solve), and ensure_hpp sees a split assembly
      fz_lambda = lamp ? std::numeric_limits<double>::infinity() : lambda;
    }
    timer.begin("linearize", stream);
    launch::linearize_fused(group_args(g), fz_chunks.get(), fz_nchunks, d_hidx[g.vtA].get(), d_hidx[g.vtB].get(),
                            g.off_dst.get(), g.off_tr.get(), dH.get(), doffslot.get(), dHll.get(), db.get(), num_poses,
                            size_poses, lm_begin, fz_lpart.get(), split ? &sp : nullptr, stream);
    timer.end(stream);
    for (const OffRed& R : offred)
      launch::offblock_reduce(R.nb, R.bsz, R.ptr.get(), R.soff.get(), doffslot.get(), dH.get(), R.dst.get(), stream);
    timer.begin("vreduce", stream);
    // split landmarks first: the camera pass reads every landmark's U and c
    launch::lm_fixup(fz_nfix, fz_fix.get(), fz_lpart.get(), dHll.get(), db.get(), num_poses, size_poses, lm_begin,
                     split ? &sp : nullptr, stream);
    EdgeArgs ca = group_args(g);
    ca.v0 = cm_v0.get();
    ca.v1 = cm_v1.get();
    ca.meas = cm_meas.get();
    ca.info = cm_info.get();
    ca.params = cm_params.get();
    if (split && ncam_list > 0)  // a sharded rank's split pass: only the cameras it needs (the rest stay zero)
      launch::cam_assemble(ca, cm_ptr.get(), ncam_list, dH.get(), db.get(), num_poses, lm_begin, &sp, stream,
                           d_cam_list.get());
    else
      launch::cam_assemble(ca, cm_ptr.get(), num_poses, dH.get(), db.get(), num_poses, lm_begin, split ? &sp : nullptr,
                           stream);
    timer.end(stream);
    if (use_cgls()) {  // JacobiSolver::buildSystem's J (jacobi_solver.hpp:479-700)
      timer.begin("cgls_jacobian", stream);
      cgls.build(group_args(g), d_hidx[g.vtA].get(), d_hidx[g.vtB].get(), stream);
      timer.end(stream);
    }
    return G2OHIP_OK;
  }
  timer.begin("linearize", stream);
  for (const EGroup& g : groups)
    launch::linearize(g.family, group_args(g), g.ne, d_hidx[g.vtA].get(), d_hidx[g.vtB].get(),
                      slot_arena(g.DA) + g.slotA * (g.DA * (g.DA + 1) / 2 + g.DA),
                      slot_arena(g.DB) + g.slotB * (g.DB * (g.DB + 1) / 2 + g.DB), g.off_dst.get(), g.off_tr.get(),
                      dH.get(), doffslot.get(), stream);
  timer.end(stream);
  for (const OffRed& R : offred)
    launch::offblock_reduce(R.nb, R.bsz, R.ptr.get(), R.soff.get(), doffslot.get(), dH.get(), R.dst.get(), stream);
  timer.begin("vreduce", stream);
  launch::vertex_reduce(pd, vr_pose.nv, vr_pose.lanes, vr_pose.ptr.get(), vr_pose.code.get(), slot_arena(pd), vr_pose.H,
                        db.get(), vr_pose.boff.get(), stream);
  if (do_schur)
    launch::vertex_reduce(ld, vr_lm.nv, vr_lm.lanes, vr_lm.ptr.get(), vr_lm.code.get(), slot_arena(ld), vr_lm.H, db.get(),
                          vr_lm.boff.get(), stream);
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
  if (use_cgls()) {  // LinearSolverPCGEigen::solve on J (x for poses and landmarks at once, no Schur)
    if (sev) HIP_CHECK(hipEventRecord(ev_[1], stream));
    timer.begin("cgls", stream);
    cgls.solve(dscal.get(), db.get(), dx.get(), stream);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
    if (sev) HIP_CHECK(hipEventRecord(ev_[3], stream));
    return;
  }
  const int lm_begin = local_lm.empty() ? 0 : local_lm.front();
  const int nLloc = (int)local_lm.size();
  const double* Hpl = dH.get() + (long long)nHpp * pd * pd;
  double* S = dS.get();
  double* bschur = dS.get() + (size_t)nS * pd * pd;
  // Schur split formed at assembly: usable as is when this trial's lambda is the one it was formed with; a trial at
  // another lambda re-assembles at the same (popped) state with its lambda. Otherwise the plain passes over Hpl.
  bool split = !std::isnan(fz_lambda);
  if (split && fz_lambda != lambda_host) split = build_system_split(lambda_host) == G2OHIP_OK && !std::isnan(fz_lambda);
  if (!split) {
    timer.begin("schur_dinv", stream);
    launch::schur_prep(ld, nLloc, lm_begin, dHll.get(), db.get() + size_poses, dscal.get(), dDinv.get(), dUfac.get(),
                       dCl.get(), failp() + 1, stream);
    timer.end(stream);
    timer.begin("schur_diag", stream);
    launch::schur_diag(pd, ld, num_poses, sch_rptr.get(), sch_robs.get(), sch_obs_lm.get(), lm_begin, Hpl, dUfac.get(),
                       dCl.get(), sch_sdiag.get(), ds_hpp.get(), dH.get(), db.get(), dscal.get() + 4,
                       dist_aligned ? d_lam_own.get() : nullptr, dscal.get(), S, bschur, dG.get(), stream);
    timer.end(stream);
  }
  // the Cholesky's pre-scattered fronts are cleared by extra workgroups of the Schur pass (they are dead since the
  // last factorization), off the factorization's own chain
  const bool zero_here = !use_pcg() && chol.nzero > 0;
  timer.begin("schur_rows", stream);
  if (split && fz_kx && nsch_tasks_kx > 0) {  // Kt records in batches of their own block size
    launch::schur_rows(pd, ld, nsch_tasks_kx, sch_tasks_kx.get(), sch_batches_kx.get(), sch_st_obs_kx.get(),
                       sch_pairs_kx.get(), sch_pp_kx.get(), dG.get(), ds_hpp.get(), dH.get(), S,
                       zero_here ? chol.nzero : 0, chol.zero_rng.get(), chol.fronts.get(), stream, true, kx_sb,
                       dSchurPart.get(), sch_gmap_kx.get());
    launch::schur_part_sum(pd, nsch_groups_kx, sch_groups_kx.get(), dSchurPart.get(), ds_hpp.get(), dH.get(), S, stream);
  } else {
    launch::schur_rows(pd, ld, nsch_tasks, sch_tasks.get(), sch_batches.get(),
                       split ? sch_st_obs_h.get() : sch_st_obs.get(), sch_pairs.get(), sch_pp.get(), dG.get(),
                       ds_hpp.get(), dH.get(), S, zero_here ? chol.nzero : 0, chol.zero_rng.get(), chol.fronts.get(),
                       stream, split && fz_kx, launch::SCHUR_SB, dSchurPart.get(), sch_gmap.get());
    launch::schur_part_sum(pd, nsch_groups, sch_groups.get(), dSchurPart.get(), ds_hpp.get(), dH.get(), S, stream);
  }
  timer.end(stream);
  const bool rs = !use_pcg() && chol.rs_on;  // distributed factorization: each rank's blocks reduce-scattered to it
  if (rs) chol.reduce_input(dS.get(), stream);
  else allreduce_sum(S, (size_t)nS * pd * pd + size_poses);
  if (sev) HIP_CHECK(hipEventRecord(ev_[1], stream));
  if (use_pcg()) {
    timer.begin("pcg", stream);
    pcg.solve(S, dscal.get() + 5, bschur, dx.get(), stream);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
  } else {
    timer.begin("chol_factor", stream);
    if (rs) chol.factor(chol.rs_buf.get(), dscal.get() + 5, chol.rs_buf.get() + chol.rs_rhs_off, failp(), stream, zero_here);
    else chol.factor(S, dscal.get() + 5, bschur, failp(), stream, zero_here);
    timer.end(stream);
    if (sev) HIP_CHECK(hipEventRecord(ev_[2], stream));
    timer.begin("chol_solve", stream);
    chol.solve(dx.get(), stream);
    timer.end(stream);
  }
  if (sev) HIP_CHECK(hipEventRecord(ev_[3], stream));
  timer.begin("backsub", stream);
  // the split's back-substitution recomputes each observation's Jacobians instead of reading its 144-byte G block
  // (k_backsub_j: C5 4.58 -> 4.48 ms per iteration, profiles/r04_ab_backsub_recompute.log); G2OHIP_BACKSUB_RECOMPUTE=0
  // reads G (k_backsub_g, dev A/B)
  const char* bsr = getenv("G2OHIP_BACKSUB_RECOMPUTE");
  const bool bs_recompute = !(bsr && atoi(bsr) == 0) || fz_kx;  // Kt records: no G to read
  if (split && bs_recompute && ld == 3 && pd == 6)
    launch::backsub_j(group_args(groups[0]), nLloc, d_bs_erng.get(), d_hidx[groups[0].vtB].get(), dUfac.get(),
                      dCl.get(), size_poses, lm_begin, dx.get(), stream);
  else if (split)
    launch::backsub_g(pd, ld, nLloc, d_lm_ptr.get(), d_blk_pose.get(), dG.get(), dUfac.get(), dCl.get(), size_poses,
                      lm_begin, dx.get(), stream);
  else
    launch::backsub(pd, ld, nLloc, d_lm_ptr.get(), d_blk_pose.get(), Hpl, dDinv.get(), db.get(), size_poses, lm_begin,
                    dx.get(), stream);
  timer.end(stream);
}

int Engine::solve_sync() {
  if (!structure_built) return G2OHIP_ERR_STATE;
  solve_async(true);
  int f[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(f, failp(), sizeof f, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  timer.collect();
  if (f[0] && write_debug && rank == 0 && !use_pcg() && !use_cgls()) write_debug_dump();
  return f[0] ? 0 : 1;
}

void Engine::update_async() {  // sparse_optimizer.cpp:441-454
  timer.begin("oplus", stream);
  launch::OplusList L;
  for (int t = 1; t < NVT; ++t) {
    const int n = (int)hg.by_type[t].size();
    if (!n) continue;
    L.vt[L.cnt] = t;
    L.n[L.cnt] = n;
    L.xoff[L.cnt] = d_xoff[t].get();
    L.st[L.cnt] = dstate[t].get();
    if (t == G2OHIP_V_SE3_QUAT) L.nopl = dnopl.get();
    ++L.cnt;
  }
  launch::oplus_multi(L, dx.get(), stream);
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

int Engine::push() { return push_set_lambda(false, 0.0); }
// push (base_vertex.h:93-95 for all active vertices, a stream-ordered device copy); with_lambda: the trial's
// setLambda (set_lambda_device(lam, true)) rides in the same launch
int Engine::push_set_lambda(bool with_lambda, double lam) {
  ensure_device_state();
  if ((int)stack_.size() <= stack_depth_) stack_.emplace_back(NVT);
  auto& lvl = stack_[stack_depth_++];
  launch::CopyList cl{};
  for (int t = 1; t < NVT; ++t) {
    if (!dstate[t].size()) continue;
    lvl[t].resize(dstate[t].size());
    cl.src[cl.n] = dstate[t].get();
    cl.dst[cl.n] = lvl[t].get();
    cl.len[cl.n++] = (long long)dstate[t].size();
  }
  if (with_lambda) {
    lambda_host = lam;
    cl.sp = dscal.get();
    cl.lam = lam;
    cl.lam_rank = rank == 0 ? lam : 0.0;
  }
  launch::copy_multi(cl, stream);  // one launch for every vertex type
  return G2OHIP_OK;
}
int Engine::pop() {
  if (stack_depth_ == 0) return G2OHIP_ERR_STATE;
  auto& lvl = stack_[--stack_depth_];
  launch::CopyList cl{};
  for (int t = 1; t < NVT; ++t)
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

int Engine::diag_absmax(double* out) {  // the vertex Hessian diagonal computeLambdaInit reads (:152-175)
  if (!structure_built) return G2OHIP_ERR_STATE;
  *out = max_diagonal();
  return G2OHIP_OK;
}

double Engine::lambda_init() { return 1e-5 * max_diagonal(); }  // optimization_algorithm_levenberg.cpp:152-175

double Engine::max_diagonal() {
  if (use_cgls()) {  // JacobiSolver leaves the vertex Hessians empty: max |diag(J^T J)| (:165-172)
    cgls.diag_max(dpartial.get(), dscal.get() + 3, stream);
    double m = 0;
    HIP_CHECK(hipMemcpyAsync(&m, dscal.get() + 3, sizeof(double), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    return m;
  }
  ensure_hpp();
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
  return m;
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
  // else enqueued by the previous iteration; lambda is known from iteration 1 on (iteration 0 derives it from H)
  if (built_ver != state_ver || iteration == 0)
    build_system_split(iteration == 0 ? std::numeric_limits<double>::quiet_NaN() : current_lambda);
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
  // the next iteration's assembly depends on the trial's decision (the state it leaves, lambda in Hll + lambda I): the
  // device takes the decision itself (lm_decide, the same arithmetic), so the assembly is enqueued behind the scalar
  // readback and the GPU starts on it while the host is still waking up; a rejected trial's speculative assembly is
  // discarded (fz_lambda stays +inf: the next trial re-assembles at the popped state). Not with the stage timer on
  // (its events would be read before the speculative work ran).
  // (the not-PD dump reads S; stage timers of the assembly would be collected while the next assembly is queued)
  const bool spec = ba_fused && fz_split_ok && !timer_times_build() && !write_debug;
  bool spec_built = false, last_accept = false, last_decide_fused = false;
  do {
    push_set_lambda(true, current_lambda);  // + setLambda, which also clears the not-PD flags, in the same launch
    if (st) st->levenbergIterations++;
    const bool ev1 = st && stats_level >= 1, ev2 = st && stats_level >= 2;
    if (ev1) HIP_CHECK(hipEventRecord(e0, stream));
    solve_async(false);
    if (ev1) HIP_CHECK(hipEventRecord(e1, stream));
    update_async();
    if (ev2) HIP_CHECK(hipEventRecord(e2, stream));
    // computeScale (:177-184) on the device, sum x (lambda x + b), while lambda is still set; the
    // restoreDiagonal that follows (:113) is the next setLambda (lambda is virtual, never in H)
    // one rank, device decision: the finals and k_lm_decide in one launch (no all-reduce between them)
    const bool decide_fused = spec && nranks <= 1 && groups.size() == 1 && groups[0].family != FAM_HOSTJ;
    last_decide_fused = decide_fused;
    if (groups.size() == 1 && groups[0].family != FAM_HOSTJ) {  // chi2 and the scale sum in one pass + one final
      timer.begin("error", stream);
      const EGroup& g = groups[0];
      const launch::LmDecide dec{currentChi, (double)ni, rank == 0, hdec_dev_};
      launch::error_scale(g.family, group_args(g), g.ne, vector_size(), size_poses, dx.get(), db.get(), dscal.get(),
                          dpartial.get(), dscal.get() + 1, dscal.get() + 2, stream, decide_fused ? &dec : nullptr);
      timer.end(stream);
    } else {
      launch::scale_sum(vector_size(), size_poses, dx.get(), db.get(), dscal.get(), dpartial.get(), dscal.get() + 2,
                        stream);
      compute_errors_async(false);
    }
    // the same collectives on every rank whatever its edge groups: chi2 is per landmark shard only in Schur mode
    if (do_schur) allreduce_sum(dscal.get() + 1, 2);
    else allreduce_sum(dscal.get() + 2, 1);
    if (ev2) HIP_CHECK(hipEventRecord(e3, stream));
    if (spec && !decide_fused) launch::lm_decide(dscal.get(), currentChi, (double)ni, rank == 0, stream);
    // lambda, chi2, scale, ... | fail flags | decision: one readback per trial into pinned memory, or (one rank) written
    // to mapped host memory by the decision kernel itself
    double* hs = decide_fused ? hdec_ : hscal_;
    if (!decide_fused) HIP_CHECK(hipMemcpyAsync(hs, dscal.get(), 16 * sizeof(double), hipMemcpyDeviceToHost, stream));
    if (spec) {
      HIP_CHECK(hipEventRecord(rb_ev_, stream));
      build_system_split(std::numeric_limits<double>::quiet_NaN(), dscal.get() + 12);
      spec_built = true;
      HIP_CHECK(hipEventSynchronize(rb_ev_));
    } else {
      HIP_CHECK(hipStreamSynchronize(stream));
    }
    timer.collect();
    tempChi = hs[1];
    int f[2];
    std::memcpy(f, hs + 8, sizeof f);
    const bool ok2 = f[0] == 0;
    if (!ok2 && write_debug && rank == 0 && !use_pcg() && !use_cgls()) write_debug_dump();
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
    bool accept;
    if (spec) {  // the device's decision (k_lm_decide restates the branch below)
      rho = hs[15];
      accept = hs[14] != 0.0;
      current_lambda = hs[12];
    } else {
      rho = currentChi - tempChi;
      double scale = hs[2];
      scale += 1e-3;
      rho /= scale;
      accept = rho > 0 && std::isfinite(tempChi);
      if (accept) {
        current_lambda *= lm_scale_factor(rho);  // optimization_algorithm_levenberg.cpp:127-136
      } else {
        current_lambda *= ni;
      }
    }
    last_accept = accept;
    if (accept) {
      ni = 2;
      currentChi = tempChi;
      discard_top();
    } else {
      ni *= 2;
      pop();
      if (!std::isfinite(current_lambda)) break;
    }
    qmax++;
  } while (rho < 0 && qmax < maxTrials);
  // restoreDiagonal of the last trial (block_solver.hpp:552-565); after an accepted trial whose decision ran in
  // k_sum_final2_decide the device has done it already
  if (last_decide_fused && last_accept) lambda_host = 0.0;
  else set_lambda_device(0.0);
  // the state left behind has chi2 currentChi (accepted: the last tempChi; rejected: popped back)
  chi_cache = currentChi;
  chi_ver = state_ver;
  // the next iteration starts with buildSystem on exactly this state: enqueue it now so the GPU works
  // while the host returns to the caller (skipped when the loop is about to stop)
  const bool more = !(qmax == maxTrials || rho == 0 || !std::isfinite(current_lambda));
  if (spec_built && last_accept) {  // the last trial was accepted: its speculative assembly is this state's, at this lambda
    fz_lambda = current_lambda;
    built_ver = state_ver;
  } else if (more) {
    build_system_split(current_lambda);
    built_ver = state_ver;
  }
  if (qmax == maxTrials || rho == 0 || !std::isfinite(current_lambda)) return 1;  // Terminate
  return 0;                                                                       // OK
}

// OptimizationAlgorithmGaussNewton::solve (optimization_algorithm_gauss_newton.cpp:50-92): errors, buildStructure on
// iteration 0, buildSystem, solve (no damping: lambda 0), update with whatever x the solve left, Fail on not-PD
int Engine::gn_solve(int iteration, g2ohip_batch_stats* st) {
  double t = wall();
  chi2_sync();  // computeActiveErrors (:56)
  if (st) st->timeResiduals = wall() - t;
  if (iteration == 0 && !structure_built) {
    if (build_structure()) return 2;
  }
  t = wall();
  if (built_ver != state_ver || iteration == 0) build_system();
  built_ver = 0;
  if (st && stats_level >= 2) {
    HIP_CHECK(hipStreamSynchronize(stream));
    st->timeQuadraticForm = wall() - t;
  }
  set_lambda_device(0.0, true);  // also clears the not-PD flags
  const bool ev1 = st && stats_level >= 1;
  if (ev1) HIP_CHECK(hipEventRecord(lm_ev_[0], stream));
  solve_async(false);
  if (ev1) HIP_CHECK(hipEventRecord(lm_ev_[1], stream));
  update_async();
  if (ev1) HIP_CHECK(hipEventRecord(lm_ev_[2], stream));
  int f[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(f, failp(), sizeof f, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  timer.collect();
  if (ev1) {
    float a = 0, b = 0;
    HIP_CHECK(hipEventElapsedTime(&a, lm_ev_[0], lm_ev_[1]));
    HIP_CHECK(hipEventElapsedTime(&b, lm_ev_[1], lm_ev_[2]));
    st->timeLinearSolution = a * 1e-3;
    st->timeUpdate = b * 1e-3;
  }
  levenberg_iterations = 0;
  if (f[0] != 0 && write_debug && rank == 0 && !use_pcg() && !use_cgls()) write_debug_dump();
  return f[0] == 0 ? 0 : 2;
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
    st->numEdges = (int)hg.num_edges();
    st->numVertices = (int)active.size();
  }
  const double ts = wall();
  const int result = levenberg ? lm_solve(i, cfg, st) : gn_solve(i, st);
  if (st || cfg.verbose) {
    const double c = chi2_sync();
    if (st) {
      st->chi2 = c;
      st->lambda = levenberg ? current_lambda : 0.0;
      st->timeIteration = wall() - ts;
      st->hessianPoseDimension = size_poses;
      st->hessianLandmarkDimension = size_landmarks;
      st->hessianDimension = size_poses + size_landmarks;
      st->choleskyNNZ = (long long)chol.sym.nnzL;
    }
    if (cfg.verbose && rank == 0)
      fprintf(stderr, "iteration= %d\t chi2= %.6f\t time= %g\t edges= %zu\t lambda= %.6f\t levenbergIter= %d\n", i, c,
              wall() - ts, (size_t)hg.num_edges(), current_lambda, levenberg_iterations);
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
  {  // G2OHIP_STAGE_SPLIT=1 (tests): stage through the Schur split formed at assembly, as the LM loop does
    const char* ev = getenv("G2OHIP_STAGE_SPLIT");
    if (ev && atoi(ev) == 1) build_system_split(lambda);
    else build_system();
  }
  set_lambda(lambda, 1);
  const int ok = solve_sync();
  // the distributed factorization reduce-scatters S (dS keeps this rank's partial sums): the whole reduced system
  // for the caller takes one more all-reduce (every rank calls stage, as it calls every other collective step)
  if ((Hs || bs) && do_schur && chol.rs_on) allreduce_sum(dS.get(), (size_t)nS * pd * pd + size_poses);
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

void BlockSymv::setup(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj, hipStream_t s) {
  nb = nblocks;
  pd = bdim;
  std::vector<int> dg(nb, -1), cnt(nb + 1, 0);
  for (size_t t = 0; t < bi.size(); ++t) {
    if (bi[t] == bj[t]) dg[bi[t]] = (int)t;
    else { ++cnt[bi[t] + 1]; ++cnt[bj[t] + 1]; }
  }
  for (int i = 0; i < nb; ++i) {
    if (dg[i] < 0) throw std::runtime_error("BlockSymv: missing diagonal block " + std::to_string(i));
    cnt[i + 1] += cnt[i];
  }
  std::vector<int2> e(std::max(cnt[nb], 1), make_int2(0, 0));
  std::vector<int> fill(cnt.begin(), cnt.end() - 1);
  for (size_t t = 0; t < bi.size(); ++t) {  // stored order: a fixed summation order per row
    if (bi[t] == bj[t]) continue;
    e[fill[bi[t]]++] = make_int2((int)t, bj[t]);
    e[fill[bj[t]]++] = make_int2((int)t, (int)((unsigned)bi[t] | 0x80000000u));
  }
  rptr.upload(cnt, s);
  diag.upload(dg, s);
  ent.upload(e, s);
}

int Engine::multiply_hessian(double* dest, const double* src) {  // block_solver.h:146
  if (!structure_built) return G2OHIP_ERR_STATE;
  if (nranks > 1) return G2OHIP_ERR_UNSUPPORTED;  // Hpp diagonal blocks are partial per landmark shard
  ensure_hpp();
  if (symv_hpp.key != structure_ver) {
    symv_hpp.setup(num_poses, pd, hpp_bi, hpp_bj, stream);
    symv_hpp.key = structure_ver;
  }
  const int n = size_poses;
  dtmp.resize(2 * (size_t)std::max(n, 1));
  HIP_CHECK(hipMemcpyAsync(dtmp.get(), src, sizeof(double) * n, hipMemcpyHostToDevice, stream));
  launch::block_symv(pd, n, symv_hpp.rptr.get(), symv_hpp.ent.get(), symv_hpp.diag.get(), dH.get(),
                     lambda_set ? dscal.get() : nullptr, dtmp.get(), dtmp.get() + n, nullptr, nullptr, nullptr, stream);
  HIP_CHECK(hipMemcpyAsync(dest, dtmp.get() + n, sizeof(double) * n, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  return G2OHIP_OK;
}

int Engine::linear_residual(double* out) {
  if (!structure_built || !out) return G2OHIP_ERR_STATE;
  // the iterative solvers never form the factorized system: PCG keeps no residual here, CGLS never assembles S
  if (use_pcg() || use_cgls()) return G2OHIP_ERR_UNSUPPORTED;
  const std::vector<int>& bi = do_schur ? s_bi : hpp_bi;
  const std::vector<int>& bj = do_schur ? s_bj : hpp_bj;
  BlockSymv& M = do_schur ? symv_s : symv_hpp;
  if (M.key != structure_ver) {
    M.setup(num_poses, pd, bi, bj, stream);
    M.key = structure_ver;
  }
  const int n = size_poses;
  // S already holds lambda on its diagonal (k_schur_diag); Hpp gets the virtual lambda like the factor
  const double* vals = do_schur ? dS.get() : dH.get();
  const double* lam = do_schur ? nullptr : dscal.get();
  const double* rhs = do_schur ? dS.get() + (size_t)nS * pd * pd : db.get();
  if (do_schur && chol.rs_on) {
    // the distributed factorization reduce-scattered S: dS holds this rank's partial sums only, so the residual is
    // taken against an all-reduced copy (a collective: every rank calls linear_residual, as it calls solve)
    const size_t len = (size_t)nS * pd * pd + size_poses;
    dsfull.resize(len);
    HIP_CHECK(hipMemcpyAsync(dsfull.get(), dS.get(), len * sizeof(double), hipMemcpyDeviceToDevice, stream));
    allreduce_sum(dsfull.get(), len);
    vals = dsfull.get();
    rhs = vals + (size_t)nS * pd * pd;
  }
  dtmp.resize(2 * (size_t)std::max(n, 1) + 2);
  launch::block_symv(pd, n, M.rptr.get(), M.ent.get(), M.diag.get(), vals, lam, dx.get(), nullptr, rhs, dtmp.get(),
                     dtmp.get() + n, stream);
  double* res = dtmp.get() + 2 * (size_t)n;
  launch::sum(dtmp.get(), n, dpartial.get(), res, stream);
  launch::sum(dtmp.get() + n, n, dpartial.get(), res + 1, stream);
  double h[2];
  HIP_CHECK(hipMemcpyAsync(h, res, sizeof h, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  *out = h[1] > 0 ? std::sqrt(h[0] / h[1]) : std::sqrt(h[0]);
  return G2OHIP_OK;
}

int Engine::compute_marginals(int nblocks, const int* brow, const int* bcol, double* out) {
  if (!structure_built) return G2OHIP_ERR_STATE;
  if (nranks > 1) return G2OHIP_ERR_UNSUPPORTED;  // Hpp diagonal blocks are partial per landmark shard
  if (nblocks < 0 || (nblocks && (!brow || !bcol || !out))) return G2OHIP_ERR_ARG;
  for (int k = 0; k < nblocks; ++k)
    if (brow[k] < 0 || brow[k] >= num_poses || bcol[k] < 0 || bcol[k] >= num_poses) return G2OHIP_ERR_ARG;
  ensure_hpp();
  // the LM's own factor is reused where it factors Hpp; otherwise (Schur complement, iterative solvers) a
  // factor of Hpp's pattern is set up once
  const bool own = !do_schur && !use_pcg() && !use_cgls();
  DeviceCholesky& C = own ? chol : marg_chol;
  if (!own && marg_ver != structure_ver) {
    marg_chol.set_replicated();
    marg_chol.setup(num_poses, pd, hpp_bi, hpp_bj, stream);
    marg_ver = structure_ver;
  }
  const int n = size_poses, K = 64 / pd * pd, bpb = K / pd;
  dmarg.resize((size_t)2 * n * K + (size_t)C.wpool + n);
  double* Y = dmarg.get();
  double* T = Y + (size_t)n * K;
  double* W = T + (size_t)n * K;
  double* zrhs = W + C.wpool;
  dmarg_fail.resize(1);
  dmarg_fail.zero(stream);
  HIP_CHECK(hipMemsetAsync(zrhs, 0, sizeof(double) * n, stream));
  // Hpp + 0 I (dscal[5] holds 0): the reference factors Hpp as buildSystem left it, lambda removed
  C.factor(dH.get(), dscal.get() + 5, zrhs, dmarg_fail.get(), stream);
  int fail = 0;
  HIP_CHECK(hipMemcpyAsync(&fail, dmarg_fail.get(), sizeof fail, hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  if (fail) return 0;
  // distinct block columns, batched K / pd per multi-right-hand-side solve
  std::vector<int> ucol(bcol, bcol + nblocks);
  std::sort(ucol.begin(), ucol.end());
  ucol.erase(std::unique(ucol.begin(), ucol.end()), ucol.end());
  const std::vector<int>& pinv = C.sym.pinv;
  const size_t bsz = (size_t)pd * pd;
  std::vector<int> prow(K);
  std::vector<long long> idx;
  std::vector<double> vals;
  for (size_t b0 = 0; b0 < ucol.size(); b0 += bpb) {
    const int nb = (int)std::min<size_t>(bpb, ucol.size() - b0), k = nb * pd;
    for (int c = 0; c < nb; ++c)
      for (int j = 0; j < pd; ++j) prow[c * pd + j] = pinv[ucol[b0 + c] * pd + j];
    HIP_CHECK(hipMemsetAsync(Y, 0, sizeof(double) * n * k, stream));
    dmarg_idx.resize(std::max<size_t>((size_t)k, bsz * nblocks));
    HIP_CHECK(hipMemcpyAsync(dmarg_idx.get(), prow.data(), sizeof(int) * k, hipMemcpyHostToDevice, stream));
    launch::marg_unit(k, reinterpret_cast<const int*>(dmarg_idx.get()), Y, n, stream);
    C.solve_multi(Y, W, T, k, stream);
    // entry (i, j) of block (r, c): Y(pinv[r pd + i], column of c's j)
    idx.clear();
    std::vector<int> which;
    for (int q = 0; q < nblocks; ++q) {
      const size_t pos = std::lower_bound(ucol.begin() + b0, ucol.begin() + b0 + nb, bcol[q]) - ucol.begin();
      if (pos >= b0 + nb || ucol[pos] != bcol[q]) continue;
      which.push_back(q);
      const int c = (int)(pos - b0);
      for (int j = 0; j < pd; ++j)
        for (int i = 0; i < pd; ++i) idx.push_back((long long)(c * pd + j) * n + pinv[brow[q] * pd + i]);
    }
    if (idx.empty()) continue;
    HIP_CHECK(hipStreamSynchronize(stream));  // dmarg_idx held the unit rows until marg_unit ran
    HIP_CHECK(hipMemcpyAsync(dmarg_idx.get(), idx.data(), sizeof(long long) * idx.size(), hipMemcpyHostToDevice, stream));
    dmarg_out.resize(idx.size());
    launch::marg_gather((long long)idx.size(), dmarg_idx.get(), Y, dmarg_out.get(), stream);
    vals.resize(idx.size());
    HIP_CHECK(hipMemcpyAsync(vals.data(), dmarg_out.get(), sizeof(double) * idx.size(), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    for (size_t w = 0; w < which.size(); ++w)
      std::copy(vals.begin() + w * bsz, vals.begin() + (w + 1) * bsz, out + (size_t)which[w] * bsz);
  }
  return 1;
}

int Engine::factor_info(double* out, int n) {
  if (!structure_built) return G2OHIP_ERR_STATE;
  const Symbolic& S = chol.sym;
  const double v[] = {(double)S.n, (double)S.nnzL, S.flops, (double)S.sn.size(), (double)S.num_levels,
                      (double)S.max_front, (double)chol.n_blocked, (double)chol.n_inplace_levels,
                      (double)chol.n_pre_levels, (double)chol.n_syrk_ops, (double)chol.n_bwd_rounds,
                      0.0 /* retired: tile-DAG levels */, (double)chol.n_owned_fronts, (double)chol.n_shared_fronts,
                      (double)chol.n_roots, (double)chol.xch_len, chol.dist_model[0], chol.dist_model[1],
                      chol.dist_model[2], chol.dist_model[3], chol.dist_model[4], chol.rs_on ? 1.0 : 0.0,
                      (double)chol.rs_seg, (double)chol.rs_tail_len, chol.rs_model[0], chol.rs_model[1],
                      0.0 /* retired: 64-column-step levels */, (double)S.band_leaf, dist_aligned ? 1.0 : 0.0,
                      (double)chol.rs_local, exchange_bytes(), (double)local_lm.size(), chol.shard_model,
                      (double)chol.n_deferred_l21};
  const int m = (int)(sizeof v / sizeof v[0]);
  for (int k = 0; k < std::min(n, m); ++k) out[k] = v[k];
  return m;
}

// Bytes this rank sends per LM trial through the collectives of the reduced system and its factorization (ring
// algorithms: a reduce-scatter or all-gather of N segments sends N-1 of them, an all-reduce 2 (N-1)/N of the buffer),
// the scalar reductions aside
double Engine::exchange_bytes() const {
  if (nranks <= 1 || !do_schur || !comm) return 0.0;
  const double N = nranks, ar = 2.0 * (N - 1) / N;
  if (!chol.distributed()) return 8.0 * ar * ((double)nS * pd * pd + size_poses);
  double b = 8.0 * (N - 1) * (double)chol.xch_seg + 8.0 * ar * (chol.sym.n + 1.0);  // root all-gather, x
  if (chol.rs_on) b += 8.0 * (N - 1) * (double)chol.rs_seg + 8.0 * ar * (double)chol.rs_tail_len;
  else b += 8.0 * ar * ((double)nS * pd * pd + size_poses);
  return b;
}

int Engine::local_landmarks(int* ids, int cap) const {
  const int n = (int)local_lm.size();
  if (ids)
    for (int k = 0; k < n && k < cap; ++k) ids[k] = hg.verts[ivmap[num_poses + local_lm[k]]].id;
  return n;
}

double Engine::kernel_bytes(const std::string& name) const {
  // algorithmic bytes per launch (SURVEY.md §8d formulas)
  const double npl = nHpl, pb = (double)pd * ld * 8;
  // the BA split's per-observation record: the 80-byte Kt record instead of the G block (assembly.hip KXB)
  const double ob = fz_kx ? 80.0 : pb;
  // Schur row pass (off-diagonal blocks): G (or its Kt record) of every observation once, the off-diagonal Hpp blocks
  // present in S, the off-diagonal S blocks written once
  if (name == "schur_rows") return npl * ob + (double)(nHppUsed - num_poses) * pd * pd * 8 +
                                   (double)(nS - num_poses) * pd * pd * 8;
  // diagonal blocks: Hpl, U and c per observation's landmark, G written, Hpp diagonal, S diagonal + bschur
  if (name == "schur_diag") return 2 * npl * pb + local_lm.size() * 9 * 8.0 + (double)num_poses * pd * pd * 8 * 2 +
                                   size_poses * 16.0;
  if (name == "schur_dinv") return local_lm.size() * ((9 + 3) * 8.0 + (9 + 6 + 3) * 8.0);
  if (name == "linearize") {  // BA groups: edge data read, the Hpl block written (+ both slots, generic path)
    double by = 0;
    for (const EGroup& g : groups)
      if (g.family == FAM_BA)
        by += g.ne * ((2 + 3 + 4) * 8.0 + 8 + (ba_fused ? 0.0 : 9.0 + 27.0) * 8 + ob) +
              (ba_fused ? local_lm.size() * 12 * 8.0 : 0.0);
    return by;
  }
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
