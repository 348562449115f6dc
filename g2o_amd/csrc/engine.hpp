// Host side of the MI355X BlockSolver backend: graph mirror, structure, LM driver.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/g2o_hip.h"
#include "comm.hpp"
#include "common.hpp"
#include "kernels.hpp"
#include "cgls.hpp"
#include "pcg.hpp"
#include "symbolic.hpp"

namespace g2ohip {

constexpr int NVT = 6;  // vertex type codes 1..5 (G2OHIP_V_*)
int vertex_dim(int vtype);
int vertex_est_dim(int vtype);
int vertex_state_stride(int vtype);
int edge_dim(int etype);
int edge_meas_dim(int etype);

// OptimizableGraph mirror (host, authoritative for I/O; the device copy is authoritative
// during optimize()).
struct HVertex {
  int id, type, dim;
  bool fixed, marg;
  int local;  // index within its type's state array
};

// one edge type of the graph (edges kept in insertion order)
struct HEdgeSet {
  int type = 0, D = 0, nm = 0;          // G2OHIP_E_*, error dimension, measurement doubles per edge
  std::vector<int> ev0, ev1;            // vertex indices
  std::vector<double> meas, info, params;  // raw: meas (as given), info D*D row-major, params 4
  int rk = 0;                           // robust kernel (G2OHIP_RK_*), delta
  double rk_delta = 1.0;
  std::vector<double> payload;          // host-J edges: latest [e | Ji | Jj] per edge from the host
  unsigned long long payload_ver = 0;   // device-state version the payload was computed at (0: set by the caller)
};

struct HostGraph {
  std::vector<HVertex> verts;
  std::unordered_map<int, int> idmap;
  std::vector<double> st[NVT];            // per type, device layout
  std::vector<std::vector<int>> by_type = std::vector<std::vector<int>>(NVT);  // local -> vertex
  std::vector<int> nopl;                // VertexSE3 oplus counters (per local SE3QUAT vertex)
  std::vector<HEdgeSet> esets;          // in first-seen type order
  long long num_edges() const {
    long long n = 0;
    for (auto& e : esets) n += (long long)e.ev0.size();
    return n;
  }
  HEdgeSet* set_of(int type) {
    for (auto& e : esets) if (e.type == type) return &e;
    return nullptr;
  }
};

// A device edge group: the local-shard edges of one edge set with one pair of endpoint vertex types,
// linearized by one kernel instantiation (family, D, DA, DB)
struct EGroup {
  int set = 0, family = 0, vtA = 0, vtB = 0, D = 0, DA = 0, DB = 0;
  std::vector<int> edges;               // indices into the edge set
  int ne = 0;
  DevBuf<int> v0, v1;                   // local vertex indices (per type)
  DevBuf<double> meas, info, params;    // meas: family payload (host-J: [e | Ji | Jj] per edge)
  int ue = 0;                           // info / params stored as one shared record (bit 0 / bit 1): all edges equal
  long long slotA = 0, slotB = 0;       // first slot of the group's A / B sides in the arenas of dims DA / DB
  DevBuf<long long> off_dst;            // per edge: offset of its off-diagonal block (bit 62: a shared-block slot)
  DevBuf<unsigned char> off_tr;
  int payload_stride() const { return D + D * DA + D * DB; }
};

void set_state_from_est(int vtype, const double* est, double* st);
void est_from_state(int vtype, const double* st, double* est);
void minimal_from_state(int vtype, const double* st, double* out);

// Device-resident multifrontal factor of one block-sparse SPD matrix.
struct DeviceCholesky {
  Symbolic sym;
  int pd = 0;
  long long nent = 0;
  DevBuf<int> colptr, ent_row, ent_src;  // input entries per permuted scalar column (k_extend_add)
  DevBuf<int> jtab;                       // per child: row ranges per parent slab (FrontDesc::jt_off)
  DevBuf<int> cmptr;                      // per front column: range of (child, child column) pairs
  DevBuf<longlong2> cment;  // per (front column, child column): U column, child relmap | jc << 32 | nr << 48
  long long npre = 0;                     // entries of pre-scattered (small-level) fronts
  long long npre_first = 0;               // of them scattered before the first level (the rest: deferred, see factor)
  int n_deferred_levels = 0;              // levels whose entries ride in the previous level's first step launch
  DevBuf<long long> pre_dst, zero_rng;
  DevBuf<int> pre_src;
  int nzero = 0;
  DevBuf<launch::FrontDesc> fd;
  DevBuf<int> children, relmap, rows, perm;
  std::vector<int> level_off;  // host offsets of each level's fronts in the level order
  std::vector<int> bwd_off;    // per level: offset of its backward-gemv tasks in `tasks` (+1 end)
  struct BwdLevel {            // backward solve of one level: (offset, count) task ranges in `tasks`
    std::pair<int, int> gemv, xall;
    std::vector<std::pair<std::pair<int, int>, std::pair<int, int>>> rounds;  // blocked fronts: (inner, x)
    bool t_is_y = false;  // every front of the level is a root (no rows below its columns): t = y, no gemv launch
  };
  std::vector<BwdLevel> bwd_ops;
  int max_ns = 0;
  int syrk_var = 4;  // the k_syrk tile variant the task lists were built for (G2OHIP_SYRK_DMA at setup)
  // schedule summary (g2ohip_solver_factor_info): blocked fronts, levels assembled in place / pre-scattered,
  // trailing-update (k_syrk) launches, big-panel backward rounds
  int n_blocked = 0, n_inplace_levels = 0, n_pre_levels = 0, n_syrk_ops = 0, n_bwd_rounds = 0;
  int n_deferred_l21 = 0;  // fronts whose L21 comes from the k_l21 GEMM after their panel steps
  struct Op { int kind, off, count; long long sc0 = 0, sc1 = 0; int b0 = 0, nb0 = 0; };  // b0/nb0: extend-add block-0 records  // sc: deferred scatter range (extend-add ops)  // kind 0 extend-add (pre-scattered level), 4 / 5 assembly + extend-add,
                                        // 2 panel step (6: with lagged-pair tasks), 3 syrk, 8 root exchange
  // ---- distributed factorization (landmark-sharded BA). Set dist_rank / dist_nranks / allreduce before
  // setup. The elimination tree is cut: every front below the cut belongs to one rank (whole subtrees, balanced by
  // modelled time), the fronts above it are factored by every rank. A rank factors its subtrees, the subtree roots'
  // contribution blocks and update vectors meet in one all-gather (each rank's roots in its own segment), every rank
  // factors the top; the backward solve runs top-down the same way and x meets in one all-reduce (with the not-PD
  // flag).
  int dist_rank = 0, dist_nranks = 1;
  std::function<void(double*, size_t)> allreduce;
  std::function<void(double*, size_t)> allgather;  // in place: nranks segments of `count` doubles
  std::vector<int> sn_owner;                 // per supernode: owning rank, -1 shared (every rank)
  int n_owned_fronts = 0, n_shared_fronts = 0, n_roots = 0;
  bool dist_on = false;                      // setup chose a cut (the model beat the replicated factorization, or forced)
  bool dist_force = false;                   // take the best cut even when the model prefers replication
  double dist_model[5] = {0, 0, 0, 0, 0};    // modelled seconds: this rank's subtrees, the shared top, replicated
                                             // factorization, the two all-reduces of the cut; 1 if distributed
  long long xch_len = 0, xch_seg = 0;         // doubles of the root exchange (nranks segments of xch_seg)
  int xch_pack_f = 0, xch_pack_v = 0, xch_unpack_f = 0, xch_unpack_v = 0;
  DevBuf<long long> xch_ranges;               // (src, dst, len): pack fronts | pack vecs | unpack fronts | unpack vecs
  DevBuf<double> xch_buf, xred;
  DevBuf<int> xzero_idx;                      // caller-order indices of the shared columns (zeroed on ranks != 0)
  int nxzero = 0;
  int* last_fail = nullptr;
  bool distributed() const { return dist_on; }
  // reduce-scatter of the input (distributed only, rs_enable set by the caller before setup): the reduced system's
  // blocks are packed by the rank whose subtrees read them — [rank 0's blocks | ... | rank N-1's (each segment padded to
  // rs_seg doubles) | shared blocks + rhs] — one reduce-scatter sums each rank's own segment, one all-reduce the tail;
  // the factor reads its entries from rs_buf (ent_src remapped), never another rank's segment
  bool rs_enable = false, rs_on = false;
  // landmark shards aligned with the cut (Engine::align_shards, set before setup): the plan's input model counts only
  // the shared tail, and blk_local (per input block) marks the blocks whose only writer is the rank that reads them —
  // read from the rank's own partial S, never exchanged
  bool aligned = false;
  std::vector<unsigned char> blk_local;
  std::vector<double> pose_work;              // per pose block: the sharded work the cut's model weighs (optional)
  // analysis already made for this pattern (Engine::align_shards plans the cut before the landmarks are placed): setup
  // takes them instead of analysing again; both are consumed (reset) by the next setup
  std::shared_ptr<const Symbolic> pre_sym;
  std::shared_ptr<const DistPlan> pre_plan;
  double shard_model = 0;                     // modelled busiest rank's sharded work (s) of the chosen layout
  long long rs_local = 0;                     // doubles of this rank's own complete blocks (rs_buf's last region)
  // a factorization of the whole system on this rank alone (pose graphs, computeMarginals' Hpp factor): clears any
  // distribution state an earlier sharded setup of the same object left behind
  void set_replicated() {
    dist_rank = 0;
    dist_nranks = 1;
    dist_force = false;
    rs_enable = false;
    aligned = false;
    blk_local.clear();
    pose_work.clear();
  }
  std::function<void(double*, size_t)> reduce_scatter;  // in place, `count` doubles per rank
  long long rs_seg = 0, rs_tail_len = 0, rs_rhs_off = 0, rs_nblk = 0;
  double rs_model[2] = {0, 0};                // modelled seconds: reduce-scatter + tail all-reduce, full all-reduce
  DevBuf<long long> rs_bmap;                  // per input block: its offset in rs_buf
  DevBuf<long long> rs_rhs_rng;               // (src, dst, len) of the rhs
  DevBuf<double> rs_buf;
  // pack this rank's partial [blocks | rhs] (the caller's layout) and reduce; factor(rs_buf, ..., rs_buf + rs_rhs_off)
  void reduce_input(const double* vals, hipStream_t s);
  std::vector<Op> ops;
  std::vector<launch::StepHead> heads;  // per op: its leading next-diagonal tasks (k_step kernel arguments)
  std::vector<launch::ScatterJob> ea_jobs;  // per extend-add op: its leading block-0 fronts (kernel arguments)
  DevBuf<launch::B0Front> b0front;          // per extend-add op (Op::b0): its fronts' block-0 records
  DevBuf<launch::B0Child> b0child;          // parallel to `children`: each child's record for its parent's block 0
  DevBuf<launch::Task> tasks;
  DevBuf<launch::StepTask> step_tasks;
  DevBuf<double> fronts, vecs, rhs_p, y_p, x_p, t_p, lbuf, linv, xinv;
  long long lpool = 0;
  void setup(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj, hipStream_t s);
  // numeric LL^T fused with the forward solve of rhs (y = L^-1 P rhs)
  // prezeroed: the pre-scattered fronts were already cleared (zero_rng, nzero) by the caller's Schur pass
  void factor(const double* vals, const double* lam, const double* rhs, int* fail, hipStream_t s, bool prezeroed = false);
  // backward solve x = P^T L^-T y
  void solve(double* x, hipStream_t s);
  // multi-right-hand-side solve with the factor in lbuf/linv (marginals.hip): Y (n x K, column-major, rows in
  // the permuted order) <- L^-T L^-1 Y; W (wpool x 64) and T (n x K) scratch, K <= 64
  DevBuf<int> lfronts;          // fronts in level order (level_off ranges)
  DevBuf<long long> woff;       // per front: offset of its below-diagonal right-hand-side block in W
  long long wpool = 0;
  void solve_multi(double* Y, double* W, double* T, int K, hipStream_t s);
};

// y = (A + lam I) x for a symmetric block matrix held as upper blocks (multiplyHessian, residual checks)
struct BlockSymv {
  int nb = 0, pd = 0;
  unsigned long long key = 0;  // Engine::structure_ver it was built for (0: never)
  DevBuf<int> rptr, diag;
  DevBuf<int2> ent;
  void setup(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj, hipStream_t s);
};

struct KernelTimer {
  bool enabled = false;
  std::string only;    // time only this kernel class (empty: all)
  bool open_ = false;  // a begin() whose end() is pending
  struct Rec { hipEvent_t a, b; std::string name; };
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;
  std::map<std::string, double> total_ms;
  std::map<std::string, long long> count;
  hipEvent_t get();
  void begin(const std::string& name, hipStream_t s);
  void end(hipStream_t s);
  void collect();  // after a sync
  void reset() { total_ms.clear(); count.clear(); }
  ~KernelTimer();
};

class Engine {
 public:
  explicit Engine(int device);
  ~Engine();
  HostGraph hg;
  int device;
  hipStream_t stream = nullptr;
  std::string algorithm = "lm_hip_var";
  // G2OBatchStatistics timers: 0 none, 1 timeLinearSolution only (2 events per trial), 2 every stage
  int stats_level = 2;
  bool levenberg = true;

  // ---- graph ops ----
  int add_vertices(int type, int n, const int* ids, const double* est, const int* fixed, const int* marg);
  int add_edges(int type, int n, const int* v0, const int* v1, const double* meas, const double* info,
                const double* params);
  // RobustKernel per edge type (base_edge.h setRobustKernel; uniform kind and delta over the type)
  int set_robust_kernel(int type, int kind, double delta);
  // host-J edges: error + Jacobians of every edge of the type (insertion order), [e | Ji | Jj] row-major
  int set_host_payload(int type, const double* payload);
  // host callback that recomputes a host-J type's payload at the current estimates (device LM loop, chi2)
  int set_host_callback(g2ohip_host_edge_fn fn, void* user);
  // computeLambdaInit (optimization_algorithm_levenberg.cpp:152-175): max |diagonal| of Hpp and Hll
  int diag_absmax(double* out);
  int load(const char* path, int marginalize_xyz);
  int save(const char* path);
  // doubles of the host payload of a host-J edge type ([e | Ji | Jj] per edge, insertion order)
  long long host_payload_len(int type);
  // Solver::saveHessian (block_solver.hpp:589-593 -> SparseBlockMatrix::writeOctave, sparse_block_matrix.hpp:579-617)
  int save_hessian(const char* path);
  // Solver::setWriteDebug (block_solver.hpp:582-586): on a not-PD factorization the LM trial writes debug.txt
  // (linear_solver_csparse.h:127-133, csparse_helper.cpp:62-111)
  bool write_debug = false;
  std::string debug_path = "debug.txt";
  int get_estimates(int type, double* out, int* ids);
  int set_estimates(int type, const double* est);
  int minimal_state(double* out);

  // ---- SparseOptimizer / Solver ----
  int initialize();
  // SparseOptimizer::updateInitialization + BlockSolver::updateStructure (online mode, non-Schur): vertices and edges
  // added after initialize() join with appended hessian indices; the existing vertices keep theirs
  int update_initialization();
  double chi2();
  int optimize(const g2ohip_config* cfg, int iterations, g2ohip_batch_stats* stats);
  // one SparseOptimizer::optimize loop body (iteration 0 rebuilds structure + lambda init);
  // returns 0 OK, 1 Terminate, 2 Fail, <0 error
  int optimize_step(const g2ohip_config* cfg, int iteration, g2ohip_batch_stats* stats);
  int build_structure();
  int build_system();
  // buildSystem with lambda known (the LM loop): where eligible the landmark side of the Schur complement is formed
  // during assembly (kernels.hpp SchurSplit); solve_async re-assembles when a trial's lambda differs
  // lamp (optional): the split's lambda pair read from the device (dscal[12..13], written by lm_decide) — the next
  // iteration's assembly enqueued before the host has read the trial's decision (fz_lambda stays NaN until it has)
  int build_system_split(double lambda, const double* lamp = nullptr);
  int set_lambda(double lambda, int backup);
  int restore_diagonal();
  int solve_sync();  // 1 ok / 0 not PD
  long long vector_size() const { return (long long)size_poses + size_landmarks; }
  int get_x(double* x);
  int get_b(double* b);
  int update_from(const double* xh);
  int push();
  int push_set_lambda(bool with_lambda, double lam);
  int pop();
  int discard_top();
  int stage(double lambda, double* b, double* x, double* Hs, double* bs, long long* dims);
  // BlockSolverBase::multiplyHessian (block_solver.h:94,146): dest = Hpp src (upper blocks mirrored, + lambda
  // while setLambda is active), host arrays of size_poses
  int multiply_hessian(double* dest, const double* src);
  // ||(A + lambda I) x - b|| / ||b|| of the last linear solve (A = Schur complement S or Hpp), on the device
  int linear_residual(double* out);
  // [n, nnz(L), flops, supernodes, levels, max front, blocked fronts, in-place levels, pre-scattered levels,
  //  k_syrk launches, backward big-panel rounds]
  int factor_info(double* out, int n);
  int block_dims(int* dims) const {
    if (!structure_built) return G2OHIP_ERR_STATE;
    dims[0] = pd; dims[1] = ld; dims[2] = num_poses; dims[3] = num_landmarks;
    return G2OHIP_OK;
  }
  // Solver::computeMarginals (block_solver.hpp:451 -> solvePattern, linear_solver_csparse.h:190-225): the pd x pd
  // blocks (rows[k], cols[k]) of Hpp^-1 (Hpp of the last buildSystem, no lambda), column-major, into out;
  // 1 done, 0 Hpp not positive definite (the reference's bool), < 0 a status code
  int compute_marginals(int nblocks, const int* rows, const int* cols, double* out);

  // comm
  int set_comm(const unsigned char* uid, int rank, int nranks);
  int set_comm_local(const std::string& key, int rank, int nranks);
  KernelTimer timer;
  double kernel_bytes(const std::string& name) const;
  double exchange_bytes() const;
  // ids of the free landmarks this rank's shard holds (landmark-sharded BA); returns the count
  int local_landmarks(int* ids, int cap) const;
  double kernel_flops(const std::string& name) const;

 private:
  // structure
  bool initialized = false, structure_built = false, device_state_dirty = true, host_state_stale = false;
  unsigned long long structure_ver = 0;  // bumped by every build_structure (block pattern, fronts, index maps)
  int pd = 0, ld = 0;
  int num_poses = 0, num_landmarks = 0, size_poses = 0, size_landmarks = 0;
  std::vector<int> active;       // active vertex indices sorted by id
  std::vector<int> ivmap;        // hessian order
  std::vector<int> hidx;         // per vertex: hessian index or -1
  bool do_schur = false;
  int ne = 0;                    // local edges over all groups
  std::vector<EGroup> groups;
  bool has_hostj = false;
  g2ohip_host_edge_fn host_fn = nullptr;
  void* host_user = nullptr;
  // sharding
  int rank = 0, nranks = 1;
  std::unique_ptr<Comm> comm;
  std::vector<int> local_lm;     // landmark (hessian - num_poses) this rank owns
  // aligned landmark shards (align_shards): per rank its landmark range of the hessian order [lm_bnd[r], lm_bnd[r+1]),
  // empty: the uniform split. The landmarks' hessian order is then grouped by rank (ivmap / hidx renumbered).
  std::vector<int> lm_bnd;
  bool dist_aligned = false;
  std::vector<int> al_bpinv, al_bowner;  // the cut's pattern: pose block -> permuted block, permuted block -> owner
  // align_shards' analysis of the Schur pattern (al_sbi, al_sbj) and its aligned plan, handed to DeviceCholesky::setup
  std::shared_ptr<const Symbolic> al_sym;
  std::shared_ptr<const DistPlan> al_plan;
  std::vector<int> al_sbi, al_sbj;
  std::vector<unsigned char> lam_own_h;  // per pose: this rank adds lambda to its diagonal block of S
  DevBuf<unsigned char> d_lam_own;
  void align_shards();
  void schur_pattern(std::vector<int>& sbi, std::vector<int>& sbj, std::vector<int>& srow_ptr) const;
  std::vector<double> pose_work() const;

  // device state
  DevBuf<double> dstate[NVT];
  DevBuf<int> dnopl;
  std::vector<std::vector<DevBuf<double>>> stack_;  // per push level: per type (buffers reused)
  int stack_depth_ = 0;
  bool edges_ready = false;
  hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};  // schur start, factor start, factor end, solve end
  bool ev_valid_ = false;
  DevBuf<int> d_xoff[NVT];         // per type local -> x offset or -1
  DevBuf<int> d_hidx[NVT];         // per type local -> hessian index (-1 fixed)
  // per-vertex-side slot arenas by vertex dimension (2, 3, 6): packed upper H + b, one slot per (edge, side)
  DevBuf<double> dslot[7];
  long long nslot[7] = {0, 0, 0, 0, 0, 0, 0};
  double* slot_arena(int dim) { return dslot[dim].get(); }
  // off-diagonal blocks several local edges share: per-edge slots reduced in edge order, one launch per block size
  DevBuf<double> doffslot;
  struct OffRed { int nb = 0, bsz = 0; DevBuf<int> ptr; DevBuf<long long> soff, dst; };
  OffRed offred[2];  // [Hpp off-diagonal blocks (pd x pd), Hpl blocks (pd x ld)]
  // fused BA assembly (assembly.hip): graphs whose only edge group is BA in Schur mode; edges landmark-major,
  // wave chunks of whole landmarks, camera-major copies of the edge data for the camera-side pass
  bool ba_fused = false;
  DevBuf<int4> fz_chunks, fz_fix;
  int fz_nchunks = 0, fz_nfix = 0;
  DevBuf<double> fz_lpart;
  // Schur split at assembly: eligible graphs (fused BA, no shared off-diagonal blocks, a Cholesky / PCG on S), and the
  // lambda the stored G = Hpl U^-T, S(i,i) and bschur were formed with (NaN: Hpl stored, the plain Schur passes run)
  bool fz_split_ok = false;
  bool fz_kx = false;  // the split stores Kt records (assembly.hip KXB) instead of G
  DevBuf<int> cm_hpl;    // per camera-major observation its Kt record (the camera pass reads it)
  DevBuf<int> kx_extra;  // per BA edge of a fixed landmark and a free camera its extra Kt record, else -1
  int n_kx_extra = 0;
  double fz_lambda = std::numeric_limits<double>::quiet_NaN();
  DevBuf<int> cm_ptr, cm_v0, cm_v1;
  DevBuf<double> cm_meas, cm_info, cm_params;
  std::vector<int> cm_ptr_h, cm_e_h, lm_eptr_h;  // host copies for the CGLS setup (camera lists, landmark edge ranges)
  // hessian storage
  int nHpp = 0, nHpl = 0;
  DevBuf<double> dH;             // [Hpp blocks | Hpl blocks]
  DevBuf<double> dHll;
  DevBuf<double> db, dx;
  // vertex reduction
  struct VRed { int dim, nv, lanes; DevBuf<int> ptr, code, boff; double* H; };
  VRed vr_pose, vr_lm;
  // schur
  DevBuf<int> d_lm_ptr, d_blk_pose, d_blk_lm;
  DevBuf<int2> d_bs_erng;  // fused BA: per local landmark its edge range (k_backsub_j)
  DevBuf<double> dDinv, dUfac, dS, dCl, dG;
  int nS = 0, nHppUsed = 0;
  long long npairs = 0, nstaged = 0;  // off-diagonal pair products, staged blocks per Schur pass
  DevBuf<int> ds_hpp;
  // row-stationary Schur pass (k_schur_rows)
  DevBuf<launch::SchurTask> sch_tasks;
  DevBuf<launch::SchurBatch> sch_batches;
  DevBuf<int> sch_st_obs, sch_pairs, sch_pp;
  DevBuf<int> sch_gmap, sch_gmap_kx;  // per Schur task its 128 lane groups (slot_groups; the Kt-record pass)
  DevBuf<int> sch_st_obs_h;  // the same staged blocks as Hpl block indices (G in Hpl's order, Schur split)
  int nsch_tasks = 0;
  // the BA split's Kt-record batches (k_schur_rows<..., KX>) when their block size differs from launch::SCHUR_SB
  DevBuf<launch::SchurTask> sch_tasks_kx;
  DevBuf<launch::SchurBatch> sch_batches_kx;
  DevBuf<int> sch_st_obs_kx, sch_pairs_kx, sch_pp_kx;
  int nsch_tasks_kx = 0, kx_sb = launch::SCHUR_SB;
  // row chunks split into parts (per-rank task lists): their reduction groups and the partial-block scratch
  DevBuf<launch::SchurPartGroup> sch_groups, sch_groups_kx;
  int nsch_groups = 0, nsch_groups_kx = 0;
  long long sch_part_blocks = 0;
  DevBuf<double> dSchurPart;
  DevBuf<int> d_cam_list;  // the split camera pass's cameras on a sharded rank (ncam_list 0: every camera)
  int ncam_list = 0;
  static int kx_batch_size();
  // diagonal Schur blocks (k_schur_diag): per camera row its observations in landmark order
  DevBuf<int> sch_rptr, sch_robs, sch_obs_lm, sch_sdiag;
  std::vector<int> s_bi, s_bj, hpp_bi, hpp_bj;
  DeviceCholesky chol;
  DeviceCholesky marg_chol;  // factor of Hpp for computeMarginals where `chol` factors S (or is not set up)
  unsigned long long marg_ver = 0;  // structure_ver marg_chol was set up for (0: never)
  DevBuf<double> dmarg, dmarg_out;  // [Y | T | W | zero rhs], gathered blocks
  DevBuf<int> dmarg_fail;
  DevBuf<long long> dmarg_idx;
  BlockSymv symv_hpp, symv_s;
  DevBuf<double> dtmp;
  DevBuf<double> dsfull;  // linear_residual under a reduce-scattered S: the all-reduced copy of [S blocks | bschur]
  DevicePCG pcg;  // {lm,gn}_pcg* algorithms (linear_solver_pcg.hpp)
  bool use_cgls() const { return algorithm.size() > 12 && algorithm.compare(algorithm.size() - 12, 12, "pcg6_3_eigen") == 0; }
  bool use_pcg() const { return algorithm.find("_pcg") != std::string::npos && !use_cgls(); }
 public:
  DeviceCGLS cgls;  // lm_pcg6_3_eigen: the fork's matrix-free CGLS (JacobiSolver_6_3 + LinearSolverPCGEigen)
 private:
  // scalars: [0] lambda, [1] chi2, [2] scale, [3] maxdiag
  DevBuf<double> dscal;
  DevBuf<double> dpartial;
  double lambda_host = 0.0;
  bool lambda_set = false;
  // LM state (optimization_algorithm_levenberg.cpp)
  double current_lambda = -1, ni = 2;
  // chi2 of the device state, cached: every state change bumps state_ver; the LM loop knows the chi2 of
  // the state it leaves behind (accepted: tempChi, rejected + pop: currentChi) and records it
  unsigned long long state_ver = 1, chi_ver = 0;
  // buildSystem of the next LM iteration is enqueued as soon as a trial loop ends (it only depends on
  // the state the loop leaves); built_ver records which state the assembled system belongs to
  unsigned long long built_ver = 0;
  double chi_cache = 0.0;
  hipEvent_t lm_ev_[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipEvent_t rb_ev_ = nullptr;   // the trial's scalar readback landed (the stream may hold more work behind it)
  // the kernel timer records events in the assembly (all classes, or one of the assembly's): the speculative next
  // assembly is off then (a timer on chol_factor alone, bench.py's, leaves it on)
  bool timer_times_build() const {
    return timer.enabled && (timer.only.empty() || timer.only == "linearize" || timer.only == "vreduce" ||
                             timer.only == "schur_rows");
  }
  double* hscal_ = nullptr;      // pinned host copy of dscal (one readback per LM trial)
  double* hdec_ = nullptr;       // mapped coherent host memory the one-rank decision kernel writes the scalars to
  double* hdec_dev_ = nullptr;   // its device address
  int levenberg_iterations = 0;

  void ensure_device_state();
  void sync_host_state();
  void setup_edges_device();
  void compute_errors_async(bool reduce = true);  // reduce: the chi2 all-reduce over landmark shards
  void refresh_host_payload(bool jacobians);  // host-J groups: payload at the current state (callback), upload
  EdgeArgs group_args(const EGroup& g) const;
  double chi2_sync();
  double lambda_init();
  double max_diagonal();
  void ensure_hpp();
  void solve_async(bool reset_fail);
  int* failp() const { return reinterpret_cast<int*>(dscal.get() + 8); }
  void update_async();
  void set_lambda_device(double l, bool reset_fail = false);
  void allreduce_sum(double* dptr, size_t n);
  int lm_solve(int iteration, const g2ohip_config& cfg, g2ohip_batch_stats* st);
  int gn_solve(int iteration, g2ohip_batch_stats* st);
  // upper blocks of the matrix the last factorization saw (S with lambda, or Hpp + lambda) as an Octave file
  void write_debug_dump();
};

}  // namespace g2ohip
