/*
 * g2o_hip.h — C ABI of the MI355X-native BlockSolver<p,l> backend (libg2o_hip.so).
 *
 * The drop-in boundary is g2o's own plugin interface for this path (paths
 * relative to the reference tree):
 *
 *   Solver (core/solver.h:44-155) ........ g2ohip_solver_*  (buildStructure /
 *        buildSystem / setLambda / restoreDiagonal / solve / x / b / vectorSize)
 *   LinearSolver<M>::solve (core/linear_solver.h:42-105) .. g2ohip_linear_solve_ccs
 *   OptimizationAlgorithmLevenberg::solve (core/optimization_algorithm_levenberg.cpp:58-150)
 *        + SparseOptimizer::optimize (core/sparse_optimizer.cpp:374-439) ... g2ohip_optimize
 *   OptimizableGraph::load / save (core/optimizable_graph.cpp:397-679) .. g2ohip_load_g2o / g2ohip_save_g2o
 *   OptimizationAlgorithmFactory::construct (core/optimization_algorithm_factory.cpp:84-93)
 *        .. g2ohip_set_algorithm("lm_hip_fix6_3" | "lm_hip_fix3_3" | "lm_hip_fix6_6" | "lm_hip_var" | "gn_hip_*"
 *           | "{lm,gn}_pcg" | "{lm,gn}_pcg6_3" (block-Jacobi PCG, solver_pcg.cpp:91-98)
 *           | "lm_pcg6_3_eigen" (fork JacobiSolver_6_3 + LinearSolverPCGEigen CGLS, solver_eigen.cpp:80,126))
 *   G2OBatchStatistics (core/batch_stats.h:42-72) .. g2ohip_batch_stats
 *
 * Plain pointers and sizes only; no torch / HIP types cross the boundary.
 * Errors follow the reference: no exceptions, int status codes; a solve that
 * meets a non-positive-definite pivot returns 0 (the reference's `false`,
 * linear_solver_csparse.h:127-133) so the LM retry logic is unchanged.
 * Every compute entry point requires a MI355X (gfx950); there is no CPU path.
 */
#ifndef G2O_HIP_H
#define G2O_HIP_H
#ifdef __cplusplus
extern "C" {
#endif

/* ---- vertex types (estimate layouts) ---- */
#define G2OHIP_V_SE3_EXPMAP 1 /* VertexSE3Expmap, types_six_dof_expmap.h:84-102: tx ty tz qx qy qz qw (world->cam) */
#define G2OHIP_V_XYZ 2        /* VertexSBAPointXYZ, types_sba.h:137: x y z */
#define G2OHIP_V_SE3_QUAT 3   /* VertexSE3, vertex_se3.h:50: x y z qx qy qz qw (toVectorQT) */
#define G2OHIP_V_SE2 4        /* VertexSE2, vertex_se2.h:40: x y theta */
#define G2OHIP_V_XY 5         /* VertexPointXY, vertex_point_xy.h:39-88: x y (a BlockSolver_3_2 landmark) */
/* ---- edge types ---- */
#define G2OHIP_E_SE3_PROJECT_XYZ 1 /* EdgeSE3ProjectXYZ, types_six_dof_expmap.h:201-229: v0 point, v1 camera;
                                      meas u v; info 2x2; params fx fy cx cy */
#define G2OHIP_E_SE3_QUAT 2        /* EdgeSE3, edge_se3.h: meas x y z qx qy qz qw; info 6x6 */
#define G2OHIP_E_SE2 3             /* EdgeSE2, edge_se2.h:46-52: meas x y theta; info 3x3 */
#define G2OHIP_E_SE2_XY 5          /* EdgeSE2PointXY, edge_se2_pointxy.h:41-75: v0 SE2 pose, v1 XY point; meas x y;
                                      info 2x2 */
/* An edge type the device does not know (any BaseBinaryEdge<D, E, Vi, Vj> between registered vertices of
 * dimension 2, 3 or 6): the host's own linearizeOplus (the type's analytic one, or BaseBinaryEdge's numeric
 * central differences, base_binary_edge.hpp:198-266) supplies the error and both Jacobians, see
 * g2ohip_set_host_jacobians; the device assembles, marginalises and solves. meas unused (may be NULL);
 * info D*D. Several host-J types (different D) may coexist with the device types in one graph. */
#define G2OHIP_E_HOSTJ(D) (32 + (D)) /* D = error dimension, 1..6 */

/* robust kernels (robust_kernel_impl.cpp; RobustKernelFactory names) */
#define G2OHIP_RK_NONE 0
#define G2OHIP_RK_HUBER 1
#define G2OHIP_RK_PSEUDO_HUBER 2
#define G2OHIP_RK_CAUCHY 3
#define G2OHIP_RK_GEMAN_MCCLURE 4
#define G2OHIP_RK_WELSCH 5
#define G2OHIP_RK_FAIR 6
#define G2OHIP_RK_TUKEY 7
#define G2OHIP_RK_SATURATED 8
#define G2OHIP_RK_DCS 9

/* status codes */
#define G2OHIP_OK 0
#define G2OHIP_ERR_ARG (-1)
#define G2OHIP_ERR_STATE (-2)
#define G2OHIP_ERR_DEVICE (-3)
#define G2OHIP_ERR_UNSUPPORTED (-4)

/* G2OBatchStatistics (core/batch_stats.h:42-72) + the current lambda */
typedef struct {
  int iteration;
  int numVertices;
  int numEdges;
  double chi2;
  double lambda;
  double timeResiduals;
  double timeQuadraticForm;
  int levenbergIterations;
  double timeSchurComplement;
  double timeSymbolicDecomposition;
  double timeNumericDecomposition;
  double timeLinearSolution;
  double timeLinearSolver;
  double timeUpdate;
  double timeIteration;
  long long hessianDimension;
  long long hessianPoseDimension;
  long long hessianLandmarkDimension;
  long long choleskyNNZ;
} g2ohip_batch_stats;

/* OptimizationAlgorithmLevenberg properties (optimization_algorithm_levenberg.cpp:48-49) */
typedef struct {
  int max_trials_after_failure; /* maxTrialsAfterFailure, default 10 */
  double user_lambda_init;      /* initialLambda, 0 -> tau * max diag (tau = 1e-5) */
  int verbose;                  /* SparseOptimizer::setVerbose: per-iteration line on stderr */
} g2ohip_config;

typedef struct g2ohip_graph g2ohip_graph;

/* ---- graph (OptimizableGraph / SparseOptimizer) ---- */
g2ohip_graph* g2ohip_graph_create(int device);
void g2ohip_graph_destroy(g2ohip_graph* g);
int g2ohip_add_vertices(g2ohip_graph* g, int type, int n, const int* ids, const double* est, const int* fixed,
                        const int* marginalized);
int g2ohip_add_edges(g2ohip_graph* g, int type, int n, const int* v0, const int* v1, const double* meas,
                     const double* info /* n * D*D row-major */, const double* params /* n*4 or NULL */);
int g2ohip_load_g2o(g2ohip_graph* g, const char* path, int marginalize_xyz);
int g2ohip_save_g2o(g2ohip_graph* g, const char* path);
int g2ohip_num_vertices(g2ohip_graph* g);
int g2ohip_num_edges(g2ohip_graph* g);
/* estimates of one vertex type in insertion order (syncs device state to host first) */
int g2ohip_get_estimates(g2ohip_graph* g, int type, double* out, int* ids_out);
/* overwrite estimates of one vertex type (insertion order) — host-authoritative Solver mode */
int g2ohip_set_estimates(g2ohip_graph* g, int type, const double* est);
/* minimal state vector concatenated in vertex-id order (parity checks) */
int g2ohip_minimal_state(g2ohip_graph* g, double* out);

/* OptimizableGraph::Edge::setRobustKernel (optimizable_graph.h; base_binary_edge.hpp:104-135 weighted
 * quadratic form, sparse_optimizer.cpp:102-116 robust chi2) for every edge of a type: kind G2OHIP_RK_*,
 * delta = RobustKernel::setDelta. G2OHIP_RK_NONE removes it. */
int g2ohip_set_robust_kernel(g2ohip_graph* g, int edge_type, int kind, double delta);
/* Host-computed linearization of the G2OHIP_E_HOSTJ(D) edges of one type, in insertion order: per edge
 * [e (D) | Ji (D x dim(v0)) | Jj (D x dim(v1))], row-major, at the estimates the device holds (call after
 * g2ohip_set_estimates, before g2ohip_solver_build_system). The J_host_fallback of SURVEY.md 8b. */
int g2ohip_set_host_jacobians(g2ohip_graph* g, int edge_type, const double* payload);
/* Callback for the device-resident loops (g2ohip_optimize / g2ohip_chi2) when host-J edges exist: fill the
 * payload of every edge of `edge_type` at the current estimates (read them with g2ohip_get_estimates);
 * with_jacobians = 0 only needs the errors. Return 0 on success. */
typedef int (*g2ohip_host_edge_fn)(void* user, int edge_type, int with_jacobians, double* payload);
int g2ohip_set_host_edge_callback(g2ohip_graph* g, g2ohip_host_edge_fn fn, void* user);
/* Length in doubles of the payload buffer of a host-J edge type (the `payload` the callback fills and
 * g2ohip_set_host_jacobians reads): sum over its edges of D * (1 + dim(v0) + dim(v1)). A callback must write exactly
 * this many doubles. */
long long g2ohip_host_payload_len(g2ohip_graph* g, int edge_type);

/* OptimizationAlgorithmFactory::construct by name; default "lm_hip_var" */
int g2ohip_set_algorithm(g2ohip_graph* g, const char* name);
/* SparseOptimizer::initializeOptimization(0): active edges/vertices, index mapping */
int g2ohip_initialize(g2ohip_graph* g);
/* SparseOptimizer::updateInitialization(vset, eset) + BlockSolver::updateStructure (sparse_optimizer.cpp:465-502,
 * block_solver.hpp:258-312), online mode: after g2ohip_initialize (and optimizing), vertices and edges added with
 * g2ohip_add_vertices / g2ohip_add_edges join the optimization without re-indexing the existing ones — each new free
 * vertex (one that has an edge) takes the next hessian index, new vertices in id order; the next optimize / build
 * continues from the current (optimized) state with the grown structure. Non-Schur graphs only, as in the reference:
 * G2OHIP_ERR_UNSUPPORTED when the graph or a new vertex is marginalized (the reference aborts), G2OHIP_ERR_STATE
 * before g2ohip_initialize. Calling g2ohip_initialize instead re-indexes every vertex in id order. */
int g2ohip_update_initialization(g2ohip_graph* g);
/* computeActiveErrors + activeRobustChi2 on the device */
double g2ohip_chi2(g2ohip_graph* g);
/* SparseOptimizer::optimize(iterations) with the device-resident LM loop.
 * stats: array of `iterations` entries or NULL. Returns iterations done, 0 on Fail, <0 on error. */
int g2ohip_optimize(g2ohip_graph* g, const g2ohip_config* cfg, int iterations, g2ohip_batch_stats* stats);
/* One iteration of the SparseOptimizer::optimize loop (iteration 0 rebuilds the structure and the
 * initial lambda, exactly as optimize() does). Returns 0 OK, 1 Terminate, 2 Fail, <0 error. */
int g2ohip_optimize_step(g2ohip_graph* g, const g2ohip_config* cfg, int iteration, g2ohip_batch_stats* stats);

/* ---- Solver-level plugin (core/solver.h:54-137) for a g2o-side BlockSolverHip adapter ---- */
int g2ohip_solver_build_structure(g2ohip_graph* g);             /* Solver::buildStructure */
int g2ohip_solver_build_system(g2ohip_graph* g);                /* Solver::buildSystem */
int g2ohip_solver_set_lambda(g2ohip_graph* g, double lambda, int backup); /* Solver::setLambda */
int g2ohip_solver_restore_diagonal(g2ohip_graph* g);            /* Solver::restoreDiagonal */
int g2ohip_solver_solve(g2ohip_graph* g);                       /* Solver::solve: 1 ok, 0 not PD, <0 error */
long long g2ohip_solver_vector_size(g2ohip_graph* g);           /* Solver::vectorSize */
/* BlockSolver<p, l> traits after build_structure: dims = [PoseDim, LandmarkDim, pose blocks, landmark blocks]
 * (block_solver.h:44-60; Solver::additionalVectorSpace etc. not needed) */
int g2ohip_solver_block_dims(g2ohip_graph* g, int* dims);
/* Solver::x() / Solver::b() (host copies) in the Hessian order: poses, then the free landmarks. On one rank the
 * landmarks follow buildIndexMapping's id order (block_solver.hpp, sparse_optimizer.cpp:207-241). With landmark shards
 * aligned to the factorization's cut (g2ohip_set_comm, N > 1) the landmarks are regrouped by owning rank (stable in
 * id order within a rank). The vectors keep a slot for every landmark, but on a sharded rank only its own landmarks'
 * slots hold this rank's values: one contiguous range of the landmark part, whose landmark ids g2ohip_local_landmarks
 * lists in the order x / b carry them. */
int g2ohip_solver_get_x(g2ohip_graph* g, double* x);
int g2ohip_solver_get_b(g2ohip_graph* g, double* b);
/* BlockSolverBase::multiplyHessian (core/block_solver.h:94,146; used by OptimizationAlgorithmDogleg
 * optimization_algorithm_dogleg.cpp:100,179): dest = Hpp src with the upper blocks mirrored (+ lambda on the
 * diagonal while a setLambda is active), host arrays of hessianPoseDimension. Single rank only. */
int g2ohip_solver_multiply_hessian(g2ohip_graph* g, double* dest, const double* src);
/* max |diagonal entry| of the vertex Hessian blocks (Hpp, Hll) after buildSystem: the quantity
 * OptimizationAlgorithmLevenberg::computeLambdaInit reads through the vertices' mapped Hessians
 * (optimization_algorithm_levenberg.cpp:152-175) in the host-authoritative Solver mode. */
int g2ohip_solver_diag_absmax(g2ohip_graph* g, double* out);
/* Solver::setEta (core/solver.h:137, jacobi_solver.h:142): forcing term of the lm_pcg6_3_eigen CGLS (stop when
 * s.s < eta s0.s0, linear_solver_pcg_eigen.h:170-176); default 0.1 (core/linear_solver.h:66). */
int g2ohip_solver_set_eta(g2ohip_graph* g, double eta);
/* G2OBatchStatistics::iterationsLinearSolver of the last lm_pcg6_3_eigen solve */
int g2ohip_solver_linear_iterations(g2ohip_graph* g);
/* ||(A + lambda I) x - b|| / ||b|| of the last Solver::solve, evaluated on the device (A = the Schur complement
 * with Schur, else Hpp): a size-independent check of the factorization at any problem size. With landmark shards
 * (g2ohip_set_comm) it is a collective: every rank calls it (the reduced system is summed over ranks first when the
 * distributed factorization reduce-scattered it). */
int g2ohip_solver_linear_residual(g2ohip_graph* g, double* rel);
/* Symbolic / schedule summary of the device factorization: out[0..20] = n, nnz(L), flops (this ordering),
 * supernodes, tree levels, largest front, blocked fronts, levels assembled in place, pre-scattered levels,
 * trailing-update launches, big-panel backward rounds, out[11] = 0 (retired slot), and for landmark
 * shards (nranks > 1) this rank's fronts, the shared fronts, the subtree roots, the doubles of the root exchange
 * buffer (nranks all-gathered segments), the cost model of the best cut of the elimination tree (modelled seconds of
 * this rank's subtrees, of the shared top, of the replicated factorization, of the cut's exchanges: root all-gather and
 * x all-reduce) and whether the factorization is distributed (1) or
 * replicated (0: the model preferred replication, or G2OHIP_DIST_FACTOR=0); then out[21..25] = whether the reduced
 * system is reduce-scattered by subtree ownership (1) instead of all-reduced, its per-rank segment and all-reduced tail
 * (doubles), and the modelled seconds of that input exchange and of the plain all-reduce; out[26] = 0 (retired slot);
 * out[27] = the band-leaf size of the ordering (blocks; 0: plain nested dissection); out[28] = 1 when the landmark
 * shards are aligned with the cut (each landmark on the rank whose subtrees its Schur blocks land in, G2OHIP_DIST_ALIGN),
 * out[29] = doubles of this rank's subtree blocks read from its own partial reduced system (never exchanged), out[30] =
 * bytes this rank sends per LM trial through the reduced system's and the factorization's collectives (ring
 * algorithms), out[31] = free landmarks in this rank's shard, out[32] = the modelled sharded work (s) of the busiest
 * rank under this layout, out[33] = fronts whose panel steps factor only their own rows, L21 then formed as one GEMM
 * with the explicit L11^-1 (deferred L21, G2OHIP_CHOL_DEFER_L21). Returns the number of entries available. */
int g2ohip_solver_factor_info(g2ohip_graph* g, double* out, int n);
/* Landmark shards (g2ohip_set_comm / _set_comm_local): the ids of the free landmarks this rank holds (their estimates
 * are current on this rank only); ids may be NULL. Returns the count. With the distributed factorization the shards
 * follow its cut (not id ranges); otherwise they are contiguous ranges of the landmark order. */
int g2ohip_local_landmarks(g2ohip_graph* g, int* ids, int cap);
/* Solver::computeMarginals (core/solver.h:108; BlockSolver::computeMarginals block_solver.hpp:451-460 ->
 * LinearSolverCSparse::solvePattern linear_solver_csparse.h:190-225, MarginalCovarianceCholesky): the pose-block
 * entries (block_rows[k], block_cols[k]) (Hessian indices) of Hpp^-1, Hpp as the last build_system left it (no
 * lambda), each a pd x pd column-major block written to out + k * pd * pd. The whole pose system is factored on the
 * device (the LM's own factor when it factors Hpp), then one multi-right-hand-side supernodal solve per 64 / pd
 * requested block columns. Returns 1, or 0 when Hpp is not positive definite (the reference's bool), or a
 * negative status (unsupported on sharded graphs). */
int g2ohip_solver_compute_marginals(g2ohip_graph* g, int nblocks, const int* block_rows, const int* block_cols,
                                    double* out);
/* SparseOptimizer::update(x) + push/pop/discardTop on the device-resident state */
int g2ohip_update(g2ohip_graph* g, const double* x_host /* NULL: use device x */);
int g2ohip_push(g2ohip_graph* g);
int g2ohip_pop(g2ohip_graph* g);
int g2ohip_discard_top(g2ohip_graph* g);

/* Stage export for parity tests (small problems): after build_system + set_lambda + solve, the
 * dense reduced system and solution. dims: [n, n_pose_scalars, n_landmark_scalars]. */
int g2ohip_stage(g2ohip_graph* g, double lambda, double* b, double* x, double* Hschur_dense, double* bschur,
                 long long* dims);

/* Solver::saveHessian (core/block_solver.hpp:589-593 -> SparseBlockMatrix::writeOctave, sparse_block_matrix.hpp:579-617):
 * Hpp of the last buildSystem (+ lambda while a setLambda is active) as an Octave sparse-matrix text file, every entry of
 * every stored block plus the mirrored off-diagonal blocks, "%.9f". Returns 1 written, 0 not written, <0 error. */
int g2ohip_solver_save_hessian(g2ohip_graph* g, const char* path);
/* Solver::setWriteDebug (core/block_solver.hpp:582-586): when on, a factorization that meets a non-positive pivot
 * writes the matrix it factored (S, or Hpp + lambda) to "debug.txt" in the format of csparse_helper.cpp:62-111, as
 * LinearSolverCSparse::solve does (linear_solver_csparse.h:127-133). Default off. */
int g2ohip_solver_set_write_debug(g2ohip_graph* g, int on);

/* ---- LinearSolver-level plugin (core/linear_solver.h:42-105, LinearSolverCCS) ----
 * Solve A x = b for symmetric PD A given as UPPER CCS (n, Ap[n+1], Ai, Ax) of scalar entries,
 * with an optional block partition (nblocks, block_ends[] cumulative end offsets as in
 * SparseBlockMatrix::rowBlockIndices) used for the block ordering. Returns 1 ok, 0 not PD. */
int g2ohip_linear_solve_ccs(int device, int n, const int* Ap, const int* Ai, const double* Ax, const double* b,
                            double* x, int nblocks, const int* block_ends);

/* ---- multi-GPU (landmark sharding + RCCL all-reduce of the reduced camera system) ---- */
int g2ohip_comm_unique_id(unsigned char out[128]);
/* this rank keeps landmark shard `rank` of `nranks` (g2ohip_local_landmarks lists it) */
int g2ohip_set_comm(g2ohip_graph* g, const unsigned char uid[128], int rank, int nranks);
/* Test transport: `nranks` graphs in ONE process (one host thread each, same GPU) that share
 * `group_key` reduce through host memory in rank order instead of RCCL. Same sharding, same
 * call sequence as g2ohip_set_comm; used to test the sharded path on a single-GPU box. A `group_key` starting with
 * "solo:" makes this graph play rank `rank` of `nranks` ALONE with every collective a no-op: the kernels rank `rank`
 * would run, for timing (tools/dist_rank_times.py); its results are not meaningful. */
int g2ohip_set_comm_local(g2ohip_graph* g, const char* group_key, int rank, int nranks);
/* RCCL transport self-test on one device (a one-rank communicator from `uid`): the product's allreduce sum and max
 * (the calls g2ohip_set_comm's ranks make) over n doubles of `in` on a stream of `device`; out (2n doubles) =
 * [sum | max]. A one-GPU box cannot host two ranks of one RCCL communicator, so this is the binding's smoke test there. */
int g2ohip_comm_selftest(int device, const unsigned char uid[128], int n, const double* in, double* out);
/* As g2ohip_comm_selftest, plus the in-place reduce-scatter sum the distributed factorization uses: rs_out (n doubles)
 * = this rank's segment, and the in-place all-gather of its root exchange (checked internally: an error if the
 * rank's own segment changes). (0.1.x wrote the segment as a third block of `out`; 0.2 restored the 2n contract.) */
int g2ohip_comm_selftest_rs(int device, const unsigned char uid[128], int n, const double* in, double* out,
                            double* rs_out);
/* The test transport's rank-ordered host reduction alone (no GPU): `nranks` host threads that share `group_key` each
 * call this with their buffer; every call is checked to be the same collective on every rank (call number, length,
 * operation) and a mismatch returns G2OHIP_ERR_DEVICE on every rank (g2ohip_last_error says which) instead of reading
 * past a buffer. RCCL ranks run the same check when G2OHIP_COMM_CHECK=1 is set. */
int g2ohip_comm_local_reduce_host(const char* group_key, int rank, int nranks, double* buf, long long n, int is_max);
/* JSON text naming the HIP runtime and RCCL libraries this library's calls are bound to (resolved paths) and their
 * versions; returns the length needed including the NUL. */
int g2ohip_runtime_info(char* out, int cap);
/* hipDeviceSynchronize on `device` in this library's HIP runtime (the benchmark's bracket around its timed region). */
int g2ohip_device_synchronize(int device);

/* ---- host-only symbolic analysis (no GPU needed) ----
 * Block pattern of a symmetric matrix given as upper blocks (bi[k] <= bj[k]) of a uniform block
 * size bdim: returns n = nblocks*bdim, fills perm[n] (new -> old scalar) and
 * stats[5] = {nnz(L), factor flops, #supernodes, #levels, level-synchronous 32-column panel steps}. */
int g2ohip_symbolic_analyze(int nblocks, int bdim, int nblk, const int* bi, const int* bj, int* perm, double* stats);
/* Host-only: the distributed factorization's cut for `nranks` landmark shards of the same block pattern (DESIGN.md §6,
 * the model the solver's setup runs; flags: 1 the input is reduce-scattered by subtree ownership, 2 the landmark shards
 * are aligned with the cut; pose_work, optional: per pose block the seconds of landmark-sharded work that follow it).
 * out[14] = {distributed (the cut beats the replicated model), this rank's subtrees s, shared top s, replicated
 * iteration s (factorization + whole-S all-reduce + uniform sharded work), exchanges s (root all-gather + x
 * all-reduce), input s, replicated input s, slowest rank's subtrees s, root all-gather doubles per rank, input
 * reduce-scatter doubles per rank, input tail all-reduce doubles, supernodes, busiest rank's sharded work s, uniform
 * sharded work s}; sn_owner (cap entries, optional): per supernode its rank, -1 shared. Returns the supernodes. */
int g2ohip_dist_plan(int nblocks, int bdim, int nblk, const int* bi, const int* bj, int nranks, int rank,
                     int flags, const double* pose_work, double* out, int* sn_owner, int cap);

/* ---- measurement hooks ---- */
void g2ohip_enable_kernel_timing(g2ohip_graph* g, int on);
/* restrict the kernel timer to one kernel class (NULL or "": every class); each timed class costs two
 * event records per launch on the stream */
void g2ohip_kernel_timing_only(g2ohip_graph* g, const char* name);
/* G2OBatchStatistics timers: 0 none, 1 timeLinearSolution only (2 events per LM trial), 2 (default)
 * every stage (timeSchurComplement, timeNumericDecomposition, timeLinearSolver, timeUpdate, timeQuadraticForm) */
void g2ohip_set_stats_level(g2ohip_graph* g, int level);
/* per-kernel-class average device time (ms) since the timer was enabled; classes: "linearize", "vreduce",
 * "schur_dinv", "schur_diag", "schur_rows", "chol_factor", "chol_solve", "backsub", "error", "oplus" */
double g2ohip_kernel_ms(g2ohip_graph* g, const char* name);
long long g2ohip_kernel_count(g2ohip_graph* g, const char* name);
/* algorithmic bytes / flops of one launch of the named kernel class (for roofline accounting) */
double g2ohip_kernel_bytes(g2ohip_graph* g, const char* name);
double g2ohip_kernel_flops(g2ohip_graph* g, const char* name);
/* development builds (-DG2OHIP_PHASES) only: per-launch phase stamps of the Cholesky kernels,
 * 8 x u64 per record {kernel id, t0, t1..t6}; returns the record count (0 in product builds) */
int g2ohip_debug_phases(unsigned long long* out, int max_records);
const char* g2ohip_last_error(void);
/* Measured roofline peaks of `device` (peaks.hip, ~1 s): out[0] HBM streaming-copy GB/s (read + written bytes of a
 * 2 GiB 16-byte-per-lane copy), out[1] FP64 MFMA TFLOP/s (v_mfma_f64_16x16x4f64 issue loop), out[2] FP64 VALU TFLOP/s (v_fma_f64
 * issue loop), out[3] compute units; n >= 4. Returns 4 or a negative error. */
int g2ohip_measure_peaks(int device, double* out, int n);
/* The accepted LM trial's lambda factor max(1/3, min(2/3, 1 - (2 rho - 1)^3)) exactly as the device decision and the
 * host loop compute it (optimization_algorithm_levenberg.cpp:127-136; the cube rounded once, like glibc's pow). */
double g2ohip_lm_scale_factor(double rho);
const char* g2ohip_version(void);

#ifdef __cplusplus
}
#endif
#endif
