/* ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
 * cpu_baseline).  C ABI of the CPU restatement of the reference BlockSolver /
 * LinearSolverCSparse / OptimizationAlgorithmLevenberg path.  Never linked into
 * the product library.  Type and statistics layouts deliberately mirror
 * include/g2o_hip.h so that tests can feed both the same arrays. */
#ifndef G2O_ORACLE_H
#define G2O_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* vertex types */
#define ORACLE_V_SE3_EXPMAP 1 /* est: tx ty tz qx qy qz qw (world->cam, SE3Quat::toVector order) */
#define ORACLE_V_XYZ 2        /* est: x y z */
#define ORACLE_V_SE3_QUAT 3   /* est: x y z qx qy qz qw (toVectorQT) */
#define ORACLE_V_SE2 4        /* est: x y theta */
#define ORACLE_V_XY 5         /* VertexPointXY (slam2d/vertex_point_xy.h:39-88), est: x y */
/* edge types */
#define ORACLE_E_SE3_PROJECT_XYZ 1 /* v0 = point, v1 = camera; meas u v; info 2x2; params fx fy cx cy */
#define ORACLE_E_SE3_QUAT 2        /* meas x y z qx qy qz qw; info 6x6 */
#define ORACLE_E_SE2 3             /* meas x y theta; info 3x3 */
#define ORACLE_E_SE3_EXPMAP 4      /* EdgeSE3Expmap (types_six_dof_expmap.h:108-127) between two VertexSE3Expmap:
                                      meas tx ty tz qx qy qz qw; info 6x6; Jacobians always numeric here */
#define ORACLE_E_SE2_XY 5          /* EdgeSE2PointXY (slam2d/edge_se2_pointxy.h:41-75): v0 = SE2 pose, v1 = XY point;
                                      meas x y; info 2x2 */

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
} oracle_batch_stats;

typedef struct {
  int max_trials_after_failure; /* 10 */
  double user_lambda_init;      /* 0 -> tau * max diag */
  int threads;                  /* OpenMP threads for assembly / Schur (1 = deterministic) */
  int use_ref_csparse;          /* 1: cs_amd + cs_chol from oracle/_ref (if loaded); 0: restated */
  int block_ordering;           /* 1: AMD on block pattern (lm_fixP_L), 0: scalar (lm_var) */
  int gauss_newton;             /* 1: OptimizationAlgorithmGaussNewton instead of Levenberg */
} oracle_config;

typedef struct OracleGraph OracleGraph;

OracleGraph* oracle_graph_new(void);
void oracle_graph_free(OracleGraph* g);
int oracle_add_vertices(OracleGraph* g, int type, int n, const int* ids, const double* est, const int* fixed,
                        const int* marginalized);
int oracle_add_edges(OracleGraph* g, int type, int n, const int* v0, const int* v1, const double* meas,
                     const double* info /* D*D row-major per edge */, const double* params /* or NULL */);
int oracle_load_g2o(OracleGraph* g, const char* path, int marginalize_xyz);
int oracle_save_g2o(OracleGraph* g, const char* path);
int oracle_num_vertices(OracleGraph* g);
int oracle_num_edges(OracleGraph* g);
/* estimates in insertion order of the given type; returns count */
int oracle_get_estimates(OracleGraph* g, int type, double* out, int* ids_out);
/* minimal state vector (SE3: toVectorMQT / SE3Quat minimal, SE2 x y th, XYZ) concatenated in vertex-id order */
int oracle_minimal_state(OracleGraph* g, double* out);

int oracle_initialize(OracleGraph* g);
/* SparseOptimizer::updateInitialization + BlockSolver::updateStructure (online, non-Schur); -3 for Schur graphs */
int oracle_update_initialization(OracleGraph* g);
double oracle_chi2(OracleGraph* g); /* computeActiveErrors + activeRobustChi2 */
int oracle_optimize(OracleGraph* g, const oracle_config* cfg, int iterations, oracle_batch_stats* stats);

/* Stage export (small problems only): runs buildStructure, computeActiveErrors,
 * buildSystem, setLambda(lambda), solve at the current state.  Dense outputs:
 *   b[n], x[n], Hschur[np*np] (full symmetric, or Hpp when no Schur),
 *   bschur[np]; sizes returned in dims[0]=n, dims[1]=np (pose scalars),
 *   dims[2]=nl (landmark scalars).  Any output pointer may be NULL. */
int oracle_stage(OracleGraph* g, const oracle_config* cfg, double lambda, double* b, double* x, double* Hschur,
                 double* bschur, long long* dims);
/* Dense Hessian blocks: Hpp[np*np] (full sym), Hll[nl*l] (diag blocks, col-major per landmark, l = dim),
 * Hpl[np*nl] dense.  Small problems only. */
int oracle_hessian_dense(OracleGraph* g, double* Hpp, double* Hll_diag, double* Hpl);

/* Jacobians of one edge at the current estimates (analytic + numeric), for unit tests. */
int oracle_edge_jacobians(OracleGraph* g, int edge_index, double* err, double* Ji_an, double* Jj_an,
                          double* Ji_num, double* Jj_num);

/* Sparse Cholesky pin: solve A x = b, A given as upper CCS (n, Ap, Ai, Ax).  mode 0 = restated
 * up-looking LL^T with natural ordering, 1 = restated with cs_amd ordering (needs _ref),
 * 2 = reference CSparse cs_cholsol (needs _ref).  Returns 1 on success, 0 not PD, -1 unavailable. */
int oracle_ccs_cholsol(int n, const int* Ap, const int* Ai, const double* Ax, double* b, int mode);
/* Symbolic stats of the CSparse block ordering (cs_amd on the block pattern when use_ref, else natural):
 * out[0] = nnz(L), out[1] = sum of squared column counts (factorization flops). */
int oracle_block_symbolic(int nblocks, int bdim, int nblk, const int* bi, const int* bj, int use_ref, double* out);
/* robust kernel (G2OHIP_RK_* numbering) for every edge of a type; numeric-Jacobian flag for listed edges */
int oracle_set_robust_kernel(OracleGraph* g, int etype, int kind, double delta);
int oracle_set_edge_numeric(OracleGraph* g, int n, const int* idx);
/* [e | Ji | Jj] row-major per listed edge at the current estimates; returns doubles written */
int oracle_edge_payload(OracleGraph* g, int n, const int* idx, int numeric, double* out);
/* SparseOptimizer::update / push / pop / discardTop (host-authoritative Solver-mode tests) */
int oracle_update(OracleGraph* g, const double* x);
int oracle_set_estimates(OracleGraph* g, int type, const double* est); /* insertion order of the type */
int oracle_push(OracleGraph* g);
int oracle_pop(OracleGraph* g);
int oracle_discard_top(OracleGraph* g);
int oracle_ref_available(void);
/* isometry3d_mappings / SE2 mappings (op codes in oracle.cpp), for the reference unit-test pins */
int oracle_mapping(int op, const double* in, double* out);
const char* oracle_ref_path(void);

#ifdef __cplusplus
}
#endif
#endif
