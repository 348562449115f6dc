// ORACLE — test infrastructure only.  Imported/executed only by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
//
// CPU restatement (plain C++, no Eigen) of the reference hot path:
//   SparseOptimizer pieces   core/sparse_optimizer.cpp:63-116,168-192,441-454,624-637
//   BlockSolver<Traits>       core/block_solver.hpp:102-256 (buildStructure),
//                             :314-447 (solve), :462-521 (buildSystem),
//                             :524-565 (setLambda/restoreDiagonal)
//   BaseBinaryEdge            core/base_binary_edge.hpp:61-137 (constructQuadraticForm),
//                             :198-266 (numeric linearizeOplus)
//   LinearSolverCSparse       solvers/csparse/linear_solver_csparse.h:106-142,246-344
//   cs_chol_workspace         solvers/csparse/csparse_extension.cpp:32-119 (up-looking LL^T)
//   OptimizationAlgorithmLevenberg  core/optimization_algorithm_levenberg.cpp:58-184
//   Types: types/sba/types_six_dof_expmap.{h,cpp}, types/slam3d/{se3quat.h,edge_se3.cpp,
//          vertex_se3.h,isometry3d_gradients.h}, types/slam2d/{edge_se2.{h,cpp},vertex_se2.h,se2.h}
//
// The vendored CSparse (EXTERNAL/csparse) is optionally dlopen()ed from
// oracle/_ref/libcsparse_ref.so (built from the reference sources by
// oracle/Makefile) for the block-AMD ordering and as a bitwise pin of the
// restated factorization.
#include "oracle.h"
#include "oracle_math.hpp"

#include <dlfcn.h>
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <limits>
#include <map>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

using namespace oracle;

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// --------------------------------------------------------------------------------------------
// Optional reference CSparse (oracle/_ref)
// --------------------------------------------------------------------------------------------
struct cs_ref {  // EXTERNAL/csparse/cs.h:47-56 (csi = int)
  int nzmax, m, n;
  int* p;
  int* i;
  double* x;
  int nz;
};
struct RefCS {
  void* h = nullptr;
  int* (*cs_amd)(int, const cs_ref*) = nullptr;
  int (*cs_cholsol)(int, const cs_ref*, double*) = nullptr;
  void* (*cs_free)(void*) = nullptr;
  std::string path;
  RefCS() {
    std::vector<std::string> cands;
    if (const char* env = getenv("G2O_ORACLE_REF")) cands.push_back(env);
    Dl_info info;
    if (dladdr((void*)&now, &info) && info.dli_fname) {
      std::string self(info.dli_fname);
      auto pos = self.rfind('/');
      std::string dir = pos == std::string::npos ? "." : self.substr(0, pos);
      cands.push_back(dir + "/_ref/libcsparse_ref.so");
    }
    for (auto& c : cands) {
      h = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (h) { path = c; break; }
    }
    if (!h) return;
    cs_amd = (int* (*)(int, const cs_ref*))dlsym(h, "cs_amd");
    cs_cholsol = (int (*)(int, const cs_ref*, double*))dlsym(h, "cs_cholsol");
    cs_free = (void* (*)(void*))dlsym(h, "cs_free");
    if (!cs_amd || !cs_cholsol || !cs_free) { dlclose(h); h = nullptr; path.clear(); }
  }
  bool ok() const { return h != nullptr; }
};
RefCS& refcs() {
  static RefCS r;
  return r;
}

// --------------------------------------------------------------------------------------------
// Restated CSparse pieces (EXTERNAL/csparse/*.c; csparse_extension.cpp:64-119)
// --------------------------------------------------------------------------------------------
struct CCS {
  int n = 0;
  std::vector<int> p, i;
  std::vector<double> x;
};

std::vector<int> make_pinv(const std::vector<int>& p) {  // cs_pinv.c
  std::vector<int> pinv(p.size());
  for (size_t k = 0; k < p.size(); ++k) pinv[p[k]] = (int)k;
  return pinv;
}

// cs_symperm.c (upper part, values via an index map so values can be refreshed)
void symperm_upper(const CCS& A, const std::vector<int>& pinv, CCS& C, std::vector<int>& map) {
  const int n = A.n;
  std::vector<int> w(n, 0);
  for (int j = 0; j < n; ++j) {
    const int j2 = pinv[j];
    for (int p = A.p[j]; p < A.p[j + 1]; ++p) {
      const int i = A.i[p];
      if (i > j) continue;
      w[std::max(pinv[i], j2)]++;
    }
  }
  C.n = n;
  C.p.assign(n + 1, 0);
  for (int k = 0; k < n; ++k) C.p[k + 1] = C.p[k] + w[k];
  for (int k = 0; k < n; ++k) w[k] = C.p[k];
  C.i.assign(C.p[n], 0);
  C.x.assign(C.p[n], 0.0);
  map.assign(C.p[n], 0);
  for (int j = 0; j < n; ++j) {
    const int j2 = pinv[j];
    for (int p = A.p[j]; p < A.p[j + 1]; ++p) {
      const int i = A.i[p];
      if (i > j) continue;
      const int i2 = pinv[i];
      const int q = w[std::max(i2, j2)]++;
      C.i[q] = std::min(i2, j2);
      map[q] = p;
    }
  }
}

// cs_etree.c (ata = 0)
std::vector<int> etree(const CCS& A) {
  const int n = A.n;
  std::vector<int> parent(n), ancestor(n);
  for (int k = 0; k < n; ++k) {
    parent[k] = -1;
    ancestor[k] = -1;
    for (int p = A.p[k]; p < A.p[k + 1]; ++p) {
      int i = A.i[p];
      int inext;
      for (; i != -1 && i < k; i = inext) {
        inext = ancestor[i];
        ancestor[i] = k;
        if (inext == -1) parent[i] = k;
      }
    }
  }
  return parent;
}

// cs_ereach.c: nonzero pattern of row k of L, in s[top..n-1] (same traversal order as CSparse)
int ereach(const CCS& A, int k, const std::vector<int>& parent, std::vector<int>& s, std::vector<int>& mark,
           int stamp) {
  const int n = A.n;
  int top = n;
  mark[k] = stamp;
  for (int p = A.p[k]; p < A.p[k + 1]; ++p) {
    int i = A.i[p];
    if (i > k) continue;
    int len = 0;
    for (; mark[i] != stamp; i = parent[i]) {
      s[len++] = i;
      mark[i] = stamp;
    }
    while (len > 0) s[--top] = s[--len];
  }
  return top;
}

// column counts of L by running the symbolic up-looking pass (same result as cs_counts)
std::vector<int> colcounts(const CCS& C, const std::vector<int>& parent) {
  const int n = C.n;
  std::vector<int> cnt(n, 1), s(n), mark(n, -1);
  for (int k = 0; k < n; ++k) {
    int top = ereach(C, k, parent, s, mark, k);
    for (; top < n; ++top) cnt[s[top]]++;
  }
  return cnt;
}

// cs_chol_workspace (csparse_extension.cpp:64-119) == cs_chol.c numerically
bool chol_numeric(const CCS& C, const std::vector<int>& parent, const std::vector<int>& cp, std::vector<int>& Li,
                  std::vector<double>& Lx) {
  const int n = C.n;
  std::vector<int> c(cp.begin(), cp.begin() + n), s(n), mark(n, -1);
  std::vector<double> x(n, 0.0);
  Li.assign(cp[n], 0);
  Lx.assign(cp[n], 0.0);
  for (int k = 0; k < n; ++k) {
    int top = ereach(C, k, parent, s, mark, k);
    x[k] = 0;
    for (int p = C.p[k]; p < C.p[k + 1]; ++p)
      if (C.i[p] <= k) x[C.i[p]] = C.x[p];
    double d = x[k];
    x[k] = 0;
    for (; top < n; ++top) {
      const int i = s[top];
      const double lki = x[i] / Lx[cp[i]];
      x[i] = 0;
      for (int p = cp[i] + 1; p < c[i]; ++p) x[Li[p]] -= Lx[p] * lki;
      d -= lki * lki;
      const int p = c[i]++;
      Li[p] = k;
      Lx[p] = lki;
    }
    if (d <= 0) return false;
    const int p = c[k]++;
    Li[p] = k;
    Lx[p] = std::sqrt(d);
  }
  return true;
}

// cs_ipvec / cs_lsolve / cs_ltsolve / cs_pvec (csparse_extension.cpp:47-52)
void chol_solve(int n, const std::vector<int>& pinv, const std::vector<int>& cp, const std::vector<int>& Li,
                const std::vector<double>& Lx, double* b, std::vector<double>& x) {
  x.assign(n, 0.0);
  for (int k = 0; k < n; ++k) x[pinv[k]] = b[k];  // cs_ipvec(pinv, b, x)
  for (int j = 0; j < n; ++j) {                   // cs_lsolve
    x[j] /= Lx[cp[j]];
    for (int p = cp[j] + 1; p < cp[j + 1]; ++p) x[Li[p]] -= Lx[p] * x[j];
  }
  for (int j = n - 1; j >= 0; --j) {  // cs_ltsolve
    for (int p = cp[j] + 1; p < cp[j + 1]; ++p) x[j] -= Lx[p] * x[Li[p]];
    x[j] /= Lx[cp[j]];
  }
  for (int k = 0; k < n; ++k) b[k] = x[pinv[k]];  // cs_pvec(pinv, x, b)
}

// --------------------------------------------------------------------------------------------
// Graph
// --------------------------------------------------------------------------------------------
int vdim(int type) {
  switch (type) {
    case ORACLE_V_SE3_EXPMAP: return 6;
    case ORACLE_V_XYZ: return 3;
    case ORACLE_V_SE3_QUAT: return 6;
    case ORACLE_V_SE2: return 3;
    case ORACLE_V_XY: return 2;
  }
  return -1;
}
int edim(int type) {
  switch (type) {
    case ORACLE_E_SE3_PROJECT_XYZ: return 2;
    case ORACLE_E_SE3_QUAT: return 6;
    case ORACLE_E_SE2: return 3;
    case ORACLE_E_SE3_EXPMAP: return 6;
    case ORACLE_E_SE2_XY: return 2;
  }
  return -1;
}

struct VState {
  SE3Quat q;
  V3 p{0, 0, 0};
  Iso3 iso;
  SE2 se2;
  int numOplus = 0;  // VertexSE3::_numOplusCalls (vertex_se3.h:124) — not part of push/pop
};

struct Vertex {
  int id = 0, type = 0, dim = 0;
  bool fixed = false, marginalized = false;
  VState est;
  std::vector<VState> stack;  // base_vertex.h:93-95
  std::vector<int> edges;
  int hessianIndex = -1;
  int colInHessian = -1;
  size_t Hoff = 0;
  bool HinHll = false;
  double b[6] = {0, 0, 0, 0, 0, 0};
};

struct Edge {
  int type = 0, D = 0;
  int v[2] = {0, 0};  // vertex slots (index into Graph::verts)
  double meas[7] = {0};
  double info[36] = {0};
  double params[4] = {0};
  double err[6] = {0};
  Iso3 Z, Zinv;   // EdgeSE3 (edge_se3.h:53-56)
  SE2 m2, m2inv;  // EdgeSE2 (edge_se2.h:58-61)
  int offKind = 0;  // 0 none, 1 Hpp block, 2 Hpl block, 3 Hll block
  size_t offOff = 0;
  bool rowMajor = false;
  int rk = 0;              // robust kernel (ORACLE_RK_* = G2OHIP_RK_*), 0 none
  double rkDelta = 1.0;
  bool numeric = false;    // linearizeOplus by BaseBinaryEdge's numeric differences (a type without analytic J)
};

// RobustKernel*::robustify (robust_kernel_impl.cpp:60-200): rho[0], rho[1]
void robustify(int kind, double delta, double e2, double& r0, double& r1) {
  switch (kind) {
    case 1: {  // Huber :65-78
      const double dsqr = delta * delta;
      if (e2 <= dsqr) { r0 = e2; r1 = 1.; }
      else { const double sqrte = std::sqrt(e2); r0 = 2 * sqrte * delta - dsqr; r1 = delta / sqrte; }
      return;
    }
    case 2: {  // PseudoHuber
      const double dsqr = delta * delta, dsqrReci = 1. / dsqr, aux1 = dsqrReci * e2 + 1.0, aux2 = std::sqrt(aux1);
      r0 = 2 * dsqr * (aux2 - 1);
      r1 = 1. / aux2;
      return;
    }
    case 3: {  // Cauchy
      const double dsqr = delta * delta, dsqrReci = 1. / dsqr, aux = dsqrReci * e2 + 1.0;
      r0 = dsqr * std::log(aux);
      r1 = 1. / aux;
      return;
    }
    case 4: {  // GemanMcClure
      const double aux = delta / (delta + e2);
      r0 = e2 * aux;
      r1 = aux * aux;
      return;
    }
    case 5: {  // Welsch
      const double dsqr = delta * delta, aux = e2 / dsqr, aux2 = std::exp(-aux);
      r0 = dsqr * (1. - aux2);
      r1 = aux2;
      return;
    }
    case 6: {  // Fair
      const double sqrte = std::sqrt(e2), aux = sqrte / delta;
      r0 = 2. * delta * delta * (aux - std::log(1. + aux));
      r1 = 1. / (1. + aux);
      return;
    }
    case 7: {  // Tukey
      const double e = std::sqrt(e2), delta2 = delta * delta;
      if (e <= delta) {
        const double aux = e2 / delta2;
        r0 = delta2 * (1. - std::pow((1. - aux), 3)) / 3.;
        r1 = std::pow((1. - aux), 2);
      } else {
        r0 = delta2 / 3.;
        r1 = 0;
      }
      return;
    }
    case 8: {  // Saturated
      const double dsqr = delta * delta;
      if (e2 <= dsqr) { r0 = e2; r1 = 1.; }
      else { r0 = dsqr; r1 = 0.; }
      return;
    }
    case 9: {  // DCS
      double scale = (2.0 * delta) / (delta + e2);
      if (scale >= 1.0) scale = 1.0;
      r0 = scale * e2 * scale;
      r1 = scale * scale;
      return;
    }
  }
  r0 = e2;
  r1 = 1.;
}

struct SBM {  // core/sparse_block_matrix.h:62-231
  std::vector<int> rowBlockIndices, colBlockIndices;  // cumulative END offsets
  std::vector<std::map<int, size_t>> cols;
  std::vector<double> arena;
  int rowsOfBlock(int r) const { return r ? rowBlockIndices[r] - rowBlockIndices[r - 1] : rowBlockIndices[0]; }
  int colsOfBlock(int c) const { return c ? colBlockIndices[c] - colBlockIndices[c - 1] : colBlockIndices[0]; }
  int rowBaseOfBlock(int r) const { return r ? rowBlockIndices[r - 1] : 0; }
  int colBaseOfBlock(int c) const { return c ? colBlockIndices[c - 1] : 0; }
  int rows() const { return rowBlockIndices.empty() ? 0 : rowBlockIndices.back(); }
  int ncols() const { return colBlockIndices.empty() ? 0 : colBlockIndices.back(); }
  void init(const std::vector<int>& rbi, const std::vector<int>& cbi) {
    rowBlockIndices = rbi;
    colBlockIndices = cbi;
    cols.assign(cbi.size(), {});
    arena.clear();
  }
  size_t block(int r, int c) {
    auto it = cols[c].find(r);
    if (it != cols[c].end()) return it->second;
    size_t off = arena.size();
    arena.resize(off + (size_t)rowsOfBlock(r) * colsOfBlock(c), 0.0);
    cols[c][r] = off;
    return off;
  }
  void clear() { std::fill(arena.begin(), arena.end(), 0.0); }
  // sparse_block_matrix.hpp:496-549 fillCCS(upper=true): structure + values
  void fillCCS(CCS& A) const {
    const int n = ncols();
    A.n = n;
    A.p.assign(n + 1, 0);
    A.i.clear();
    A.x.clear();
    for (size_t bc = 0; bc < cols.size(); ++bc) {
      const int cstart = colBaseOfBlock((int)bc), csize = colsOfBlock((int)bc);
      for (int c = 0; c < csize; ++c) {
        A.p[cstart + c] = (int)A.i.size();
        for (auto& kv : cols[bc]) {
          const int rstart = rowBaseOfBlock(kv.first), rsz = rowsOfBlock(kv.first);
          int elems = rsz;
          if (rstart == cstart) elems = c + 1;
          const double* b = arena.data() + kv.second + (size_t)c * rsz;
          for (int r = 0; r < elems; ++r) {
            A.i.push_back(rstart + r);
            A.x.push_back(b[r]);
          }
        }
      }
    }
    A.p[n] = (int)A.i.size();
  }
  void fillCCSValues(CCS& A) const {
    size_t k = 0;
    for (size_t bc = 0; bc < cols.size(); ++bc) {
      const int cstart = colBaseOfBlock((int)bc), csize = colsOfBlock((int)bc);
      for (int c = 0; c < csize; ++c)
        for (auto& kv : cols[bc]) {
          const int rstart = rowBaseOfBlock(kv.first), rsz = rowsOfBlock(kv.first);
          int elems = rstart == cstart ? c + 1 : rsz;
          const double* b = arena.data() + kv.second + (size_t)c * rsz;
          for (int r = 0; r < elems; ++r) A.x[k++] = b[r];
        }
    }
  }
};

struct Config {
  int maxTrials = 10;
  double userLambdaInit = 0;
  int threads = 1;
  bool useRef = true;
  bool blockOrdering = true;
  bool gaussNewton = false;
};

struct Stats {
  oracle_batch_stats* cur = nullptr;
};

// linear_solver_csparse.h
struct LinearSolverCSparse {
  bool blockOrdering = true;
  bool useRef = true;
  bool haveSymbolic = false;
  CCS A, C;
  std::vector<int> Cmap, pinv, parent, cp, Li;
  std::vector<double> Lx, xw;
  long long lnz = 0;
  void reset() { haveSymbolic = false; }

  void computeSymbolic(const SBM& M, oracle_batch_stats* st) {  // :246-308
    double t = now();
    const int n = A.n;
    std::vector<int> P;
    if (blockOrdering) {
      // fillBlockStructure (sparse_block_matrix.hpp:551-577): block pattern, r <= c
      const int nb = (int)M.cols.size();
      std::vector<int> bp(nb + 1, 0), bi;
      for (int c = 0; c < nb; ++c) {
        bp[c] = (int)bi.size();
        for (auto& kv : M.cols[c])
          if (kv.first <= c) bi.push_back(kv.first);
      }
      bp[nb] = (int)bi.size();
      std::vector<int> bperm(nb);
      if (useRef && refcs().ok()) {
        cs_ref aux{(int)bi.size(), nb, nb, bp.data(), bi.data(), nullptr, -1};
        int* p = refcs().cs_amd(1, &aux);
        for (int k = 0; k < nb; ++k) bperm[k] = p[k];
        refcs().cs_free(p);
      } else {
        for (int k = 0; k < nb; ++k) bperm[k] = k;
      }
      for (int k = 0; k < nb; ++k) {
        int base = M.colBaseOfBlock(bperm[k]), nc = M.colsOfBlock(bperm[k]);
        for (int j = 0; j < nc; ++j) P.push_back(base + j);
      }
    } else {
      P.resize(n);
      if (useRef && refcs().ok()) {
        cs_ref aux{(int)A.i.size(), n, n, A.p.data(), A.i.data(), A.x.data(), -1};
        int* p = refcs().cs_amd(1, &aux);
        for (int k = 0; k < n; ++k) P[k] = p[k];
        refcs().cs_free(p);
      } else {
        for (int k = 0; k < n; ++k) P[k] = k;
      }
    }
    pinv = make_pinv(P);
    symperm_upper(A, pinv, C, Cmap);
    parent = etree(C);
    std::vector<int> cnt = colcounts(C, parent);
    cp.assign(n + 1, 0);
    for (int k = 0; k < n; ++k) cp[k + 1] = cp[k] + cnt[k];
    lnz = cp[n];
    haveSymbolic = true;
    if (st) st->timeSymbolicDecomposition = now() - t;
  }

  bool solve(const SBM& M, double* x, double* b, oracle_batch_stats* st) {  // :106-142
    if (!haveSymbolic) M.fillCCS(A);
    else M.fillCCSValues(A);
    if (!haveSymbolic) computeSymbolic(M, st);
    double t = now();
    for (size_t k = 0; k < Cmap.size(); ++k) C.x[k] = A.x[Cmap[k]];
    if (x != b) std::memcpy(x, b, sizeof(double) * A.n);
    bool ok = chol_numeric(C, parent, cp, Li, Lx);
    if (!ok) return false;
    chol_solve(A.n, pinv, cp, Li, Lx, x, xw);
    if (st) {
      st->timeNumericDecomposition = now() - t;
      st->choleskyNNZ = lnz;
    }
    return true;
  }
};

struct Graph;

// block_solver.hpp
struct BlockSolver {
  Graph* g = nullptr;
  int numPoses = 0, numLandmarks = 0, sizePoses = 0, sizeLandmarks = 0;
  bool doSchur = false;
  SBM Hpp, Hll, Hpl, Hschur;
  std::vector<std::vector<std::pair<int, size_t>>> HplCCS;            // per landmark: (pose row, off) sorted
  std::vector<std::vector<std::pair<int, size_t>>> HschurTransposed;  // per pose row i1: (i2>=i1, off)
  std::vector<double> DInv;   // per landmark l*l
  std::vector<size_t> DInvOff;
  std::vector<double> x, b, coefficients, bschur;
  std::vector<std::vector<double>> diagBackupPose, diagBackupLandmark;
  LinearSolverCSparse lin;
  std::vector<omp_lock_t> vlocks, coeffLocks;
  ~BlockSolver() {
    for (auto& l : vlocks) omp_destroy_lock(&l);
    for (auto& l : coeffLocks) omp_destroy_lock(&l);
  }
  bool buildStructure(Graph& G);
  void buildSystem(Graph& G, int threads);
  void setLambda(double lambda, bool backup);
  void restoreDiagonal();
  bool solve(int threads, oracle_batch_stats* st);
};

struct Graph {
  std::vector<Vertex> verts;
  std::unordered_map<int, int> idmap;
  std::vector<Edge> edges;
  // SparseOptimizer state (sparse_optimizer.h:193-197)
  std::vector<int> activeVertices;  // sorted by id
  std::vector<int> ivMap;           // index mapping: poses first, then landmarks
  bool initialized = false;
  BlockSolver solver;
  bool structureBuilt = false;
  double* vH(Vertex& v) {
    return v.HinHll ? solver.Hll.arena.data() + v.Hoff : solver.Hpp.arena.data() + v.Hoff;
  }
};

// ---------------- vertex ops ----------------
void vertexOplus(Vertex& v, const double* u) {
  switch (v.type) {
    case ORACLE_V_SE3_EXPMAP:  // types_six_dof_expmap.h:97-100
      v.est.q = se3mul(se3exp(u), v.est.q);
      break;
    case ORACLE_V_XYZ:  // types_sba.h:149-153
      v.est.p = add(v.est.p, V3{u[0], u[1], u[2]});
      break;
    case ORACLE_V_SE3_QUAT: {  // vertex_se3.h:105-113
      Iso3 inc = fromVectorMQT(u);
      v.est.iso = isomul(v.est.iso, inc);
      if (++v.est.numOplus > 1000) {
        v.est.numOplus = 0;
        approximateNearestOrthogonalMatrix(v.est.iso.R);
      }
      break;
    }
    case ORACLE_V_SE2: {  // vertex_se2.h:51-58
      v.est.se2.x += u[0];
      v.est.se2.y += u[1];
      v.est.se2.th = normalize_theta(v.est.se2.th + u[2]);
      break;
    }
    case ORACLE_V_XY:  // vertex_point_xy.h:77-81
      v.est.p.x += u[0];
      v.est.p.y += u[1];
      break;
  }
}
void vpush(Vertex& v) { v.stack.push_back(v.est); }
void vpop(Vertex& v) {
  int n = v.est.numOplus;
  v.est = v.stack.back();
  v.est.numOplus = n;
  v.stack.pop_back();
}
void vdiscard(Vertex& v) { v.stack.pop_back(); }

// ---------------- edge error / Jacobians ----------------
void computeError(const Graph& G, Edge& e) {
  const Vertex& a = G.verts[e.v[0]];
  const Vertex& b = G.verts[e.v[1]];
  switch (e.type) {
    case ORACLE_E_SE3_PROJECT_XYZ: {  // types_six_dof_expmap.h:211-216
      V3 pc = se3map(b.est.q, a.est.p);
      const double u = pc.x / pc.z * e.params[0] + e.params[2];
      const double w = pc.y / pc.z * e.params[1] + e.params[3];
      e.err[0] = e.meas[0] - u;
      e.err[1] = e.meas[1] - w;
      break;
    }
    case ORACLE_E_SE3_QUAT: {  // edge_se3.cpp:77-82
      Iso3 delta = isomul(isomul(e.Zinv, isoinv(a.est.iso)), b.est.iso);
      toVectorMQT(delta, e.err);
      break;
    }
    case ORACLE_E_SE3_EXPMAP: {  // types_six_dof_expmap.h:117-124: (v2^-1 * C * v1).log()
      SE3Quat C;
      C.t = {e.meas[0], e.meas[1], e.meas[2]};
      C.r = Quat{e.meas[6], e.meas[3], e.meas[4], e.meas[5]};
      se3log(se3mul(se3mul(se3inv(b.est.q), C), a.est.q), e.err);
      break;
    }
    case ORACLE_E_SE2: {  // edge_se2.h:46-52
      SE2 delta = se2mul(e.m2inv, se2mul(se2inv(a.est.se2), b.est.se2));
      e.err[0] = delta.x;
      e.err[1] = delta.y;
      e.err[2] = delta.th;
      break;
    }
    case ORACLE_E_SE2_XY: {  // edge_se2_pointxy.h:44-49: v1^-1 * l - z (se2.h:77-80 SE2 * Vector2 = t + R v)
      const SE2 inv = se2inv(a.est.se2);
      const double c = std::cos(inv.th), s = std::sin(inv.th);
      e.err[0] = (inv.x + (c * b.est.p.x - s * b.est.p.y)) - e.meas[0];
      e.err[1] = (inv.y + (s * b.est.p.x + c * b.est.p.y)) - e.meas[1];
      break;
    }
  }
}

double edgeChi2(const Edge& e) {  // base_edge.h chi2() = e' * Omega * e
  double s = 0;
  for (int i = 0; i < e.D; ++i) {
    double r = 0;
    for (int j = 0; j < e.D; ++j) r += e.info[i * e.D + j] * e.err[j];
    s += e.err[i] * r;
  }
  return s;
}

// Analytic Jacobians, row-major D x dim
void linearizeOplus(const Graph& G, const Edge& e, double* Ji, double* Jj) {
  const Vertex& va = G.verts[e.v[0]];
  const Vertex& vb = G.verts[e.v[1]];
  switch (e.type) {
    case ORACLE_E_SE3_PROJECT_XYZ: {  // types_six_dof_expmap.cpp:395-447
      const SE3Quat& T = vb.est.q;
      V3 xt = se3map(T, va.est.p);
      const double x = xt.x, y = xt.y, z = xt.z, z2 = z * z;
      const double fx = e.params[0], fy = e.params[1];
      M3 R = qToR(T.r);
      double tmp[2][3] = {{fx, 0, -x / z * fx}, {0, fy, -y / z * fy}};
      for (int r = 0; r < 2; ++r)
        for (int c = 0; c < 3; ++c) {
          double s = 0;
          for (int k = 0; k < 3; ++k) s += (-1. / z * tmp[r][k]) * R.m[k][c];
          Ji[r * 3 + c] = s;
        }
      Jj[0] = x * y / z2 * fx;
      Jj[1] = -(1 + (x * x / z2)) * fx;
      Jj[2] = y / z * fx;
      Jj[3] = -1. / z * fx;
      Jj[4] = 0;
      Jj[5] = x / z2 * fx;
      Jj[6] = (1 + y * y / z2) * fy;
      Jj[7] = -x * y / z2 * fy;
      Jj[8] = -x / z * fy;
      Jj[9] = 0;
      Jj[10] = -1. / z * fy;
      Jj[11] = y / z2 * fy;
      break;
    }
    case ORACLE_E_SE3_QUAT: {  // isometry3d_gradients.h:194-260 (computeEdgeSE3Gradient, no offsets)
      const Iso3& Xi = va.est.iso;
      const Iso3& Xj = vb.est.iso;
      Iso3 A = e.Zinv;  // Z.inverse()
      Iso3 B = isomul(isoinv(Xi), Xj);
      Iso3 E = isomul(A, B);
      const M3& Re = E.R;
      const M3& Ra = A.R;
      const M3& Rb = B.R;
      V3 tb = B.t;
      double dq[27];
      compute_dq_dR(dq, Re);
      for (int i = 0; i < 36; ++i) Ji[i] = Jj[i] = 0;
      auto setblk = [](double* J, int r0, int c0, const M3& M) {
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) J[(r0 + r) * 6 + c0 + c] = M.m[r][c];
      };
      setblk(Ji, 0, 0, mscale(Ra, -1.0));  // dte/dti
      setblk(Jj, 0, 0, Re);                // dte/dtj
      {                                    // dte/dqi: Ra * skewT(tb)
        const double X = 2 * tb.x, Y = 2 * tb.y, Zz = 2 * tb.z;
        M3 S;  // skewT: s << 0,-z,y, z,0,-x, -y,x,0  (comma init is row-major)
        S.m[0][0] = 0;  S.m[0][1] = -Zz; S.m[0][2] = Y;
        S.m[1][0] = Zz; S.m[1][1] = 0;   S.m[1][2] = -X;
        S.m[2][0] = -Y; S.m[2][1] = X;   S.m[2][2] = 0;
        setblk(Ji, 0, 3, mmul(Ra, S));
      }
      // skewT(Sx,Sy,Sz,R) (isometry3d_gradients.h:76-86), comma initialisers are row-major
      auto skewT3 = [](const M3& R, M3& Sx, M3& Sy, M3& Sz, bool transposed) {
        const double r11 = 2 * R.m[0][0], r12 = 2 * R.m[0][1], r13 = 2 * R.m[0][2];
        const double r21 = 2 * R.m[1][0], r22 = 2 * R.m[1][1], r23 = 2 * R.m[1][2];
        const double r31 = 2 * R.m[2][0], r32 = 2 * R.m[2][1], r33 = 2 * R.m[2][2];
        const double sg = transposed ? 1.0 : -1.0;
        double sx[9] = {0, 0, 0, sg * r31, sg * r32, sg * r33, -sg * r21, -sg * r22, -sg * r23};
        double sy[9] = {-sg * r31, -sg * r32, -sg * r33, 0, 0, 0, sg * r11, sg * r12, sg * r13};
        double sz[9] = {sg * r21, sg * r22, sg * r23, -sg * r11, -sg * r12, -sg * r13, 0, 0, 0};
        for (int k = 0; k < 9; ++k) {
          Sx.m[k / 3][k % 3] = sx[k];
          Sy.m[k / 3][k % 3] = sy[k];
          Sz.m[k / 3][k % 3] = sz[k];
        }
      };
      auto dqM = [&](double* J, const M3& Mx, const M3& My, const M3& Mz) {
        // M (9x3, col-major buf): column c = vec(M_c) column-major; J(3+r, 3+c) = sum_k dq[r][k] * M[k][c]
        const M3* Ms[3] = {&Mx, &My, &Mz};
        for (int r = 0; r < 3; ++r)
          for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 9; ++k) s += dq[r * 9 + k] * Ms[c]->m[k % 3][k / 3];
            J[(3 + r) * 6 + 3 + c] = s;
          }
      };
      {  // dre/dqi
        M3 Sx, Sy, Sz;
        skewT3(Rb, Sx, Sy, Sz, true);
        dqM(Ji, mmul(Ra, Sx), mmul(Ra, Sy), mmul(Ra, Sz));
      }
      {  // dre/dqj: skew(Sx,Sy,Sz, I) (non-transposed form)
        M3 Sx, Sy, Sz;
        skewT3(meye(), Sx, Sy, Sz, false);
        dqM(Jj, mmul(Re, Sx), mmul(Re, Sy), mmul(Re, Sz));
      }
      break;
    }
    case ORACLE_E_SE2: {  // edge_se2.cpp:77-103
      const SE2& si = va.est.se2;
      const SE2& sj = vb.est.se2;
      const double thetai = si.th;
      const double dtx = sj.x - si.x, dty = sj.y - si.y;
      const double s = std::sin(thetai), c = std::cos(thetai);
      double A[9] = {-c, -s, -s * dtx + c * dty, s, -c, -c * dtx - s * dty, 0, 0, -1};
      double B[9] = {c, s, 0, -s, c, 0, 0, 0, 1};
      const double rc = std::cos(e.m2inv.th), rs = std::sin(e.m2inv.th);
      double Z[9] = {rc, -rs, 0, rs, rc, 0, 0, 0, 1};
      for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) {
          double a = 0, b = 0;
          for (int k = 0; k < 3; ++k) {
            a += Z[r * 3 + k] * A[k * 3 + cc];
            b += Z[r * 3 + k] * B[k * 3 + cc];
          }
          Ji[r * 3 + cc] = a;
          Jj[r * 3 + cc] = b;
        }
      break;
    }
    case ORACLE_E_SE2_XY: {  // edge_se2_pointxy.cpp:63-87
      const double x1 = va.est.se2.x, y1 = va.est.se2.y, th1 = va.est.se2.th;
      const double x2 = vb.est.p.x, y2 = vb.est.p.y;
      const double aux_1 = std::cos(th1), aux_2 = -aux_1, aux_3 = std::sin(th1);
      Ji[0] = aux_2;
      Ji[1] = -aux_3;
      Ji[2] = aux_1 * y2 - aux_1 * y1 - aux_3 * x2 + aux_3 * x1;
      Ji[3] = aux_3;
      Ji[4] = aux_2;
      Ji[5] = -aux_3 * y2 + aux_3 * y1 - aux_1 * x2 + aux_1 * x1;
      Jj[0] = aux_1;
      Jj[1] = aux_3;
      Jj[2] = -aux_3;
      Jj[3] = aux_1;
      break;
    }
  }
}

// base_binary_edge.hpp:198-266 numeric Jacobian (delta = 1e-9, central differences)
void linearizeNumeric(Graph& G, Edge& e, double* Ji, double* Jj) {
  const double delta = 1e-9, scal = 1 / (2 * delta);
  double ebak[6];
  std::memcpy(ebak, e.err, sizeof ebak);
  for (int side = 0; side < 2; ++side) {
    Vertex& v = G.verts[e.v[side]];
    double* J = side == 0 ? Ji : Jj;
    double add[6] = {0, 0, 0, 0, 0, 0};
    for (int d = 0; d < v.dim; ++d) {
      double ep[6];
      vpush(v);
      add[d] = delta;
      vertexOplus(v, add);
      computeError(G, e);
      std::memcpy(ep, e.err, sizeof ep);
      vpop(v);
      vpush(v);
      add[d] = -delta;
      vertexOplus(v, add);
      computeError(G, e);
      for (int k = 0; k < e.D; ++k) ep[k] -= e.err[k];
      vpop(v);
      add[d] = 0;
      for (int k = 0; k < e.D; ++k) J[k * v.dim + d] = scal * ep[k];
    }
  }
  std::memcpy(e.err, ebak, sizeof ebak);
}

// ---------------- SparseOptimizer ----------------
void initializeOptimization(Graph& G) {  // sparse_optimizer.cpp:201-279 (level 0, all edges)
  G.activeVertices.clear();
  for (size_t k = 0; k < G.verts.size(); ++k)
    if (!G.verts[k].edges.empty()) G.activeVertices.push_back((int)k);
  std::sort(G.activeVertices.begin(), G.activeVertices.end(),
            [&](int a, int b) { return G.verts[a].id < G.verts[b].id; });
  G.ivMap.clear();  // buildIndexMapping (:168-192)
  for (int k = 0; k < 2; ++k)
    for (int vi : G.activeVertices) {
      Vertex& v = G.verts[vi];
      if (!v.fixed) {
        if ((int)v.marginalized == k) {
          v.hessianIndex = (int)G.ivMap.size();
          G.ivMap.push_back(vi);
        }
      } else {
        v.hessianIndex = -1;
      }
    }
  G.initialized = true;
  G.structureBuilt = false;
}

// sparse_optimizer.cpp:465-502 (updateInitialization) + block_solver.hpp:258-312 (updateStructure), online mode: the
// vertices that gained edges since the last initialization are appended to the index mapping (free ones take the next
// hessian indices; the reference walks the caller's vertex set, here the new vertices in id order); the existing
// vertices keep their indices. The next LM iteration 0 rebuilds Hpp over the grown mapping — the same blocks the
// reference's updateStructure adds to its Hpp — and the linear solver re-analyses (LinearSolverCSparse::init).
// Marginalized vertices: -3 (the reference aborts, sparse_optimizer.cpp:491-492; Schur unsupported :274-277).
int updateInitialization(Graph& G) {
  if (G.ivMap.empty()) return -1;
  for (int vi : G.ivMap)
    if (G.verts[vi].marginalized) return -3;
  std::vector<char> was(G.verts.size(), 0);
  for (int vi : G.activeVertices) was[vi] = 1;
  std::vector<int> fresh;
  for (size_t k = 0; k < G.verts.size(); ++k)
    if (!was[k] && !G.verts[k].edges.empty()) fresh.push_back((int)k);
  std::sort(fresh.begin(), fresh.end(), [&](int a, int b) { return G.verts[a].id < G.verts[b].id; });
  for (int vi : fresh)
    if (!G.verts[vi].fixed && G.verts[vi].marginalized) return -3;
  for (int vi : fresh) {
    G.activeVertices.push_back(vi);
    Vertex& v = G.verts[vi];
    if (v.fixed) {
      v.hessianIndex = -1;
      continue;
    }
    v.hessianIndex = (int)G.ivMap.size();
    G.ivMap.push_back(vi);
  }
  G.initialized = true;
  G.structureBuilt = false;
  return 0;
}

void computeActiveErrors(Graph& G, int threads) {  // sparse_optimizer.cpp:63-90
  const int ne = (int)G.edges.size();
#pragma omp parallel for num_threads(threads) if (ne > 50)
  for (int k = 0; k < ne; ++k) computeError(G, G.edges[k]);
}
double activeRobustChi2(const Graph& G) {  // :102-116
  double chi = 0;
  for (const Edge& e : G.edges) {
    if (e.rk) {
      double r0, r1;
      robustify(e.rk, e.rkDelta, edgeChi2(e), r0, r1);
      chi += r0;
    } else {
      chi += edgeChi2(e);
    }
  }
  return chi;
}
void update(Graph& G, const double* upd) {  // :441-454
  for (int vi : G.ivMap) {
    Vertex& v = G.verts[vi];
    vertexOplus(v, upd);
    upd += v.dim;
  }
}
void push(Graph& G) { for (int vi : G.activeVertices) vpush(G.verts[vi]); }
void pop(Graph& G) { for (int vi : G.activeVertices) vpop(G.verts[vi]); }
void discardTop(Graph& G) { for (int vi : G.activeVertices) vdiscard(G.verts[vi]); }

// ---------------- BlockSolver ----------------
bool BlockSolver::buildStructure(Graph& G) {  // block_solver.hpp:102-256
  g = &G;
  numPoses = numLandmarks = sizePoses = sizeLandmarks = 0;
  std::vector<int> blockPoseIndices, blockLandmarkIndices;
  for (int vi : G.ivMap) {
    Vertex& v = G.verts[vi];
    if (!v.marginalized) {
      v.colInHessian = sizePoses;
      sizePoses += v.dim;
      blockPoseIndices.push_back(sizePoses);
      ++numPoses;
    } else {
      v.colInHessian = sizeLandmarks;
      sizeLandmarks += v.dim;
      blockLandmarkIndices.push_back(sizeLandmarks);
      ++numLandmarks;
    }
  }
  doSchur = numLandmarks > 0;  // optimization_algorithm_with_hessian.cpp:48-73
  Hpp.init(blockPoseIndices, blockPoseIndices);
  if (doSchur) {
    Hll.init(blockLandmarkIndices, blockLandmarkIndices);
    Hpl.init(blockPoseIndices, blockLandmarkIndices);
    Hschur.init(blockPoseIndices, blockPoseIndices);
  }
  const int n = sizePoses + sizeLandmarks;
  x.assign(n, 0.0);
  b.assign(n, 0.0);
  coefficients.assign(sizePoses, 0.0);
  bschur.assign(sizePoses, 0.0);
  int poseIdx = 0, landmarkIdx = 0;
  for (int vi : G.ivMap) {
    Vertex& v = G.verts[vi];
    if (!v.marginalized) {
      v.Hoff = Hpp.block(poseIdx, poseIdx);
      v.HinHll = false;
      ++poseIdx;
    } else {
      v.Hoff = Hll.block(landmarkIdx, landmarkIdx);
      v.HinHll = true;
      ++landmarkIdx;
    }
  }
  std::map<std::pair<int, int>, int> schurLookup;  // SparseBlockMatrixHashMap
  for (Edge& e : G.edges) {
    e.offKind = 0;
    Vertex& v1 = G.verts[e.v[0]];
    Vertex& v2 = G.verts[e.v[1]];
    int ind1 = v1.hessianIndex, ind2 = v2.hessianIndex;
    if (ind1 == -1 || ind2 == -1) continue;
    bool transposed = ind1 > ind2;
    if (transposed) std::swap(ind1, ind2);
    if (!v1.marginalized && !v2.marginalized) {
      e.offKind = 1;
      e.offOff = Hpp.block(ind1, ind2);
      e.rowMajor = transposed;
      if (doSchur) schurLookup[{ind1, ind2}] = 1;
    } else if (v1.marginalized && v2.marginalized) {
      e.offKind = 3;
      e.offOff = Hll.block(ind1 - numPoses, ind2 - numPoses);
      e.rowMajor = false;
    } else if (v1.marginalized) {
      e.offKind = 2;
      e.offOff = Hpl.block(v2.hessianIndex, v1.hessianIndex - numPoses);
      e.rowMajor = true;
    } else {
      e.offKind = 2;
      e.offOff = Hpl.block(v1.hessianIndex, v2.hessianIndex - numPoses);
      e.rowMajor = false;
    }
  }
  if (!doSchur) return true;
  DInvOff.assign(numLandmarks, 0);
  size_t dsz = 0;
  for (int l = 0; l < numLandmarks; ++l) {
    DInvOff[l] = dsz;
    int d = Hll.rowsOfBlock(l);
    dsz += (size_t)d * d;
  }
  DInv.assign(dsz, 0.0);
  HplCCS.assign(numLandmarks, {});
  for (int l = 0; l < numLandmarks; ++l)
    for (auto& kv : Hpl.cols[l]) HplCCS[l].push_back({kv.first, kv.second});
  for (int vi : G.ivMap) {
    Vertex& v = G.verts[vi];
    if (!v.marginalized) continue;
    for (int e1 : v.edges)
      for (int a = 0; a < 2; ++a) {
        Vertex& va = G.verts[G.edges[e1].v[a]];
        if (va.hessianIndex == -1 || &va == &v) continue;
        for (int e2 : v.edges)
          for (int bb = 0; bb < 2; ++bb) {
            Vertex& vb = G.verts[G.edges[e2].v[bb]];
            if (vb.hessianIndex == -1 || &vb == &v) continue;
            if (va.hessianIndex <= vb.hessianIndex) schurLookup[{va.hessianIndex, vb.hessianIndex}] = 1;
          }
      }
  }
  for (int i = 0; i < numPoses; ++i) schurLookup[{i, i}] = 1;
  for (auto& kv : schurLookup) Hschur.block(kv.first.first, kv.first.second);  // takePatternFromHash
  HschurTransposed.assign(numPoses, {});
  for (int c = 0; c < numPoses; ++c)
    for (auto& kv : Hschur.cols[c]) HschurTransposed[kv.first].push_back({c, kv.second});
  return true;
}

void BlockSolver::buildSystem(Graph& G, int threads) {  // block_solver.hpp:462-521
  for (int vi : G.ivMap) {
    Vertex& v = G.verts[vi];
    for (int k = 0; k < 6; ++k) v.b[k] = 0;
  }
  Hpp.clear();
  if (doSchur) {
    Hll.clear();
    Hpl.clear();
  }
  if ((int)vlocks.size() != (int)G.verts.size()) {
    for (auto& l : vlocks) omp_destroy_lock(&l);
    vlocks.assign(G.verts.size(), omp_lock_t());
    for (auto& l : vlocks) omp_init_lock(&l);
  }
  const int ne = (int)G.edges.size();
  // numeric Jacobians perturb vertex estimates (push / oplus / pop, base_binary_edge.hpp:198-266, which the
  // reference guards with the vertex's QuadraticFormLock): computed serially up front, before the parallel loop
  std::vector<int> numIdx(ne, -1);
  std::vector<double> numJ;
  for (int k = 0; k < ne; ++k)
    if (G.edges[k].numeric) {
      numIdx[k] = (int)(numJ.size() / 72);
      numJ.resize(numJ.size() + 72);
      linearizeNumeric(G, G.edges[k], numJ.data() + (size_t)numIdx[k] * 72, numJ.data() + (size_t)numIdx[k] * 72 + 36);
    }
#pragma omp parallel for num_threads(threads) schedule(static) if (ne > 100)
  for (int k = 0; k < ne; ++k) {
    Edge& e = G.edges[k];
    Vertex& from = G.verts[e.v[0]];
    Vertex& to = G.verts[e.v[1]];
    const bool fromNotFixed = !from.fixed, toNotFixed = !to.fixed;
    if (!fromNotFixed && !toNotFixed) continue;
    double A[36], B[36];
    if (e.numeric) {
      std::memcpy(A, numJ.data() + (size_t)numIdx[k] * 72, sizeof A);
      std::memcpy(B, numJ.data() + (size_t)numIdx[k] * 72 + 36, sizeof B);
    } else {
      linearizeOplus(G, e, A, B);
    }
    const int D = e.D, di = from.dim, dj = to.dim;
    // base_binary_edge.hpp:61-137: omega_r = -Omega e; robust: weightedOmega = rho' Omega, omega_r *= rho'
    double Om[36];
    for (int k = 0; k < D * D; ++k) Om[k] = e.info[k];
    double w = 1.0;
    if (e.rk) {
      double r0;
      robustify(e.rk, e.rkDelta, edgeChi2(e), r0, w);
      for (int k = 0; k < D * D; ++k) Om[k] = w * e.info[k];
    }
    double omega_r[6];
    for (int r = 0; r < D; ++r) {
      double s = 0;
      for (int c = 0; c < D; ++c) s += e.info[r * D + c] * e.err[c];
      omega_r[r] = -s * w;
    }
    double AtO[6 * 6];  // di x D
    for (int i = 0; i < di; ++i)
      for (int c = 0; c < D; ++c) {
        double s = 0;
        for (int r = 0; r < D; ++r) s += A[r * di + i] * Om[r * D + c];
        AtO[i * D + c] = s;
      }
    if (fromNotFixed) {
      omp_set_lock(&vlocks[e.v[0]]);
      double* H = G.vH(from);  // col-major di x di
      for (int i = 0; i < di; ++i) {
        double s = 0;
        for (int r = 0; r < D; ++r) s += A[r * di + i] * omega_r[r];
        from.b[i] += s;
      }
      for (int cc = 0; cc < di; ++cc)
        for (int i = 0; i < di; ++i) {
          double s = 0;
          for (int r = 0; r < D; ++r) s += AtO[i * D + r] * A[r * di + cc];
          H[cc * di + i] += s;
        }
      omp_unset_lock(&vlocks[e.v[0]]);
      if (toNotFixed && e.offKind) {
        SBM& M = e.offKind == 1 ? Hpp : (e.offKind == 2 ? Hpl : Hll);
        double* H01 = M.arena.data() + e.offOff;
        if (e.rowMajor) {  // _hessianTransposed (dj x di, col-major) += B' * AtO'
          for (int cc = 0; cc < di; ++cc)
            for (int j = 0; j < dj; ++j) {
              double s = 0;
              for (int r = 0; r < D; ++r) s += B[r * dj + j] * AtO[cc * D + r];
              H01[cc * dj + j] += s;
            }
        } else {  // _hessian (di x dj, col-major) += AtO * B
          for (int cc = 0; cc < dj; ++cc)
            for (int i = 0; i < di; ++i) {
              double s = 0;
              for (int r = 0; r < D; ++r) s += AtO[i * D + r] * B[r * dj + cc];
              H01[cc * di + i] += s;
            }
        }
      }
    }
    if (toNotFixed) {
      omp_set_lock(&vlocks[e.v[1]]);
      double* H = G.vH(to);
      for (int j = 0; j < dj; ++j) {
        double s = 0;
        for (int r = 0; r < D; ++r) s += B[r * dj + j] * omega_r[r];
        to.b[j] += s;
      }
      double BtO[6 * 6];
      for (int j = 0; j < dj; ++j)
        for (int c = 0; c < D; ++c) {
          double s = 0;
          for (int r = 0; r < D; ++r) s += B[r * dj + j] * Om[r * D + c];
          BtO[j * D + c] = s;
        }
      for (int cc = 0; cc < dj; ++cc)
        for (int j = 0; j < dj; ++j) {
          double s = 0;
          for (int r = 0; r < D; ++r) s += BtO[j * D + r] * B[r * dj + cc];
          H[cc * dj + j] += s;
        }
      omp_unset_lock(&vlocks[e.v[1]]);
    }
  }
  for (int vi : G.ivMap) {  // copyB
    Vertex& v = G.verts[vi];
    int iBase = v.colInHessian + (v.marginalized ? sizePoses : 0);
    for (int k = 0; k < v.dim; ++k) b[iBase + k] = v.b[k];
  }
}

void BlockSolver::setLambda(double lambda, bool backup) {  // :524-550
  if (backup) {
    diagBackupPose.assign(numPoses, {});
    diagBackupLandmark.assign(numLandmarks, {});
  }
  for (int i = 0; i < numPoses; ++i) {
    double* B = Hpp.arena.data() + Hpp.cols[i].at(i);
    int d = Hpp.rowsOfBlock(i);
    if (backup) { diagBackupPose[i].resize(d); for (int k = 0; k < d; ++k) diagBackupPose[i][k] = B[k * d + k]; }
    for (int k = 0; k < d; ++k) B[k * d + k] += lambda;
  }
  for (int i = 0; i < numLandmarks; ++i) {
    double* B = Hll.arena.data() + Hll.cols[i].at(i);
    int d = Hll.rowsOfBlock(i);
    if (backup) { diagBackupLandmark[i].resize(d); for (int k = 0; k < d; ++k) diagBackupLandmark[i][k] = B[k * d + k]; }
    for (int k = 0; k < d; ++k) B[k * d + k] += lambda;
  }
}
void BlockSolver::restoreDiagonal() {  // :552-565
  for (int i = 0; i < numPoses; ++i) {
    double* B = Hpp.arena.data() + Hpp.cols[i].at(i);
    int d = Hpp.rowsOfBlock(i);
    for (int k = 0; k < d; ++k) B[k * d + k] = diagBackupPose[i][k];
  }
  for (int i = 0; i < numLandmarks; ++i) {
    double* B = Hll.arena.data() + Hll.cols[i].at(i);
    int d = Hll.rowsOfBlock(i);
    for (int k = 0; k < d; ++k) B[k * d + k] = diagBackupLandmark[i][k];
  }
}

bool BlockSolver::solve(int threads, oracle_batch_stats* st) {  // :314-447
  if (!doSchur) {
    double t = now();
    bool ok = lin.solve(Hpp, x.data(), b.data(), st);
    if (st) {
      st->timeLinearSolver = now() - t;
      st->hessianDimension = st->hessianPoseDimension = Hpp.ncols();
    }
    return ok;
  }
  double t = now();
  // Hschur = Hpp keeping the pattern of Hschur
  Hschur.clear();
  for (size_t c = 0; c < Hpp.cols.size(); ++c)
    for (auto& kv : Hpp.cols[c]) {
      const size_t so = Hschur.cols[c].at(kv.first);
      const int sz = Hpp.rowsOfBlock(kv.first) * Hpp.colsOfBlock((int)c);
      for (int k = 0; k < sz; ++k) Hschur.arena[so + k] += Hpp.arena[kv.second + k];
    }
  std::fill(coefficients.begin(), coefficients.end(), 0.0);
  if ((int)coeffLocks.size() != numPoses) {
    for (auto& l : coeffLocks) omp_destroy_lock(&l);
    coeffLocks.assign(numPoses, omp_lock_t());
    for (auto& l : coeffLocks) omp_init_lock(&l);
  }
#pragma omp parallel for num_threads(threads) schedule(dynamic, 10)
  for (int l = 0; l < numLandmarks; ++l) {
    const int ld = Hll.rowsOfBlock(l);
    const double* Dm = Hll.arena.data() + Hll.cols[l].at(l);
    double* Dinv = DInv.data() + DInvOff[l];
    if (ld == 3) {
      inverse3(Dm, Dinv);
    } else if (ld == 2) {  // Eigen compute_inverse_size2 (BlockSolver_3_2's Matrix2 inverse)
      const double invdet = 1.0 / (Dm[0] * Dm[3] - Dm[1] * Dm[2]);
      Dinv[0] = Dm[3] * invdet;
      Dinv[1] = -Dm[1] * invdet;
      Dinv[2] = -Dm[2] * invdet;
      Dinv[3] = Dm[0] * invdet;
    } else {  // generic: Gauss-Jordan (only used for other landmark dims)
      std::vector<double> M(Dm, Dm + ld * ld), I(ld * ld, 0.0);
      for (int k = 0; k < ld; ++k) I[k * ld + k] = 1;
      for (int c = 0; c < ld; ++c) {
        int piv = c;
        for (int r = c + 1; r < ld; ++r) if (std::fabs(M[c * ld + r]) > std::fabs(M[c * ld + piv])) piv = r;
        for (int k = 0; k < ld; ++k) { std::swap(M[k * ld + c], M[k * ld + piv]); std::swap(I[k * ld + c], I[k * ld + piv]); }
        double dv = M[c * ld + c];
        for (int k = 0; k < ld; ++k) { M[k * ld + c] /= dv; I[k * ld + c] /= dv; }
        for (int r = 0; r < ld; ++r) if (r != c) {
          double f = M[c * ld + r];
          for (int k = 0; k < ld; ++k) { M[k * ld + r] -= f * M[k * ld + c]; I[k * ld + r] -= f * I[k * ld + c]; }
        }
      }
      std::copy(I.begin(), I.end(), Dinv);
    }
    double db[6];
    const int lbase = Hll.rowBaseOfBlock(l) + sizePoses;
    for (int r = 0; r < ld; ++r) {
      double s = 0;
      for (int k = 0; k < ld; ++k) s += Dinv[k * ld + r] * b[lbase + k];
      db[r] = s;
    }
    const auto& col = HplCCS[l];
    for (size_t o = 0; o < col.size(); ++o) {
      const int i1 = col[o].first;
      const int pd = Hpl.rowsOfBlock(i1);
      const double* Bi = Hpl.arena.data() + col[o].second;  // pd x ld col-major
      double BDinv[6 * 6];                                  // pd x ld col-major
      for (int c = 0; c < ld; ++c)
        for (int r = 0; r < pd; ++r) {
          double s = 0;
          for (int k = 0; k < ld; ++k) s += Bi[k * pd + r] * Dinv[c * ld + k];
          BDinv[c * pd + r] = s;
        }
      omp_set_lock(&coeffLocks[i1]);
      const int base = Hpl.rowBaseOfBlock(i1);
      for (int r = 0; r < pd; ++r) {
        double s = 0;
        for (int k = 0; k < ld; ++k) s += Bi[k * pd + r] * db[k];
        coefficients[base + r] += s;
      }
      auto tIt = HschurTransposed[i1].begin();
      for (size_t in = o; in < col.size(); ++in) {
        const int i2 = col[in].first;
        const int pd2 = Hpl.rowsOfBlock(i2);
        const double* Bj = Hpl.arena.data() + col[in].second;
        while (tIt->first < i2) ++tIt;
        double* Hi = Hschur.arena.data() + tIt->second;  // pd x pd2 col-major
        for (int c = 0; c < pd2; ++c)
          for (int r = 0; r < pd; ++r) {
            double s = 0;
            for (int k = 0; k < ld; ++k) s += BDinv[k * pd + r] * Bj[k * pd2 + c];
            Hi[c * pd + r] -= s;
          }
      }
      omp_unset_lock(&coeffLocks[i1]);
    }
  }
  for (int i = 0; i < sizePoses; ++i) bschur[i] = b[i] - coefficients[i];
  if (st) st->timeSchurComplement = now() - t;
  t = now();
  bool solvedPoses = lin.solve(Hschur, x.data(), bschur.data(), st);
  if (st) {
    st->timeLinearSolver = now() - t;
    st->hessianPoseDimension = Hpp.ncols();
    st->hessianLandmarkDimension = Hll.ncols();
    st->hessianDimension = st->hessianPoseDimension + st->hessianLandmarkDimension;
  }
  if (!solvedPoses) return false;
  // back-substitution :420-446
  double* xp = x.data();
  double* xl = x.data() + sizePoses;
  const double* bl = b.data() + sizePoses;
#pragma omp parallel for num_threads(threads) schedule(static)
  for (int l = 0; l < numLandmarks; ++l) {
    const int ld = Hll.rowsOfBlock(l);
    const int lb = Hll.rowBaseOfBlock(l);
    double cl[6];
    for (int r = 0; r < ld; ++r) cl[r] = bl[lb + r];
    for (auto& rb : HplCCS[l]) {  // cl = bl - B' * xp (rightMultiply with cp = -xp)
      const int pd = Hpl.rowsOfBlock(rb.first), pb = Hpl.rowBaseOfBlock(rb.first);
      const double* Bm = Hpl.arena.data() + rb.second;
      for (int c = 0; c < ld; ++c) {
        double s = 0;
        for (int r = 0; r < pd; ++r) s += Bm[c * pd + r] * (-xp[pb + r]);
        cl[c] += s;
      }
    }
    const double* Dinv = DInv.data() + DInvOff[l];
    for (int r = 0; r < ld; ++r) {
      double s = 0;
      for (int k = 0; k < ld; ++k) s += Dinv[k * ld + r] * cl[k];
      xl[lb + r] = s;
    }
  }
  return true;
}

double computeLambdaInit(Graph& G, const Config& cfg) {  // optimization_algorithm_levenberg.cpp:152-175
  if (cfg.userLambdaInit > 0) return cfg.userLambdaInit;
  double maxDiagonal = 0;
  for (int vi : G.ivMap) {
    Vertex& v = G.verts[vi];
    double* H = G.vH(v);
    for (int j = 0; j < v.dim; ++j) maxDiagonal = std::max(std::fabs(H[j * v.dim + j]), maxDiagonal);
  }
  return 1e-5 * maxDiagonal;
}

struct LM {  // optimization_algorithm_levenberg.cpp
  double currentLambda = -1;
  double ni = 2;
  int levenbergIterations = 0;
  enum Result { OK = 0, Terminate = 1, Fail = 2 };

  Result solve(Graph& G, const Config& cfg, int iteration, oracle_batch_stats* st) {
    BlockSolver& S = G.solver;
    if (iteration == 0) {
      if (!S.buildStructure(G)) return Fail;
      G.structureBuilt = true;
      S.lin.blockOrdering = cfg.blockOrdering;
      S.lin.useRef = cfg.useRef;
      S.lin.reset();
    }
    double t = now();
    computeActiveErrors(G, cfg.threads);
    if (st) { st->timeResiduals = now() - t; t = now(); }
    double currentChi = activeRobustChi2(G);
    double tempChi = currentChi;
    S.buildSystem(G, cfg.threads);
    if (st) st->timeQuadraticForm = now() - t;
    if (iteration == 0) {
      currentLambda = computeLambdaInit(G, cfg);
      ni = 2;
    }
    double rho = 0;
    int& qmax = levenbergIterations;
    qmax = 0;
    do {
      push(G);
      if (st) { st->levenbergIterations++; t = now(); }
      S.setLambda(currentLambda, true);
      bool ok2 = S.solve(cfg.threads, st);
      if (st) { st->timeLinearSolution += now() - t; t = now(); }
      update(G, S.x.data());
      if (st) st->timeUpdate = now() - t;
      S.restoreDiagonal();
      computeActiveErrors(G, cfg.threads);
      tempChi = activeRobustChi2(G);
      if (!ok2) tempChi = std::numeric_limits<double>::max();
      rho = (currentChi - tempChi);
      double scale = 0;  // computeScale :177-184
      for (size_t j = 0; j < S.x.size(); ++j) scale += S.x[j] * (currentLambda * S.x[j] + S.b[j]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi)) {
        double alpha = 1. - std::pow((2 * rho - 1), 3);
        alpha = std::min(alpha, 2. / 3.);
        double scaleFactor = std::max(1. / 3., alpha);
        currentLambda *= scaleFactor;
        ni = 2;
        currentChi = tempChi;
        discardTop(G);
      } else {
        currentLambda *= ni;
        ni *= 2;
        pop(G);
        if (!std::isfinite(currentLambda)) break;
      }
      qmax++;
    } while (rho < 0 && qmax < cfg.maxTrials);
    if (qmax == cfg.maxTrials || rho == 0 || !std::isfinite(currentLambda)) return Terminate;
    return OK;
  }
};

// optimization_algorithm_gauss_newton.cpp:50-92
LM::Result gaussNewtonSolve(Graph& G, const Config& cfg, int iteration, oracle_batch_stats* st) {
  BlockSolver& S = G.solver;
  double t = now();
  computeActiveErrors(G, cfg.threads);
  if (st) st->timeResiduals = now() - t;
  if (iteration == 0) {
    if (!S.buildStructure(G)) return LM::Fail;
    G.structureBuilt = true;
    S.lin.blockOrdering = cfg.blockOrdering;
    S.lin.useRef = cfg.useRef;
    S.lin.reset();
  }
  t = now();
  S.buildSystem(G, cfg.threads);
  if (st) { st->timeQuadraticForm = now() - t; t = now(); }
  const bool ok = S.solve(cfg.threads, st);
  if (st) { st->timeLinearSolution = now() - t; t = now(); }
  update(G, S.x.data());
  if (st) st->timeUpdate = now() - t;
  return ok ? LM::OK : LM::Fail;
}

Config toConfig(const oracle_config* c) {
  Config cfg;
  if (c) {
    cfg.maxTrials = c->max_trials_after_failure > 0 ? c->max_trials_after_failure : 10;
    cfg.userLambdaInit = c->user_lambda_init;
    cfg.threads = c->threads > 0 ? c->threads : 1;
    cfg.useRef = c->use_ref_csparse != 0;
    cfg.blockOrdering = c->block_ordering != 0;
    cfg.gaussNewton = c->gauss_newton != 0;
  }
  return cfg;
}

void setEdgeDerived(Edge& e) {
  if (e.type == ORACLE_E_SE3_QUAT) {
    double m[7];
    std::memcpy(m, e.meas, sizeof m);
    double nq = std::sqrt(m[3] * m[3] + m[4] * m[4] + m[5] * m[5] + m[6] * m[6]);  // edge_se3.cpp:46-47
    for (int k = 3; k < 7; ++k) m[k] /= nq;
    e.Z = fromVectorQT(m);
    e.Zinv = isoinv(e.Z);
  } else if (e.type == ORACLE_E_SE2) {
    e.m2.x = e.meas[0]; e.m2.y = e.meas[1]; e.m2.th = e.meas[2];
    e.m2inv = se2inv(e.m2);
  }
}

int addEdgeRaw(Graph& G, int type, int id0, int id1, const double* meas, const double* info, const double* params) {
  auto a = G.idmap.find(id0), b = G.idmap.find(id1);
  if (a == G.idmap.end() || b == G.idmap.end()) return -1;
  Edge e;
  e.type = type;
  e.D = edim(type);
  e.v[0] = a->second;
  e.v[1] = b->second;
  const int nm = type == ORACLE_E_SE3_PROJECT_XYZ || type == ORACLE_E_SE2_XY ? 2 : (type == ORACLE_E_SE3_QUAT || type == ORACLE_E_SE3_EXPMAP ? 7 : 3);
  std::memcpy(e.meas, meas, sizeof(double) * nm);
  e.numeric = type == ORACLE_E_SE3_EXPMAP;  // no analytic Jacobian restated: base_binary_edge.hpp:198-266
  std::memcpy(e.info, info, sizeof(double) * e.D * e.D);
  if (params && type == ORACLE_E_SE3_PROJECT_XYZ) std::memcpy(e.params, params, sizeof(double) * 4);
  setEdgeDerived(e);
  int idx = (int)G.edges.size();
  G.verts[e.v[0]].edges.push_back(idx);
  G.verts[e.v[1]].edges.push_back(idx);
  G.edges.push_back(e);
  G.initialized = false;
  return 0;
}

void setVertexEstimate(Vertex& v, const double* est) {
  switch (v.type) {
    case ORACLE_V_SE3_EXPMAP:
      v.est.q.t = {est[0], est[1], est[2]};
      v.est.q.r = Quat{est[6], est[3], est[4], est[5]};
      v.est.q.normalizeRotation();  // SE3Quat::fromVector + setEstimate
      break;
    case ORACLE_V_XYZ: v.est.p = {est[0], est[1], est[2]}; break;
    case ORACLE_V_SE3_QUAT: v.est.iso = fromVectorQT(est); break;  // vertex_se3.cpp:49-55
    case ORACLE_V_SE2: v.est.se2.x = est[0]; v.est.se2.y = est[1]; v.est.se2.th = est[2]; break;
    case ORACLE_V_XY: v.est.p = {est[0], est[1], 0.0}; break;
  }
}
int estDim(int type) {
  return type == ORACLE_V_SE3_EXPMAP || type == ORACLE_V_SE3_QUAT ? 7 : (type == ORACLE_V_XY ? 2 : 3);
}
void getVertexEstimate(const Vertex& v, double* out) {
  switch (v.type) {
    case ORACLE_V_SE3_EXPMAP:
      out[0] = v.est.q.t.x; out[1] = v.est.q.t.y; out[2] = v.est.q.t.z;
      out[3] = v.est.q.r.x; out[4] = v.est.q.r.y; out[5] = v.est.q.r.z; out[6] = v.est.q.r.w;
      break;
    case ORACLE_V_XYZ: out[0] = v.est.p.x; out[1] = v.est.p.y; out[2] = v.est.p.z; break;
    case ORACLE_V_SE3_QUAT: toVectorQT(v.est.iso, out); break;
    case ORACLE_V_SE2: out[0] = v.est.se2.x; out[1] = v.est.se2.y; out[2] = v.est.se2.th; break;
    case ORACLE_V_XY: out[0] = v.est.p.x; out[1] = v.est.p.y; break;
  }
}
void minimalEstimate(const Vertex& v, double* out) {
  switch (v.type) {
    case ORACLE_V_SE3_EXPMAP:  // SE3Quat::toMinimalVector (se3quat.h:143-152)
      out[0] = v.est.q.t.x; out[1] = v.est.q.t.y; out[2] = v.est.q.t.z;
      out[3] = v.est.q.r.x; out[4] = v.est.q.r.y; out[5] = v.est.q.r.z;
      break;
    case ORACLE_V_SE3_QUAT: toVectorMQT(v.est.iso, out); break;
    default: getVertexEstimate(v, out); break;
  }
}

}  // namespace

struct OracleGraph {
  Graph g;
  LM lm;
};

extern "C" {

OracleGraph* oracle_graph_new(void) { return new OracleGraph(); }
void oracle_graph_free(OracleGraph* g) { delete g; }

int oracle_add_vertices(OracleGraph* og, int type, int n, const int* ids, const double* est, const int* fixed,
                        const int* marginalized) {
  Graph& G = og->g;
  if (vdim(type) < 0) return -1;
  const int ed = estDim(type);
  for (int k = 0; k < n; ++k) {
    if (G.idmap.count(ids[k])) return -2;
    Vertex v;
    v.id = ids[k];
    v.type = type;
    v.dim = vdim(type);
    v.fixed = fixed ? fixed[k] != 0 : false;
    v.marginalized = marginalized ? marginalized[k] != 0 : false;
    setVertexEstimate(v, est + (size_t)k * ed);
    G.idmap[v.id] = (int)G.verts.size();
    G.verts.push_back(std::move(v));
  }
  G.initialized = false;
  return 0;
}

int oracle_add_edges(OracleGraph* og, int type, int n, const int* v0, const int* v1, const double* meas,
                     const double* info, const double* params) {
  Graph& G = og->g;
  const int D = edim(type);
  if (D < 0) return -1;
  const int nm = type == ORACLE_E_SE3_PROJECT_XYZ || type == ORACLE_E_SE2_XY ? 2 : (type == ORACLE_E_SE3_QUAT || type == ORACLE_E_SE3_EXPMAP ? 7 : 3);
  G.edges.reserve(G.edges.size() + n);
  for (int k = 0; k < n; ++k) {
    int r = addEdgeRaw(G, type, v0[k], v1[k], meas + (size_t)k * nm, info + (size_t)k * D * D,
                       params ? params + (size_t)k * 4 : nullptr);
    if (r) return r;
  }
  return 0;
}

// optimizable_graph.cpp:397-661 (tags used by the BASELINE configs only)
int oracle_load_g2o(OracleGraph* og, const char* path, int marginalize_xyz) {
  std::ifstream in(path);
  if (!in) return -1;
  Graph& G = og->g;
  std::string line, tag;
  std::vector<int> fixIds;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    if (!(ss >> tag)) continue;
    if (tag[0] == '#') continue;
    if (tag == "VERTEX_SE3:EXPMAP") {  // types_six_dof_expmap.cpp:93-101: file holds cam2world
      int id; double v[7];
      ss >> id; for (double& d : v) ss >> d;
      SE3Quat c2w; c2w.t = {v[0], v[1], v[2]}; c2w.r = Quat{v[6], v[3], v[4], v[5]};
      SE3Quat w2c = se3inv(c2w);
      double est[7] = {w2c.t.x, w2c.t.y, w2c.t.z, w2c.r.x, w2c.r.y, w2c.r.z, w2c.r.w};
      int z = 0;
      oracle_add_vertices(og, ORACLE_V_SE3_EXPMAP, 1, &id, est, &z, &z);
    } else if (tag == "VERTEX_XYZ") {
      int id; double v[3];
      ss >> id >> v[0] >> v[1] >> v[2];
      int z = 0, m = marginalize_xyz ? 1 : 0;
      oracle_add_vertices(og, ORACLE_V_XYZ, 1, &id, v, &z, &m);
    } else if (tag == "VERTEX_SE3:QUAT") {
      int id; double v[7];
      ss >> id; for (double& d : v) ss >> d;
      int z = 0;
      oracle_add_vertices(og, ORACLE_V_SE3_QUAT, 1, &id, v, &z, &z);
    } else if (tag == "VERTEX_SE2") {
      int id; double v[3];
      ss >> id >> v[0] >> v[1] >> v[2];
      int z = 0;
      oracle_add_vertices(og, ORACLE_V_SE2, 1, &id, v, &z, &z);
    } else if (tag == "VERTEX_XY") {  // vertex_point_xy.cpp:46-50
      int id; double v[2];
      ss >> id >> v[0] >> v[1];
      int z = 0, m = marginalize_xyz ? 1 : 0;
      oracle_add_vertices(og, ORACLE_V_XY, 1, &id, v, &z, &m);
    } else if (tag == "FIX") {
      int id;
      while (ss >> id) fixIds.push_back(id);
    } else if (tag == "EDGE_SE3_PROJECT_XYZ:EXPMAP") {  // :363-378
      int a, b; double m[2], o[3], p[4];
      ss >> a >> b >> m[0] >> m[1] >> o[0] >> o[1] >> o[2] >> p[0] >> p[1] >> p[2] >> p[3];
      double info[4] = {o[0], o[1], o[1], o[2]};
      if (addEdgeRaw(G, ORACLE_E_SE3_PROJECT_XYZ, a, b, m, info, p)) return -3;
    } else if (tag == "EDGE_SE3:QUAT") {  // edge_se3.cpp:42-65
      int a, b; double m[7], info[36];
      ss >> a >> b; for (double& d : m) ss >> d;
      for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j) { ss >> info[i * 6 + j]; info[j * 6 + i] = info[i * 6 + j]; }
      if (addEdgeRaw(G, ORACLE_E_SE3_QUAT, a, b, m, info, nullptr)) return -3;
    } else if (tag == "EDGE_SE2") {  // edge_se2.cpp:41-53
      int a, b; double m[3], info[9];
      ss >> a >> b >> m[0] >> m[1] >> m[2];
      for (int i = 0; i < 3; ++i)
        for (int j = i; j < 3; ++j) { ss >> info[i * 3 + j]; info[j * 3 + i] = info[i * 3 + j]; }
      if (addEdgeRaw(G, ORACLE_E_SE2, a, b, m, info, nullptr)) return -3;
    } else if (tag == "EDGE_SE2_XY") {  // edge_se2_pointxy.cpp:46-52
      int a, b; double m[2], o[3];
      ss >> a >> b >> m[0] >> m[1] >> o[0] >> o[1] >> o[2];
      double info[4] = {o[0], o[1], o[1], o[2]};
      if (addEdgeRaw(G, ORACLE_E_SE2_XY, a, b, m, info, nullptr)) return -3;
    }
  }
  for (int id : fixIds) {
    auto it = G.idmap.find(id);
    if (it != G.idmap.end()) G.verts[it->second].fixed = true;
  }
  return 0;
}

int oracle_save_g2o(OracleGraph* og, const char* path) {
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  Graph& G = og->g;
  for (auto& v : G.verts) {
    double e[7];
    getVertexEstimate(v, e);
    if (v.type == ORACLE_V_SE3_EXPMAP) {
      SE3Quat c2w = se3inv(v.est.q);
      fprintf(f, "VERTEX_SE3:EXPMAP %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", v.id, c2w.t.x, c2w.t.y, c2w.t.z,
              c2w.r.x, c2w.r.y, c2w.r.z, c2w.r.w);
    } else if (v.type == ORACLE_V_XYZ) {
      fprintf(f, "VERTEX_XYZ %d %.17g %.17g %.17g\n", v.id, e[0], e[1], e[2]);
    } else if (v.type == ORACLE_V_SE3_QUAT) {
      fprintf(f, "VERTEX_SE3:QUAT %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", v.id, e[0], e[1], e[2], e[3], e[4],
              e[5], e[6]);
    } else if (v.type == ORACLE_V_XY) {
      fprintf(f, "VERTEX_XY %d %.17g %.17g\n", v.id, e[0], e[1]);
    } else {
      fprintf(f, "VERTEX_SE2 %d %.17g %.17g %.17g\n", v.id, e[0], e[1], e[2]);
    }
    if (v.fixed) fprintf(f, "FIX %d\n", v.id);
  }
  for (auto& e : G.edges) {
    int a = G.verts[e.v[0]].id, b = G.verts[e.v[1]].id;
    if (e.type == ORACLE_E_SE3_PROJECT_XYZ) {
      fprintf(f, "EDGE_SE3_PROJECT_XYZ:EXPMAP %d %d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", a, b,
              e.meas[0], e.meas[1], e.info[0], e.info[1], e.info[3], e.params[0], e.params[1], e.params[2],
              e.params[3]);
    } else {
      const char* tag = e.type == ORACLE_E_SE3_QUAT ? "EDGE_SE3:QUAT" : (e.type == ORACLE_E_SE2_XY ? "EDGE_SE2_XY" : "EDGE_SE2");
      int nm = e.type == ORACLE_E_SE3_QUAT ? 7 : (e.type == ORACLE_E_SE2_XY ? 2 : 3);
      fprintf(f, "%s %d %d", tag, a, b);
      for (int k = 0; k < nm; ++k) fprintf(f, " %.17g", e.meas[k]);
      for (int i = 0; i < e.D; ++i)
        for (int j = i; j < e.D; ++j) fprintf(f, " %.17g", e.info[i * e.D + j]);
      fprintf(f, "\n");
    }
  }
  fclose(f);
  return 0;
}

int oracle_num_vertices(OracleGraph* og) { return (int)og->g.verts.size(); }
int oracle_num_edges(OracleGraph* og) { return (int)og->g.edges.size(); }

int oracle_get_estimates(OracleGraph* og, int type, double* out, int* ids_out) {
  int n = 0;
  const int ed = estDim(type);
  for (auto& v : og->g.verts)
    if (v.type == type) {
      if (out) getVertexEstimate(v, out + (size_t)n * ed);
      if (ids_out) ids_out[n] = v.id;
      ++n;
    }
  return n;
}

int oracle_minimal_state(OracleGraph* og, double* out) {
  Graph& G = og->g;
  std::vector<int> order(G.verts.size());
  for (size_t k = 0; k < order.size(); ++k) order[k] = (int)k;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return G.verts[a].id < G.verts[b].id; });
  int n = 0;
  for (int k : order) {
    const Vertex& v = G.verts[k];
    if (out) minimalEstimate(v, out + n);
    n += v.dim;
  }
  return n;
}

int oracle_initialize(OracleGraph* og) {
  initializeOptimization(og->g);
  return 0;
}

int oracle_update_initialization(OracleGraph* og) { return updateInitialization(og->g); }

double oracle_chi2(OracleGraph* og) {
  computeActiveErrors(og->g, 1);
  return activeRobustChi2(og->g);
}

// sparse_optimizer.cpp:374-439
int oracle_optimize(OracleGraph* og, const oracle_config* c, int iterations, oracle_batch_stats* stats) {
  Graph& G = og->g;
  Config cfg = toConfig(c);
  if (!G.initialized) initializeOptimization(G);
  if (G.ivMap.empty()) return -1;
  int cj = 0;
  LM::Result result = LM::OK;
  bool ok = true;
  for (int i = 0; i < iterations && ok; ++i) {
    oracle_batch_stats* st = stats ? stats + i : nullptr;
    if (st) {
      std::memset(st, 0, sizeof *st);
      st->iteration = i;
      st->numEdges = (int)G.edges.size();
      st->numVertices = (int)G.activeVertices.size();
    }
    double ts = now();
    result = cfg.gaussNewton ? gaussNewtonSolve(G, cfg, i, st) : og->lm.solve(G, cfg, i, st);
    ok = result == LM::OK;
    if (st) {
      computeActiveErrors(G, cfg.threads);
      st->chi2 = activeRobustChi2(G);
      st->lambda = cfg.gaussNewton ? 0.0 : og->lm.currentLambda;
      st->timeIteration = now() - ts;
    }
    ++cj;
  }
  if (result == LM::Fail) return 0;
  return cj;
}

int oracle_stage(OracleGraph* og, const oracle_config* c, double lambda, double* b, double* x, double* Hschur,
                 double* bschur, long long* dims) {
  Graph& G = og->g;
  Config cfg = toConfig(c);
  if (!G.initialized) initializeOptimization(G);
  BlockSolver& S = G.solver;
  if (!S.buildStructure(G)) return -1;
  S.lin.blockOrdering = cfg.blockOrdering;
  S.lin.useRef = cfg.useRef;
  S.lin.reset();
  computeActiveErrors(G, cfg.threads);
  S.buildSystem(G, cfg.threads);
  S.setLambda(lambda, true);
  bool ok = S.solve(cfg.threads, nullptr);
  const int n = S.sizePoses + S.sizeLandmarks, np = S.sizePoses;
  if (dims) { dims[0] = n; dims[1] = np; dims[2] = S.sizeLandmarks; }
  if (b) std::memcpy(b, S.b.data(), sizeof(double) * n);
  if (x) std::memcpy(x, S.x.data(), sizeof(double) * n);
  if (Hschur) {
    SBM& M = S.doSchur ? S.Hschur : S.Hpp;
    std::fill(Hschur, Hschur + (size_t)np * np, 0.0);
    for (size_t cb = 0; cb < M.cols.size(); ++cb)
      for (auto& kv : M.cols[cb]) {
        int rb = kv.first, r0 = M.rowBaseOfBlock(rb), c0 = M.colBaseOfBlock((int)cb);
        int rs = M.rowsOfBlock(rb), cs = M.colsOfBlock((int)cb);
        for (int cc = 0; cc < cs; ++cc)
          for (int r = 0; r < rs; ++r) {
            double v = M.arena[kv.second + (size_t)cc * rs + r];
            Hschur[(size_t)(r0 + r) * np + c0 + cc] = v;
            Hschur[(size_t)(c0 + cc) * np + r0 + r] = v;
          }
      }
  }
  if (bschur) {
    if (S.doSchur) std::memcpy(bschur, S.bschur.data(), sizeof(double) * np);
    else std::memcpy(bschur, S.b.data(), sizeof(double) * np);
  }
  S.restoreDiagonal();
  return ok ? 1 : 0;
}

int oracle_hessian_dense(OracleGraph* og, double* Hpp, double* Hll_diag, double* Hpl) {
  Graph& G = og->g;
  BlockSolver& S = G.solver;
  const int np = S.sizePoses, nl = S.sizeLandmarks;
  if (Hpp) {
    std::fill(Hpp, Hpp + (size_t)np * np, 0.0);
    for (size_t cb = 0; cb < S.Hpp.cols.size(); ++cb)
      for (auto& kv : S.Hpp.cols[cb]) {
        int r0 = S.Hpp.rowBaseOfBlock(kv.first), c0 = S.Hpp.colBaseOfBlock((int)cb);
        int rs = S.Hpp.rowsOfBlock(kv.first), cs = S.Hpp.colsOfBlock((int)cb);
        for (int cc = 0; cc < cs; ++cc)
          for (int r = 0; r < rs; ++r) {
            double v = S.Hpp.arena[kv.second + (size_t)cc * rs + r];
            Hpp[(size_t)(r0 + r) * np + c0 + cc] = v;
            Hpp[(size_t)(c0 + cc) * np + r0 + r] = v;
          }
      }
  }
  if (!S.doSchur) return 0;
  if (Hll_diag)
    for (int l = 0; l < S.numLandmarks; ++l) {
      const double* B = S.Hll.arena.data() + S.Hll.cols[l].at(l);
      int d = S.Hll.rowsOfBlock(l);
      std::memcpy(Hll_diag + (size_t)S.Hll.rowBaseOfBlock(l) * d, B, sizeof(double) * d * d);
    }
  if (Hpl) {
    std::fill(Hpl, Hpl + (size_t)np * nl, 0.0);
    for (int l = 0; l < S.numLandmarks; ++l)
      for (auto& kv : S.Hpl.cols[l]) {
        int r0 = S.Hpl.rowBaseOfBlock(kv.first), c0 = S.Hpl.colBaseOfBlock(l);
        int rs = S.Hpl.rowsOfBlock(kv.first), cs = S.Hpl.colsOfBlock(l);
        for (int cc = 0; cc < cs; ++cc)
          for (int r = 0; r < rs; ++r) Hpl[(size_t)(r0 + r) * nl + c0 + cc] = S.Hpl.arena[kv.second + (size_t)cc * rs + r];
      }
  }
  return 0;
}

int oracle_edge_jacobians(OracleGraph* og, int k, double* err, double* Ji_an, double* Jj_an, double* Ji_num,
                          double* Jj_num) {
  Graph& G = og->g;
  if (k < 0 || k >= (int)G.edges.size()) return -1;
  Edge& e = G.edges[k];
  computeError(G, e);
  if (err) std::memcpy(err, e.err, sizeof(double) * e.D);
  double A[36], B[36];
  linearizeOplus(G, e, A, B);
  const int di = G.verts[e.v[0]].dim, dj = G.verts[e.v[1]].dim;
  if (Ji_an) std::memcpy(Ji_an, A, sizeof(double) * e.D * di);
  if (Jj_an) std::memcpy(Jj_an, B, sizeof(double) * e.D * dj);
  linearizeNumeric(G, e, A, B);
  if (Ji_num) std::memcpy(Ji_num, A, sizeof(double) * e.D * di);
  if (Jj_num) std::memcpy(Jj_num, B, sizeof(double) * e.D * dj);
  return 0;
}

int oracle_ccs_cholsol(int n, const int* Ap, const int* Ai, const double* Ax, double* b, int mode) {
  CCS A;
  A.n = n;
  A.p.assign(Ap, Ap + n + 1);
  A.i.assign(Ai, Ai + Ap[n]);
  A.x.assign(Ax, Ax + Ap[n]);
  if (mode == 2) {
    if (!refcs().ok()) return -1;
    cs_ref a{Ap[n], n, n, A.p.data(), A.i.data(), A.x.data(), -1};
    return refcs().cs_cholsol(1, &a, b) ? 1 : 0;
  }
  std::vector<int> P(n);
  if (mode == 1) {
    if (!refcs().ok()) return -1;
    cs_ref a{Ap[n], n, n, A.p.data(), A.i.data(), A.x.data(), -1};
    int* p = refcs().cs_amd(1, &a);
    for (int k = 0; k < n; ++k) P[k] = p[k];
    refcs().cs_free(p);
  } else {
    for (int k = 0; k < n; ++k) P[k] = k;
  }
  std::vector<int> pinv = make_pinv(P), map, Li;
  CCS C;
  symperm_upper(A, pinv, C, map);
  for (size_t k = 0; k < map.size(); ++k) C.x[k] = A.x[map[k]];
  std::vector<int> parent = etree(C);
  std::vector<int> cnt = colcounts(C, parent);
  std::vector<int> cp(n + 1, 0);
  for (int k = 0; k < n; ++k) cp[k + 1] = cp[k] + cnt[k];
  std::vector<double> Lx, xw;
  if (!chol_numeric(C, parent, cp, Li, Lx)) return 0;
  chol_solve(n, pinv, cp, Li, Lx, b, xw);
  return 1;
}

// Symbolic statistics of LinearSolverCSparse::computeSymbolicDecomposition (linear_solver_csparse.h:246-308) for
// a block pattern (upper blocks bi <= bj of uniform size bdim): cs_amd on the block pattern (reference CSparse
// when use_ref and loaded, else natural order) expanded to scalars, symperm, etree, column counts.
// out[0] = nnz(L) = sum c_k, out[1] = sum c_k^2 (the factorization flop count of SURVEY.md 8d, cs_demo's "fl").
int oracle_block_symbolic(int nblocks, int bdim, int nblk, const int* bi, const int* bj, int use_ref, double* out) {
  if (nblocks <= 0 || bdim <= 0 || nblk < 0 || !out) return -1;
  std::vector<std::vector<int>> colrows(nblocks);
  for (int k = 0; k < nblk; ++k) {
    const int r = std::min(bi[k], bj[k]), c = std::max(bi[k], bj[k]);
    if (r < 0 || c >= nblocks) return -1;
    colrows[c].push_back(r);
  }
  for (int c = 0; c < nblocks; ++c) {
    colrows[c].push_back(c);
    std::sort(colrows[c].begin(), colrows[c].end());
    colrows[c].erase(std::unique(colrows[c].begin(), colrows[c].end()), colrows[c].end());
  }
  std::vector<int> bp(nblocks + 1, 0), bix;
  for (int c = 0; c < nblocks; ++c) {
    bp[c] = (int)bix.size();
    bix.insert(bix.end(), colrows[c].begin(), colrows[c].end());
  }
  bp[nblocks] = (int)bix.size();
  std::vector<int> bperm(nblocks);
  if (use_ref && refcs().ok()) {
    cs_ref aux{(int)bix.size(), nblocks, nblocks, bp.data(), bix.data(), nullptr, -1};
    int* pp = refcs().cs_amd(1, &aux);
    if (!pp) return -1;
    for (int k = 0; k < nblocks; ++k) bperm[k] = pp[k];
    refcs().cs_free(pp);
  } else {
    for (int k = 0; k < nblocks; ++k) bperm[k] = k;
  }
  const int n = nblocks * bdim;
  std::vector<int> P;
  P.reserve(n);
  for (int k = 0; k < nblocks; ++k)
    for (int j = 0; j < bdim; ++j) P.push_back(bperm[k] * bdim + j);
  CCS A;  // scalar upper pattern (fillCCS(upper=true), sparse_block_matrix.hpp:496-549)
  A.n = n;
  A.p.assign(n + 1, 0);
  for (int bc = 0; bc < nblocks; ++bc)
    for (int c = 0; c < bdim; ++c) {
      A.p[bc * bdim + c] = (int)A.i.size();
      for (int br : colrows[bc]) {
        const int elems = br == bc ? c + 1 : bdim;
        for (int r = 0; r < elems; ++r) A.i.push_back(br * bdim + r);
      }
    }
  A.p[n] = (int)A.i.size();
  A.x.assign(A.i.size(), 1.0);
  CCS C;
  std::vector<int> map;
  symperm_upper(A, make_pinv(P), C, map);
  const std::vector<int> parent = etree(C);
  const std::vector<int> cnt = colcounts(C, parent);
  double lnz = 0, fl = 0;
  for (int k = 0; k < n; ++k) {
    lnz += cnt[k];
    fl += (double)cnt[k] * cnt[k];
  }
  out[0] = lnz;
  out[1] = fl;
  return 0;
}

int oracle_set_robust_kernel(OracleGraph* og, int etype, int kind, double delta) {
  for (Edge& e : og->g.edges)
    if (e.type == etype) { e.rk = kind; e.rkDelta = delta; }
  return 0;
}
int oracle_set_edge_numeric(OracleGraph* og, int n, const int* idx) {
  for (int k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= (int)og->g.edges.size()) return -1;
    og->g.edges[idx[k]].numeric = true;
  }
  return 0;
}
// [e | Ji | Jj] row-major per listed edge at the current estimates (the host side of a host-Jacobian edge)
int oracle_edge_payload(OracleGraph* og, int n, const int* idx, int numeric, double* out) {
  Graph& G = og->g;
  size_t o = 0;
  for (int k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= (int)G.edges.size()) return -1;
    Edge& e = G.edges[idx[k]];
    computeError(G, e);
    double A[36], B[36];
    if (numeric) linearizeNumeric(G, e, A, B);
    else linearizeOplus(G, e, A, B);
    const int di = G.verts[e.v[0]].dim, dj = G.verts[e.v[1]].dim;
    for (int i = 0; i < e.D; ++i) out[o++] = e.err[i];
    for (int i = 0; i < e.D * di; ++i) out[o++] = A[i];
    for (int i = 0; i < e.D * dj; ++i) out[o++] = B[i];
  }
  return (int)o;
}
int oracle_update(OracleGraph* og, const double* x) {
  if (!og->g.initialized) initializeOptimization(og->g);
  update(og->g, x);
  return 0;
}
int oracle_set_estimates(OracleGraph* og, int type, const double* est) {
  const int ed = estDim(type);
  int n = 0;
  for (auto& v : og->g.verts)
    if (v.type == type) setVertexEstimate(v, est + (size_t)(n++) * ed);
  return n;
}
int oracle_push(OracleGraph* og) { push(og->g); return 0; }
int oracle_pop(OracleGraph* og) { pop(og->g); return 0; }
int oracle_discard_top(OracleGraph* og) { discardTop(og->g); return 0; }

// The rotation / isometry mappings of isometry3d_mappings.{h,cpp} and the SE2 constructors, for the CPU pins of the
// reference's own unit tests (unit_test/slam3d/mappings_slam3d.cpp, orthogonal_matrix.cpp, slam2d/mappings_se2.cpp).
// Matrices col-major (Eigen), an isometry as [R (9) | t (3)]. Returns the number of doubles written, -1 for an unknown op.
int oracle_mapping(int op, const double* in, double* out) {
  auto getR = [](const double* p) { M3 R; for (int c = 0; c < 3; ++c) for (int r = 0; r < 3; ++r) R.m[r][c] = p[c * 3 + r]; return R; };
  auto putR = [](const M3& R, double* p) { for (int c = 0; c < 3; ++c) for (int r = 0; r < 3; ++r) p[c * 3 + r] = R.m[r][c]; return 9; };
  auto getI = [&](const double* p) { Iso3 a; a.R = getR(p); a.t = {p[9], p[10], p[11]}; return a; };
  auto putI = [&](const Iso3& a, double* p) { putR(a.R, p); p[9] = a.t.x; p[10] = a.t.y; p[11] = a.t.z; return 12; };
  switch (op) {
    case 0: return putR(fromEuler(V3{in[0], in[1], in[2]}), out);
    case 1: { const V3 e = toEuler(getR(in)); out[0] = e.x; out[1] = e.y; out[2] = e.z; return 3; }
    case 2: { const V3 q = toCompactQuaternion(getR(in)); out[0] = q.x; out[1] = q.y; out[2] = q.z; return 3; }
    case 3: return putR(fromCompactQuaternion(V3{in[0], in[1], in[2]}), out);
    case 4: return putI(fromVectorET(in), out);
    case 5: toVectorET(getI(in), out); return 6;
    case 6: toVectorMQT(getI(in), out); return 6;
    case 7: return putI(fromVectorMQT(in), out);
    case 8: toVectorQT(getI(in), out); return 7;
    case 9: return putI(fromVectorQT(in), out);
    case 10: { M3 R = getR(in); approximateNearestOrthogonalMatrix(R); return putR(R, out); }
    case 11: { M3 R = getR(in); nearestOrthogonalMatrix(R); return putR(R, out); }
    case 12: { const SE2 s = se2FromIso(in, in + 4); out[0] = s.x; out[1] = s.y; out[2] = s.th; return 3; }
    default: return -1;
  }
}

int oracle_ref_available(void) { return refcs().ok() ? 1 : 0; }
const char* oracle_ref_path(void) { return refcs().path.c_str(); }

}  // extern "C"
