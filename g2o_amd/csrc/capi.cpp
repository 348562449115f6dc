// extern "C" entry points of libg2o_hip.so (include/g2o_hip.h).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <vector>
#include <cstring>
#include <string>

#include "../../include/g2o_hip.h"
#include "engine.hpp"

struct g2ohip_graph {
  g2ohip::Engine* e;
};

namespace {
thread_local std::string g_err;

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return G2OHIP_ERR_DEVICE;
  }
}
// 1 known, 0 unknown, -1 a reference name this backend does not build (with g_err set)
int algorithm_known(const std::string& n) {
  // {gn,lm}_hip_{var,fix6_3,fix3_2,fix3_3,fix6_6} (cf. solver_csparse.cpp:51-84 name parsing)
  if (n.size() < 6) return 0;
  const std::string m = n.substr(0, 3), rest = n.substr(3);
  if (m != "lm_" && m != "gn_") return 0;
  if (rest == "hip_var" || rest == "hip_fix6_3" || rest == "hip_fix3_2" || rest == "hip_fix3_3" || rest == "hip_fix6_6")
    return 1;
  // g2o/solvers/pcg registry (solver_pcg.cpp:91-98): pcg (variable block size), pcg3_2, pcg6_3, pcg7_3.
  // Block-Jacobi PCG on the device replaces the Cholesky; pose blocks of 3 or 6 only.
  if (rest == "pcg" || rest == "pcg6_3" || rest == "pcg3_2") return 1;
  // fork solvers/eigen/solver_eigen.cpp:80,126: JacobiSolver_6_3 + LinearSolverPCGEigen (matrix-free CGLS)
  if (m == "lm_" && rest == "pcg6_3_eigen") return 1;
  if (rest == "pcg7_3") {
    g_err = n + ": fixed block size 7_3 is not supported by the device PCG (pose blocks of 3 or 6 only; "
                "use " + m + "pcg)";
    return -1;
  }
  return 0;
}
// the kernels are built for gfx950 only (MFMA f64 16x16x4, 160 KB LDS, 8 XCDs): refuse anything else
bool gfx950_device(int device) {
  int n = 0;
  if (device < 0 || hipGetDeviceCount(&n) != hipSuccess || n <= device) {
    g_err = "no HIP device " + std::to_string(device) + " (libg2o_hip requires a gfx950 GPU)";
    return false;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_err = "HIP device " + std::to_string(device) + " is not gfx950 (" +
            std::string(hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.gcnArchName : "unknown") +
            "): libg2o_hip requires a MI355X";
    return false;
  }
  return true;
}
}  // namespace

extern "C" {

g2ohip_graph* g2ohip_graph_create(int device) {
  try {
    int n = 0;
    if (!gfx950_device(device)) return nullptr;
    return new g2ohip_graph{new g2ohip::Engine(device)};
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return nullptr;
  }
}
void g2ohip_graph_destroy(g2ohip_graph* g) {
  if (!g) return;
  delete g->e;
  delete g;
}
int g2ohip_add_vertices(g2ohip_graph* g, int type, int n, const int* ids, const double* est, const int* fixed,
                        const int* marginalized) {
  if (!g || (n > 0 && (!ids || !est))) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->add_vertices(type, n, ids, est, fixed, marginalized); });
}
int g2ohip_add_edges(g2ohip_graph* g, int type, int n, const int* v0, const int* v1, const double* meas,
                     const double* info, const double* params) {
  if (!g || (n > 0 && (!v0 || !v1 || !info))) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->add_edges(type, n, v0, v1, meas, info, params); });
}
int g2ohip_load_g2o(g2ohip_graph* g, const char* path, int marginalize_xyz) {
  if (!g || !path) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->load(path, marginalize_xyz); });
}
int g2ohip_save_g2o(g2ohip_graph* g, const char* path) {
  if (!g || !path) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->save(path); });
}
int g2ohip_num_vertices(g2ohip_graph* g) { return g ? (int)g->e->hg.verts.size() : G2OHIP_ERR_ARG; }
int g2ohip_num_edges(g2ohip_graph* g) { return g ? (int)g->e->hg.num_edges() : G2OHIP_ERR_ARG; }
int g2ohip_set_robust_kernel(g2ohip_graph* g, int edge_type, int kind, double delta) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->set_robust_kernel(edge_type, kind, delta); });
}
int g2ohip_set_host_jacobians(g2ohip_graph* g, int edge_type, const double* payload) {
  if (!g || !payload) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->set_host_payload(edge_type, payload); });
}
int g2ohip_set_host_edge_callback(g2ohip_graph* g, g2ohip_host_edge_fn fn, void* user) {
  if (!g) return G2OHIP_ERR_ARG;
  return g->e->set_host_callback(fn, user);
}
int g2ohip_solver_set_eta(g2ohip_graph* g, double eta) {
  if (!g || !(eta > 0)) return G2OHIP_ERR_ARG;
  g->e->cgls.eta = eta;
  return G2OHIP_OK;
}
int g2ohip_solver_linear_iterations(g2ohip_graph* g) { return g ? g->e->cgls.last_iterations : G2OHIP_ERR_ARG; }
int g2ohip_solver_diag_absmax(g2ohip_graph* g, double* out) {
  if (!g || !out) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->diag_absmax(out); });
}
int g2ohip_get_estimates(g2ohip_graph* g, int type, double* out, int* ids_out) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->get_estimates(type, out, ids_out); });
}
int g2ohip_set_estimates(g2ohip_graph* g, int type, const double* est) {
  if (!g || !est) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->set_estimates(type, est); });
}
int g2ohip_minimal_state(g2ohip_graph* g, double* out) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->minimal_state(out); });
}
int g2ohip_set_algorithm(g2ohip_graph* g, const char* name) {
  if (!g || !name) return G2OHIP_ERR_ARG;
  const int k = algorithm_known(name);
  if (k < 0) return G2OHIP_ERR_UNSUPPORTED;
  if (k == 0) {
    g_err = std::string("unknown optimization algorithm ") + name;
    return G2OHIP_ERR_ARG;
  }
  g->e->algorithm = name;
  g->e->levenberg = std::string(name).rfind("lm_", 0) == 0;
  return G2OHIP_OK;
}
int g2ohip_initialize(g2ohip_graph* g) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->initialize(); });
}

int g2ohip_update_initialization(g2ohip_graph* g) {
  if (!g) return G2OHIP_ERR_ARG;
  const int r = guarded([&] { return g->e->update_initialization(); });
  if (r == G2OHIP_ERR_STATE) g_err = "updateInitialization: initializeOptimization first";
  if (r == G2OHIP_ERR_UNSUPPORTED)
    g_err = "updateInitialization: online updates of a Schur (marginalized) graph or of another pose block size are "
            "not supported (block_solver.hpp:274-277)";
  return r;
}
double g2ohip_chi2(g2ohip_graph* g) {
  if (!g) return std::nan("");
  try {
    return g->e->chi2();
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return std::nan("");
  }
}
int g2ohip_optimize(g2ohip_graph* g, const g2ohip_config* cfg, int iterations, g2ohip_batch_stats* stats) {
  if (!g || iterations < 0) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->optimize(cfg, iterations, stats); });
}
int g2ohip_optimize_step(g2ohip_graph* g, const g2ohip_config* cfg, int iteration, g2ohip_batch_stats* stats) {
  if (!g || iteration < 0) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->optimize_step(cfg, iteration, stats); });
}
int g2ohip_solver_build_structure(g2ohip_graph* g) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->build_structure(); });
}
int g2ohip_solver_build_system(g2ohip_graph* g) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->build_system(); });
}
int g2ohip_solver_set_lambda(g2ohip_graph* g, double lambda, int backup) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->set_lambda(lambda, backup); });
}
int g2ohip_solver_restore_diagonal(g2ohip_graph* g) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->restore_diagonal(); });
}
int g2ohip_solver_solve(g2ohip_graph* g) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->solve_sync(); });
}
long long g2ohip_solver_vector_size(g2ohip_graph* g) { return g ? g->e->vector_size() : G2OHIP_ERR_ARG; }
int g2ohip_solver_block_dims(g2ohip_graph* g, int* dims) {
  if (!g || !dims) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->block_dims(dims); });
}
int g2ohip_solver_get_x(g2ohip_graph* g, double* x) {
  if (!g || !x) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->get_x(x); });
}
int g2ohip_solver_get_b(g2ohip_graph* g, double* b) {
  if (!g || !b) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->get_b(b); });
}
int g2ohip_solver_multiply_hessian(g2ohip_graph* g, double* dest, const double* src) {
  if (!g || !dest || !src) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->multiply_hessian(dest, src); });
}
int g2ohip_solver_linear_residual(g2ohip_graph* g, double* rel) {
  if (!g || !rel) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->linear_residual(rel); });
}
int g2ohip_local_landmarks(g2ohip_graph* g, int* ids, int cap) {
  if (!g || cap < 0) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->local_landmarks(ids, cap); });
}
int g2ohip_solver_factor_info(g2ohip_graph* g, double* out, int n) {
  if (!g || !out || n < 0) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->factor_info(out, n); });
}
int g2ohip_solver_compute_marginals(g2ohip_graph* g, int nblocks, const int* block_rows, const int* block_cols,
                                    double* out) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->compute_marginals(nblocks, block_rows, block_cols, out); });
}
int g2ohip_update(g2ohip_graph* g, const double* x_host) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->update_from(x_host); });
}
int g2ohip_push(g2ohip_graph* g) { return g ? guarded([&] { return g->e->push(); }) : G2OHIP_ERR_ARG; }
int g2ohip_pop(g2ohip_graph* g) { return g ? guarded([&] { return g->e->pop(); }) : G2OHIP_ERR_ARG; }
int g2ohip_discard_top(g2ohip_graph* g) { return g ? guarded([&] { return g->e->discard_top(); }) : G2OHIP_ERR_ARG; }
int g2ohip_stage(g2ohip_graph* g, double lambda, double* b, double* x, double* Hs, double* bs, long long* dims) {
  if (!g) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->stage(lambda, b, x, Hs, bs, dims); });
}

int g2ohip_linear_solve_ccs(int device, int n, const int* Ap, const int* Ai, const double* Ax, const double* b,
                            double* x, int nblocks, const int* block_ends) {
  if (n <= 0 || !Ap || !Ai || !Ax || !b || !x) return G2OHIP_ERR_ARG;
  if (!gfx950_device(device)) return G2OHIP_ERR_DEVICE;
  return guarded([&]() -> int {
    // Uniform block partition required (BlockSolver<p,l> pose blocks); default 1x1 blocks.
    int bd = 1;
    if (nblocks > 0 && block_ends) {
      bd = block_ends[0];
      for (int k = 0; k < nblocks; ++k)
        if (block_ends[k] != (k + 1) * bd) return G2OHIP_ERR_UNSUPPORTED;
      if (nblocks * bd != n) return G2OHIP_ERR_ARG;
    }
    const int nb = n / bd;
    // collect upper blocks from the scalar CCS
    std::map<std::pair<int, int>, int> bid;
    std::vector<int> bi, bj;
    for (int j = 0; j < n; ++j)
      for (int p = Ap[j]; p < Ap[j + 1]; ++p) {
        const int i = Ai[p];
        if (i > j) continue;
        auto key = std::make_pair(i / bd, j / bd);
        if (!bid.count(key)) { bid[key] = (int)bi.size(); bi.push_back(key.first); bj.push_back(key.second); }
      }
    for (int k = 0; k < nb; ++k) {
      auto key = std::make_pair(k, k);
      if (!bid.count(key)) { bid[key] = (int)bi.size(); bi.push_back(k); bj.push_back(k); }
    }
    std::vector<double> vals(bi.size() * bd * bd, 0.0);
    for (int j = 0; j < n; ++j)
      for (int p = Ap[j]; p < Ap[j + 1]; ++p) {
        const int i = Ai[p];
        if (i > j) continue;
        const int t = bid[{i / bd, j / bd}];
        const int r = i % bd, c = j % bd;
        vals[(size_t)t * bd * bd + c * bd + r] = Ax[p];
        if (i / bd == j / bd) vals[(size_t)t * bd * bd + r * bd + c] = Ax[p];
      }
    HIP_CHECK(hipSetDevice(device));
    hipStream_t s;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int ok = 0;
    {
      g2ohip::DeviceCholesky ch;
      ch.setup(nb, bd, bi, bj, s);
      g2ohip::DevBuf<double> dv, db, dx, dl;
      g2ohip::DevBuf<int> df;
      dv.upload(vals, s);
      db.upload(b, n, s);
      dx.resize(n);
      std::vector<double> zero{0.0};
      dl.upload(zero, s);
      df.resize(1);
      df.zero(s);
      ch.factor(dv.get(), dl.get(), db.get(), df.get(), s);
      ch.solve(dx.get(), s);
      int f = 0;
      HIP_CHECK(hipMemcpyAsync(&f, df.get(), sizeof f, hipMemcpyDeviceToHost, s));
      dx.download(x, n, s);
      HIP_CHECK(hipStreamSynchronize(s));
      ok = f ? 0 : 1;
    }
    (void)hipStreamDestroy(s);
    return ok;
  });
}

int g2ohip_comm_unique_id(unsigned char out[128]) {
  if (!out) return G2OHIP_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return G2OHIP_ERR_DEVICE;
  std::memcpy(out, &id, 128);
  return G2OHIP_OK;
}
int g2ohip_set_comm(g2ohip_graph* g, const unsigned char uid[128], int rank, int nranks) {
  if (!g || !uid || rank < 0 || rank >= nranks) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->set_comm(uid, rank, nranks); });
}
int g2ohip_comm_selftest(int device, const unsigned char uid[128], int n, const double* in, double* out) {
  return g2ohip_comm_selftest_rs(device, uid, n, in, out, nullptr);
}
int g2ohip_comm_selftest_rs(int device, const unsigned char uid[128], int n, const double* in, double* out,
                            double* rs_out) {
  if (!uid || n <= 0 || !in || !out) return G2OHIP_ERR_ARG;
  return guarded([&] {
    HIP_CHECK(hipSetDevice(device));
    std::string err;
    std::unique_ptr<g2ohip::Comm> c(g2ohip::make_rccl_comm(uid, 0, 1, err));
    if (!c) throw g2ohip::DeviceError(err);
    hipStream_t s = nullptr;
    HIP_CHECK(hipStreamCreate(&s));
    double* d = nullptr;
    HIP_CHECK(hipMalloc(&d, sizeof(double) * 4 * (size_t)n));
    for (int k = 0; k < 4; ++k) HIP_CHECK(hipMemcpyAsync(d + (size_t)k * n, in, sizeof(double) * n, hipMemcpyHostToDevice, s));
    c->allreduce_sum(d, (size_t)n, s);
    c->allreduce_max(d + n, (size_t)n, s);
    c->reduce_scatter_sum(d + 2 * (size_t)n, (size_t)n, s);  // in place: rank r's segment is [r n, (r + 1) n)
    c->allgather(d + 3 * (size_t)n, (size_t)n, s);           // in place: the distributed factorization's root exchange
    HIP_CHECK(hipMemcpyAsync(out, d, sizeof(double) * 2 * (size_t)n, hipMemcpyDeviceToHost, s));
    if (rs_out) HIP_CHECK(hipMemcpyAsync(rs_out, d + 2 * (size_t)n, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    std::vector<double> ag((size_t)n);
    HIP_CHECK(hipMemcpyAsync(ag.data(), d + 3 * (size_t)n, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (std::memcmp(ag.data(), in, sizeof(double) * n) != 0)
      throw g2ohip::DeviceError("ncclAllGather (in place, one rank) changed its segment");
    HIP_CHECK(hipFree(d));
    HIP_CHECK(hipStreamDestroy(s));
    c.reset();  // ncclCommDestroy
    return G2OHIP_OK;
  });
}
int g2ohip_set_comm_local(g2ohip_graph* g, const char* key, int rank, int nranks) {
  if (!g || !key || rank < 0 || rank >= nranks) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->set_comm_local(key, rank, nranks); });
}
int g2ohip_comm_local_reduce_host(const char* key, int rank, int nranks, double* buf, long long n, int is_max) {
  if (!key || rank < 0 || rank >= nranks || n < 0 || (n > 0 && !buf)) return G2OHIP_ERR_ARG;
  return guarded([&] {
    g2ohip::local_comm_reduce_host(key, rank, nranks, buf, (size_t)n, is_max != 0);
    return G2OHIP_OK;
  });
}

int g2ohip_runtime_info(char* out, int cap) {
  // which HIP runtime and RCCL this library's calls actually bound to (dladdr of the resolved symbols), and their
  // versions: a process that loaded another copy first (e.g. torch's bundled RCCL / HIP) is visible here
  auto where = [](const void* sym) -> std::string {
    Dl_info di;
    return dladdr(sym, &di) && di.dli_fname ? di.dli_fname : "?";
  };
  int hipv = 0, ncv = 0;
  (void)hipRuntimeGetVersion(&hipv);
  (void)ncclGetVersion(&ncv);
  const std::string s = std::string("{\"libamdhip64\": \"") + where((const void*)&hipStreamSynchronize) +
                        "\", \"hip_runtime_version\": " + std::to_string(hipv) + ", \"librccl\": \"" +
                        where((const void*)&ncclGetVersion) + "\", \"rccl_version\": " + std::to_string(ncv) +
                        ", \"libg2o_hip\": \"" + where((const void*)&g2ohip_runtime_info) + "\"}";
  if (out && cap > 0) {
    std::strncpy(out, s.c_str(), (size_t)cap - 1);
    out[cap - 1] = 0;
  }
  return (int)s.size() + 1;
}
int g2ohip_device_synchronize(int device) {
  return guarded([&] {
    HIP_CHECK(hipSetDevice(device));
    HIP_CHECK(hipDeviceSynchronize());
    return G2OHIP_OK;
  });
}
long long g2ohip_host_payload_len(g2ohip_graph* g, int edge_type) {
  if (!g) return G2OHIP_ERR_ARG;
  try {
    return g->e->host_payload_len(edge_type);
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return G2OHIP_ERR_DEVICE;
  }
}
int g2ohip_solver_save_hessian(g2ohip_graph* g, const char* path) {
  if (!g || !path) return G2OHIP_ERR_ARG;
  return guarded([&] { return g->e->save_hessian(path); });
}
int g2ohip_solver_set_write_debug(g2ohip_graph* g, int on) {
  if (!g) return G2OHIP_ERR_ARG;
  g->e->write_debug = on != 0;
  return G2OHIP_OK;
}

int g2ohip_debug_phases(unsigned long long* out, int max_records) {
  try {
    return g2ohip::launch::debug_phases(out, max_records);
  } catch (...) {
    return 0;
  }
}

int g2ohip_dist_plan(int nblocks, int bdim, int nblk, const int* bi, const int* bj, int nranks, int rank,
                     int flags, const double* pose_work, double* out, int* sn_owner, int cap) {
  if (nblocks <= 0 || bdim <= 0 || nblk < 0 || (nblk > 0 && (!bi || !bj)) || nranks < 1 || rank < 0 ||
      rank >= nranks || !out)
    return G2OHIP_ERR_ARG;
  try {
    for (int k = 0; k < nblk; ++k)
      if (bi[k] < 0 || bj[k] < 0 || bi[k] >= nblocks || bj[k] >= nblocks) return G2OHIP_ERR_ARG;
    const std::vector<int> vbi(bi, bi + nblk), vbj(bj, bj + nblk);
    const g2ohip::Symbolic S = g2ohip::analyze(g2ohip::block_pattern(nblocks, bdim, vbi, vbj));
    std::vector<double> pw;
    if (pose_work) pw.assign(pose_work, pose_work + nblocks);
    const g2ohip::DistPlan D = g2ohip::plan_distribution(S, vbi, vbj, bdim, nblocks, nranks, rank, flags & 1, false,
                                                         (flags & 2) != 0, pose_work ? &pw : nullptr);
    const double v[14] = {D.on ? 1.0 : 0.0, D.rank_s, D.shared_s, D.repl_s, D.xch_s, D.input_s, D.input_repl_s,
                          D.max_rank_s, (double)D.xch_seg, (double)D.rs_seg, (double)D.tail, (double)S.sn.size(),
                          D.shard_s, D.shard_repl_s};
    std::memcpy(out, v, sizeof v);
    if (sn_owner)
      for (int k = 0; k < (int)S.sn.size() && k < cap; ++k) sn_owner[k] = D.owner.empty() ? -1 : D.owner[k];
    return (int)S.sn.size();
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return G2OHIP_ERR_STATE;
  }
}

int g2ohip_symbolic_analyze(int nblocks, int bdim, int nblk, const int* bi, const int* bj, int* perm, double* stats) {
  if (nblocks <= 0 || bdim <= 0 || nblk < 0 || (nblk > 0 && (!bi || !bj))) return G2OHIP_ERR_ARG;
  try {
    for (int k = 0; k < nblk; ++k)
      if (bi[k] < 0 || bj[k] < 0 || bi[k] >= nblocks || bj[k] >= nblocks) return G2OHIP_ERR_ARG;
    // the pattern exactly as the solver's setup builds it (adjacency in block order): the same analysis
    g2ohip::Symbolic S = g2ohip::analyze(g2ohip::block_pattern(nblocks, bdim, std::vector<int>(bi, bi + nblk),
                                                               std::vector<int>(bj, bj + nblk)));
    if (perm) std::memcpy(perm, S.perm.data(), sizeof(int) * S.n);
    if (stats) {
      stats[0] = S.nnzL;
      stats[1] = S.flops;
      stats[2] = (double)S.sn.size();
      stats[3] = (double)S.num_levels;
      int lsteps = 0;  // level-synchronous 32-column panel steps (the factor's dependent launch chain)
      for (const auto& lv : S.levels) {
        int mx = 0;
        for (int sn : lv) mx = std::max(mx, (S.sn[sn].ns + 31) / 32);
        lsteps += mx;
      }
      stats[4] = (double)lsteps;
    }
    return S.n;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return G2OHIP_ERR_STATE;
  }
}

void g2ohip_enable_kernel_timing(g2ohip_graph* g, int on) {
  if (!g) return;
  g->e->timer.enabled = on != 0;
  g->e->timer.reset();
}
void g2ohip_kernel_timing_only(g2ohip_graph* g, const char* name) {
  if (!g) return;
  g->e->timer.only = name ? name : "";
}
void g2ohip_set_stats_level(g2ohip_graph* g, int level) {
  if (!g) return;
  g->e->stats_level = level < 0 ? 0 : (level > 2 ? 2 : level);
}
double g2ohip_kernel_ms(g2ohip_graph* g, const char* name) {
  if (!g || !name) return -1;
  auto& t = g->e->timer;
  auto it = t.total_ms.find(name);
  auto ct = t.count.find(name);
  if (it == t.total_ms.end() || ct == t.count.end() || ct->second == 0) return 0;
  return it->second / (double)ct->second;
}
long long g2ohip_kernel_count(g2ohip_graph* g, const char* name) {
  if (!g || !name) return -1;
  auto ct = g->e->timer.count.find(name);
  return ct == g->e->timer.count.end() ? 0 : ct->second;
}
double g2ohip_kernel_bytes(g2ohip_graph* g, const char* name) { return g && name ? g->e->kernel_bytes(name) : -1; }
double g2ohip_kernel_flops(g2ohip_graph* g, const char* name) { return g && name ? g->e->kernel_flops(name) : -1; }
const char* g2ohip_last_error(void) { return g_err.c_str(); }
int g2ohip_measure_peaks(int device, double* out, int n) {
  if (!out || n < 4) return G2OHIP_ERR_ARG;
  return guarded([&] {
    g2ohip::launch::measure_peaks(device, out);
    return 4;
  });
}
double g2ohip_lm_scale_factor(double rho) { return g2ohip::lm_scale_factor(rho); }
const char* g2ohip_version(void) { return "g2o_hip 0.2.0 (gfx950)"; }

}  // extern "C"
