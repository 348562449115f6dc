// Block-Jacobi preconditioned conjugate gradient on the block-sparse reduced system, device resident.
// Replaces LinearSolverPCG<MatrixType>::solve (g2o/solvers/pcg/linear_solver_pcg.hpp:80-159) behind the
// same BlockSolver seam as DeviceCholesky (§8f rank 3): A is given as the upper block triangle the
// engine already holds in HBM (S for the Schur case, Hpp otherwise), pd x pd col-major blocks, with a
// virtual λ added to the diagonal.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "common.hpp"

namespace g2ohip {

struct DevicePCG {
  // linear_solver_pcg.h:51-58 defaults
  double tolerance = 1e-6;
  bool absolute_tolerance = true;
  int max_iter = -1;  // < 0: A.rows()
  int last_iterations = 0;

  // bi/bj: block row/col of every stored block (each unordered pair once, diagonal blocks present)
  void setup(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj, hipStream_t s);
  // x = (A + λ I)^-1 b by PCG; synchronises `s` every CHUNK iterations to test convergence
  void solve(const double* vals, const double* lam, const double* b, double* x, hipStream_t s);
  // LinearSolverPCG::init (linear_solver_pcg.h:63-68): forget the carried residual
  void reset(hipStream_t s);
  DevicePCG() = default;
  DevicePCG(const DevicePCG&) = delete;
  DevicePCG& operator=(const DevicePCG&) = delete;
  ~DevicePCG() {
    if (chunk_exec) (void)hipGraphExecDestroy(chunk_exec);
  }

 private:
  int nb = 0, pd = 0, n = 0, npa = 0, npb = 0;
  DevBuf<int> rptr, diag;
  DevBuf<int2> ent;  // (block index, other block row | 0x80000000 when the block is used transposed)
  DevBuf<double> J, r, sv, q, dbuf, part, sc;
  hipGraphExec_t chunk_exec = nullptr;  // CHUNK iterations captured once per (vals, λ, x, maxIter)
  const void* chunk_key[4] = {};
};

}  // namespace g2ohip
