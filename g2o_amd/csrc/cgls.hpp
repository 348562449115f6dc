// Matrix-free preconditioned CGLS on the bundle-adjustment Jacobian, device resident: the fork's
// JacobiSolver_6_3 + LinearSolverPCGEigen ("lm_pcg6_3_eigen", solvers/eigen/solver_eigen.cpp:80,126).
//
//   JacobiSolver::buildSystem (core/jacobi_solver.hpp:479-700): J has two rows per observation, each scaled by
//   sqrt(Omega(0,0)), columns [cameras 6 | points 3]; below it one identity row per unknown scaled by sqrt(lambda)
//   (setLambda, :703-718). b = -sum J^T Omega e as BlockSolver's (copyB).
//   LinearSolverPCGEigen::solve (solvers/eigen/linear_solver_pcg_eigen.h:70-248): block preconditioner R = diag(R_c,
//   R_p) from the QR of every camera's / point's column block of J (computeRc_inverse / computeRp_inverse,
//   :378-517), then CG on the normal equations of J R^-1 started at y = (0, R_p^-T b_p): the preconditioned normal
//   matrix has identity diagonal blocks, so the residual lives in the camera block on odd and in the point block on
//   even iterations; stop when s.s < eta s0.s0; x = R^-1 y.
// Here R comes from the Cholesky factor of the block Gram matrix J_b^T J_b + lambda I (R^T R is the same matrix; a
// QR's R differs by the signs of its rows, which CG's iterates x do not depend on).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace g2ohip {

struct DeviceCGLS {
  double eta = 0.1;  // LinearSolver::solve default forcing term (core/linear_solver.h:66)
  int last_iterations = 0;

  // edges in the BA group's (landmark-major) order; pt_ptr: per local landmark its edge range; cam_ptr/cam_e: per
  // camera its edges (indices into the group order)
  void setup(int ncam, int npt, int ne, const std::vector<int>& pt_ptr, const std::vector<int>& cam_ptr,
             const std::vector<int>& cam_e, const std::vector<int>& e_cam, const std::vector<int>& e_pt,
             hipStream_t s);
  // per LM iteration: J (sqrt(Omega00)-scaled Jacobian blocks of the edges) and the block Gram matrices
  void build(const EdgeArgs& a, const int* h0, const int* h1, hipStream_t s);
  // max |diag(J^T J)| (computeLambdaInit's fallback when the vertex Hessians are empty,
  // optimization_algorithm_levenberg.cpp:165-172) into *out
  void diag_max(double* partial, double* out, hipStream_t s);
  // x = argmin ||J x - r|| with the lambda rows, b = J^T r given (poses first, then landmarks); lam = device lambda
  void solve(const double* lam, const double* b, double* x, hipStream_t s);
  DeviceCGLS() = default;
  DeviceCGLS(const DeviceCGLS&) = delete;
  DeviceCGLS& operator=(const DeviceCGLS&) = delete;
  ~DeviceCGLS();

 private:
  int ncam = 0, npt = 0, ne = 0, n = 0, npart = 0;
  DevBuf<int> pt_ptr, cam_ptr, cam_e, e_cam, e_pt;  // e_cam / e_pt: per edge its camera / local point (-1 fixed)
  DevBuf<double> JA, JB, JBc;  // 2x3 / 2x6 row-major per edge (edge order); JB again camera-major
  DevBuf<double> Gc, Gp;       // Gram blocks (full 6x6 / 3x3)
  DevBuf<double> Rc, Rp;       // R^-1 blocks (upper triangular, full storage, row-major)
  DevBuf<double> y, p, sv, z, q, part, sc;
  hipGraphExec_t chunk_exec = nullptr;
  void iterate(int k0, int cnt, hipStream_t s);
};

}  // namespace g2ohip
