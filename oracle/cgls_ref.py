"""TEST INFRASTRUCTURE ONLY (checker, never shipped or measured): numpy restatement of the fork's matrix-free
solver "lm_pcg6_3_eigen" (solvers/eigen/solver_eigen.cpp:80,126):

* JacobiSolver<6,3>::buildSystem (core/jacobi_solver.hpp:479-700): J with two rows per observation scaled by
  sqrt(Omega(0,0)), columns [cameras (6 each) | points (3 each)] in Hessian order, one identity row per unknown
  below it scaled by sqrt(lambda) (setLambda, :703-718); b = -sum J^T Omega e (copyB).
* LinearSolverPCGEigen::solve (solvers/eigen/linear_solver_pcg_eigen.h:70-248) with computeRc_inverse /
  computeRp_inverse (:378-517): R_b from the Householder QR of each camera's / point's column block of J (lambda rows
  included), y0 = (0, R_p^-T b_p), CG on the normal equations of J R^-1 with the residual alternating between the
  camera block (odd iterations) and the point block (even iterations), stop when s.s < eta s0.s0, x = R^-1 y.
* OptimizationAlgorithmLevenberg (optimization_algorithm_levenberg.cpp:58-184) around it, computeLambdaInit falling
  back to max diag(J^T J) because JacobiSolver leaves the vertex Hessians empty (:165-172).

Parity status: the fork's solver is Eigen code (absent here): "parity unpinned" against reference outputs; the
device CGLS (g2o_amd/csrc/cgls.hip) is checked against this restatement, the restatement against a direct solve.
"""
import math

import numpy as np


def jacobian(payload, cam_col, pt_col, sqrt_info, ncam, npt):
    """Edge rows of J from [e (2) | A (2x3) | B (2x6)] payloads; cam_col / pt_col: Hessian block index or -1."""
    ne = len(cam_col)
    n = 6 * ncam + 3 * npt
    rows = 2 * ne
    J = np.zeros((rows + n, n))
    P = payload.reshape(ne, 20)
    for e in range(ne):
        A = P[e, 2:8].reshape(2, 3) * sqrt_info[e]
        B = P[e, 8:20].reshape(2, 6) * sqrt_info[e]
        if pt_col[e] >= 0:
            c = 6 * ncam + 3 * pt_col[e]
            J[2 * e:2 * e + 2, c:c + 3] = A
        if cam_col[e] >= 0:
            c = 6 * cam_col[e]
            J[2 * e:2 * e + 2, c:c + 6] = B
    return J


def cgls_solve(J, b, ncam, npt, sqrt_lam, eta=0.1):
    """LinearSolverPCGEigen::solve. J: dense (2 ne + n) x n with the lambda rows still zero. Returns (x, iterations)."""
    n = J.shape[1]
    rows = J.shape[0] - n
    J = J.copy()
    J[rows:, :] = np.eye(n) * sqrt_lam  # setLambda: the scale entries are sqrt(lambda)
    Rinv = []
    for c in range(ncam):  # computeRc_inverse: QR of the camera's column block (its rows + lambda rows)
        blk = J[:, 6 * c:6 * c + 6]
        nz = np.nonzero(np.any(blk != 0, axis=1))[0]
        R = np.linalg.qr(blk[nz], mode="r")[:6, :6]
        Rinv.append(np.linalg.inv(R))
    for p in range(npt):  # computeRp_inverse: QR of [point rows; sqrt(lambda) I]
        c = 6 * ncam + 3 * p
        blk = J[:rows, c:c + 3]
        nz = np.nonzero(np.any(blk != 0, axis=1))[0]
        R = np.linalg.qr(np.vstack([blk[nz], np.eye(3) * sqrt_lam]), mode="r")[:3, :3]
        Rinv.append(np.linalg.inv(R))
    offs = [6 * c for c in range(ncam)] + [6 * ncam + 3 * p for p in range(npt)]
    dims = [6] * ncam + [3] * npt

    def rmul(v, tr):
        out = np.empty_like(v)
        for Ri, o, d in zip(Rinv, offs, dims):
            out[o:o + d] = (Ri.T if tr else Ri) @ v[o:o + d]
        return out

    nc = 6 * ncam
    pb = rmul(b, True)  # R^-T b
    x = np.zeros(n)
    x[nc:] = pb[nc:]  # xC = 0, xP = bP
    p = pb - rmul(J.T @ (J @ rmul(x, False)), True)
    s = p.copy()
    q = J @ rmul(p, False)
    maxit = J.shape[0] + J.shape[0] % 2
    gamma = float(s @ s)
    gamma_old = gamma
    thr = eta * float(s @ s)
    it = 0
    while it < maxit:
        if gamma < thr:
            break
        even = it % 2 == 0
        alpha = gamma / float(q @ q)
        x += alpha * p
        s = np.zeros(n)
        if not even:  # cameras
            s[:nc] = rmul(np.concatenate([-alpha * (J[:, :nc].T @ q), np.zeros(n - nc)]), True)[:nc]
        else:  # points
            s[nc:] = rmul(np.concatenate([np.zeros(nc), -alpha * (J[:, nc:].T @ q)]), True)[nc:]
        gamma = float(s @ s)
        beta = gamma / gamma_old
        gamma_old = gamma
        p = s + beta * p
        if not even:
            z = rmul(np.concatenate([s[:nc], np.zeros(n - nc)]), False)
            q = beta * q + J[:, :nc] @ z[:nc]
        else:
            z = rmul(np.concatenate([np.zeros(nc), s[nc:]]), False)
            q = beta * q + J[:, nc:] @ z[nc:]
        it += 1
    return rmul(x, False), it


def jacobi_lm(host, prob, iterations, eta=0.1, max_trials=10):
    """OptimizationAlgorithmLevenberg + JacobiSolver_6_3 + LinearSolverPCGEigen on a pure BA problem; host is an
    oracle graph of `prob` (errors, Jacobians, update, push/pop). Returns [(chi2, trials, lambda, cg_iters)]."""
    cams, pts = prob.vertices
    e = prob.edges[0]
    free = cams.fixed == 0
    cam_idx = {int(i): k for k, i in enumerate(np.sort(cams.ids[free]))}
    pt_idx = {int(i): k for k, i in enumerate(np.sort(pts.ids))}
    ncam, npt = len(cam_idx), len(pt_idx)
    cam_col = np.array([cam_idx.get(int(c), -1) for c in e.v1])
    pt_col = np.array([pt_idx.get(int(p), -1) for p in e.v0])
    sqrt_info = np.sqrt(e.info[:, 0, 0])
    idx = np.arange(len(e.v0))
    n = 6 * ncam + 3 * npt
    stats = []
    lam, ni = None, 2.0
    for it in range(iterations):
        current = host.chi2()
        pay = host.edge_payload(idx, 20 * len(idx), numeric=False)
        J = jacobian(pay, cam_col, pt_col, sqrt_info, ncam, npt)
        P = pay.reshape(-1, 20)
        b = np.zeros(n)  # copyB: b = -sum J^T Omega e with the full information
        for k in range(len(idx)):
            om = e.info[k] @ P[k, :2]
            if pt_col[k] >= 0:
                o = 6 * ncam + 3 * pt_col[k]
                b[o:o + 3] -= P[k, 2:8].reshape(2, 3).T @ om
            if cam_col[k] >= 0:
                o = 6 * cam_col[k]
                b[o:o + 6] -= P[k, 8:20].reshape(2, 6).T @ om
        if it == 0:
            lam = 1e-5 * float(np.max(np.abs(np.einsum("ij,ij->j", J, J))))
            ni = 2.0
        q, rho, cg = 0, 0.0, 0
        while True:
            host.push()
            x, cg = cgls_solve(J, b, ncam, npt, math.sqrt(lam), eta)
            host.update(x)
            temp = host.chi2()
            rho = (current - temp) / (float(x @ (lam * x + b)) + 1e-3)
            if rho > 0 and math.isfinite(temp):
                lam *= max(1.0 / 3.0, min(1.0 - (2 * rho - 1) ** 3, 2.0 / 3.0))
                ni = 2.0
                current = temp
                host.discard_top()
            else:
                lam *= ni
                ni *= 2
                host.pop()
                if not math.isfinite(lam):
                    break
            q += 1
            if not (rho < 0 and q < max_trials):
                break
        stats.append((host.chi2(), q, lam, cg))
        if q == max_trials or rho == 0 or not math.isfinite(lam):
            break
    return stats
