"""TEST INFRASTRUCTURE ONLY (checker, never shipped or measured): numpy restatement of g2o's
block-Jacobi preconditioned conjugate gradient, LinearSolverPCG<MatrixType>::solve
(g2o/solvers/pcg/linear_solver_pcg.hpp:80-159), defaults from linear_solver_pcg.h:51-58.

Parity status: the reference PCG is header-only C++ over Eigen (absent here), so this restatement is
pinned by construction against np.linalg.solve (tests/test_pcg_oracle.py) — "parity unpinned" against
reference outputs; the GPU path is checked against this restatement.
"""
import math

import numpy as np


def pcg_solve(A, b, pd, tolerance=1e-6, absolute_tolerance=True, residual=-1.0, max_iter=-1):
    """Solve A x = b (A dense symmetric, block size pd). Returns (x, iterations, new_residual).

    `residual` is the value the solver carries between calls (`_residual`, -1 after init(),
    linear_solver_pcg.h:56,66); the returned one is 0.5 * dn (linear_solver_pcg.hpp:153).
    """
    n = len(b)
    nb = n // pd
    # _J: inverses of the diagonal blocks (:92-96)
    J = [np.linalg.inv(A[i * pd:(i + 1) * pd, i * pd:(i + 1) * pd]) for i in range(nb)]

    def mult_diag(v):  # multDiag (:162-170)
        out = np.empty_like(v)
        for i in range(nb):
            sl = slice(i * pd, (i + 1) * pd)
            out[sl] = J[i] @ v[sl]
        return out

    x = np.zeros(n)
    r = b.astype(np.float64).copy()
    d = mult_diag(r)  # :118-121
    dn = float(r @ d)
    d0 = tolerance * dn
    if absolute_tolerance and residual > 0.0 and residual > d0:  # :125-128
        d0 = residual
    maxit = n if max_iter < 0 else max_iter  # :130
    it = 0
    while it < maxit:  # :133-151
        if dn <= d0:
            break
        q = A @ d
        a = dn / float(d @ q)
        x += a * d
        r -= a * q
        s = mult_diag(r)
        dold = dn
        dn = float(r @ s)
        d = s + (dn / dold) * d
        it += 1
    return x, it, 0.5 * dn


def pcg_lm(host, iterations, pd, max_trials=10, tolerance=1e-6):
    """OptimizationAlgorithmLevenberg (optimization_algorithm_levenberg.cpp:58-184) around LinearSolverPCG on a
    pose graph (no Schur): the reduced system of every trial from the oracle's stage(lambda) (Hpp + lambda I, b), the
    PCG's `_residual` carried across every trial and iteration (set once by init(), linear_solver_pcg.h:66).
    host: an oracle graph. Returns [(chi2, trials, lambda, pcg_iterations_of_the_last_trial)]."""
    stats = []
    lam, ni, carry = None, 2.0, -1.0
    for it in range(iterations):
        current = host.chi2()
        if it == 0:  # computeLambdaInit: tau * max diagonal entry of the Hessian (:152-175)
            H0 = host.stage(0.0)["Hschur"]
            lam = 1e-5 * float(np.max(np.abs(np.diag(H0))))
            ni = 2.0
        q, rho, cg = 0, 0.0, 0
        while True:
            st = host.stage(lam)
            b = st["bschur"]
            x, cg, carry = pcg_solve(st["Hschur"], b, pd, tolerance=tolerance, residual=carry)
            host.push()
            host.update(x)
            temp = host.chi2()
            rho = (current - temp) / (float(x @ (lam * x + b)) + 1e-3)  # computeScale (:177-184)
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
