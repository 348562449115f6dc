"""The fork's matrix-free solver lm_pcg6_3_eigen (JacobiSolver_6_3 + LinearSolverPCGEigen).

CPU: the numpy restatement (oracle/cgls_ref.py) solves the damped normal equations exactly when eta -> 0 and its LM
loop reduces chi2. GPU: the device CGLS (g2o_amd/csrc/cgls.hip) behind the LM loop follows the restatement's LM
trajectory (chi2 and trial counts per iteration, final state) within the north_star 1e-6; "parity unpinned" against
reference outputs (the fork's solver needs Eigen).
"""
import math

import numpy as np
import pytest

import cgls_ref
from g2o_amd import synth

RTOL = 1e-6


def _tiny():
    return synth.ba(num_cameras=12, num_points=200, obs_per_point=5, window=8)


def _system(oracle, prob):
    host = oracle.OracleGraph(prob)
    host.chi2()
    cams, pts = prob.vertices
    e = prob.edges[0]
    free = cams.fixed == 0
    cam_idx = {int(i): k for k, i in enumerate(np.sort(cams.ids[free]))}
    pt_idx = {int(i): k for k, i in enumerate(np.sort(pts.ids))}
    cam_col = np.array([cam_idx.get(int(c), -1) for c in e.v1])
    pt_col = np.array([pt_idx.get(int(p), -1) for p in e.v0])
    pay = host.edge_payload(np.arange(len(e.v0)), 20 * len(e.v0), numeric=False)
    J = cgls_ref.jacobian(pay, cam_col, pt_col, np.sqrt(e.info[:, 0, 0]), len(cam_idx), len(pt_idx))
    return J, len(cam_idx), len(pt_idx)


def test_cgls_restatement_direct(oracle):
    J, nc, npt = _system(oracle, _tiny())
    rng = np.random.default_rng(2)
    b = rng.standard_normal(J.shape[1])
    lam = 0.3
    x, it = cgls_ref.cgls_solve(J, b, nc, npt, math.sqrt(lam), eta=1e-28)
    Jr = J[: J.shape[0] - J.shape[1]]
    xd = np.linalg.solve(Jr.T @ Jr + lam * np.eye(J.shape[1]), b)
    assert 0 < it and np.linalg.norm(x - xd) <= 1e-8 * np.linalg.norm(xd)
    # the forcing term stops early: fewer iterations, an inexact but useful step
    x1, it1 = cgls_ref.cgls_solve(J, b, nc, npt, math.sqrt(lam), eta=0.1)
    assert it1 < it and np.linalg.norm(x1 - xd) < np.linalg.norm(xd)


def test_cgls_restatement_lm(oracle):
    prob = _tiny()
    host = oracle.OracleGraph(prob)
    c0 = host.chi2()
    st = cgls_ref.jacobi_lm(host, prob, 5)
    assert st[-1][0] < 0.05 * c0 and all(s[3] > 0 for s in st)


@pytest.mark.gpu
@pytest.mark.parametrize("eta", [0.1, 1e-3])
def test_gpu_cgls_lm_matches_restatement(g2o_amd_mod, oracle, eta):
    for prob in (_tiny(), synth.ba(num_cameras=20, num_points=400, obs_per_point=6, window=10, seed=9)):
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
        opt.set_algorithm("lm_pcg6_3_eigen")
        opt.set_eta(eta)
        n, st = opt.optimize(5)
        host = oracle.OracleGraph(prob)
        sr = cgls_ref.jacobi_lm(host, prob, 5, eta=eta)
        assert n == len(sr)
        for a, b in zip(st, sr):
            assert a.levenbergIterations == b[1]
            assert abs(a.chi2 - b[0]) <= RTOL * b[0], (a.chi2, b[0])
        xg, xr = opt.minimal_state(), host.minimal_state()
        assert np.linalg.norm(xg - xr) <= RTOL * np.linalg.norm(xr)


@pytest.mark.gpu
def test_gpu_cgls_c4_small_reaches_cholesky_chi2(g2o_amd_mod):
    """On C4-small the inexact CGLS steps (eta 0.1) still converge to the Cholesky path's chi2 within 1 %."""
    prob = synth.by_name("C4", "small")
    a = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    a.set_algorithm("lm_pcg6_3_eigen")
    n, st = a.optimize(10)
    b = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    nb, sb = b.optimize(10)
    assert abs(st[-1].chi2 - sb[-1].chi2) <= 1e-2 * sb[-1].chi2 and a.linear_iterations() > 0
