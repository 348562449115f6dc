"""Block-Jacobi PCG (linear_solver_pcg.hpp:80-159; §8f rank 3).

CPU: the numpy restatement (oracle/pcg_ref.py) converges to np.linalg.solve and honours the carried
absolute residual. GPU: the device PCG behind the `lm_pcg*` algorithms against that restatement on the
reduced system the engine stages. Tolerance: both sides run the same recurrence in a different
summation order, stopping at a relative preconditioned residual of 1e-6, so the iterates agree to
1e-5 relative (not bitwise); both are equally inexact against the direct solution.
"""
import numpy as np
import pytest

import pcg_ref
from g2o_amd import synth

PCG_RTOL = 1e-5


def _block_spd(nb, pd, seed):
    rng = np.random.default_rng(seed)
    n = nb * pd
    M = rng.standard_normal((n, n)) * (rng.random((n, n)) < 0.1)
    return M @ M.T + n * 0.05 * np.eye(n), rng.standard_normal(n)


def test_pcg_restatement_converges():
    A, b = _block_spd(40, 6, 1)
    x, it, res = pcg_ref.pcg_solve(A, b, 6, tolerance=1e-14)
    assert 0 < it <= len(b)
    assert np.linalg.norm(x - np.linalg.solve(A, b)) <= 1e-6 * np.linalg.norm(x)
    assert res >= 0.0


def test_pcg_restatement_absolute_residual_carry():
    A, b = _block_spd(30, 3, 2)
    _, it0, res = pcg_ref.pcg_solve(A, b, 3)
    # a carried residual larger than tol*dn ends the next solve earlier (linear_solver_pcg.hpp:125-128)
    _, it1, _ = pcg_ref.pcg_solve(A, b, 3, residual=res * 1e6)
    assert it1 < it0
    _, it2, _ = pcg_ref.pcg_solve(A, b, 3, residual=res * 1e6, absolute_tolerance=False)
    assert it2 == it0
    _, it3, _ = pcg_ref.pcg_solve(A, b, 3, max_iter=2)
    assert it3 == 2


def test_pcg_restatement_indefinite_block():
    """An indefinite diagonal block (the Jacobi preconditioner is its plain inverse, linear_solver_pcg.hpp:92-96):
    r.(J r) < 0 at the start satisfies dn <= tol dn at once — zero iterations, x = 0 — both here and on the
    device (k_pcg_start: the same test); a singular block gives a non-finite preconditioner and a NaN x,
    which the LM rejects like a failed factorization."""
    A, b = _block_spd(10, 3, 4)
    A[:3, :3] = np.diag([1.0, -2.0, 3.0])
    # make r.(J r) negative: b concentrated on the negative direction of the indefinite block
    b = np.zeros_like(b)
    b[1] = 1.0
    x, it, res = pcg_ref.pcg_solve(A, b, 3)
    assert it == 0 and not np.any(x) and res < 0
    A[:3, :3] = 0.0
    with np.errstate(all="ignore"):
        try:
            x, it, _ = pcg_ref.pcg_solve(A, b, 3)
            assert not np.all(np.isfinite(x))
        except np.linalg.LinAlgError:  # numpy refuses the singular block outright
            pass


@pytest.mark.gpu
@pytest.mark.parametrize("name,pd,rtol", [("C1", 6, 1e-6), ("C2", 3, 1e-4)])
def test_gpu_pcg_lm_matches_restatement(g2o_amd_mod, oracle, name, pd, rtol):
    """The whole LM loop around the PCG (lm_pcg) against pcg_ref.pcg_lm: per-iteration chi2, lambda and trial
    counts, with the PCG's absolute-tolerance residual carried across every trial and iteration.
    Both sides see the same reduced systems up to summation order. On C1 (14-60 CG iterations) chi2 and lambda
    agree to 1e-6; the SE2 grid (150-210 iterations per solve on an ill-conditioned system) amplifies the
    summation-order rounding to ~1e-5 in chi2 — even two runs of the multithreaded oracle differ that much."""
    prob = synth.by_name(name, "small")
    iters = 6 if name == "C1" else 4
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm("lm_pcg")
    n, st = opt.optimize(iters)
    ref = pcg_ref.pcg_lm(oracle.OracleGraph(prob), iters, pd)
    assert n == len(ref)
    for a, (chi2, trials, lam, _) in zip(st, ref):
        assert a.levenbergIterations == trials
        assert abs(a.chi2 - chi2) <= rtol * chi2, (a.chi2, chi2)
        assert abs(a.lambda_ - lam) <= rtol * lam, (a.lambda_, lam)


@pytest.mark.gpu
@pytest.mark.parametrize("name,algo,pd", [("C4", "lm_pcg6_3", 6), ("C1", "lm_pcg", 6), ("C2", "lm_pcg", 3)])
def test_gpu_pcg_matches_restatement(g2o_amd_mod, name, algo, pd):
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm(algo)
    g = opt.stage(1e-3)
    A, bs = g["Hschur"], g["bschur"]
    x_ref, it, _ = pcg_ref.pcg_solve(A, bs, pd)
    assert it > 0
    xg = g["x"][:g["np"]]
    # CG amplifies the summation-order rounding over its iterations (hundreds on the SE2 pose graph)
    assert np.linalg.norm(xg - x_ref) <= PCG_RTOL * np.linalg.norm(x_ref), (np.linalg.norm(xg - x_ref), it)
    # the reference stops at dn <= 1e-6 dn_0 (preconditioned residual): an inexact solve (a few % off
    # the direct solution on BA, far more on the ill-conditioned pose graphs) — the GPU result must be
    # exactly as inexact as the restatement's
    x_direct = np.linalg.solve(A, bs)
    e_g, e_r = np.linalg.norm(xg - x_direct), np.linalg.norm(x_ref - x_direct)
    assert abs(e_g - e_r) <= PCG_RTOL * np.linalg.norm(x_direct)


@pytest.mark.gpu
def test_gpu_pcg_lm_reduces_chi2(g2o_amd_mod, oracle):
    """LM with the PCG linear solver follows the Cholesky trajectory closely (inexact solves)."""
    prob = synth.by_name("C4", "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm("lm_pcg6_3")
    n, st = opt.optimize(6)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.optimize(6, oracle.make_config(threads=4))
    assert n == 6 and nr == 6
    chis = [s.chi2 for s in st]
    assert all(b <= a * (1 + 1e-12) for a, b in zip(chis, chis[1:])), chis
    assert abs(chis[-1] - sr[-1].chi2) <= 1e-2 * sr[-1].chi2, (chis[-1], sr[-1].chi2)
