"""Solver::computeMarginals on the device (block_solver.hpp:451-460 -> LinearSolverCSparse::solvePattern,
linear_solver_csparse.h:190-225, MarginalCovarianceCholesky): the requested blocks of Hpp^-1 against numpy's inverse
of the oracle's dense Hpp at the same state.

Block pattern as g2o_cli requests it (apps/g2o_cli/g2o.cpp:581-595): (i, i) for every pose and (i-1, i).
Tolerance: 1e-9 relative (Frobenius over all requested blocks) at the same linearization point — both sides are
fp64 with a different summation order; pose graphs here have condition numbers up to ~1e5.
"""
import numpy as np
import pytest

from g2o_amd import synth

pytestmark = pytest.mark.gpu


def _pattern(npose):
    return [(i, i) for i in range(npose)] + [(i - 1, i) for i in range(1, npose)]


def _dense_inverse(oracle, prob):
    ref = oracle.OracleGraph(prob)
    r = ref.stage(0.0)
    Hpp, _, _ = ref.hessian_dense(r["np"], r["nl"])
    return np.linalg.inv(Hpp)


def _compare(blocks, Hinv, pd, tol):
    num = den = 0.0
    for (r, c), B in blocks.items():
        R = Hinv[r * pd:(r + 1) * pd, c * pd:(c + 1) * pd]
        num += float(np.sum((B - R) ** 2))
        den += float(np.sum(R ** 2))
    rel = np.sqrt(num / den)
    assert rel <= tol, rel


@pytest.mark.parametrize("name,algo", [("C1", "lm_hip_var"), ("C2", "lm_hip_var"), ("C4", "lm_hip_var"),
                                       ("C1", "lm_pcg")])
def test_marginals_vs_dense_inverse(g2o_amd_mod, oracle, name, algo):
    """C1 / C2 reuse the LM's own factor of Hpp (pd 6 / 3: 10 / 21 block columns per batch), C4 (Schur mode: the
    LM factors S) and the PCG algorithm set up a separate factor of Hpp."""
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm(algo)
    opt.initialize_optimization()
    opt.build_structure()
    opt.build_system()
    pd, _, npose, _ = opt.block_dims()
    pat = _pattern(npose)
    blocks = opt.compute_marginals(pat)
    assert blocks is not None and len(blocks) == len(pat)
    _compare(blocks, _dense_inverse(oracle, prob), pd, 1e-9)


def test_marginals_after_optimize(g2o_amd_mod, oracle):
    """After LM iterations (the factor's buffers last held a damped system): Hpp of a fresh buildSystem at the
    optimized state, against the oracle optimized the same way (states agree to the trajectory tolerance)."""
    prob = synth.by_name("C1", "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.optimize(3)
    opt.build_system()
    ref = oracle.OracleGraph(prob)
    ref.optimize(3, oracle.make_config(threads=8))
    r = ref.stage(0.0)
    Hpp, _, _ = ref.hessian_dense(r["np"], r["nl"])
    pd, _, npose, _ = opt.block_dims()
    pat = [(i, i) for i in range(0, npose, 7)] + [(0, npose - 1), (3, 40)]
    blocks = opt.compute_marginals(pat)
    _compare(blocks, np.linalg.inv(Hpp), pd, 1e-6)
    # the LM still runs after the marginals borrowed its factor
    n, st = opt.optimize(2)
    nr, sr = ref.optimize(2, oracle.make_config(threads=8))
    assert n == nr
    assert abs(st[-1].chi2 - sr[-1].chi2) <= 1e-6 * abs(sr[-1].chi2)


def test_marginals_many_batches(g2o_amd_mod, oracle):
    """Every pose's diagonal block and a full block row of C2 (800 poses, pd 3: 39 batches of 21 block columns),
    arbitrary request order with repeats."""
    prob = synth.by_name("C2", "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.initialize_optimization()
    opt.build_structure()
    opt.build_system()
    pd, _, npose, _ = opt.block_dims()
    rng = np.random.default_rng(3)
    pat = [(i, i) for i in rng.permutation(npose)] + [(5, j) for j in range(npose)] + [(7, 7), (7, 7)]
    blocks = opt.compute_marginals(pat)
    _compare(blocks, _dense_inverse(oracle, prob), pd, 1e-9)
    assert opt.compute_marginals([]) == {}


@pytest.mark.parametrize("knobs", [
    {"G2OHIP_CHOL_FUSED_MAX": "0", "G2OHIP_CHOL_BLOCK_MIN": "64", "G2OHIP_CHOL_PB": "64", "G2OHIP_CHOL_WIDE_PB": "64"},
    {"G2OHIP_CHOL_LAG": "2"},
    {"G2OHIP_CHOL_FUSED_MAX": "0", "G2OHIP_CHOL_LAG": "1"},
], ids=["blocked_fronts", "lagged_all_levels", "lagged_separate_contrib"])
@pytest.mark.parametrize("name", ["C1", "C3"])
def test_marginals_blocked_and_lagged_schedules(g2o_amd_mod, oracle, monkeypatch, knobs, name):
    """The marginal solves read the factor's layout (L21 per front, L_kk^-1 per panel, no stored diagonal blocks).
    The full-size schedules — blocked fronts with big-panel trailing updates and backward rounds, lagged rank-64 pair
    steps — only appear on large systems; the schedule knobs force them on the small C1 / C3 pose graphs, so the
    marginals are checked against the dense inverse on exactly those factor layouts."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.initialize_optimization()
    opt.build_structure()
    opt.build_system()
    info = opt.factor_info()
    if "G2OHIP_CHOL_BLOCK_MIN" in knobs:
        assert info["blocked_fronts"] > 0 and info["bwd_rounds"] > 0, info
    pd, _, npose, _ = opt.block_dims()
    pat = _pattern(npose)
    blocks = opt.compute_marginals(pat)
    assert blocks is not None
    _compare(blocks, _dense_inverse(oracle, prob), pd, 1e-9)
