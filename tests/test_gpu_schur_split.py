"""Schur split formed at assembly (kernels.hpp SchurSplit): the LM loop's buildSystem knows lambda, so the
linearize waves store G = Hpl U^-T (Hll + lambda I = U U^T) and the camera pass forms S(i,i) and bschur
directly (block_solver.hpp:341-400). Checked against the oracle's BlockSolver at the stage level (reduced
system, solution) and through LM trajectories whose rejected trials re-assemble at another lambda; the plain
passes (G2OHIP_SCHUR_SPLIT=0) give the same trajectory.
"""
import numpy as np
import pytest

from g2o_amd import synth

pytestmark = pytest.mark.gpu


def _stage(g2o_amd_mod, oracle, prob, lam, monkeypatch):
    monkeypatch.setenv("G2OHIP_STAGE_SPLIT", "1")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    g = opt.stage(lam)
    r = oracle.OracleGraph(prob).stage(lam)
    assert g["ok"] == r["ok"] == 1
    for k in ("b", "bschur", "x"):
        assert np.linalg.norm(g[k] - r[k]) <= 1e-9 * np.linalg.norm(r[k]), k
    assert np.linalg.norm(g["Hschur"] - r["Hschur"]) <= 1e-11 * np.linalg.norm(r["Hschur"])


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_split_stage_reduced_system(g2o_amd_mod, oracle, name, monkeypatch):
    _stage(g2o_amd_mod, oracle, synth.by_name(name, "small"), 1e-3, monkeypatch)


def test_split_stage_long_tracks(g2o_amd_mod, oracle, monkeypatch):
    """Landmarks seen by more than 64 cameras span several linearize waves: their U, c and G are formed by
    k_lm_fixup after the partial sums (mixed with short tracks)."""
    prob = synth.ba(num_cameras=140, num_points=300, obs_per_point=90, window=120, seed=7)
    _stage(g2o_amd_mod, oracle, prob, 1e-2, monkeypatch)


def _traj(g2o_amd_mod, oracle, prob, iters):
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    ref = oracle.OracleGraph(prob)
    n, st = opt.optimize(iters)
    nr, sr = ref.optimize(iters, oracle.make_config(threads=8))
    assert n == nr
    for a, b in zip(st, sr):
        assert abs(a.chi2 - b.chi2) <= 1e-6 * abs(b.chi2), (a.chi2, b.chi2)
        assert a.levenbergIterations == b.levenbergIterations
    xg, xr = opt.minimal_state(), ref.minimal_state()
    assert np.linalg.norm(xg - xr) <= 1e-6 * np.linalg.norm(xr)
    return opt, st


def test_split_trajectory_with_rejected_trials(g2o_amd_mod, oracle):
    """Heavy pixel noise: iterations 0 and 1 reject a trial (oracle: [2, 2, 1, ...]); iteration 1's retry
    re-assembles the split at the new lambda from the popped state."""
    prob = synth.ba(num_cameras=40, num_points=1500, obs_per_point=8, window=24, cam_rot_noise=0.02,
                    cam_trans_noise=0.05, point_noise=0.1, pixel_noise=200.0, seed=11)
    _, st = _traj(g2o_amd_mod, oracle, prob, 10)
    assert st[1].levenbergIterations > 1, "no rejected trial after iteration 0"


def test_split_trajectory_long_tracks(g2o_amd_mod, oracle):
    prob = synth.ba(num_cameras=140, num_points=300, obs_per_point=90, window=120, seed=7)
    _traj(g2o_amd_mod, oracle, prob, 5)


def test_split_equals_plain_passes(g2o_amd_mod, monkeypatch):
    """The split and the plain passes (k_schur_prep / k_schur_diag over Hpl) follow the same trajectory."""
    prob = synth.by_name("C4", "small")
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("G2OHIP_SCHUR_SPLIT", flag)
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
        n, st = opt.optimize(6)
        runs.append((n, [s.chi2 for s in st], [s.levenbergIterations for s in st], opt.minimal_state()))
    (n1, c1, t1, x1), (n0, c0, t0, x0) = runs
    assert n1 == n0 and t1 == t0
    assert np.allclose(c1, c0, rtol=1e-10, atol=0)
    assert np.linalg.norm(x1 - x0) <= 1e-10 * np.linalg.norm(x0)


def test_split_hpp_consumers_after_optimize(g2o_amd_mod, oracle):
    """After optimize() the engine holds a split assembly of the final state (no Hpp stored): multiplyHessian
    and computeMarginals still see Hpp of that state (a plain buildSystem runs first)."""
    prob = synth.by_name("C4", "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.optimize(3)
    npose = opt.block_dims()[2] * 6
    v = np.random.default_rng(0).standard_normal(npose)
    y = opt.multiply_hessian(v)
    ref = oracle.OracleGraph(prob)
    ref.optimize(3, oracle.make_config(threads=8))
    r = ref.stage(0.0)  # buildSystem at the optimized state
    Hpp, _, _ = ref.hessian_dense(r["np"], r["nl"])
    assert np.linalg.norm(y - Hpp @ v) <= 1e-8 * np.linalg.norm(Hpp @ v)


def _ba_fixed_points_varied_intrinsics(seed=5):
    """BA where every 7th point is fixed (observations of a fixed landmark only feed the camera's blocks: the Kt
    record of such an observation is zero), intrinsics differ per edge (no shared record: the Kt record folds each
    edge's fx, fy) and a few gross outliers for a robust kernel."""
    base = synth.ba(num_cameras=30, num_points=900, obs_per_point=6, window=16, seed=seed)
    cams, pts = base.vertices
    fixed = pts.fixed.copy()
    fixed[::7] = 1
    pv = synth.VertexSet(pts.vtype, pts.ids, pts.est, fixed, pts.marginalized)
    e = base.edges[0]
    rng = np.random.default_rng(seed)
    par = e.params * (1.0 + 0.02 * rng.standard_normal(e.params.shape))
    meas = e.meas.copy()
    out = rng.random(len(meas)) < 0.05
    meas[out] += rng.standard_normal((int(out.sum()), 2)) * 30.0
    ev = synth.EdgeSet(e.etype, e.v0, e.v1, meas, e.info, par)
    return synth.Problem(base.name + "_fixedpts", [cams, pv], [ev], 6, 3)


@pytest.mark.parametrize("kx,cam", [("1", "1"), ("1", "0"), ("0", "0")])
def test_split_fixed_points_varied_intrinsics_robust(g2o_amd_mod, oracle, monkeypatch, kx, cam):
    """The Schur split with Kt records (default; the camera pass from the records or re-linearising, G2OHIP_CAM_KX) and
    with G blocks (G2OHIP_SCHUR_KX=0): stage-level reduced system and a Huber-robustified LM trajectory against the
    oracle on a graph with fixed points and per-edge intrinsics."""
    monkeypatch.setenv("G2OHIP_SCHUR_KX", kx)
    monkeypatch.setenv("G2OHIP_CAM_KX", cam)
    prob = _ba_fixed_points_varied_intrinsics()
    _stage(g2o_amd_mod, oracle, prob, 1e-3, monkeypatch)
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, "Huber", 2.447)
    ref = oracle.OracleGraph(prob)
    ref.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, 1, 2.447)
    n, st = opt.optimize(6)
    nr, sr = ref.optimize(6, oracle.make_config(threads=8))
    assert n == nr
    for a, b in zip(st, sr):
        assert abs(a.chi2 - b.chi2) <= 1e-6 * abs(b.chi2), (a.chi2, b.chi2)
        assert a.levenbergIterations == b.levenbergIterations
    xg, xr = opt.minimal_state(), ref.minimal_state()
    assert np.linalg.norm(xg - xr) <= 1e-6 * np.linalg.norm(xr)


@pytest.mark.parametrize("which", ["C4", "fixedpts"])
def test_split_kx_records_match_g_blocks(g2o_amd_mod, monkeypatch, which):
    """The Kt-record path rebuilds G_a G_b^T, S(i,i) and bschur from (Kt, x/z, y/z, 1/z) with arithmetic different from
    the G-block path's (which follows EdgeSE3ProjectXYZ::linearizeOplus, types_six_dof_expmap.cpp:395-447, term by
    term). Entry by entry the two reduced systems must agree to within a few ulp of the matrix scale: every entry of
    Hschur and bschur within 1e-13 of max|Hschur| / max|bschur| (an f64 sum of O(100) terms of that scale), so a later
    change to the rebuild that loses digits in a few entries is caught even where the norm-wise oracle check is not."""
    prob = synth.by_name("C4", "small") if which == "C4" else _ba_fixed_points_varied_intrinsics()
    monkeypatch.setenv("G2OHIP_STAGE_SPLIT", "1")
    out = {}
    for kx in ("1", "0"):
        monkeypatch.setenv("G2OHIP_SCHUR_KX", kx)
        monkeypatch.setenv("G2OHIP_CAM_KX", kx)
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
        out[kx] = opt.stage(1e-3)
    a, b = out["1"], out["0"]
    assert a["ok"] == b["ok"] == 1
    for k in ("Hschur", "bschur"):
        x, y = np.asarray(a[k]), np.asarray(b[k])
        scale = np.abs(y).max()
        assert np.abs(x - y).max() <= 1e-13 * scale, (k, np.abs(x - y).max() / scale)


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_split_row_parts(g2o_amd_mod, oracle, name, monkeypatch):
    """Row chunks split into parts (G2OHIP_SCHUR_SPLIT_TASKS: the sharded path's default, forced here on one GPU): each
    part's partial blocks, then k_schur_part_sum's fixed-order sum into S. The reduced system against the oracle, and
    the LM trajectory against the unsplit pass."""
    monkeypatch.setenv("G2OHIP_SCHUR_SPLIT_TASKS", "1000000")
    prob = synth.by_name(name, "small")
    _stage(g2o_amd_mod, oracle, prob, 1e-3, monkeypatch)
    runs = []
    for flag in ("1000000", "0"):
        monkeypatch.setenv("G2OHIP_SCHUR_SPLIT_TASKS", flag)
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
        n, st = opt.optimize(5)
        runs.append((n, [s.chi2 for s in st], [s.levenbergIterations for s in st], opt.minimal_state()))
    (n1, c1, t1, x1), (n0, c0, t0, x0) = runs
    assert n1 == n0 and t1 == t0
    assert np.allclose(c1, c0, rtol=1e-10, atol=0)
    assert np.linalg.norm(x1 - x0) <= 1e-10 * np.linalg.norm(x0)
