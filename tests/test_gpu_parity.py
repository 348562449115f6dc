"""GPU parity tests: the HIP backend (through the C ABI) against the oracle.

Tolerance (north_star): state vector and final chi2 within 1e-6 relative of the
CSparse reference path; the stage-level checks (reduced system, solution) use
1e-9 because both sides do the same fp64 arithmetic in a different order.
"""
import numpy as np
import pytest

from g2o_amd import synth

pytestmark = pytest.mark.gpu

STATE_RTOL = 1e-6
CHI2_RTOL = 1e-6


def _run_both(g2o_amd_mod, oracle, prob, iters, threads=8):
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    n, st = opt.optimize(iters)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.optimize(iters, oracle.make_config(threads=threads))
    return opt, n, st, ref, nr, sr


def _check(opt, n, st, ref, nr, sr):
    assert n == nr
    for a, b in zip(st, sr):
        assert abs(a.chi2 - b.chi2) <= CHI2_RTOL * abs(b.chi2), (a.chi2, b.chi2)
        assert a.levenbergIterations == b.levenbergIterations
    xg, xr = opt.minimal_state(), ref.minimal_state()
    rel = np.linalg.norm(xg - xr) / np.linalg.norm(xr)
    assert rel <= STATE_RTOL, rel


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C4", "C5"])
def test_lm_trajectory_small(g2o_amd_mod, oracle, name):
    prob = synth.by_name(name, "small")
    _check(*_run_both(g2o_amd_mod, oracle, prob, 6))


def test_ba_sphere2500_full(g2o_amd_mod, oracle):
    """C1 at its real size (sphere2500 recipe, 2500 poses / 9799 edges)."""
    prob = synth.by_name("C1")
    _check(*_run_both(g2o_amd_mod, oracle, prob, 5))


@pytest.mark.slow
def test_c4_full_size_parity(g2o_amd_mod, oracle):
    """BASELINE config C4 at full size (1k cameras x 100k points x 1M observations)."""
    prob = synth.by_name("C4")
    _check(*_run_both(g2o_amd_mod, oracle, prob, 2, threads=16))


@pytest.mark.parametrize("name", ["C1", "C2", "C4"])
def test_stage_reduced_system(g2o_amd_mod, oracle, name):
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    ref = oracle.OracleGraph(prob)
    lam = 1e-3
    g = opt.stage(lam)
    r = ref.stage(lam)
    assert g["ok"] == r["ok"] == 1
    for k in ("b", "bschur", "x"):
        assert np.linalg.norm(g[k] - r[k]) <= 1e-9 * np.linalg.norm(r[k]), k
    assert np.linalg.norm(g["Hschur"] - r["Hschur"]) <= 1e-11 * np.linalg.norm(r["Hschur"])


def test_solver_plugin_interface(g2o_amd_mod, oracle):
    """Solver-level contract (core/solver.h): buildStructure / buildSystem / setLambda / solve /
    x() / b() / restoreDiagonal, driven step by step like OptimizationAlgorithmLevenberg."""
    prob = synth.by_name("C4", "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.initialize_optimization()
    opt.build_structure()
    opt.build_system()
    opt.set_lambda(1e-2, True)
    assert opt.solve()
    x = opt.x()
    b = opt.b()
    opt.restore_diagonal()
    r = oracle.OracleGraph(prob).stage(1e-2)
    assert np.linalg.norm(x - r["x"]) <= 1e-9 * np.linalg.norm(r["x"])
    assert np.linalg.norm(b - r["b"]) <= 1e-12 * np.linalg.norm(r["b"])
    # update / push / pop on the device-resident state
    s0 = opt.minimal_state()
    lib = g2o_amd_mod.lib()
    assert lib.g2ohip_push(opt.h) == 0
    assert lib.g2ohip_update(opt.h, None) == 0
    assert not np.array_equal(opt.minimal_state(), s0)
    assert lib.g2ohip_pop(opt.h) == 0
    assert np.array_equal(opt.minimal_state(), s0)


def test_linear_solver_ccs(g2o_amd_mod):
    rng = np.random.default_rng(3)
    n = 90
    A = rng.standard_normal((n, n)) * (rng.random((n, n)) < 0.1)
    A = A @ A.T + n * np.eye(n)
    Ap, Ai, Ax = [0], [], []
    for j in range(n):
        rows = np.nonzero(A[: j + 1, j])[0]
        Ai += rows.tolist()
        Ax += A[rows, j].tolist()
        Ap.append(len(Ai))
    b = rng.standard_normal(n)
    ok, x = g2o_amd_mod.linear_solve_ccs(n, Ap, Ai, Ax, b, block_dim=3)
    assert ok
    np.testing.assert_allclose(A @ x, b, rtol=1e-10, atol=1e-10)
    # not positive definite -> false (linear_solver_csparse.h:127-133)
    Ax2 = list(Ax)
    Ax2[Ap[5]:Ap[6]][-1:] = [-1.0]
    for k in range(Ap[5], Ap[6]):
        if Ai[k] == 5:
            Ax2[k] = -50.0
    ok2, _ = g2o_amd_mod.linear_solve_ccs(n, Ap, Ai, Ax2, b, block_dim=3)
    assert not ok2


def _dense_spd_ccs(rng, n, density):
    nb = n // 6
    mask = np.kron(rng.random((nb, nb)) < density, np.ones((6, 6))) > 0
    mask = mask | mask.T
    A = rng.standard_normal((n, n)) * mask
    A = A @ A.T + n * np.eye(n)
    Ap, Ai, Ax = [0], [], []
    for j in range(n):
        rows = np.nonzero(A[: j + 1, j])[0]
        Ai += rows.tolist()
        Ax += A[rows, j].tolist()
        Ap.append(len(Ai))
    return A, Ap, Ai, Ax


@pytest.mark.parametrize("pb,pre_max", [(64, "0"), (128, "1000000000000"), (256, "0")])
def test_linear_solver_blocked_fronts(g2o_amd_mod, monkeypatch, pb, pre_max):
    """Wide supernodes factored in big panels (rank-32 steps inside a panel, one rank-PB trailing update
    per panel, first block of the next panel on its own): same solution as the unblocked schedule."""
    rng = np.random.default_rng(11)
    n = 1800
    A, Ap, Ai, Ax = _dense_spd_ccs(rng, n, 0.05)
    b = rng.standard_normal(n)
    monkeypatch.setenv("G2OHIP_CHOL_PRE_MAX", pre_max)
    monkeypatch.setenv("G2OHIP_CHOL_FUSED_MAX", "0")
    monkeypatch.setenv("G2OHIP_CHOL_BLOCK_MIN", "1000000")
    ok0, x0 = g2o_amd_mod.linear_solve_ccs(n, Ap, Ai, Ax, b, block_dim=6)
    monkeypatch.setenv("G2OHIP_CHOL_BLOCK_MIN", "32")
    monkeypatch.setenv("G2OHIP_CHOL_PB", str(pb))
    ok1, x1 = g2o_amd_mod.linear_solve_ccs(n, Ap, Ai, Ax, b, block_dim=6)
    assert ok0 and ok1
    np.testing.assert_allclose(A @ x1, b, rtol=1e-10, atol=1e-10)
    assert np.linalg.norm(x1 - x0) <= 1e-12 * np.linalg.norm(x0)


@pytest.mark.parametrize("pre_max", ["0", "1000000000000"])
def test_lm_blocked_fronts_sphere2500(g2o_amd_mod, oracle, monkeypatch, pre_max):
    """C1 full size with every supernode wider than 32 columns blocked (PB = 64); fronts assembled in
    place by the level launches (pre_max 0) or zeroed + scattered before the first level (all levels)."""
    monkeypatch.setenv("G2OHIP_CHOL_PRE_MAX", pre_max)
    monkeypatch.setenv("G2OHIP_CHOL_FUSED_MAX", "0")
    monkeypatch.setenv("G2OHIP_CHOL_BLOCK_MIN", "32")
    monkeypatch.setenv("G2OHIP_CHOL_PB", "64")
    prob = synth.by_name("C1")
    _check(*_run_both(g2o_amd_mod, oracle, prob, 3))


def test_lm_ba_random_covisibility(g2o_amd_mod, oracle):
    """SURVEY.md §8d's C4 variant covis=random at reduced size: every point seen by 10 of all 450 cameras, so the
    reduced camera system is dense (2688 columns, one wide supernode) and takes the blocked dense-front schedule
    (big panels, rank-256 trailing updates) with the default settings."""
    prob = synth.ba(450, 8000, window=450)
    opt, n, st, ref, nr, sr = _run_both(g2o_amd_mod, oracle, prob, 2, threads=16)
    _check(opt, n, st, ref, nr, sr)
    fi = opt.factor_info()
    assert fi["blocked_fronts"] >= 1 and fi["max_front"] >= 2000, fi


def test_g2o_file_roundtrip_parity(g2o_amd_mod, oracle, tmp_path):
    prob = synth.by_name("C4", "small")
    path = str(tmp_path / "ba.g2o")
    oracle.OracleGraph(prob).save(path)
    opt = g2o_amd_mod.SparseOptimizer(0)
    opt.load(path, True)
    ref = oracle.OracleGraph.load(path, True)
    n, st = opt.optimize(4)
    nr, sr = ref.optimize(4)
    _check(opt, n, st, ref, nr, sr)
    out = str(tmp_path / "out.g2o")
    opt.save(out)
    back = oracle.OracleGraph.load(out, True)
    np.testing.assert_allclose(back.minimal_state(), opt.minimal_state(), rtol=0, atol=1e-12)


@pytest.mark.parametrize("kind", ["translation", "rotation"])
def test_reference_optimization_slam3d_on_gpu(g2o_amd_mod, kind):
    """unit_test/slam3d/optimization_slam3d.cpp:38-126 through the HIP backend."""
    import math
    ident = np.array([0, 0, 0, 0, 0, 0, 1.0])
    if kind == "translation":
        p2 = np.array([10, 10, 10, 0, 0, 0, 1.0])
    else:
        R = synth._axis_angle(np.ones((1, 3)) / math.sqrt(3), np.array([math.radians(2)]))
        p2 = np.concatenate([np.zeros(3), synth.rot_to_quat(R)[0]])
    vs = synth.VertexSet(synth.V_SE3_QUAT, np.array([0, 1], np.int32), np.stack([ident, p2]),
                         np.array([1, 0], np.int32), np.zeros(2, np.int32))
    es = synth.EdgeSet(synth.E_SE3_QUAT, np.array([0], np.int32), np.array([1], np.int32), ident[None], np.eye(6)[None])
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(synth.Problem("t", [vs], [es], 6, 0))
    assert opt.chi2() > 0
    n, st = opt.optimize(100)
    assert n > 0 and st[-1].chi2 < 1e-6
    est = opt.estimates(synth.V_SE3_QUAT)[1]
    assert np.linalg.norm(est[:3]) < 1e-12 and np.linalg.norm(est[3:6]) < 1e-12


def test_deterministic_bitwise(g2o_amd_mod):
    prob = synth.by_name("C4", "small")
    a = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    b = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    a.optimize(4)
    b.optimize(4)
    assert np.array_equal(a.minimal_state(), b.minimal_state())


def test_full_size_properties_c4(g2o_amd_mod):
    """Size-independent properties at the bench size: chi2 decreases monotonically and reaches
    the noise floor (~ #residuals - #dof for unit pixel noise)."""
    prob = synth.by_name("C4")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    c0 = opt.chi2()
    n, st = opt.optimize(8)
    chis = [c0] + [s.chi2 for s in st]
    assert all(b <= a for a, b in zip(chis, chis[1:]))
    dof = 2 * prob.num_edges - (6 * 998 + 3 * 100_000)
    assert abs(chis[-1] / dof - 1.0) < 0.05


def _ragged_ba(seed=11, dup=40):
    """BA with ragged observation counts (1..12 per point, not the recipe's fixed k), duplicate
    observations of a point by the same camera (two Hpl contributions into one block: the duplicate
    off-diagonal path: block_solver.hpp:181-205 maps both edges onto the one block `block(i, j, true)` returns), and the edges in a
    random order (the reference takes edges in any order)."""
    base = synth.ba(num_cameras=40, num_points=1500, obs_per_point=12, window=16, seed=seed)
    e = base.edges[0]
    rng = np.random.default_rng(seed)
    npts = len(base.vertices[1].ids)
    keep = np.zeros(len(e.v0), bool)
    kper = rng.integers(1, 13, size=npts)
    for p in range(npts):  # edges of point p are rows 12p .. 12p+11
        keep[12 * p + rng.permutation(12)[: kper[p]]] = True
    idx = np.nonzero(keep)[0]
    idx = np.concatenate([idx, rng.choice(idx, size=dup, replace=False)])  # duplicate observations
    idx = idx[rng.permutation(len(idx))]
    meas = e.meas[idx] + rng.standard_normal((len(idx), 2)) * 0.5
    edges = synth.EdgeSet(e.etype, e.v0[idx], e.v1[idx], meas, e.info[idx], e.params[idx])
    return synth.Problem(base.name + "_ragged", base.vertices, [edges], 6, 3)


def test_lm_ragged_ba_duplicates_shuffled(g2o_amd_mod, oracle):
    prob = _ragged_ba()
    _check(*_run_both(g2o_amd_mod, oracle, prob, 6))


def test_lm_pose_graph_shuffled_edges(g2o_amd_mod, oracle):
    """SE3 and SE2 pose graphs with their edges in random order and some edges reversed in the
    file sense (i > j: the Hessian block lands transposed, block_solver.hpp:181-184)."""
    for name in ("C1", "C2"):
        base = synth.by_name(name, "small")
        e = base.edges[0]
        rng = np.random.default_rng(5)
        perm = rng.permutation(len(e.v0))
        edges = synth.EdgeSet(e.etype, e.v0[perm], e.v1[perm], e.meas[perm], e.info[perm], None)
        prob = synth.Problem(base.name + "_shuffled", base.vertices, [edges], base.pose_dim, base.landmark_dim)
        _check(*_run_both(g2o_amd_mod, oracle, prob, 5))


@pytest.mark.parametrize("name", ["C1", "C4"])
def test_gauss_newton_trajectory(g2o_amd_mod, oracle, name):
    """gn_hip_*: OptimizationAlgorithmGaussNewton (optimization_algorithm_gauss_newton.cpp:50-92) — no damping,
    no trial loop — against the oracle's GN, and a different trajectory from LM on the same problem."""
    prob = synth.by_name(name, "small")
    algo = "gn_hip_fix6_3" if prob.landmark_dim else "gn_hip_fix6_6"
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm(algo)
    n, st = opt.optimize(4)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.optimize(4, oracle.make_config(threads=4, gauss_newton=True))
    assert n == nr == 4
    for a, b in zip(st, sr):
        assert a.levenbergIterations == 0
        assert abs(a.chi2 - b.chi2) <= CHI2_RTOL * abs(b.chi2), (a.chi2, b.chi2)
    xg, xr = opt.minimal_state(), ref.minimal_state()
    assert np.linalg.norm(xg - xr) <= STATE_RTOL * np.linalg.norm(xr)
    lm = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    lm.optimize(4)
    assert np.linalg.norm(lm.minimal_state() - xg) > 1e-9 * np.linalg.norm(xg)


@pytest.mark.parametrize("name", ["C1", "C4"])
def test_multiply_hessian(g2o_amd_mod, oracle, name):
    """BlockSolverBase::multiplyHessian (block_solver.h:146): Hpp (upper blocks mirrored) times a vector,
    against the oracle's dense Hpp; with setLambda active the damped diagonal is used."""
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.initialize_optimization()
    opt.build_structure()
    opt.build_system()
    ref = oracle.OracleGraph(prob)
    r = ref.stage(0.0)
    Hpp, _, _ = ref.hessian_dense(r["np"], r["nl"])
    v = np.random.default_rng(1).standard_normal(r["np"])
    y = opt.multiply_hessian(v)
    assert np.linalg.norm(y - Hpp @ v) <= 1e-12 * np.linalg.norm(Hpp @ v)
    opt.set_lambda(0.5, True)
    y2 = opt.multiply_hessian(v)
    assert np.linalg.norm(y2 - (Hpp @ v + 0.5 * v)) <= 1e-12 * np.linalg.norm(Hpp @ v)
    opt.restore_diagonal()


def test_linear_residual_small(g2o_amd_mod):
    for name, lam in (("C1", 1e-3), ("C4", 1e-2)):
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(synth.by_name(name, "small"))
        opt.initialize_optimization()
        opt.build_structure()
        opt.build_system()
        opt.set_lambda(lam, True)
        assert opt.solve()
        assert opt.linear_residual() <= 1e-12
        opt.restore_diagonal()


@pytest.mark.parametrize("fused", ["1", "0"])
def test_ba_assembly_paths(g2o_amd_mod, oracle, monkeypatch, fused):
    """BA assembly: the fused path (assembly.hip: landmark sums inside the linearize waves, camera blocks from a
    camera-major pass; landmarks with > 64 observations split over chunks + fix-up) and the generic per-edge
    slot path (G2OHIP_ASM_FUSED=0) both follow the oracle; points seen by 80 cameras exercise the split chunks."""
    monkeypatch.setenv("G2OHIP_ASM_FUSED", fused)
    for prob in (synth.ba(num_cameras=100, num_points=60, obs_per_point=80, window=100), _ragged_ba(seed=5)):
        _check(*_run_both(g2o_amd_mod, oracle, prob, 4))


SCHEDULES = {
    "default": {},
    "lagged_all_levels": {"G2OHIP_CHOL_LAG": "2"},
    "blocked_separate_contrib": {"G2OHIP_CHOL_FUSED_MAX": "0", "G2OHIP_CHOL_BLOCK_MIN": "64", "G2OHIP_CHOL_PB": "64",
                                 "G2OHIP_CHOL_WIDE_PB": "64"},
    # band leaves forced small: sequentially ordered leaf parts amalgamated into band supernodes whose structural-zero
    # tiles the steps, the trailing updates and the contribution passes skip
    "band_leaves": {"G2OHIP_BAND_LEAF": "24"},
    "band_leaves_blocked": {"G2OHIP_BAND_LEAF": "24", "G2OHIP_CHOL_FUSED_MAX": "0", "G2OHIP_CHOL_BLOCK_MIN": "64",
                            "G2OHIP_CHOL_PB": "64", "G2OHIP_CHOL_WIDE_PB": "64"},
    # the in-place assembly zeroing childless fronts' contribution blocks too (default: their k_syrk pass writes them)
    "assembly_cb_zeroed": {"G2OHIP_EA_CB_ZERO": "1"},
    # every input entry scattered before the first level (default: later levels' entries ride in earlier launches)
    "scatter_up_front": {"G2OHIP_SCATTER_DEFER": "0"},
    # no small leaf absorption in the symbolic analysis (the r03 tree shapes)
    "no_leaf_absorption": {"G2OHIP_ND_ABSORB": "0"},
    # the Schur split's back-substitution from the stored G blocks (default: Jacobians recomputed per observation)
    "backsub_from_g": {"G2OHIP_BACKSUB_RECOMPUTE": "0"},
    # the Schur row pass with two index buffers drained by each batch's barrier (default: three, counted vmcnt)
    "schur_rows_pipe0": {"G2OHIP_SCHUR_PIPE": "0"},
    # contribution / trailing GEMM tiles: the register-staged GemmNT (default: the LDS-DMA ring GemmNTd (16, 2))
    "syrk_register_staged": {"G2OHIP_SYRK_DMA": "0"},
    "syrk_dma_32x2": {"G2OHIP_SYRK_DMA": "1"},
    # 128 x 64 contribution / trailing tiles (row tiles of 128 in the task lists), blocked fronts forced
    "syrk_128x64_blocked": {"G2OHIP_SYRK_DMA": "6", "G2OHIP_CHOL_FUSED_MAX": "0", "G2OHIP_CHOL_BLOCK_MIN": "64",
                            "G2OHIP_CHOL_PB": "64", "G2OHIP_CHOL_WIDE_PB": "64"},
    "syrk_128x64_deferred_l21": {"G2OHIP_SYRK_DMA": "5", "G2OHIP_CHOL_DEFER_L21": "2", "G2OHIP_CHOL_FUSED_MAX": "0"},
    # in-place extend-add column buffers of 512 / 2048 rows (default 1024)
    "extend_add_512": {"G2OHIP_EA_BIG": "512"},
    "extend_add_2048": {"G2OHIP_EA_BIG": "2048"},
    # deferred L21 forced on every eligible level (default: levels of >= 16 fronts) and switched off
    "deferred_l21_all": {"G2OHIP_CHOL_DEFER_L21": "2", "G2OHIP_CHOL_FUSED_MAX": "0"},
    "deferred_l21_off": {"G2OHIP_CHOL_DEFER_L21": "0"},
    # the Schur split storing G blocks instead of the Kt records
    "schur_g_blocks": {"G2OHIP_SCHUR_KX": "0"},
    "schur_kx_batch128": {"G2OHIP_SCHUR_SB_KX": "128"},
    # recomputing back-substitution with 4 / 8 / 16 lanes per landmark (default 2)
    "backsub_j_lanes4": {"G2OHIP_BACKSUB_J_LANES": "4"},
    "backsub_j_lanes8": {"G2OHIP_BACKSUB_J_LANES": "8"},
    "backsub_j_lanes16": {"G2OHIP_BACKSUB_J_LANES": "16"},
}


@pytest.mark.parametrize("mode", list(SCHEDULES))
@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C4", "C5"])
def test_factor_schedules(g2o_amd_mod, oracle, monkeypatch, name, mode):
    """The factorization schedules of a tree level against the oracle: the default launch-per-panel 32-column steps,
    lagged rank-64 pair steps forced on every level, and blocked fronts (big-panel trailing updates, separate
    contribution passes, backward rounds) forced on the small configs. Reduced system, solution, an LM trajectory and
    marginals from the same factor layout."""
    for k, v in SCHEDULES[mode].items():
        monkeypatch.setenv(k, v)
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    ref = oracle.OracleGraph(prob)
    g = opt.stage(1e-3)
    r = ref.stage(1e-3)
    assert g["ok"] == r["ok"] == 1
    for k in ("bschur", "x"):
        assert np.linalg.norm(g[k] - r[k]) <= 1e-9 * np.linalg.norm(r[k]), k
    info = opt.factor_info()
    if mode == "blocked_separate_contrib" and name in ("C1", "C3"):
        assert info["blocked_fronts"] > 0, info
    if mode == "deferred_l21_all" and info["levels"] > 1:  # every front below the root has rows below its supernode
        assert info["deferred_l21_fronts"] > 0, info
    opt.build_system()
    opt.set_lambda(1e-3)
    assert opt.solve()
    assert opt.linear_residual() <= 1e-10
    opt.restore_diagonal()
    _check(*_run_both(g2o_amd_mod, oracle, prob, 4))


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_schur_rows_pipe_bitwise(g2o_amd_mod, monkeypatch, name):
    """k_schur_rows' pipelined index loads (PIPE 1: three index buffers, counted vmcnt waits that trust the number of
    index loads idx_load3 issues) against the plain double-buffered pass (PIPE 0): both are deterministic with the same
    summation order, so the reduced camera system must be BITWISE equal; a miscounted wait would read G blocks before
    they land."""
    prob = synth.by_name(name, "small")
    out = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("G2OHIP_SCHUR_PIPE", pipe)
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
        out[pipe] = opt.stage(1e-3)
        opt.close()
    assert np.array_equal(out["0"]["Hschur"], out["1"]["Hschur"])
    assert np.array_equal(out["0"]["bschur"], out["1"]["bschur"])
    assert np.array_equal(out["0"]["x"], out["1"]["x"])


def test_syrk_variant_pinned_per_factorization(g2o_amd_mod, monkeypatch):
    """The k_syrk tile variant is read once, when a factorization builds its row-tile task lists, and kept with them:
    optimizer A is built with the 128 x 64 tile (G2OHIP_SYRK_DMA=5, row tiles of 128), the knob then changes and optimizer
    B is built with the 64 x 64 tile (row tiles of 64); A's next solve must still launch the tile its lists were built for
    (a 64-row tile over 128-row lists would skip half the rows, the reverse would apply rows twice)."""
    prob = synth.by_name("C3", "small")
    sched = {"G2OHIP_CHOL_FUSED_MAX": "0", "G2OHIP_CHOL_BLOCK_MIN": "64", "G2OHIP_CHOL_PB": "64", "G2OHIP_CHOL_WIDE_PB": "64"}
    for k, v in sched.items():
        monkeypatch.setenv(k, v)
    ref = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    r0 = ref.stage(1e-3)
    monkeypatch.setenv("G2OHIP_SYRK_DMA", "5")
    a = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    ga = a.stage(1e-3)
    monkeypatch.setenv("G2OHIP_SYRK_DMA", "4")
    b = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    gb = b.stage(1e-3)
    ga2 = a.stage(1e-3)  # A again, after B's build bumped the knob epoch
    for g in (ga, gb, ga2):
        assert g["ok"] == 1
        assert np.linalg.norm(g["x"] - r0["x"]) <= 1e-9 * np.linalg.norm(r0["x"])
