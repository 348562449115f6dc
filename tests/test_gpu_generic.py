"""Boundary cases a real g2o graph hits, on the GPU against the oracle:

* robust kernels: the weighted quadratic form of BaseBinaryEdge::constructQuadraticForm
  (base_binary_edge.hpp:104-135, RobustKernel*::robustify robust_kernel_impl.cpp:60-200) and the robust chi2
  (sparse_optimizer.cpp:102-116) in the device LM loop;
* host-authoritative Solver mode: g2o's own LM loop on the host drives buildStructure / buildSystem /
  setLambda / solve / x() / b() / restoreDiagonal of the device solver (tests/solver_mode.py);
* edge types the device does not know (host-Jacobian edges, the J_host_fallback): the host supplies error and
  Jacobians (BaseBinaryEdge's numeric linearizeOplus, base_binary_edge.hpp:198-266), mixed in one graph with
  device-linearized edges and sharing Hessian blocks with them; through the Solver mode and through the device
  LM loop with a host callback;
* the .g2o loader skipping unknown tags (optimizable_graph.cpp:455-460).
Tolerance: the north_star 1e-6 relative on chi2 and state; trial counts identical.
"""
import numpy as np
import pytest

import solver_mode
from g2o_amd import synth

pytestmark = pytest.mark.gpu

RTOL = 1e-6
RK = {"Huber": 1, "PseudoHuber": 2, "Cauchy": 3, "GemanMcClure": 4, "Welsch": 5, "Fair": 6, "Tukey": 7,
      "Saturated": 8, "DCS": 9}
ORACLE_E_SE3_EXPMAP = 4


def _check_stats(st, sr):
    assert len(st) == len(sr)
    for a, b in zip(st, sr):
        ca, cb = (a.chi2 if hasattr(a, "chi2") else a[0]), b.chi2
        qa = a.levenbergIterations if hasattr(a, "levenbergIterations") else a[1]
        assert qa == b.levenbergIterations, (qa, b.levenbergIterations)
        assert abs(ca - cb) <= RTOL * abs(cb), (ca, cb)


def _state_close(xg, xr, tol=RTOL):
    assert np.linalg.norm(xg - xr) <= tol * np.linalg.norm(xr), np.linalg.norm(xg - xr) / np.linalg.norm(xr)


def _ba_with_outliers(seed=3, frac=0.05, px=40.0):
    base = synth.by_name("C4", "small")
    e = base.edges[0]
    rng = np.random.default_rng(seed)
    meas = e.meas.copy()
    out = rng.random(len(meas)) < frac
    meas[out] += rng.standard_normal((int(out.sum()), 2)) * px
    edges = synth.EdgeSet(e.etype, e.v0, e.v1, meas, e.info, e.params)
    return synth.Problem(base.name + "_outliers", base.vertices, [edges], 6, 3)


@pytest.mark.parametrize("kind,delta", [("Huber", 2.447), ("Cauchy", 2.0), ("Tukey", 8.0), ("DCS", 5.0),
                                        ("PseudoHuber", 3.0), ("Welsch", 6.0), ("Fair", 3.0),
                                        ("GemanMcClure", 9.0), ("Saturated", 12.0)])
def test_robust_kernel_lm(g2o_amd_mod, oracle, kind, delta):
    """BA with 5% gross outliers, every observation robustified (ba_demo.cpp's ROBUST_KERNEL: Huber,
    delta = sqrt(5.991)); the other kernels of the factory with deltas that split inliers from outliers."""
    prob = _ba_with_outliers()
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, kind, delta)
    ref = oracle.OracleGraph(prob)
    ref.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, RK[kind], delta)
    assert abs(opt.chi2() - ref.chi2()) <= 1e-12 * ref.chi2()
    n, st = opt.optimize(6)
    nr, sr = ref.optimize(6, oracle.make_config(threads=4))
    assert n == nr
    _check_stats(st, sr)
    _state_close(opt.minimal_state(), ref.minimal_state())


def test_robust_pose_graph(g2o_amd_mod, oracle):
    prob = synth.by_name("C2", "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_robust_kernel(synth.E_SE2, "Cauchy", 1.0)
    ref = oracle.OracleGraph(prob)
    ref.set_robust_kernel(synth.E_SE2, RK["Cauchy"], 1.0)
    n, st = opt.optimize(5)
    nr, sr = ref.optimize(5, oracle.make_config(threads=4))
    _check_stats(st, sr)
    _state_close(opt.minimal_state(), ref.minimal_state())


def test_solver_mode_host_authoritative(g2o_amd_mod, oracle):
    """g2o's LM on the host, the device as the Solver: the trajectory matches the oracle's own LM."""
    prob = synth.by_name("C4", "small")
    gpu = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    host = oracle.OracleGraph(prob)
    st = solver_mode.solver_mode_lm(gpu, host, 5, [synth.V_SE3_EXPMAP, synth.V_XYZ])
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.optimize(5, oracle.make_config(threads=4))
    _check_stats(st, sr)
    _state_close(host.minimal_state(), ref.minimal_state())


def _quat_mul(a, b):  # (x, y, z, w)
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def _mixed_ba(frac_hostj=0.3, seed=7, odometry=True):
    """BA (C4-small) where a fraction of the observations arrive as an edge type the device does not know
    (G2OHIP_E_HOSTJ(2): same projection, Jacobians from the host), plus camera-to-camera relative-pose edges
    (EdgeSE3Expmap, types_six_dof_expmap.h:108-127, G2OHIP_E_HOSTJ(6)) between consecutive cameras, which
    put pose-pose blocks into Hpp and so into the Schur complement. Some host-J observations duplicate device
    ones (shared Hpl blocks across edge types)."""
    import g2o_amd
    base = synth.by_name("C4", "small")
    cams, pts = base.vertices
    e = base.edges[0]
    rng = np.random.default_rng(seed)
    n = len(e.v0)
    hj = rng.random(n) < frac_hostj
    dup = np.nonzero(~hj)[0][:25]  # 25 device observations also arrive as host-J (duplicate blocks)
    hj_idx = np.concatenate([np.nonzero(hj)[0], dup])
    dev = synth.EdgeSet(e.etype, e.v0[~hj], e.v1[~hj], e.meas[~hj], e.info[~hj], e.params[~hj])
    meas_hj = e.meas[hj_idx] + rng.standard_normal((len(hj_idx), 2)) * 0.3
    gpu_edges = [dev, synth.EdgeSet(g2o_amd.E_HOSTJ(2), e.v0[hj_idx], e.v1[hj_idx], None, e.info[hj_idx], None)]
    ora_edges = [dev, synth.EdgeSet(e.etype, e.v0[hj_idx], e.v1[hj_idx], meas_hj, e.info[hj_idx], e.params[hj_idx])]
    hostj = [(g2o_amd.E_HOSTJ(2), np.arange(len(dev.v0), len(dev.v0) + len(hj_idx)), len(hj_idx) * 2 * (1 + 3 + 6))]
    if odometry:
        C = cams.ids.size
        t, q = cams.est[:, :3], cams.est[:, 3:]
        a, b = np.arange(C - 1), np.arange(1, C)
        meas = np.zeros((C - 1, 7))
        for k in range(C - 1):  # C = T_b T_a^-1 (so that log(T_b^-1 C T_a) = 0), perturbed
            qa_inv = np.array([-q[a[k], 0], -q[a[k], 1], -q[a[k], 2], q[a[k], 3]])
            qc = _quat_mul(q[b[k]], qa_inv)
            Rc = synth.quat_to_rot(qc[None])[0]
            tc = t[b[k]] - Rc @ t[a[k]]
            dq = np.concatenate([rng.standard_normal(3) * 1e-3, [1.0]])
            qc = _quat_mul(dq / np.linalg.norm(dq), qc)
            meas[k] = np.concatenate([tc + rng.standard_normal(3) * 1e-3, qc / np.linalg.norm(qc)])
        info = np.broadcast_to(np.eye(6) * 50.0, (C - 1, 6, 6)).copy()
        ida, idb = cams.ids[a], cams.ids[b]
        gpu_edges.append(synth.EdgeSet(g2o_amd.E_HOSTJ(6), ida, idb, None, info, None))
        ora_edges.append(synth.EdgeSet(ORACLE_E_SE3_EXPMAP, ida, idb, meas, info, None))
        n0 = len(dev.v0) + len(hj_idx)
        hostj.append((g2o_amd.E_HOSTJ(6), np.arange(n0, n0 + C - 1), (C - 1) * 6 * (1 + 6 + 6)))
    gpu = synth.Problem("mixed_gpu", base.vertices, gpu_edges, 6, 3)
    ora = synth.Problem("mixed_oracle", base.vertices, ora_edges, 6, 3)
    return gpu, ora, hostj


def _oracle_mixed(oracle, ora, hostj):
    g = oracle.OracleGraph(ora)
    g.set_numeric(np.concatenate([idx for _, idx, _ in hostj]))
    return g


@pytest.mark.parametrize("odometry", [False, True])
def test_solver_mode_mixed_host_jacobian_edges(g2o_amd_mod, oracle, odometry):
    gp, ora, hostj = _mixed_ba(odometry=odometry)
    gpu = g2o_amd_mod.SparseOptimizer(0).add_problem(gp)
    # the oracle robustifies every projection edge, host-J ones included: so does the device (robust weighting
    # of the host-supplied error and Jacobians)
    gpu.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, "Huber", 2.447)
    gpu.set_robust_kernel(g2o_amd_mod.E_HOSTJ(2), "Huber", 2.447)
    host = _oracle_mixed(oracle, ora, hostj)
    host.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, RK["Huber"], 2.447)
    st = solver_mode.solver_mode_lm(gpu, host, 5, [synth.V_SE3_EXPMAP, synth.V_XYZ], hostj)
    ref = _oracle_mixed(oracle, ora, hostj)
    ref.set_robust_kernel(synth.E_SE3_PROJECT_XYZ, RK["Huber"], 2.447)
    nr, sr = ref.optimize(5, oracle.make_config(threads=4))
    _check_stats(st, sr)
    _state_close(host.minimal_state(), ref.minimal_state())


def test_device_lm_host_jacobian_callback(g2o_amd_mod, oracle):
    """The device-resident LM loop with host-J edges: a host callback recomputes their errors / Jacobians at
    the device's estimates (the CPU fallback path), everything else stays on the GPU."""
    gp, ora, hostj = _mixed_ba(odometry=True)
    gpu = g2o_amd_mod.SparseOptimizer(0).add_problem(gp)
    mirror = _oracle_mixed(oracle, ora, hostj)  # the host's view of the edges, fed the device's estimates
    calls = {"n": 0}

    def cb(etype, with_jac):
        calls["n"] += 1
        for vt in (synth.V_SE3_EXPMAP, synth.V_XYZ):
            mirror.set_estimates(vt, gpu.estimates(vt))
        for t, idx, size in hostj:
            if t == etype:
                return mirror.edge_payload(idx, size, numeric=True)
        raise KeyError(etype)

    gpu.set_host_edge_callback(cb)
    n, st = gpu.optimize(5)
    ref = _oracle_mixed(oracle, ora, hostj)
    nr, sr = ref.optimize(5, oracle.make_config(threads=4))
    assert n == nr and calls["n"] > 0
    _check_stats(st, sr)
    _state_close(gpu.minimal_state(), ref.minimal_state())


def test_host_jacobian_edges_need_payload(g2o_amd_mod):
    gp, _, _ = _mixed_ba(odometry=False)
    gpu = g2o_amd_mod.SparseOptimizer(0).add_problem(gp)
    with pytest.raises(g2o_amd_mod.G2OHipError):
        gpu.optimize(1)  # neither a payload nor a callback: fails loudly, no silent zero Jacobians


def test_load_skips_unknown_tags(g2o_amd_mod, oracle, tmp_path):
    prob = synth.by_name("C1", "small")
    path = str(tmp_path / "a.g2o")
    oracle.OracleGraph(prob).save(path)
    lines = open(path).read().splitlines()
    lines.insert(3, "PARAMS_SE3OFFSET 0 0 0 0 0 0 0 1")
    lines.insert(10, "EDGE_SE3_PRIOR 0 0 0 0 0 0 0 1 1 0 0 0 0 0 1 0 0 0 0 1 0 0 0 1 0 0 1 0 1")
    open(path, "w").write("\n".join(lines) + "\n")
    opt = g2o_amd_mod.SparseOptimizer(0)
    opt.load(path)
    assert g2o_amd_mod.lib().g2ohip_num_edges(opt.h) == prob.num_edges
    n, st = opt.optimize(3)
    ref = oracle.OracleGraph(prob)
    nr, sr = ref.optimize(3, oracle.make_config(threads=4))
    _check_stats(st, sr)


def _clear_and_redo_graph():
    """unit_test/general/clear_and_redo.cpp:38-107: three VertexSE3 at the origin, a loop of EdgeSE3 with
    translations (1,0,0), (0,1,0), (-0.8,-0.7,0.1), identity information, vertex 0 fixed."""
    ident = np.array([0, 0, 0, 0, 0, 0, 1.0])
    vs = synth.VertexSet(synth.V_SE3_QUAT, np.arange(3, dtype=np.int32), np.tile(ident, (3, 1)),
                         np.array([1, 0, 0], np.int32), np.zeros(3, np.int32))
    meas = np.array([[1, 0, 0, 0, 0, 0, 1.0], [0, 1, 0, 0, 0, 0, 1.0], [-0.8, -0.7, 0.1, 0, 0, 0, 1.0]])
    es = synth.EdgeSet(synth.E_SE3_QUAT, np.array([0, 1, 2], np.int32), np.array([1, 2, 0], np.int32), meas,
                       np.tile(np.eye(6), (3, 1, 1)))
    return synth.Problem("clear_and_redo", [vs], [es], 6, 0)


def test_reference_clear_and_redo_gauss_newton(g2o_amd_mod, oracle):
    """The reference test runs Gauss-Newton (var block ordering off) twice on a fresh graph and asserts
    optimize() > 0; here each run also matches the oracle's Gauss-Newton."""
    for _ in range(2):
        prob = _clear_and_redo_graph()
        opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
        opt.set_algorithm("gn_hip_var")
        n, st = opt.optimize(10)
        assert n > 0
        ref = oracle.OracleGraph(prob)
        nr, sr = ref.optimize(10, oracle.make_config(threads=1, gauss_newton=True, block_ordering=False))
        assert n == nr
        for a, b in zip(st, sr):
            assert abs(a.chi2 - b.chi2) <= RTOL * abs(b.chi2) + 1e-12
        opt.close()
