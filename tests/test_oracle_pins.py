"""Pins of the oracle (CPU restatement) against what the reference itself fixes.

* unit_test/slam3d/jacobians_slam3d.cpp:56-81, unit_test/slam2d/jacobians_slam2d.cpp:47-72 and
  test_helper/evaluate_jacobian.h:40-88: analytic vs numeric (BaseBinaryEdge::linearizeOplus,
  base_binary_edge.hpp:198-266) Jacobians agree within 1e-6.  The same test is applied to
  EdgeSE3ProjectXYZ (no reference test exists for it; same strategy).
* unit_test/slam3d/optimization_slam3d.cpp:38-126: two-vertex EdgeSE3 LM converges to chi2 < 1e-6
  with the free pose at the identity.
* The restated CSparse factorization is bitwise identical to the reference's vendored CSparse
  (oracle/_ref, compiled from /root/reference/EXTERNAL/csparse) with the same cs_amd ordering.
"""
import math

import numpy as np
import pytest

from g2o_amd import synth

RNG = np.random.default_rng(20261015)


def _eigen_random(n):  # Eigen::Vector3d::Random(): uniform [-1, 1]
    return RNG.uniform(-1.0, 1.0, size=n)


def random_isometry():
    """unit_test/slam3d/jacobians_slam3d.cpp:46-54 randomIsometry3d()."""
    aa = _eigen_random(3) + _eigen_random(3)
    ang = np.linalg.norm(aa)
    R = synth._axis_angle(aa[None], np.array([ang]))[0]
    t = _eigen_random(3)
    q = synth.rot_to_quat(R[None])[0]
    return np.concatenate([t, q])


def random_se2():
    """unit_test/slam2d/jacobians_slam2d.cpp randomSE2(): x,y uniform, theta uniform(-pi, pi)."""
    return np.array([RNG.uniform(-1, 1), RNG.uniform(-1, 1), RNG.uniform(-math.pi, math.pi)])


def _two_vertex_problem(vt, et, est, meas, D, d):
    vs = synth.VertexSet(vt, np.array([0, 1], np.int32), np.asarray(est), np.zeros(2, np.int32), np.zeros(2, np.int32))
    es = synth.EdgeSet(et, np.array([0], np.int32), np.array([1], np.int32), np.asarray(meas)[None],
                       np.eye(D)[None])
    return synth.Problem("j", [vs], [es], d, 0)


@pytest.mark.parametrize("trials", [2000])
def test_edge_se3_jacobian_vs_numeric(oracle, trials):
    worst = 0.0
    for _ in range(trials):
        prob = _two_vertex_problem(synth.V_SE3_QUAT, synth.E_SE3_QUAT, [random_isometry(), random_isometry()],
                                   random_isometry(), 6, 6)
        g = oracle.OracleGraph(prob)
        _, Ja, Jb, Na, Nb = g.edge_jacobians(0, 6, 6, 6)
        worst = max(worst, np.abs(Ja - Na).max(), np.abs(Jb - Nb).max())
    assert worst < 1e-6, worst  # evaluate_jacobian.h:60 EXPECT_NEAR(n, a, 1e-6)


@pytest.mark.parametrize("trials", [2000])
def test_edge_se2_jacobian_vs_numeric(oracle, trials):
    worst = 0.0
    for _ in range(trials):
        prob = _two_vertex_problem(synth.V_SE2, synth.E_SE2, [random_se2(), random_se2()], random_se2(), 3, 3)
        g = oracle.OracleGraph(prob)
        _, Ja, Jb, Na, Nb = g.edge_jacobians(0, 3, 3, 3)
        worst = max(worst, np.abs(Ja - Na).max(), np.abs(Jb - Nb).max())
    assert worst < 1e-6, worst


@pytest.mark.parametrize("trials", [2000])
def test_edge_se2_pointxy_jacobian_vs_numeric(oracle, trials):
    """unit_test/slam2d/jacobians_slam2d.cpp:123-150 (EdgeSE2PointXYJacobian): analytic vs numeric, 1e-6."""
    worst = 0.0
    for _ in range(trials):
        vs = [synth.VertexSet(synth.V_SE2, np.array([0], np.int32), random_se2()[None], np.zeros(1, np.int32),
                              np.zeros(1, np.int32)),
              synth.VertexSet(synth.V_XY, np.array([1], np.int32), RNG.uniform(-1, 1, (1, 2)), np.zeros(1, np.int32),
                              np.ones(1, np.int32))]
        es = synth.EdgeSet(synth.E_SE2_XY, np.array([0], np.int32), np.array([1], np.int32),
                           RNG.uniform(-1, 1, (1, 2)), np.eye(2)[None])
        g = oracle.OracleGraph(synth.Problem("j", vs, [es], 3, 2))
        _, Ja, Jb, Na, Nb = g.edge_jacobians(0, 2, 3, 2)
        worst = max(worst, np.abs(Ja - Na).max(), np.abs(Jb - Nb).max())
    assert worst < 1e-6, worst


def test_slam2d_oracle_file_roundtrip(oracle, tmp_path):
    """VERTEX_XY / EDGE_SE2_XY reader and writer of the oracle (vertex_point_xy.cpp:46-56,
    edge_se2_pointxy.cpp:46-61): same chi2 after a save/load cycle, and the LM converges."""
    prob = synth.slam2d(200)
    g = oracle.OracleGraph(prob)
    path = str(tmp_path / "s.g2o")
    g.save(path)
    h = oracle.OracleGraph.load(path)
    chi0 = g.chi2()
    assert abs(h.chi2() - chi0) <= 1e-12 * chi0
    n, st = h.optimize(8)
    assert n == 8 and st[-1].chi2 < 0.05 * chi0
    assert st[-1].hessianPoseDimension == 3 * 199 and st[-1].hessianLandmarkDimension == 2 * prob.vertices[1].ids.size


def test_edge_se3_project_xyz_jacobian_vs_numeric(oracle):
    prob = synth.ba(12, 300, 5, 8)
    g = oracle.OracleGraph(prob)
    worst = 0.0
    for k in range(0, 1500, 3):
        _, Ja, Jb, Na, Nb = g.edge_jacobians(k, 2, 3, 6)
        # pixel-scale Jacobians (fx = 1000): compare relative to the focal length
        worst = max(worst, np.abs(Ja - Na).max() / 1000.0, np.abs(Jb - Nb).max() / 1000.0)
    assert worst < 1e-6, worst


def _iso_vec(R, t):
    return np.concatenate([t, synth.rot_to_quat(R[None])[0]])


@pytest.mark.parametrize("kind", ["translation", "rotation"])
def test_reference_optimization_slam3d(oracle, kind):
    """unit_test/slam3d/optimization_slam3d.cpp:38-126 (BlockSolverX + LM, 100 iterations)."""
    ident = _iso_vec(np.eye(3), np.zeros(3))
    if kind == "translation":
        p2 = _iso_vec(np.eye(3), np.array([10.0, 10.0, 10.0]))
    else:
        R = synth._axis_angle(np.ones((1, 3)) / math.sqrt(3), np.array([math.radians(2)]))[0]
        p2 = _iso_vec(R, np.zeros(3))
    vs = synth.VertexSet(synth.V_SE3_QUAT, np.array([0, 1], np.int32), np.stack([ident, p2]),
                         np.array([1, 0], np.int32), np.zeros(2, np.int32))
    es = synth.EdgeSet(synth.E_SE3_QUAT, np.array([0], np.int32), np.array([1], np.int32), ident[None], np.eye(6)[None])
    g = oracle.OracleGraph(synth.Problem("t", [vs], [es], 6, 0))
    assert g.chi2() > 0.0
    n, st = g.optimize(100, oracle.make_config(block_ordering=False))
    assert n > 0
    assert st[-1].chi2 < 1e-6
    est = g.estimates(synth.V_SE3_QUAT)[1]
    assert np.linalg.norm(est[:3]) < 1e-12  # ASSERT_DOUBLE_EQ(0, |t|) in the reference
    assert np.linalg.norm(est[3:6]) < 1e-12   # rotation == identity


def _random_spd_ccs(n, density, rng):
    A = np.zeros((n, n))
    mask = rng.random((n, n)) < density
    A[mask] = rng.standard_normal(mask.sum())
    A = A @ A.T + n * np.eye(n)
    Ap, Ai, Ax = [0], [], []
    for j in range(n):
        rows = np.nonzero(A[: j + 1, j])[0]
        Ai.extend(rows.tolist())
        Ax.extend(A[rows, j].tolist())
        Ap.append(len(Ai))
    return A, np.array(Ap), np.array(Ai), np.array(Ax)


def test_restated_cholesky_bitwise_equals_reference_csparse(oracle):
    if not oracle.ref_available():
        pytest.skip("oracle/_ref (reference CSparse) not built")
    rng = np.random.default_rng(7)
    for n in (1, 5, 40, 150):
        A, Ap, Ai, Ax = _random_spd_ccs(n, 0.08, rng)
        b = rng.standard_normal(n)
        r1, x1 = oracle.ccs_cholsol(n, Ap, Ai, Ax, b, mode=1)  # restated LL^T, cs_amd order
        r2, x2 = oracle.ccs_cholsol(n, Ap, Ai, Ax, b, mode=2)  # reference cs_cholsol
        assert r1 == r2 == 1
        assert np.array_equal(x1, x2)  # bitwise
        np.testing.assert_allclose(A @ x1, b, rtol=1e-9, atol=1e-9)


def test_restated_cholesky_detects_not_pd(oracle):
    n = 4
    A = np.diag([1.0, 2.0, -3.0, 4.0])
    Ap = np.arange(n + 1)
    Ai = np.arange(n)
    r, _ = oracle.ccs_cholsol(n, Ap, Ai, np.diag(A), np.ones(n), mode=0)
    assert r == 0
    if oracle.ref_available():
        r2, _ = oracle.ccs_cholsol(n, Ap, Ai, np.diag(A), np.ones(n), mode=2)
        assert r2 == 0


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C4"])
def test_oracle_ordering_independence(oracle, name):
    """cs_amd block ordering (reference) vs natural ordering: same LM trajectory up to roundoff."""
    prob = synth.by_name(name, "small")
    a = oracle.OracleGraph(prob)
    b = oracle.OracleGraph(prob)
    na, sa = a.optimize(4, oracle.make_config(use_ref=True))
    nb, sb = b.optimize(4, oracle.make_config(use_ref=False))
    assert na == nb
    for x, y in zip(sa, sb):
        assert abs(x.chi2 - y.chi2) <= 1e-9 * abs(y.chi2)
    xa, xb = a.minimal_state(), b.minimal_state()
    assert np.linalg.norm(xa - xb) <= 1e-9 * np.linalg.norm(xb)


def test_g2o_roundtrip(oracle, tmp_path):
    prob = synth.by_name("C4", "small")
    g = oracle.OracleGraph(prob)
    p = str(tmp_path / "ba.g2o")
    g.save(p)
    h = oracle.OracleGraph.load(p, marginalize_xyz=True)
    np.testing.assert_allclose(h.minimal_state(), g.minimal_state(), rtol=0, atol=1e-12)
    assert abs(h.chi2() - g.chi2()) <= 1e-10 * g.chi2()


def test_oracle_deterministic_single_thread(oracle):
    prob = synth.by_name("C4", "small")
    a = oracle.OracleGraph(prob)
    b = oracle.OracleGraph(prob)
    a.optimize(3)
    b.optimize(3)
    assert np.array_equal(a.minimal_state(), b.minimal_state())


def test_oracle_gauss_newton_clear_and_redo(oracle):
    """unit_test/general/clear_and_redo.cpp:38-107 through the oracle's Gauss-Newton: optimize() > 0 and chi2
    decreasing on the 3-pose loop."""
    import test_gpu_generic as T
    g = oracle.OracleGraph(T._clear_and_redo_graph())
    c0 = g.chi2()
    n, st = g.optimize(10, oracle.make_config(threads=1, gauss_newton=True, block_ordering=False))
    assert n > 0 and st[-1].chi2 < c0


def test_oracle_block_symbolic_natural_order(oracle):
    """sum c_k^2 / nnz(L) of the CSparse symbolic path against a dense boolean elimination (natural order)."""
    rng = np.random.default_rng(4)
    nb, bd = 30, 3
    M = rng.random((nb, nb)) < 0.12
    bi, bj = np.nonzero(np.triu(M | M.T, 1))
    lnz, fl = oracle.block_symbolic(nb, bd, bi, bj, use_ref=False)
    n = nb * bd
    P = np.kron(np.eye(nb, dtype=bool) | M | M.T, np.ones((bd, bd), bool))
    L = np.tril(P).copy()
    for k in range(n):  # symbolic elimination: column k's pattern fills below
        rows = np.nonzero(L[k + 1:, k])[0] + k + 1
        L[np.ix_(rows, rows)] |= np.tril(np.ones((len(rows), len(rows)), bool))
    cnt = L.sum(axis=0)
    assert lnz == cnt.sum() and fl == float((cnt.astype(np.float64) ** 2).sum())


# ---- the reference's own mapping tests, restated against the oracle's mappings (oracle_math.hpp) ----
# EXPECT_DOUBLE_EQ is gtest's 4-ulp comparison; EXPECT_NEAR / EXPECT_EQ / EXPECT_LE / EXPECT_GE as written.

def _double_eq(a, b):
    a, b = float(a), float(b)
    if a == b:
        return True
    ia = np.array([a]).view(np.int64)[0]
    ib = np.array([b]).view(np.int64)[0]
    ia = ia if ia >= 0 else -(ia & 0x7FFFFFFFFFFFFFFF)  # sign-magnitude -> biased, as gtest's FloatingPoint
    ib = ib if ib >= 0 else -(ib & 0x7FFFFFFFFFFFFFFF)
    return abs(int(ia) - int(ib)) <= 4


def _R(v9):
    return np.asarray(v9).reshape(3, 3).T  # col-major -> matrix


def _flat(R):
    return np.asarray(R).T.ravel()


EULER = np.array([.1, .2, .3])
ET = np.array([1., 2., 3., .1, .2, .3])


def test_mappings_slam3d_euler_conversion(oracle):
    """unit_test/slam3d/mappings_slam3d.cpp:35-42 (EulerConversion): toEuler(fromEuler(e)) == e to 4 ulps."""
    m1 = oracle.mapping("fromEuler", EULER)
    back = oracle.mapping("toEuler", m1)
    for i in range(3):
        assert _double_eq(EULER[i], back[i]), (i, EULER[i], back[i])


def test_mappings_slam3d_quaternion_conversion(oracle):
    """mappings_slam3d.cpp:44-53 (QuaternionConversion): fromCompactQuaternion(toCompactQuaternion(R)) == R to 4 ulps
    entry by entry — the compact (x, y, z; w >= 0) quaternion EdgeSE3's error (toVectorMQT) is built on."""
    m1 = oracle.mapping("fromEuler", EULER)
    q = oracle.mapping("toCompactQuaternion", m1)
    m2 = oracle.mapping("fromCompactQuaternion", q)
    for k in range(9):
        assert _double_eq(m1[k], m2[k]), (k, m1[k], m2[k])


def test_mappings_slam3d_et(oracle):
    """mappings_slam3d.cpp:55-72 (ET): fromVectorET keeps the translation exactly and the rotation of fromEuler to 1e-6;
    toVectorET inverts it to 1e-6."""
    m1 = _R(oracle.mapping("fromEuler", EULER))
    i1 = oracle.mapping("fromVectorET", ET)
    for r in range(3):
        assert ET[r] == i1[9 + r]
    assert np.abs(_R(i1[:9]) - m1).max() <= 1e-6
    et2 = oracle.mapping("toVectorET", i1)
    assert np.abs(ET - et2).max() <= 1e-6


def test_mappings_slam3d_mqt(oracle):
    """mappings_slam3d.cpp:74-88 (MQT): fromVectorMQT(toVectorMQT(T)) == T to 1e-6 (rotation and translation)."""
    i1 = oracle.mapping("fromVectorET", ET)
    qt1 = oracle.mapping("toVectorMQT", i1)
    assert qt1.size == 6
    i2 = oracle.mapping("fromVectorMQT", qt1)
    assert np.abs(_R(i1[:9]) - _R(i2[:9])).max() <= 1e-6
    assert np.abs(i1[9:] - i2[9:]).max() <= 1e-6


def test_mappings_slam3d_qt(oracle):
    """mappings_slam3d.cpp:90-104 (QT): fromVectorQT(toVectorQT(T)) == T to 1e-6 — the (x y z qx qy qz qw) layout of the
    VERTEX_SE3:QUAT / EDGE_SE3:QUAT tags."""
    i1 = oracle.mapping("fromVectorET", ET)
    qt2 = oracle.mapping("toVectorQT", i1)
    assert qt2.size == 7
    assert abs(np.linalg.norm(qt2[3:]) - 1.0) <= 1e-15
    i2 = oracle.mapping("fromVectorQT", qt2)
    assert np.abs(_R(i1[:9]) - _R(i2[:9])).max() <= 1e-6
    assert np.abs(i1[9:] - i2[9:]).max() <= 1e-6


def _angle_axis(angle, axis):
    """Eigen AngleAxis::toRotationMatrix (Rodrigues) for a unit axis — the test's input construction."""
    a = np.asarray(axis, float)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) * math.cos(angle) + math.sin(angle) * K + (1 - math.cos(angle)) * np.outer(a, a)


def test_orthogonal_matrix(oracle):
    """unit_test/slam3d/orthogonal_matrix.cpp:33-77 (Slam3D.OrthogonalMatrix): 10000 products of a small rotation
    drift off orthogonality; nearestOrthogonalMatrix brings det and R R^T back to 1e-7, and the approximate form that
    VertexSE3::oplusImpl applies every 1000 updates (vertex_se3.h:110-113) to 1e-6, never closer than the exact one."""
    R = np.eye(3)
    rot = _angle_axis(0.01, [0, 0, 1]) @ _angle_axis(0.01, [1, 0, 0])
    initial = np.abs(R @ R.T - np.eye(3)).max()
    assert _double_eq(0.0, initial)
    for _ in range(10000):
        R = R @ rot
    after = np.abs(R @ R.T - np.eye(3)).max()
    assert after >= initial
    inaccurate_det = np.linalg.det(R)
    approx = _R(oracle.mapping("approximateNearestOrthogonalMatrix", _flat(R)))
    Rn = _R(oracle.mapping("nearestOrthogonalMatrix", _flat(R)))
    assert abs(np.linalg.det(Rn) - 1.0) <= abs(inaccurate_det - 1.0)
    assert abs(1.0 - np.linalg.det(Rn)) <= 1e-7
    assert np.abs(Rn @ Rn.T - np.eye(3)).max() <= 1e-7
    for i in range(3):
        assert abs(1.0 - np.linalg.norm(Rn[:, i])) <= 1e-7
    assert np.abs(approx @ approx.T - np.eye(3)).max() <= 1e-6
    assert abs(np.linalg.det(Rn) - 1.0) <= abs(np.linalg.det(approx) - 1.0)
    assert abs(1.0 - np.linalg.det(approx)) <= 1e-6
    for i in range(3):
        assert abs(1.0 - np.linalg.norm(approx[:, i])) <= 1e-6


def test_nearest_orthogonal_matrix_is_the_polar_factor(oracle):
    """The restated one-sided Jacobi SVD behind nearestOrthogonalMatrix: for det > 0 the result is the orthogonal polar
    factor U V^T (numpy's SVD), for det < 0 U's first column (largest singular value) flips, as the reference divides
    it by det(U V^T) = -1."""
    rng = np.random.default_rng(3)
    for k in range(200):
        A = rng.normal(size=(3, 3))
        U, s, Vt = np.linalg.svd(A)
        d = np.linalg.det(U @ Vt)
        U[:, 0] /= d
        want = U @ Vt
        got = _R(oracle.mapping("nearestOrthogonalMatrix", _flat(A)))
        assert np.abs(got - want).max() <= 1e-12, (k, np.abs(got - want).max())


def test_mappings_se2(oracle, tmp_path):
    """unit_test/slam2d/mappings_se2.cpp:34-55 (MappingsSlam2D.SE2): the three SE2 constructors. From three values and
    from a vector the (x, y, theta) are kept exactly — checked through the oracle's VERTEX_SE2 reader / writer, the path
    those values take into the oracle; from an Isometry2 of Rotation2D(1) the angle comes back as 1 (4 ulps) and the
    translation as 0."""
    for vals in ((0., 1., 2.), (0.1, 0.2, 0.3)):
        path = tmp_path / "se2.g2o"
        path.write_text(f"VERTEX_SE2 0 {vals[0]!r} {vals[1]!r} {vals[2]!r}\nFIX 0\n")
        g = oracle.OracleGraph.load(str(path))
        est = g.estimates(synth.V_SE2)
        for k in range(3):
            assert _double_eq(vals[k], est[0][k]), (vals, est)
    c, s = math.cos(1.0), math.sin(1.0)
    s3 = oracle.mapping("SE2fromIsometry2", [c, s, -s, c, 0.0, 0.0])
    assert _double_eq(0., s3[0]) and _double_eq(0., s3[1])
    assert _double_eq(1., s3[2]), s3
