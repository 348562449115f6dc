"""The rest of the Solver contract and the boundary's failure modes, on the GPU:

* caches keyed on the block pattern follow a re-initialization that changes it (computeMarginals' separate factor,
  multiplyHessian's and linear_residual's block-row maps) — the incremental workflow of adding edges to a graph and
  calling initializeOptimization again (sparse_optimizer.cpp:201-279);
* Solver::saveHessian (block_solver.hpp:589-593 -> SparseBlockMatrix::writeOctave, sparse_block_matrix.hpp:579-617) and
  Solver::setWriteDebug's not-PD dump (linear_solver_csparse.h:127-133 -> csparse_helper.cpp:62-111), parsed back and
  compared with the matrices the oracle / the device staged;
* the host-edge callback refusing a payload of the wrong length instead of writing past the engine's buffer;
* the .g2o loader on a file without its final newline and on a truncated last line; the parallel writer's save ->
  load round trip (bit-identical state and chi2).
"""
import numpy as np
import pytest

from g2o_amd import synth

pytestmark = pytest.mark.gpu


def _sub(prob, mask, name):
    e = prob.edges[0]
    es = synth.EdgeSet(e.etype, e.v0[mask], e.v1[mask], e.meas[mask], e.info[mask],
                       None if e.params is None else e.params[mask])
    return synth.Problem(name, prob.vertices, [es], prob.pose_dim, prob.landmark_dim)


def _dense_hpp(oracle, prob):
    ref = oracle.OracleGraph(prob)
    r = ref.stage(0.0)
    Hpp, _, _ = ref.hessian_dense(r["np"], r["nl"])
    return Hpp


def _marg_rel(blocks, Hinv, pd):
    num = den = 0.0
    for (r, c), B in blocks.items():
        R = Hinv[r * pd:(r + 1) * pd, c * pd:(c + 1) * pd]
        num += float(np.sum((B - R) ** 2))
        den += float(np.sum(R ** 2))
    return np.sqrt(num / den)


@pytest.mark.parametrize("algo", ["lm_pcg", "lm_hip_var"])
def test_pattern_caches_follow_reinitialize(g2o_amd_mod, oracle, algo):
    """Marginals, multiplyHessian and the linear residual before and after edges are added and the optimizer is
    re-initialized: the second pattern has more active poses (block count 49 -> 99) and more off-diagonal blocks.
    lm_pcg: computeMarginals sets up its own factor of Hpp (the cache the advisor found never invalidated);
    lm_hip_var: it reuses the LM's factor, and the residual's block-row map is rebuilt."""
    prob = synth.by_name("C1", "small")
    e = prob.edges[0]
    first = np.maximum(e.v0, e.v1) < 50
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(_sub(prob, first, "first"))
    opt.set_algorithm(algo)
    for stage, p in ((0, _sub(prob, first, "first")), (1, prob)):
        if stage == 1:
            rest = _sub(prob, ~first, "rest")
            opt.add_edges(rest.edges[0])
        opt.initialize_optimization()
        opt.build_structure()
        opt.build_system()
        pd, _, npose, _ = opt.block_dims()
        Hpp = _dense_hpp(oracle, p)
        assert Hpp.shape[0] == npose * pd
        pat = [(i, i) for i in range(npose)] + [(i - 1, i) for i in range(1, npose)]
        blocks = opt.compute_marginals(pat)
        assert blocks is not None
        assert _marg_rel(blocks, np.linalg.inv(Hpp), pd) <= 1e-9
        x = np.random.default_rng(stage).standard_normal(npose * pd)
        y = opt.multiply_hessian(x)
        np.testing.assert_allclose(y, Hpp @ x, rtol=0, atol=1e-9 * np.abs(Hpp).max() * np.abs(x).max() * 10)
        if algo == "lm_hip_var":
            opt.set_lambda(1e-3)
            assert opt.solve()
            assert opt.linear_residual() <= 1e-9
            opt.restore_diagonal()


def _read_octave(path):
    lines = open(path).read().splitlines()
    head = {}
    k = 0
    while lines[k].startswith("#"):
        key, val = lines[k][2:].split(":", 1)
        head[key.strip()] = val.strip()
        k += 1
    assert lines[k] == ""  # the blank line after the header (setprecision(...) << std::endl)
    ent = np.array([[float(t) for t in ln.split()] for ln in lines[k + 1:] if ln.strip()])
    n = int(head["rows"])
    A = np.zeros((n, int(head["columns"])))
    A[ent[:, 0].astype(int) - 1, ent[:, 1].astype(int) - 1] = ent[:, 2]
    rc = ent[:, 1] * (n + 1) + ent[:, 0]
    assert np.all(np.diff(rc) > 0), "entries must be sorted by (column, row) and unique"
    assert int(head["nnz"]) == len(ent)
    assert head["type"] == "sparse matrix"
    return head, A, lines[k + 1:]


@pytest.mark.parametrize("name", ["C1", "C4"])
def test_save_hessian_octave(g2o_amd_mod, oracle, name, tmp_path):
    """saveHessian writes Hpp (pose part) in writeOctave's format: '%.9f' entries, 1-based, sorted by column, every
    stored block entry plus the mirror of each off-diagonal block."""
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.initialize_optimization()
    opt.build_structure()
    opt.build_system()
    path = str(tmp_path / "hpp.txt")
    assert opt.save_hessian(path)
    head, A, body = _read_octave(path)
    assert head["name"] == str(tmp_path / "hpp")
    Hpp = _dense_hpp(oracle, prob)
    assert A.shape == Hpp.shape
    assert np.abs(A - Hpp).max() <= 1e-9 * np.abs(Hpp).max() + 6e-10
    assert all(len(ln.split()[2].split(".")[1]) == 9 for ln in body[:50])  # std::fixed, precision 9


@pytest.mark.parametrize("name,algo", [("C1", "lm_hip_var"), ("C4", "lm_hip_fix6_3")])
def test_write_debug_dump_on_not_pd(g2o_amd_mod, oracle, tmp_path, monkeypatch, name, algo):
    """setWriteDebug(true): a factorization that meets a non-positive pivot writes debug.txt with the matrix it
    factored, and the solve still returns false. C1: Hpp + lambda I with a negative lambda below -max diag(Hpp); C4:
    the Schur complement at a lambda that keeps every Hll + lambda I positive definite but not S + lambda I."""
    monkeypatch.chdir(tmp_path)
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm(algo)
    opt.initialize_optimization()
    opt.build_structure()
    r = opt.stage(1e-3)
    assert r["ok"] == 1 and not (tmp_path / "debug.txt").exists()
    opt.set_write_debug(True)
    if name == "C1":
        lam = -2.0 * float(np.abs(np.diag(r["Hschur"])).max())
    else:
        ref = oracle.OracleGraph(prob)
        st = ref.stage(0.0)
        _, Hll, _ = ref.hessian_dense(st["np"], st["nl"])
        # Hll as packed 3x3 blocks: lambda just above -min eig keeps every Hll + lambda I PD, while the landmark with
        # the weakest direction inflates (Hll + lambda I)^-1 there and drives S + lambda I indefinite
        lam = -0.99 * float(np.linalg.eigvalsh(Hll.reshape(-1, 3, 3)).min())
    r = opt.stage(lam)
    if r["ok"]:
        pytest.skip("lambda did not make the system indefinite")
    head, A, _ = _read_octave(str(tmp_path / "debug.txt"))
    assert head["name"] == "debug"
    S = r["Hschur"]
    assert np.isfinite(S).all()
    assert np.abs(A - S).max() <= 5e-9 * np.abs(S).max()


def test_host_callback_wrong_payload_length(g2o_amd_mod, oracle):
    """A callback returning a payload of the wrong size is refused (the call fails with an error) instead of
    overflowing the engine's payload buffer."""
    from test_gpu_generic import _mixed_ba, _oracle_mixed
    gp, ora, hostj = _mixed_ba(odometry=False)
    gpu = g2o_amd_mod.SparseOptimizer(0).add_problem(gp)
    mirror = _oracle_mixed(oracle, ora, hostj)
    t, idx, size = hostj[0]
    assert g2o_amd_mod.lib().g2ohip_host_payload_len(gpu.h, t) == size

    def cb(etype, with_jac):
        for vt in (synth.V_SE3_EXPMAP, synth.V_XYZ):
            mirror.set_estimates(vt, gpu.estimates(vt))
        pay = mirror.edge_payload(idx, size, numeric=True)
        return np.concatenate([pay, np.zeros(7)])  # 7 doubles too many

    gpu.set_host_edge_callback(cb)
    with pytest.raises(g2o_amd_mod.G2OHipError):
        gpu.optimize(1)


def test_load_without_final_newline_and_truncated(g2o_amd_mod, oracle, tmp_path):
    prob = synth.by_name("C1", "small")
    path = tmp_path / "a.g2o"
    oracle.OracleGraph(prob).save(str(path))
    text = open(path).read().rstrip("\n")
    (tmp_path / "nonl.g2o").write_text(text)  # last line without its newline
    opt = g2o_amd_mod.SparseOptimizer(0)
    opt.load(str(tmp_path / "nonl.g2o"))
    assert opt.num_edges() == prob.num_edges
    ref = oracle.OracleGraph(prob)
    assert abs(opt.chi2() - ref.chi2()) <= 1e-12 * ref.chi2()
    last = text.splitlines()[-1].split()
    for cut in (3, len(last) - 1):  # a truncated last edge line, no newline after it
        bad = "\n".join(text.splitlines()[:-1] + [" ".join(last[:cut])])
        (tmp_path / "trunc.g2o").write_text(bad)
        o2 = g2o_amd_mod.SparseOptimizer(0)
        with pytest.raises(g2o_amd_mod.G2OHipError):
            o2.load(str(tmp_path / "trunc.g2o"))


@pytest.mark.parametrize("name", ["C2", "C4"])
def test_save_load_round_trip(g2o_amd_mod, tmp_path, name):
    """The parallel writer after LM iterations: reloading its file gives the same state and chi2. The decimals are
    shortest round-trip, so every stored double reads back bit for bit; VERTEX_SE3:EXPMAP is written as the
    camera-to-world pose (types_six_dof_expmap.cpp:93-101, the inverse of the estimate) and inverted again on load,
    which leaves the cameras within a few ulps (SE2 poses: exact)."""
    prob = synth.by_name(name, "small")
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(prob)
    opt.optimize(2)
    path = str(tmp_path / "out.g2o")
    opt.save(path)
    o2 = g2o_amd_mod.SparseOptimizer(0)
    o2.load(path)
    assert o2.num_vertices() == prob.num_vertices and o2.num_edges() == prob.num_edges
    x1, x2 = opt.minimal_state(), o2.minimal_state()
    if name == "C2":
        np.testing.assert_array_equal(x2, x1)
        assert o2.chi2() == opt.chi2()
    else:
        assert np.abs(x2 - x1).max() <= 1e-14 * np.abs(x1).max()
        assert abs(o2.chi2() - opt.chi2()) <= 1e-12 * opt.chi2()
