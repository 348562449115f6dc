"""Host-side checks that need no GPU: the C-ABI library loads and exports every
symbol include/g2o_hip.h declares, refuses to run without a GPU (no CPU fallback),
the host symbolic analysis (ordering / supernodes / frontal maps), and the
synthetic generators."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, gpu_available
from g2o_amd import synth


def test_header_symbols_exported(g2o_amd_mod):
    hdr = open(os.path.join(ROOT, "include", "g2o_hip.h")).read()
    declared = set(re.findall(r"\b(g2ohip_[a-z0-9_]+)\s*\(", hdr))
    L = g2o_amd_mod.lib()
    missing = [s for s in sorted(declared) if not hasattr(L, s)]
    assert not missing, missing
    assert set(g2o_amd_mod.EXPORTS) <= declared


def test_no_cpu_fallback(g2o_amd_mod):
    if gpu_available():
        pytest.skip("a GPU is present")
    with pytest.raises(g2o_amd_mod.G2OHipError, match="requires a gfx950 GPU"):
        g2o_amd_mod.SparseOptimizer(0)


def test_version(g2o_amd_mod):
    assert b"gfx950" in g2o_amd_mod.lib().g2ohip_version()


def test_lm_scale_factor_matches_pow(g2o_amd_mod):
    """The LM trial's lambda factor max(1/3, min(2/3, 1 - (2 rho - 1)^3)) (optimization_algorithm_levenberg.cpp:127-136)
    as the library computes it on host and device (one shared __host__ __device__ function): bitwise the formula with
    the cube rounded once (exact rational arithmetic), and within one ulp of the C library's pow (glibc's pow is
    accurate to 0.52 ulp, not correctly rounded), over a sweep of gain ratios."""
    import math
    from fractions import Fraction
    f = g2o_amd_mod.lib().g2ohip_lm_scale_factor
    rng = np.random.default_rng(11)
    rhos = np.concatenate([rng.uniform(0.0, 1.2, 6000), 10.0 ** rng.uniform(-12, 2, 6000),
                           0.5 + rng.uniform(-1e-3, 1e-3, 6000), [1e-300, 0.5, 1.0, 1.5]])
    for rho in rhos.tolist():
        t = 2 * rho - 1
        exact = max(1.0 / 3.0, min(1.0 - float(Fraction(t) ** 3), 2.0 / 3.0))
        libm = max(1.0 / 3.0, min(1.0 - math.pow(t, 3), 2.0 / 3.0))
        got = f(rho)
        assert got == exact, (rho, got, exact)
        assert abs(got - libm) <= np.spacing(libm), (rho, got, libm)


def _pose_pattern(prob):
    e = prob.edges[0]
    fixed = set(prob.vertices[0].ids[prob.vertices[0].fixed.astype(bool)].tolist())
    ids = [v for v in prob.vertices[0].ids.tolist() if v not in fixed]
    idx = {v: i for i, v in enumerate(ids)}
    bi, bj = [], []
    for a, b in zip(e.v0.tolist(), e.v1.tolist()):
        if a in idx and b in idx:
            bi.append(min(idx[a], idx[b]))
            bj.append(max(idx[a], idx[b]))
    n = len(ids)
    return n, bi + list(range(n)), bj + list(range(n))


def _schur_pattern(prob):
    e = prob.edges[0]
    cams = prob.vertices[0]
    fixed = set(cams.ids[cams.fixed.astype(bool)].tolist())
    ids = [c for c in cams.ids.tolist() if c not in fixed]
    idx = {c: i for i, c in enumerate(ids)}
    by_pt = {}
    for p, c in zip(e.v0.tolist(), e.v1.tolist()):
        if c in idx:
            by_pt.setdefault(p, []).append(idx[c])
    pairs = set()
    for cs in by_pt.values():
        cs = sorted(cs)
        for a in range(len(cs)):
            for b in range(a, len(cs)):
                pairs.add((cs[a], cs[b]))
    n = len(ids)
    bi = [a for a, _ in pairs] + list(range(n))
    bj = [b for _, b in pairs] + list(range(n))
    return n, bi, bj


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C4"])
def test_symbolic_covers_factor_pattern(g2o_amd_mod, name):
    prob = synth.by_name(name, "small")
    bd = prob.pose_dim
    nb, bi, bj = _schur_pattern(prob) if name == "C4" else _pose_pattern(prob)
    perm, st = g2o_amd_mod.symbolic_analyze(nb, bd, bi, bj)
    n = nb * bd
    assert sorted(perm.tolist()) == list(range(n))
    # block structure kept together: scalar perm is a block perm
    blocks = perm.reshape(nb, bd)
    assert np.all(blocks % bd == np.arange(bd)) and np.all(blocks // bd == (blocks[:, :1] // bd))
    rng = np.random.default_rng(1)
    A = np.zeros((n, n))
    for a, b in zip(bi, bj):
        B = rng.standard_normal((bd, bd)) * 0.1
        A[a * bd:(a + 1) * bd, b * bd:(b + 1) * bd] += B
        if a != b:
            A[b * bd:(b + 1) * bd, a * bd:(a + 1) * bd] += B.T
    A = A + A.T + n * np.eye(n)
    L = np.linalg.cholesky(A[np.ix_(perm, perm)])
    assert np.count_nonzero(np.abs(L) > 0) <= st["nnzL"]
    assert st["flops"] > 0 and st["supernodes"] >= 1 and st["levels"] >= 1


@pytest.mark.parametrize("leaf", [8, 16, 32])
def test_symbolic_band_leaves(g2o_amd_mod, monkeypatch, leaf):
    """Band leaves (G2OHIP_BAND_LEAF forces the hybrid ordering: dissection down to parts of `leaf` blocks, each ordered
    sequentially and amalgamated into one band supernode): a valid block permutation, and the envelope counts the
    factor relies on (its structural-zero tiles are skipped) bound the true nonzeros of L. Fewer flops than the
    dense fronts of the same tree would do."""
    prob = synth.ba(num_cameras=160, num_points=6000, obs_per_point=6, window=12)
    bd = prob.pose_dim
    nb, bi, bj = _schur_pattern(prob)
    monkeypatch.setenv("G2OHIP_BAND_LEAF", str(leaf))
    perm, st = g2o_amd_mod.symbolic_analyze(nb, bd, bi, bj)
    n = nb * bd
    assert sorted(perm.tolist()) == list(range(n))
    blocks = perm.reshape(nb, bd)
    assert np.all(blocks % bd == np.arange(bd)) and np.all(blocks // bd == (blocks[:, :1] // bd))
    rng = np.random.default_rng(2)
    A = np.zeros((n, n))
    for a, b in zip(bi, bj):
        B = rng.standard_normal((bd, bd)) * 0.1
        A[a * bd:(a + 1) * bd, b * bd:(b + 1) * bd] += B
        if a != b:
            A[b * bd:(b + 1) * bd, a * bd:(a + 1) * bd] += B.T
    A = A + A.T + n * np.eye(n)
    L = np.linalg.cholesky(A[np.ix_(perm, perm)])
    assert np.count_nonzero(np.abs(L) > 1e-300) <= st["nnzL"]
    monkeypatch.setenv("G2OHIP_BAND_LEAF", "0")
    _, st0 = g2o_amd_mod.symbolic_analyze(nb, bd, bi, bj)
    assert st["supernodes"] < st0["supernodes"] or st["flops"] <= st0["flops"], (st, st0)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_dist_plan_model(g2o_amd_mod, nranks):
    """The distributed factorization's cut (plan_distribution, the model DeviceCholesky::setup and the landmark
    alignment run) on a 400-camera BA pattern: every supernode owned by a rank or shared; aligned shards
    reduce only the shared tail (no reduce-scattered segment) and never cost more input than uniform shards; the
    replicated alternative is priced with the same sharded work."""
    prob = synth.ba(num_cameras=400, num_points=20000, obs_per_point=8, window=40)
    nb, bi, bj = _schur_pattern(prob)
    pw = np.full(nb, 20000 * 8 / nb * 0.3e-9)
    a, own_a = g2o_amd_mod.dist_plan(nb, prob.pose_dim, bi, bj, nranks, pose_work=pw)
    u, own_u = g2o_amd_mod.dist_plan(nb, prob.pose_dim, bi, bj, nranks, aligned=False, pose_work=pw)
    _, st = g2o_amd_mod.symbolic_analyze(nb, prob.pose_dim, bi, bj)
    assert a["supernodes"] == u["supernodes"] == st["supernodes"] == own_a.size
    for d, own in ((a, own_a), (u, own_u)):
        assert np.all((own >= -1) & (own < nranks))
        if (own >= 0).any():
            assert (own < 0).any(), "a cut keeps at least the root shared"
        assert d["shard_replicated_s"] == pytest.approx(pw.sum() / nranks)
    assert a["rs_segment_doubles"] == 0 and a["rs_tail_doubles"] > 0
    assert a["input_s"] <= u["input_s"] + 1e-12
    # the aligned layout's chosen total is no worse than the uniform one's
    tot = lambda d: d["max_rank_subtrees_s"] + d["shared_s"] + d["exchange_s"] + d["input_s"] + d["shard_s"]
    assert tot(a) <= tot(u) + 1e-12 or not u["distributed"]


def test_symbolic_disconnected_and_trivial(g2o_amd_mod):
    # three disconnected cliques + isolated blocks
    bi, bj = [], []
    for base in (0, 5, 11):
        for a in range(base, base + 4):
            for b in range(a, base + 4):
                bi.append(a)
                bj.append(b)
    nb = 16
    bi += list(range(nb))
    bj += list(range(nb))
    perm, st = g2o_amd_mod.symbolic_analyze(nb, 3, bi, bj)
    assert sorted(perm.tolist()) == list(range(48))
    perm1, st1 = g2o_amd_mod.symbolic_analyze(1, 6, [0], [0])
    assert perm1.tolist() == list(range(6)) and st1["supernodes"] == 1


def test_symbolic_band_windows(g2o_amd_mod, monkeypatch):
    """C4's reduced camera system is a band (cameras within a 64-camera window share points): 998 camera blocks
    of dimension 6, half-bandwidth 63 blocks — a path of 15.8 bandwidths. Level separators from a path's end cut
    only at multiples of the bandwidth (5 levels of 12 panel steps); the window separators at the exact middles
    give the optimum for the band: 3 separator levels over 8 segments, each segment split once more into a
    separator and two small leaves. The two 3-block leaves of each segment are absorbed into its separator (small
    leaf absorption), so the segment is one 69-block front: 4 levels, 13 + 3 x 12 = 49-50 level-synchronous panel
    steps, 15 supernodes."""
    nb, w = 998, 63
    bi = [i for i in range(nb) for j in range(i, min(nb, i + w + 1))]
    bj = [j for i in range(nb) for j in range(i, min(nb, i + w + 1))]
    monkeypatch.setenv("G2OHIP_BAND_LEAF", "0")  # the dissection itself (band leaves are a separate candidate)
    perm, st = g2o_amd_mod.symbolic_analyze(nb, 6, bi, bj)
    assert sorted(perm.tolist()) == list(range(nb * 6))
    assert st["panel_steps"] <= 50, st
    assert st["levels"] == 4, st
    assert st["supernodes"] == 15, st


def test_symbolic_rejects_bad_input(g2o_amd_mod):
    with pytest.raises(g2o_amd_mod.G2OHipError):
        g2o_amd_mod.symbolic_analyze(2, 3, [0, 5], [1, 1])


def test_synth_deterministic_and_shapes():
    a = synth.ba(30, 500, 6, 10)
    b = synth.ba(30, 500, 6, 10)
    for x, y in zip(a.edges[0].meas, b.edges[0].meas):
        assert np.array_equal(x, y)
    assert a.num_edges == 3000 and a.num_vertices == 530
    # every point observed by exactly k distinct cameras inside a window
    cams = a.edges[0].v1.reshape(500, 6)
    assert np.all(np.diff(np.sort(cams, 1), axis=1) > 0)
    assert np.all(cams.max(1) - cams.min(1) < 10)
    s = synth.sphere(10, 10)
    assert s.num_edges == 9 * 10 * 3 - 10 + 99  # create_sphere.cpp recipe (2500 -> 9799 at 50x50)
    full = synth.sphere(50, 50)
    assert full.num_edges == 9799


def test_synth_c4_full_counts():
    p = synth.by_name("C4")
    assert p.num_edges == 1_000_000
    assert p.num_vertices == 101_000
    assert int(p.vertices[0].fixed.sum()) == 2


def test_runtime_binding(g2o_amd_mod):
    """The product's HIP runtime and RCCL calls resolve to /opt/rocm (ROCm 7.2, what libg2o_hip.so is built against),
    not to the copies torch bundles under the same sonames: conftest.py binds the library before any test imports
    torch, as bench.py does before its torch.distributed control plane."""
    import torch  # noqa: F401  (loaded after the library: must not rebind it)
    info = g2o_amd_mod.runtime_info()
    assert info["libamdhip64"].startswith("/opt/rocm"), info
    assert info["librccl"].startswith("/opt/rocm"), info
    assert info["hip_runtime_version"] >= 70200000, info


def _reduce_threads(g2o_amd_mod, key, sizes, is_max=False):
    import threading
    bufs = [np.arange(n, dtype=np.float64) + 10 * r for r, n in enumerate(sizes)]
    errs = [None] * len(sizes)

    def run(r):
        try:
            g2o_amd_mod.comm_local_reduce_host(key, r, len(sizes), bufs[r], is_max)
        except g2o_amd_mod.G2OHipError as ex:
            errs[r] = str(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(len(sizes))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    assert not any(t.is_alive() for t in th), "a rank hung in the collective"
    return bufs, errs


def test_local_comm_rank_ordered_sum(g2o_amd_mod):
    bufs, errs = _reduce_threads(g2o_amd_mod, "sum-ok", [5, 5, 5])
    assert errs == [None] * 3
    want = sum(np.arange(5.0) + 10 * r for r in range(3))
    for b in bufs:
        np.testing.assert_array_equal(b, want)
    bufs, errs = _reduce_threads(g2o_amd_mod, "max-ok", [4, 4], is_max=True)
    assert errs == [None, None]
    np.testing.assert_array_equal(bufs[0], np.arange(4.0) + 10)


def test_local_comm_mismatch_raises(g2o_amd_mod):
    """A rank-dependent collective sequence (the r02 segfault: ranks entering all-reduces of different lengths) is an
    error on every rank, not a heap over-read or a hang."""
    bufs, errs = _reduce_threads(g2o_amd_mod, "mismatch-n", [6, 3])
    assert all(e and "collective mismatch" in e for e in errs), errs
    np.testing.assert_array_equal(bufs[1], np.arange(3.0) + 10)  # untouched
    # a different operation on one rank is a mismatch too
    import threading
    b = [np.ones(2), np.ones(2)]
    errs = [None, None]

    def run(r):
        try:
            g2o_amd_mod.comm_local_reduce_host("mismatch-op", r, 2, b[r], is_max=(r == 1))
        except g2o_amd_mod.G2OHipError as ex:
            errs[r] = str(ex)

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join(timeout=30) for t in th]
    assert all(e and "collective mismatch" in e for e in errs), errs


def test_pmc_traffic_factor_per_factorization(tmp_path):
    """tools/pmc_traffic.py: the factorization's traffic is the sum over its kernel chain divided by the number of
    factorizations, counted by the scatter launch (which also initialises the front vectors; k_vec_init only where no
    level is pre-scattered). Two factorizations of scatter + two panel steps + a contribution pass."""
    import csv
    import json
    import subprocess
    import sys
    names = ["g2ohip::k_chol_scatter(long long)", "void g2ohip::k_step<false>(int)", "void g2ohip::k_step<true>(int)",
             "g2ohip::k_syrk(int)", "void g2ohip::k_schur_rows<6, 3>(int)"]
    vals = {"FETCH_SIZE": [10.0, 20.0, 30.0, 40.0, 7.0], "WRITE_SIZE": [1.0, 2.0, 3.0, 4.0, 5.0]}
    dirs = {}
    for counter, v in vals.items():
        d = tmp_path / counter
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for _ in range(2):  # two factorizations
                for n, x in zip(names, v):
                    w.writerow({"Kernel_Name": n, "Counter_Name": counter, "Counter_Value": x})
        dirs[counter] = str(d)
    out = tmp_path / "traffic.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(out), dirs["FETCH_SIZE"],
                    dirs["WRITE_SIZE"]], check=True, capture_output=True)
    res = json.load(open(out))
    assert res["chol_factor"]["bytes_per_launch"] == (100.0 + 10.0) * 1024  # one factorization's chain
    assert res["schur_rows"]["bytes_per_launch"] == (7.0 + 5.0) * 1024
