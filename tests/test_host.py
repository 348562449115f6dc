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


def test_symbolic_band_windows(g2o_amd_mod):
    """C4's reduced camera system is a band (cameras within a 64-camera window share points): 998 camera blocks
    of dimension 6, half-bandwidth 63 blocks — a path of 15.8 bandwidths. Level separators from a path's end cut
    only at multiples of the bandwidth (5 levels of 12 panel steps); the window separators at the exact middles
    give the optimum for the band: 3 separator levels over 8 segments, each segment split once more into a
    separator and two small leaves — 1 + 4 x 12 = 49 level-synchronous panel steps."""
    nb, w = 998, 63
    bi = [i for i in range(nb) for j in range(i, min(nb, i + w + 1))]
    bj = [j for i in range(nb) for j in range(i, min(nb, i + w + 1))]
    perm, st = g2o_amd_mod.symbolic_analyze(nb, 6, bi, bj)
    assert sorted(perm.tolist()) == list(range(nb * 6))
    assert st["panel_steps"] <= 50, st
    assert st["levels"] == 5, st


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
