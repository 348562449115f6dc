"""Online mode: SparseOptimizer::updateInitialization + BlockSolver::updateStructure
(/root/reference/g2o/core/sparse_optimizer.cpp:465-502, block_solver.hpp:258-312).

A pose graph is optimized, then grows (new poses and edges, ids interleaved with the existing ones) and is optimized
on, without re-initialization: the existing vertices keep their hessian indices and the new free ones are appended.
CPU tests pin the oracle's online path against a fresh initialization of the grown graph from the same state (the
linear system is the same up to a block permutation; within 1e-9). GPU tests (marked) check the device's online path
against the oracle's: trajectory within the parity tolerances of test_gpu_parity.py, solver-level x / b in the
appended block order within 1e-9, and the reference's refusals (Schur graphs).
"""
import dataclasses

import numpy as np
import pytest

from g2o_amd import synth

STATE_RTOL = 1e-6
CHI2_RTOL = 1e-6


def grow_split(prob, frac=0.6):
    """(before, added vertex sets, added edge sets, grown) with ids relabelled so that the added poses' ids interleave
    with the first part's (even ids for poses < K, odd for the rest): id order != hessian order after the update."""
    vs = prob.vertices[0]
    es = prob.edges[0]
    n = len(vs.ids)
    K = int(n * frac)
    idx = np.arange(n)
    new_id = np.where(idx < K, 2 * idx, 2 * (idx - K) + 1).astype(np.int32)
    remap = dict(zip(vs.ids.tolist(), new_id.tolist()))
    v0 = np.array([remap[int(a)] for a in es.v0], np.int32)
    v1 = np.array([remap[int(b)] for b in es.v1], np.int32)
    old_v = idx < K
    pos = {int(i): k for k, i in enumerate(vs.ids)}
    e_old = np.array([pos[int(a)] < K and pos[int(b)] < K for a, b in zip(es.v0, es.v1)])

    def vsub(mask):
        return dataclasses.replace(vs, ids=new_id[mask], est=vs.est[mask], fixed=vs.fixed[mask],
                                   marginalized=vs.marginalized[mask])

    def esub(mask):
        return dataclasses.replace(es, v0=v0[mask], v1=v1[mask], meas=es.meas[mask], info=es.info[mask])

    before = synth.Problem(prob.name + "/before", [vsub(old_v)], [esub(e_old)], prob.pose_dim, 0)
    grown = synth.Problem(prob.name + "/grown", [vsub(old_v), vsub(~old_v)], [esub(e_old), esub(~e_old)],
                          prob.pose_dim, 0)
    return before, [vsub(~old_v)], [esub(~e_old)], grown


def _problem(name):
    return synth.sphere(10, 12) if name == "se3" else synth.se2_grid(300)


def _oracle_online(oracle, before, add_v, add_e, it1, it2, threads=1):
    g = oracle.OracleGraph(before)
    g.optimize(it1, oracle.make_config(threads=threads))
    for v in add_v:
        g.add_vertices(v)
    for e in add_e:
        g.add_edges(e)
    assert g.update_initialization() == 0
    n, st = g.optimize(it2, oracle.make_config(threads=threads))
    return g, n, st


@pytest.mark.parametrize("name", ["se3", "se2"])
def test_oracle_online_matches_fresh_initialization(oracle, name):
    before, add_v, add_e, grown = grow_split(_problem(name))
    on, n_on, st_on = _oracle_online(oracle, before, add_v, add_e, 3, 4)
    # the same continuation from a fresh initializeOptimization (vertices re-indexed in id order)
    first = oracle.OracleGraph(before)
    first.optimize(3, oracle.make_config())
    vt = before.vertices[0].vtype
    fresh = oracle.OracleGraph(grown)
    est = fresh.estimates(vt)
    est[: len(before.vertices[0].ids)] = first.estimates(vt)
    fresh.set_estimates(vt, est)
    n_fr, st_fr = fresh.optimize(4, oracle.make_config())
    assert n_on == n_fr == 4
    for a, b in zip(st_on, st_fr):
        assert abs(a.chi2 - b.chi2) <= 1e-9 * abs(b.chi2), (a.chi2, b.chi2)
        assert a.levenbergIterations == b.levenbergIterations
    xo, xf = on.minimal_state(), fresh.minimal_state()
    assert np.linalg.norm(xo - xf) <= 1e-9 * np.linalg.norm(xf)


def _block_perm(prob_order_ids, pd):
    """hessian blocks of the fresh (id-sorted) order, listed in the online (appended) order"""
    rank = np.argsort(np.argsort(prob_order_ids))
    return (rank[:, None] * pd + np.arange(pd)).ravel()


def _free_ids_online(before, add_v):
    """hessian order after the update: the first part's free vertices by id, then the added free ones by id"""
    a = before.vertices[0]
    b = add_v[0]
    ia = np.sort(a.ids[a.fixed == 0])
    ib = np.sort(b.ids[b.fixed == 0])
    return np.concatenate([ia, ib])


def test_oracle_online_appends_hessian_blocks(oracle):
    before, add_v, add_e, grown = grow_split(_problem("se2"))
    g = oracle.OracleGraph(before)
    g.optimize(2, oracle.make_config())
    for v in add_v:
        g.add_vertices(v)
    for e in add_e:
        g.add_edges(e)
    assert g.update_initialization() == 0
    r_on = g.stage(1e-3)
    fresh = oracle.OracleGraph(grown)
    vt = before.vertices[0].vtype
    fresh.set_estimates(vt, g.estimates(vt))
    r_fr = fresh.stage(1e-3)
    perm = _block_perm(_free_ids_online(before, add_v), 3)
    assert r_on["n"] == r_fr["n"] == len(perm)
    assert np.linalg.norm(r_on["x"] - r_fr["x"][perm]) <= 1e-9 * np.linalg.norm(r_fr["x"])
    assert np.linalg.norm(r_on["b"] - r_fr["b"][perm]) <= 1e-12 * np.linalg.norm(r_fr["b"])


def test_oracle_online_refuses_schur(oracle):
    prob = synth.by_name("C4", "small")
    g = oracle.OracleGraph(prob)
    g.optimize(1, oracle.make_config())
    assert g.update_initialization() == -3


# ---------------------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("name", ["se3", "se2"])
def test_online_trajectory(g2o_amd_mod, oracle, name):
    before, add_v, add_e, _ = grow_split(_problem(name))
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(before)
    opt.optimize(3)
    for v in add_v:
        opt.add_vertices(v)
    for e in add_e:
        opt.add_edges(e)
    opt.update_initialization()
    n, st = opt.optimize(4)
    ref, nr, sr = _oracle_online(oracle, before, add_v, add_e, 3, 4, threads=8)
    assert n == nr == 4
    for a, b in zip(st, sr):
        assert abs(a.chi2 - b.chi2) <= CHI2_RTOL * abs(b.chi2), (a.chi2, b.chi2)
        assert a.levenbergIterations == b.levenbergIterations
        assert a.numVertices == b.numVertices and a.numEdges == b.numEdges
    xg, xr = opt.minimal_state(), ref.minimal_state()
    assert np.linalg.norm(xg - xr) <= STATE_RTOL * np.linalg.norm(xr)


@pytest.mark.gpu
def test_online_solver_level_block_order(g2o_amd_mod, oracle):
    """Solver-level plugin after updateStructure: x / b in the appended hessian order (the order the host's
    SparseOptimizer::update reads them in), against the oracle's online stage."""
    before, add_v, add_e, _ = grow_split(_problem("se2"))
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(before)
    opt.optimize(2)
    ref = oracle.OracleGraph(before)
    ref.optimize(2, oracle.make_config())
    for v in add_v:
        opt.add_vertices(v)
        ref.add_vertices(v)
    for e in add_e:
        opt.add_edges(e)
        ref.add_edges(e)
    opt.update_initialization()
    assert ref.update_initialization() == 0
    vt = before.vertices[0].vtype
    ref.set_estimates(vt, opt.estimates(vt))  # the same linearization point (device state after its 2 iterations)
    opt.build_structure()
    opt.build_system()
    opt.set_lambda(1e-3, True)
    assert opt.solve()
    x, b = opt.x(), opt.b()
    opt.restore_diagonal()
    r = ref.stage(1e-3)
    assert len(x) == r["n"] == 3 * len(_free_ids_online(before, add_v))
    assert np.linalg.norm(b - r["b"]) <= 1e-12 * np.linalg.norm(r["b"])
    assert np.linalg.norm(x - r["x"]) <= 1e-9 * np.linalg.norm(r["x"])


@pytest.mark.gpu
def test_online_refusals(g2o_amd_mod):
    lib = g2o_amd_mod.lib()
    before, add_v, _, _ = grow_split(_problem("se2"))
    opt = g2o_amd_mod.SparseOptimizer(0).add_problem(before)
    assert lib.g2ohip_update_initialization(opt.h) == -2  # G2OHIP_ERR_STATE: initializeOptimization first
    ba = g2o_amd_mod.SparseOptimizer(0).add_problem(synth.by_name("C4", "small"))
    ba.optimize(1)
    with pytest.raises(g2o_amd_mod.G2OHipError, match="Schur"):
        ba.update_initialization()
