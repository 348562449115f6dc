"""Host-authoritative Solver mode, as g2o drives a BlockSolver plugin (test infrastructure).

g2o's own OptimizationAlgorithmLevenberg (optimization_algorithm_levenberg.cpp:58-150) keeps running on the CPU
and owns the vertices; only the Solver virtuals (core/solver.h:54-137: buildStructure, buildSystem, setLambda,
solve, restoreDiagonal, x(), b()) go to the device. Here the "g2o CPU side" is the oracle graph (the CPU
restatement of g2o): it computes errors / chi2, applies x with update(), and push/pop/discardTop; before every
buildSystem its estimates are copied to the device (g2ohip_set_estimates) together with the host-computed
linearization of the host-Jacobian edge types (g2ohip_set_host_jacobians, the J_host_fallback).
"""
import math

import numpy as np

DBL_MAX = np.finfo(np.float64).max


def payload_size(prob, etype_edges):
    """Doubles of a host-J payload: per edge D * (1 + dim(v0) + dim(v1))."""
    return sum(D * (1 + di + dj) for D, di, dj in etype_edges)


def solver_mode_lm(gpu, host, iterations, vertex_types, hostj=(), max_trials=10):
    """Run `iterations` LM iterations with g2o's loop on the host and the device as its Solver.

    gpu: g2o_amd.SparseOptimizer holding the same vertices (insertion order) and edges (host-J types as
    G2OHIP_E_HOSTJ(D)); host: oracle_py.OracleGraph of the full graph; vertex_types: device vertex types whose
    estimates are pushed before buildSystem; hostj: list of (gpu_edge_type, oracle_edge_indices, payload_size).
    Returns a list of (chi2, levenbergIterations, lambda) per iteration (the G2OBatchStatistics fields)."""
    gpu.initialize_optimization()
    stats = []
    lam, ni = None, 2.0
    for it in range(iterations):
        if it == 0:
            gpu.build_structure()  # :63-69
        current = host.chi2()  # computeActiveErrors + activeRobustChi2 (:76-80)
        for vt in vertex_types:
            gpu.set_estimates(vt, host.estimates(vt))
        for etype, idx, size in hostj:
            gpu.set_host_jacobians(etype, host.edge_payload(idx, size, numeric=True))
        gpu.build_system()  # :82
        if it == 0:
            lam = 1e-5 * gpu.diag_absmax()  # computeLambdaInit (:152-175)
            ni = 2.0
        rho, q = 0.0, 0
        while True:  # :102-145
            host.push()
            gpu.set_lambda(lam, True)
            ok = gpu.solve()
            x, b = gpu.x(), gpu.b()
            host.update(x)  # SparseOptimizer::update
            gpu.restore_diagonal()
            temp = host.chi2()
            if not ok:
                temp = DBL_MAX
            rho = (current - temp) / (float(x @ (lam * x + b)) + 1e-3)  # computeScale (:177-184)
            if rho > 0 and math.isfinite(temp):
                alpha = min(1.0 - (2 * rho - 1) ** 3, 2.0 / 3.0)
                lam *= max(1.0 / 3.0, alpha)
                ni = 2.0
                current = temp
                host.discard_top()
            else:
                lam *= ni
                ni *= 2
                host.pop()
                if not math.isfinite(lam):
                    break
            q += 1
            if not (rho < 0 and q < max_trials):
                break
        stats.append((host.chi2(), q, lam))
        if q == max_trials or rho == 0 or not math.isfinite(lam):
            break  # Terminate
    return stats
