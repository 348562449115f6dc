"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

ctypes wrapper over oracle/liboracle.so, the CPU restatement of the reference
BlockSolver / LinearSolverCSparse / LM path (see oracle/oracle.cpp header for
the file:line map).  Never imported by the product package ``g2o_amd``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class BatchStats(C.Structure):
    _fields_ = [
        ("iteration", C.c_int), ("numVertices", C.c_int), ("numEdges", C.c_int),
        ("chi2", C.c_double), ("lambda_", C.c_double),
        ("timeResiduals", C.c_double), ("timeQuadraticForm", C.c_double),
        ("levenbergIterations", C.c_int),
        ("timeSchurComplement", C.c_double), ("timeSymbolicDecomposition", C.c_double),
        ("timeNumericDecomposition", C.c_double), ("timeLinearSolution", C.c_double),
        ("timeLinearSolver", C.c_double), ("timeUpdate", C.c_double), ("timeIteration", C.c_double),
        ("hessianDimension", C.c_longlong), ("hessianPoseDimension", C.c_longlong),
        ("hessianLandmarkDimension", C.c_longlong), ("choleskyNNZ", C.c_longlong),
    ]


class Config(C.Structure):
    _fields_ = [("max_trials_after_failure", C.c_int), ("user_lambda_init", C.c_double),
                ("threads", C.c_int), ("use_ref_csparse", C.c_int), ("block_ordering", C.c_int),
                ("gauss_newton", C.c_int)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P, I, D = C.c_void_p, C.c_int, C.c_double
        L.oracle_graph_new.restype = P
        L.oracle_graph_free.argtypes = [P]
        L.oracle_add_vertices.argtypes = [P, I, I, P, P, P, P]
        L.oracle_add_edges.argtypes = [P, I, I, P, P, P, P, P]
        L.oracle_load_g2o.argtypes = [P, C.c_char_p, I]
        L.oracle_save_g2o.argtypes = [P, C.c_char_p]
        L.oracle_num_vertices.argtypes = [P]
        L.oracle_num_edges.argtypes = [P]
        L.oracle_get_estimates.argtypes = [P, I, P, P]
        L.oracle_minimal_state.argtypes = [P, P]
        L.oracle_initialize.argtypes = [P]
        L.oracle_update_initialization.argtypes = [P]
        L.oracle_chi2.argtypes = [P]
        L.oracle_chi2.restype = D
        L.oracle_optimize.argtypes = [P, P, I, P]
        L.oracle_stage.argtypes = [P, P, D, P, P, P, P, P]
        L.oracle_hessian_dense.argtypes = [P, P, P, P]
        L.oracle_edge_jacobians.argtypes = [P, I, P, P, P, P, P]
        L.oracle_ccs_cholsol.argtypes = [I, P, P, P, P, I]
        L.oracle_block_symbolic.argtypes = [I, I, I, P, P, I, P]
        L.oracle_set_robust_kernel.argtypes = [P, I, I, D]
        L.oracle_set_edge_numeric.argtypes = [P, I, P]
        L.oracle_edge_payload.argtypes = [P, I, P, I, P]
        L.oracle_update.argtypes = [P, P]
        L.oracle_set_estimates.argtypes = [P, I, P]
        L.oracle_push.argtypes = [P]
        L.oracle_pop.argtypes = [P]
        L.oracle_discard_top.argtypes = [P]
        L.oracle_ref_available.restype = I
        L.oracle_mapping.argtypes = [I, P, P]
        L.oracle_mapping.restype = I
        L.oracle_ref_path.restype = C.c_char_p
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


MAPPING_OPS = {"fromEuler": 0, "toEuler": 1, "toCompactQuaternion": 2, "fromCompactQuaternion": 3, "fromVectorET": 4,
               "toVectorET": 5, "toVectorMQT": 6, "fromVectorMQT": 7, "toVectorQT": 8, "fromVectorQT": 9,
               "approximateNearestOrthogonalMatrix": 10, "nearestOrthogonalMatrix": 11, "SE2fromIsometry2": 12}


def mapping(name: str, x) -> np.ndarray:
    """isometry3d_mappings / SE2 as the oracle restates them: matrices col-major (9), isometries [R col-major | t]
    (12), vectors as the reference orders them."""
    x = np.ascontiguousarray(x, np.float64).ravel()
    out = np.zeros(16)
    n = lib().oracle_mapping(MAPPING_OPS[name], x.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
    assert n > 0, name
    return out[:n].copy()


def ref_available() -> bool:
    return bool(lib().oracle_ref_available())


def make_config(threads=1, use_ref=True, block_ordering=True, max_trials=10, lambda_init=0.0,
                gauss_newton=False) -> Config:
    return Config(max_trials, lambda_init, threads, 1 if use_ref else 0, 1 if block_ordering else 0,
                  1 if gauss_newton else 0)


class OracleGraph:
    def __init__(self, problem=None):
        self.h = lib().oracle_graph_new()
        if problem is not None:
            self.add_problem(problem)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_graph_free(self.h)
            self.h = None

    def add_problem(self, prob):
        for vs in prob.vertices:
            ids = np.ascontiguousarray(vs.ids, np.int32)
            est = np.ascontiguousarray(vs.est, np.float64)
            fx = np.ascontiguousarray(vs.fixed, np.int32)
            mg = np.ascontiguousarray(vs.marginalized, np.int32)
            r = lib().oracle_add_vertices(self.h, vs.vtype, len(ids), _p(ids), _p(est), _p(fx), _p(mg))
            assert r == 0, r
        for es in prob.edges:
            v0 = np.ascontiguousarray(es.v0, np.int32)
            v1 = np.ascontiguousarray(es.v1, np.int32)
            meas = np.ascontiguousarray(es.meas, np.float64)
            info = np.ascontiguousarray(es.info, np.float64)
            par = None if es.params is None else np.ascontiguousarray(es.params, np.float64)
            r = lib().oracle_add_edges(self.h, es.etype, len(v0), _p(v0), _p(v1), _p(meas), _p(info), _p(par))
            assert r == 0, r

    @classmethod
    def load(cls, path, marginalize_xyz=True):
        g = cls()
        r = lib().oracle_load_g2o(g.h, path.encode(), 1 if marginalize_xyz else 0)
        assert r == 0, r
        return g

    def save(self, path):
        assert lib().oracle_save_g2o(self.h, path.encode()) == 0

    def chi2(self) -> float:
        lib().oracle_initialize(self.h)
        return lib().oracle_chi2(self.h)

    def initialize(self):
        lib().oracle_initialize(self.h)

    def update_initialization(self) -> int:
        """sparse_optimizer.cpp:465-502 + block_solver.hpp:258-312 (online, non-Schur): 0 ok, <0 refused."""
        return lib().oracle_update_initialization(self.h)

    def add_vertices(self, vs):
        ids = np.ascontiguousarray(vs.ids, np.int32)
        est = np.ascontiguousarray(vs.est, np.float64)
        fx = np.ascontiguousarray(vs.fixed, np.int32)
        mg = np.ascontiguousarray(vs.marginalized, np.int32)
        assert lib().oracle_add_vertices(self.h, vs.vtype, len(ids), _p(ids), _p(est), _p(fx), _p(mg)) == 0

    def add_edges(self, es):
        v0 = np.ascontiguousarray(es.v0, np.int32)
        v1 = np.ascontiguousarray(es.v1, np.int32)
        meas = np.ascontiguousarray(es.meas, np.float64)
        info = np.ascontiguousarray(es.info, np.float64)
        par = None if es.params is None else np.ascontiguousarray(es.params, np.float64)
        assert lib().oracle_add_edges(self.h, es.etype, len(v0), _p(v0), _p(v1), _p(meas), _p(info), _p(par)) == 0

    def optimize(self, iterations=10, cfg: Config | None = None):
        cfg = cfg or make_config()
        stats = (BatchStats * max(iterations, 1))()
        n = lib().oracle_optimize(self.h, C.byref(cfg), iterations, stats)
        return n, [stats[i] for i in range(max(n, 0))]

    def minimal_state(self) -> np.ndarray:
        n = lib().oracle_minimal_state(self.h, None)
        out = np.zeros(n)
        lib().oracle_minimal_state(self.h, _p(out))
        return out

    def estimates(self, vtype: int) -> np.ndarray:
        from g2o_amd.synth import EST_DIM
        n = lib().oracle_get_estimates(self.h, vtype, None, None)
        out = np.zeros((n, EST_DIM[vtype]))
        lib().oracle_get_estimates(self.h, vtype, _p(out), None)
        return out

    def set_robust_kernel(self, etype, kind, delta):
        assert lib().oracle_set_robust_kernel(self.h, etype, kind, delta) == 0

    def set_numeric(self, idx):
        idx = np.ascontiguousarray(idx, np.int32)
        assert lib().oracle_set_edge_numeric(self.h, len(idx), _p(idx)) == 0

    def edge_payload(self, idx, size, numeric=True):
        """[e | Ji | Jj] per listed edge (row-major) at the current estimates; `size` = total doubles."""
        idx = np.ascontiguousarray(idx, np.int32)
        out = np.zeros(size)
        n = lib().oracle_edge_payload(self.h, len(idx), _p(idx), 1 if numeric else 0, _p(out))
        assert n == size, (n, size)
        return out

    def update(self, x):
        x = np.ascontiguousarray(x, np.float64)
        lib().oracle_update(self.h, _p(x))

    def set_estimates(self, vtype, est):
        est = np.ascontiguousarray(est, np.float64)
        lib().oracle_set_estimates(self.h, vtype, _p(est))

    def push(self):
        lib().oracle_push(self.h)

    def pop(self):
        lib().oracle_pop(self.h)

    def discard_top(self):
        lib().oracle_discard_top(self.h)

    def stage(self, lam: float, cfg: Config | None = None):
        """buildStructure/buildSystem/setLambda/solve at the current state; dense outputs."""
        cfg = cfg or make_config()
        dims = np.zeros(3, np.int64)
        lib().oracle_stage(self.h, C.byref(cfg), 0.0, None, None, None, None, _p(dims))
        n, npose = int(dims[0]), int(dims[1])
        b = np.zeros(n)
        x = np.zeros(n)
        H = np.zeros((npose, npose))
        bs = np.zeros(npose)
        ok = lib().oracle_stage(self.h, C.byref(cfg), lam, _p(b), _p(x), _p(H), _p(bs), _p(dims))
        return dict(ok=ok, b=b, x=x, Hschur=H, bschur=bs, n=n, np=npose, nl=int(dims[2]))

    def hessian_dense(self, npose, nl):
        Hpp = np.zeros((npose, npose))
        Hll = np.zeros(nl * 3)
        Hpl = np.zeros((npose, nl))
        lib().oracle_hessian_dense(self.h, _p(Hpp), _p(Hll) if nl else None, _p(Hpl) if nl else None)
        return Hpp, Hll, Hpl

    def edge_jacobians(self, k: int, D: int, di: int, dj: int):
        err = np.zeros(D)
        Ja, Jb, Na, Nb = np.zeros((D, di)), np.zeros((D, dj)), np.zeros((D, di)), np.zeros((D, dj))
        assert lib().oracle_edge_jacobians(self.h, k, _p(err), _p(Ja), _p(Jb), _p(Na), _p(Nb)) == 0
        return err, Ja, Jb, Na, Nb


def ccs_cholsol(n, Ap, Ai, Ax, b, mode):
    Ap = np.ascontiguousarray(Ap, np.int32)
    Ai = np.ascontiguousarray(Ai, np.int32)
    Ax = np.ascontiguousarray(Ax, np.float64)
    x = np.array(b, dtype=np.float64, copy=True)
    r = lib().oracle_ccs_cholsol(n, _p(Ap), _p(Ai), _p(Ax), _p(x), mode)
    return r, x


def block_symbolic(nblocks, bdim, bi, bj, use_ref=True):
    """(nnz(L), sum c_k^2) of LinearSolverCSparse's block-AMD symbolic analysis for an upper block pattern."""
    bi = np.ascontiguousarray(bi, np.int32)
    bj = np.ascontiguousarray(bj, np.int32)
    out = np.zeros(2)
    r = lib().oracle_block_symbolic(nblocks, bdim, len(bi), _p(bi), _p(bj), 1 if use_ref else 0, _p(out))
    assert r == 0, r
    return float(out[0]), float(out[1])
