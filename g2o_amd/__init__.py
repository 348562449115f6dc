"""g2o_amd — MI355X-native BlockSolver<p,l> backend for g2o.

Python mirror of the reference's operator/plugin interface for this path
(``g2o::SparseOptimizer`` + ``OptimizationAlgorithmLevenberg`` + the ``Solver``
plugin, see ``include/g2o_hip.h``) over the C ABI of ``libg2o_hip.so``.
The library is hand-written HIP for gfx950; there is no CPU fallback: every
compute call fails loudly when the library or a GPU is missing.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import synth  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("G2OHIP_LIB") or os.path.join(HERE, "libg2o_hip.so")


class BatchStats(C.Structure):
    """G2OBatchStatistics (core/batch_stats.h:42-72) + lambda."""
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
    _fields_ = [("max_trials_after_failure", C.c_int), ("user_lambda_init", C.c_double), ("verbose", C.c_int)]


# edge types the device does not know: host-supplied error + Jacobians (include/g2o_hip.h G2OHIP_E_HOSTJ)
def E_HOSTJ(D: int) -> int:
    return 32 + D


# robust kernels (G2OHIP_RK_*, robust_kernel_impl.cpp)
RK = {"none": 0, "Huber": 1, "PseudoHuber": 2, "Cauchy": 3, "GemanMcClure": 4, "Welsch": 5, "Fair": 6, "Tukey": 7,
      "Saturated": 8, "DCS": 9}

HOST_EDGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double))

EXPORTS = [
    "g2ohip_graph_create", "g2ohip_graph_destroy", "g2ohip_add_vertices", "g2ohip_add_edges",
    "g2ohip_load_g2o", "g2ohip_save_g2o", "g2ohip_num_vertices", "g2ohip_num_edges",
    "g2ohip_set_robust_kernel", "g2ohip_set_host_jacobians", "g2ohip_set_host_edge_callback",
    "g2ohip_solver_diag_absmax", "g2ohip_solver_set_eta", "g2ohip_solver_linear_iterations",
    "g2ohip_get_estimates", "g2ohip_set_estimates", "g2ohip_minimal_state", "g2ohip_set_algorithm",
    "g2ohip_initialize", "g2ohip_chi2", "g2ohip_optimize", "g2ohip_optimize_step",
    "g2ohip_solver_build_structure", "g2ohip_solver_build_system", "g2ohip_solver_set_lambda",
    "g2ohip_solver_restore_diagonal", "g2ohip_solver_solve", "g2ohip_solver_vector_size", "g2ohip_solver_block_dims",
    "g2ohip_solver_get_x", "g2ohip_solver_get_b", "g2ohip_solver_multiply_hessian",
    "g2ohip_solver_linear_residual", "g2ohip_solver_factor_info", "g2ohip_solver_compute_marginals", "g2ohip_update", "g2ohip_push", "g2ohip_pop",
    "g2ohip_discard_top", "g2ohip_stage", "g2ohip_linear_solve_ccs", "g2ohip_comm_unique_id",
    "g2ohip_set_comm", "g2ohip_set_comm_local", "g2ohip_comm_selftest", "g2ohip_comm_selftest_rs", "g2ohip_symbolic_analyze", "g2ohip_dist_plan", "g2ohip_local_landmarks", "g2ohip_enable_kernel_timing",
    "g2ohip_kernel_timing_only", "g2ohip_set_stats_level", "g2ohip_kernel_ms",
    "g2ohip_kernel_count", "g2ohip_kernel_bytes", "g2ohip_kernel_flops", "g2ohip_last_error",
    "g2ohip_version", "g2ohip_host_payload_len", "g2ohip_solver_save_hessian", "g2ohip_solver_set_write_debug",
    "g2ohip_comm_local_reduce_host", "g2ohip_runtime_info", "g2ohip_device_synchronize", "g2ohip_lm_scale_factor",
    "g2ohip_measure_peaks",
]


def build(arch: str = "gfx950") -> None:
    """Compile libg2o_hip.so in-tree with hipcc (cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", HERE, f"ARCH={arch}", "-j8"], check=True)


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run g2o_amd.build() (hipcc --offload-arch=gfx950)")
    L = C.CDLL(LIB_PATH)
    P, I, D, LL = C.c_void_p, C.c_int, C.c_double, C.c_longlong
    sig = {
        "g2ohip_graph_create": ([I], P),
        "g2ohip_graph_destroy": ([P], None),
        "g2ohip_add_vertices": ([P, I, I, P, P, P, P], I),
        "g2ohip_add_edges": ([P, I, I, P, P, P, P, P], I),
        "g2ohip_load_g2o": ([P, C.c_char_p, I], I),
        "g2ohip_save_g2o": ([P, C.c_char_p], I),
        "g2ohip_num_vertices": ([P], I),
        "g2ohip_num_edges": ([P], I),
        "g2ohip_set_robust_kernel": ([P, I, I, D], I),
        "g2ohip_set_host_jacobians": ([P, I, P], I),
        "g2ohip_set_host_edge_callback": ([P, HOST_EDGE_FN, P], I),
        "g2ohip_solver_diag_absmax": ([P, P], I),
        "g2ohip_solver_set_eta": ([P, D], I),
        "g2ohip_solver_linear_iterations": ([P], I),
        "g2ohip_get_estimates": ([P, I, P, P], I),
        "g2ohip_set_estimates": ([P, I, P], I),
        "g2ohip_minimal_state": ([P, P], I),
        "g2ohip_set_algorithm": ([P, C.c_char_p], I),
        "g2ohip_initialize": ([P], I),
        "g2ohip_update_initialization": ([P], I),
        "g2ohip_chi2": ([P], D),
        "g2ohip_optimize": ([P, P, I, P], I),
        "g2ohip_optimize_step": ([P, P, I, P], I),
        "g2ohip_solver_build_structure": ([P], I),
        "g2ohip_solver_build_system": ([P], I),
        "g2ohip_solver_set_lambda": ([P, D, I], I),
        "g2ohip_solver_restore_diagonal": ([P], I),
        "g2ohip_solver_solve": ([P], I),
        "g2ohip_solver_vector_size": ([P], LL),
        "g2ohip_solver_block_dims": ([P, P], I),
        "g2ohip_solver_get_x": ([P, P], I),
        "g2ohip_solver_get_b": ([P, P], I),
        "g2ohip_solver_multiply_hessian": ([P, P, P], I),
        "g2ohip_solver_linear_residual": ([P, P], I),
        "g2ohip_solver_factor_info": ([P, P, I], I),
        "g2ohip_solver_compute_marginals": ([P, I, P, P, P], I),
        "g2ohip_update": ([P, P], I),
        "g2ohip_push": ([P], I),
        "g2ohip_pop": ([P], I),
        "g2ohip_discard_top": ([P], I),
        "g2ohip_stage": ([P, D, P, P, P, P, P], I),
        "g2ohip_linear_solve_ccs": ([I, I, P, P, P, P, P, I, P], I),
        "g2ohip_comm_unique_id": ([P], I),
        "g2ohip_set_comm": ([P, P, I, I], I),
        "g2ohip_set_comm_local": ([P, C.c_char_p, I, I], I),
        "g2ohip_comm_selftest": ([I, P, I, P, P], I),
        "g2ohip_comm_selftest_rs": ([I, P, I, P, P, P], I),
        "g2ohip_debug_phases": ([P, I], I),
        "g2ohip_symbolic_analyze": ([I, I, I, P, P, P, P], I),
        "g2ohip_dist_plan": ([I, I, I, P, P, I, I, I, P, P, P, I], I),
        "g2ohip_local_landmarks": ([P, P, I], I),
        "g2ohip_enable_kernel_timing": ([P, I], None),
        "g2ohip_kernel_timing_only": ([P, C.c_char_p], None),
        "g2ohip_set_stats_level": ([P, I], None),
        "g2ohip_kernel_ms": ([P, C.c_char_p], D),
        "g2ohip_kernel_count": ([P, C.c_char_p], LL),
        "g2ohip_kernel_bytes": ([P, C.c_char_p], D),
        "g2ohip_kernel_flops": ([P, C.c_char_p], D),
        "g2ohip_last_error": ([], C.c_char_p),
        "g2ohip_version": ([], C.c_char_p),
        "g2ohip_lm_scale_factor": ([D], D),
        "g2ohip_measure_peaks": ([I, P, I], I),
        "g2ohip_host_payload_len": ([P, I], LL),
        "g2ohip_solver_save_hessian": ([P, C.c_char_p], I),
        "g2ohip_solver_set_write_debug": ([P, I], I),
        "g2ohip_comm_local_reduce_host": ([C.c_char_p, I, I, P, LL, I], I),
        "g2ohip_runtime_info": ([C.c_char_p, I], I),
        "g2ohip_device_synchronize": ([I], I),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def runtime_info() -> dict:
    """The HIP runtime / RCCL this library is bound to (resolved library paths + versions)."""
    import json
    buf = C.create_string_buffer(2048)
    lib().g2ohip_runtime_info(buf, len(buf))
    return json.loads(buf.value.decode())


def device_synchronize(device: int = 0) -> None:
    _check(lib().g2ohip_device_synchronize(device), "device_synchronize")


def measure_peaks(device: int = 0) -> dict:
    """Measured roofline peaks of the device (g2ohip_measure_peaks): HBM streaming copy, FP64 MFMA and VALU issue rates."""
    out = np.zeros(4)
    _check(lib().g2ohip_measure_peaks(device, _p(out), 4), "measure_peaks")
    return {"hbm_copy_GBps": float(out[0]), "fp64_mfma_TFps": float(out[1]), "fp64_valu_TFps": float(out[2]),
            "cus": int(out[3])}


def comm_local_reduce_host(group_key: str, rank: int, nranks: int, buf, is_max: bool = False):
    """The in-process test transport's host reduction (collective-consistency checked); buf is reduced in place."""
    _check(lib().g2ohip_comm_local_reduce_host(group_key.encode(), rank, nranks, _p(buf), buf.size, int(is_max)),
           "comm_local_reduce_host")
    return buf


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def last_error() -> str:
    return lib().g2ohip_last_error().decode()


class G2OHipError(RuntimeError):
    pass


def _check(code, what):
    if code < 0:
        raise G2OHipError(f"{what} failed ({code}): {last_error()}")
    return code


def symbolic_analyze(nblocks: int, bdim: int, bi, bj):
    """Host-only symbolic analysis (ordering + supernodes); returns (perm, stats dict)."""
    bi = np.ascontiguousarray(bi, np.int32)
    bj = np.ascontiguousarray(bj, np.int32)
    perm = np.zeros(nblocks * bdim, np.int32)
    st = np.zeros(5)
    n = lib().g2ohip_symbolic_analyze(nblocks, bdim, len(bi), _p(bi), _p(bj), _p(perm), _p(st))
    _check(n, "symbolic_analyze")
    return perm, dict(nnzL=st[0], flops=st[1], supernodes=int(st[2]), levels=int(st[3]), panel_steps=int(st[4]))


DIST_PLAN_KEYS = ("distributed", "rank_subtrees_s", "shared_s", "replicated_s", "exchange_s", "input_s",
                  "input_replicated_s", "max_rank_subtrees_s", "root_allgather_doubles", "rs_segment_doubles",
                  "rs_tail_doubles", "supernodes", "shard_s", "shard_replicated_s")


def dist_plan(nblocks: int, bdim: int, bi, bj, nranks: int, rank: int = 0, reduce_scatter: bool = True,
              aligned: bool = True, pose_work=None):
    """Host-only: the distributed factorization's cut for `nranks` landmark shards (the model the solver's setup
    runs; aligned: shards follow the cut, the default); returns (model dict, per-supernode owner
    array: rank, -1 shared)."""
    bi = np.ascontiguousarray(bi, np.int32)
    bj = np.ascontiguousarray(bj, np.int32)
    out = np.zeros(len(DIST_PLAN_KEYS))
    cap = 4 * nblocks + 16
    owner = np.full(cap, -1, np.int32)
    pw = None if pose_work is None else np.ascontiguousarray(pose_work, np.float64)
    n = lib().g2ohip_dist_plan(nblocks, bdim, len(bi), _p(bi), _p(bj), nranks, rank,
                               int(reduce_scatter) | (2 if aligned else 0), None if pw is None else _p(pw), _p(out),
                               _p(owner), cap)
    _check(n, "dist_plan")
    d = dict(zip(DIST_PLAN_KEYS, out.tolist()))
    return d, owner[:n]


def linear_solve_ccs(n, Ap, Ai, Ax, b, block_dim=1, device=0):
    """LinearSolver::solve on an upper-CCS matrix (LinearSolverCCS contract)."""
    Ap = np.ascontiguousarray(Ap, np.int32)
    Ai = np.ascontiguousarray(Ai, np.int32)
    Ax = np.ascontiguousarray(Ax, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    x = np.zeros(n)
    nb = n // block_dim
    ends = np.arange(1, nb + 1, dtype=np.int32) * block_dim
    r = lib().g2ohip_linear_solve_ccs(device, n, _p(Ap), _p(Ai), _p(Ax), _p(b), _p(x), nb, _p(ends))
    _check(r, "linear_solve_ccs")
    return bool(r), x


class SparseOptimizer:
    """g2o::SparseOptimizer with a device-resident ``lm_hip_*`` algorithm
    (sparse_optimizer.h; optimization_algorithm_levenberg.h)."""

    def __init__(self, device: int = 0):
        self.h = lib().g2ohip_graph_create(device)
        if not self.h:
            raise G2OHipError(f"g2ohip_graph_create failed: {last_error()}")

    def close(self):
        if getattr(self, "h", None):
            lib().g2ohip_graph_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---- OptimizableGraph ----
    def add_vertices(self, vs):
        ids = np.ascontiguousarray(vs.ids, np.int32)
        est = np.ascontiguousarray(vs.est, np.float64)
        fx = np.ascontiguousarray(vs.fixed, np.int32)
        mg = np.ascontiguousarray(vs.marginalized, np.int32)
        _check(lib().g2ohip_add_vertices(self.h, vs.vtype, len(ids), _p(ids), _p(est), _p(fx), _p(mg)),
               "add_vertices")

    def add_edges(self, es):
        v0 = np.ascontiguousarray(es.v0, np.int32)
        v1 = np.ascontiguousarray(es.v1, np.int32)
        meas = None if es.meas is None else np.ascontiguousarray(es.meas, np.float64)
        info = np.ascontiguousarray(es.info, np.float64)
        par = None if es.params is None else np.ascontiguousarray(es.params, np.float64)
        _check(lib().g2ohip_add_edges(self.h, es.etype, len(v0), _p(v0), _p(v1), _p(meas), _p(info), _p(par)),
               "add_edges")

    def add_problem(self, prob):
        for vs in prob.vertices:
            self.add_vertices(vs)
        for es in prob.edges:
            self.add_edges(es)
        return self

    def set_robust_kernel(self, etype: int, kind, delta: float):
        """Edge::setRobustKernel for every edge of a type; kind = RK name or G2OHIP_RK_* number."""
        k = RK[kind] if isinstance(kind, str) else int(kind)
        _check(lib().g2ohip_set_robust_kernel(self.h, etype, k, float(delta)), "set_robust_kernel")

    def set_host_jacobians(self, etype: int, payload):
        """[e | Ji | Jj] row-major per edge of a host-J type (insertion order), at the device's estimates."""
        payload = np.ascontiguousarray(payload, np.float64)
        _check(lib().g2ohip_set_host_jacobians(self.h, etype, _p(payload)), "set_host_jacobians")

    def set_host_edge_callback(self, fn):
        """fn(edge_type, with_jacobians) -> payload ndarray, called by the device-resident loops for host-J edges."""
        if fn is None:
            self._host_cb = None
            _check(lib().g2ohip_set_host_edge_callback(self.h, HOST_EDGE_FN(), None), "set_host_edge_callback")
            return

        def tramp(user, etype, with_jac, out):
            try:
                pay = np.ascontiguousarray(fn(etype, bool(with_jac)), np.float64)
                want = lib().g2ohip_host_payload_len(self.h, etype)
                if want < 0 or pay.size != want:  # never write past the engine's payload buffer
                    raise G2OHipError(f"host edge callback returned {pay.size} doubles for edge type {etype}, "
                                      f"expected {want} (D * (1 + dim(v0) + dim(v1)) per edge)")
                C.memmove(out, pay.ctypes.data, pay.nbytes)
                return 0
            except Exception:  # reported as a failed callback by the engine
                import traceback
                traceback.print_exc()
                return 1

        self._host_cb = HOST_EDGE_FN(tramp)  # keep alive
        _check(lib().g2ohip_set_host_edge_callback(self.h, self._host_cb, None), "set_host_edge_callback")

    def set_estimates(self, vtype: int, est):
        """Overwrite the estimates of one vertex type (insertion order): host-authoritative Solver mode."""
        est = np.ascontiguousarray(est, np.float64)
        _check(lib().g2ohip_set_estimates(self.h, vtype, _p(est)), "set_estimates")

    def load(self, path: str, marginalize_xyz: bool = True):
        _check(lib().g2ohip_load_g2o(self.h, path.encode(), int(marginalize_xyz)), "load")

    def num_vertices(self) -> int:
        return int(lib().g2ohip_num_vertices(self.h))

    def num_edges(self) -> int:
        return int(lib().g2ohip_num_edges(self.h))

    def save(self, path: str):
        _check(lib().g2ohip_save_g2o(self.h, path.encode()), "save")

    def save_hessian(self, path: str) -> bool:
        """Solver::saveHessian (block_solver.hpp:589-593): Hpp in Octave sparse-matrix text."""
        return bool(_check(lib().g2ohip_solver_save_hessian(self.h, path.encode()), "saveHessian"))

    def set_write_debug(self, on: bool = True):
        """Solver::setWriteDebug: a not-PD factorization writes debug.txt (linear_solver_csparse.h:127-133)."""
        _check(lib().g2ohip_solver_set_write_debug(self.h, int(on)), "setWriteDebug")

    def set_algorithm(self, name: str):
        _check(lib().g2ohip_set_algorithm(self.h, name.encode()), "set_algorithm")

    def initialize_optimization(self):
        _check(lib().g2ohip_initialize(self.h), "initializeOptimization")

    def update_initialization(self):
        """SparseOptimizer::updateInitialization (online mode, non-Schur): vertices / edges added since
        initialize_optimization join with appended hessian indices; optimize() then continues from the current state."""
        _check(lib().g2ohip_update_initialization(self.h), "updateInitialization")

    def chi2(self) -> float:
        return lib().g2ohip_chi2(self.h)

    def optimize(self, iterations: int, max_trials: int = 10, lambda_init: float = 0.0, verbose: bool = False):
        cfg = Config(max_trials, lambda_init, int(verbose))
        stats = (BatchStats * max(iterations, 1))()
        n = _check(lib().g2ohip_optimize(self.h, C.byref(cfg), iterations, stats), "optimize")
        return n, [stats[i] for i in range(n)]

    def optimize_step(self, iteration: int, max_trials: int = 10, lambda_init: float = 0.0, stats: bool = True):
        cfg = Config(max_trials, lambda_init, 0)
        st = BatchStats()
        r = _check(lib().g2ohip_optimize_step(self.h, C.byref(cfg), iteration, C.byref(st) if stats else None),
                   "optimize_step")
        return r, st

    def minimal_state(self) -> np.ndarray:
        n = _check(lib().g2ohip_minimal_state(self.h, None), "minimal_state")
        out = np.zeros(n)
        lib().g2ohip_minimal_state(self.h, _p(out))
        return out

    def estimates(self, vtype: int) -> np.ndarray:
        n = _check(lib().g2ohip_get_estimates(self.h, vtype, None, None), "get_estimates")
        out = np.zeros((n, synth.EST_DIM[vtype]))
        lib().g2ohip_get_estimates(self.h, vtype, _p(out), None)
        return out

    # ---- Solver plugin (core/solver.h) ----
    def build_structure(self):
        _check(lib().g2ohip_solver_build_structure(self.h), "buildStructure")

    def build_system(self):
        _check(lib().g2ohip_solver_build_system(self.h), "buildSystem")

    def set_lambda(self, lam: float, backup: bool = True):
        _check(lib().g2ohip_solver_set_lambda(self.h, lam, int(backup)), "setLambda")

    def restore_diagonal(self):
        _check(lib().g2ohip_solver_restore_diagonal(self.h), "restoreDiagonal")

    def solve(self) -> bool:
        return bool(_check(lib().g2ohip_solver_solve(self.h), "solve"))

    def vector_size(self) -> int:
        return int(lib().g2ohip_solver_vector_size(self.h))

    def block_dims(self):
        """[PoseDim, LandmarkDim, pose blocks, landmark blocks] of the built structure."""
        d = np.zeros(4, np.int32)
        _check(lib().g2ohip_solver_block_dims(self.h, _p(d)), "block_dims")
        return [int(v) for v in d]

    def x(self) -> np.ndarray:
        out = np.zeros(self.vector_size())
        _check(lib().g2ohip_solver_get_x(self.h, _p(out)), "x")
        return out

    def b(self) -> np.ndarray:
        out = np.zeros(self.vector_size())
        _check(lib().g2ohip_solver_get_b(self.h, _p(out)), "b")
        return out

    def multiply_hessian(self, src) -> np.ndarray:
        """BlockSolverBase::multiplyHessian (block_solver.h:146): Hpp @ src (pose part)."""
        src = np.ascontiguousarray(src, np.float64)
        out = np.zeros_like(src)
        _check(lib().g2ohip_solver_multiply_hessian(self.h, _p(out), _p(src)), "multiplyHessian")
        return out

    def set_eta(self, eta: float):
        """Solver::setEta: forcing term of the lm_pcg6_3_eigen CGLS (default 0.1)."""
        _check(lib().g2ohip_solver_set_eta(self.h, float(eta)), "set_eta")

    def linear_iterations(self) -> int:
        return int(lib().g2ohip_solver_linear_iterations(self.h))

    def diag_absmax(self) -> float:
        """max |diag| of the vertex Hessians (computeLambdaInit's input) after buildSystem."""
        r = np.zeros(1)
        _check(lib().g2ohip_solver_diag_absmax(self.h, _p(r)), "diag_absmax")
        return float(r[0])

    def linear_residual(self) -> float:
        """||(A + lambda I) x - b|| / ||b|| of the last solve, computed on the device."""
        r = np.zeros(1)
        _check(lib().g2ohip_solver_linear_residual(self.h, _p(r)), "linear_residual")
        return float(r[0])

    def compute_marginals(self, block_indices):
        """SparseOptimizer::computeMarginals(spinv, blockIndices) (sparse_optimizer.h:129): {(r, c): pd x pd block
        of Hpp^-1} for the Hessian block index pairs, or None when the factorization fails (the reference's false)."""
        pairs = [(int(r), int(c)) for r, c in block_indices]
        rows = np.ascontiguousarray([p[0] for p in pairs] or [0], np.int32)
        cols = np.ascontiguousarray([p[1] for p in pairs] or [0], np.int32)
        pd = self.block_dims()[0]
        out = np.zeros(max(len(pairs), 1) * pd * pd)
        rc = lib().g2ohip_solver_compute_marginals(self.h, len(pairs), _p(rows), _p(cols), _p(out))
        _check(min(rc, 0), "computeMarginals")
        if rc == 0:
            return None
        return {p: out[k * pd * pd:(k + 1) * pd * pd].reshape(pd, pd).T.copy() for k, p in enumerate(pairs)}

    FACTOR_INFO_KEYS = ("n", "nnzL", "flops", "supernodes", "levels", "max_front", "blocked_fronts",
                        "inplace_levels", "prescatter_levels", "syrk_launches", "bwd_rounds", None,
                        "owned_fronts", "shared_fronts", "subtree_roots", "root_exchange_doubles",
                        "model_rank_subtrees_s", "model_shared_s", "model_single_gpu_s", "model_exchange_s",
                        "distributed", "reduce_scatter", "rs_segment_doubles", "rs_tail_doubles", "model_input_s",
                        "model_input_allreduce_s", None,  # None: retired slots (always 0), kept for the ABI layout
                        "band_leaf", "aligned_shards", "local_block_doubles", "exchange_bytes_per_rank",
                        "local_landmarks", "model_shard_s", "deferred_l21_fronts")

    def factor_info(self) -> dict:
        out = np.zeros(len(self.FACTOR_INFO_KEYS))
        _check(lib().g2ohip_solver_factor_info(self.h, _p(out), len(out)), "factor_info")
        return {k: v for k, v in zip(self.FACTOR_INFO_KEYS, out.tolist()) if k is not None}

    def local_landmark_ids(self) -> np.ndarray:
        """Ids of the free landmarks this rank's shard holds (landmark sharding; all of them on one rank)."""
        n = _check(lib().g2ohip_local_landmarks(self.h, None, 0), "local_landmarks")
        ids = np.zeros(max(n, 1), np.int32)
        lib().g2ohip_local_landmarks(self.h, _p(ids), n)
        return ids[:n]

    def stage(self, lam: float):
        dims = np.zeros(3, np.int64)
        _check(lib().g2ohip_stage(self.h, 0.0, None, None, None, None, _p(dims)), "stage")
        n, npose = int(dims[0]), int(dims[1])
        b, x, H, bs = np.zeros(n), np.zeros(n), np.zeros((npose, npose)), np.zeros(npose)
        ok = _check(lib().g2ohip_stage(self.h, lam, _p(b), _p(x), _p(H), _p(bs), _p(dims)), "stage")
        return dict(ok=ok, b=b, x=x, Hschur=H, bschur=bs, n=n, np=npose, nl=int(dims[2]))

    # ---- multi-GPU ----
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_ubyte * 128)()
        _check(lib().g2ohip_comm_unique_id(buf), "comm_unique_id")
        return bytes(buf)

    @staticmethod
    def comm_selftest(values, device: int = 0):
        """RCCL binding smoke test on one device (one-rank communicator): allreduce sum, allreduce max and the
        in-place reduce-scatter sum (rank 0's segment), each over `values`."""
        v = np.ascontiguousarray(values, np.float64)
        out = np.zeros(2 * v.size)
        rs = np.zeros(v.size)
        uid = (C.c_ubyte * 128).from_buffer_copy(SparseOptimizer.comm_unique_id())
        _check(lib().g2ohip_comm_selftest_rs(device, uid, v.size, _p(v), _p(out), _p(rs)), "comm_selftest")
        return out[: v.size], out[v.size:], rs

    def set_comm(self, uid: bytes, rank: int, nranks: int):
        buf = (C.c_ubyte * 128).from_buffer_copy(uid)
        _check(lib().g2ohip_set_comm(self.h, buf, rank, nranks), "set_comm")

    def set_comm_local(self, group_key: str, rank: int, nranks: int):
        """In-process test transport (see g2ohip_set_comm_local); one host thread per rank."""
        _check(lib().g2ohip_set_comm_local(self.h, group_key.encode(), rank, nranks), "set_comm_local")

    # ---- measurement ----
    def enable_kernel_timing(self, on: bool = True, only: str | None = None):
        """Per-kernel-class HIP-event timing; ``only`` restricts it to one class."""
        lib().g2ohip_kernel_timing_only(self.h, (only or "").encode())
        lib().g2ohip_enable_kernel_timing(self.h, int(on))

    def set_stats_level(self, level: int):
        """G2OBatchStatistics timers: 0 none, 1 timeLinearSolution only, 2 every stage (default)."""
        lib().g2ohip_set_stats_level(self.h, int(level))

    def kernel_ms(self, name: str) -> float:
        return lib().g2ohip_kernel_ms(self.h, name.encode())

    def kernel_count(self, name: str) -> int:
        return lib().g2ohip_kernel_count(self.h, name.encode())

    def kernel_bytes(self, name: str) -> float:
        return lib().g2ohip_kernel_bytes(self.h, name.encode())

    def kernel_flops(self, name: str) -> float:
        return lib().g2ohip_kernel_flops(self.h, name.encode())
