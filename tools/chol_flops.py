"""Algorithmic flop count of the reduced-system Cholesky (sum_k c_k^2 under the reference's own
ordering) for every BASELINE config, written to profiles/chol_flops.json for bench.py's roofline.

The reference (LinearSolverCSparse with blockOrdering, linear_solver_csparse.h:246-308) orders the block pattern
with CSparse cs_amd; the counts come from the oracle (oracle/oracle.cpp oracle_block_symbolic) driving the
reference's vendored CSparse compiled from source (oracle/_ref). This runs in the development container (it
needs oracle/_ref); the committed JSON is what travels. The backend's own nested-dissection ordering is
reported beside it (g2o_amd.symbolic_analyze: supernodal flop count including relaxed-amalgamation zeros).

    python tools/chol_flops.py [C1 C2 C3 C4 C5]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.environ.get("ORACLE_DIR", os.path.join(ROOT, "oracle")))

import oracle_py  # noqa: E402
import g2o_amd  # noqa: E402
from g2o_amd import synth  # noqa: E402


def reduced_pattern(prob):
    """Upper block pattern (bi <= bj) of the matrix the linear solver factors: the Schur complement
    for BA (block_solver.hpp:216-251 Schur pattern), Hpp for pose graphs (:142-210)."""
    poses = prob.vertices[0]
    free = poses.fixed == 0
    hidx = np.full(int(poses.ids.max()) + 1, -1, np.int64)
    hidx[poses.ids[free]] = np.arange(int(free.sum()))
    npose = int(free.sum())
    e = prob.edges[0]
    if prob.landmark_dim:
        cams = hidx[e.v1]
        pts = e.v0 - e.v0.min()
        keep = cams >= 0
        cams, pts = cams[keep], pts[keep]
        order = np.lexsort((cams, pts))
        cams, pts = cams[order], pts[order]
        starts = np.flatnonzero(np.r_[True, pts[1:] != pts[:-1]])
        ends = np.r_[starts[1:], len(pts)]
        keys = []
        for k in np.unique(ends - starts):  # group points by observation count: vectorised pairs
            sel = starts[(ends - starts) == k]
            blk = cams[sel[:, None] + np.arange(k)[None, :]]  # [npoints_k, k] sorted camera indices
            iu, ju = np.triu_indices(k)
            keys.append((blk[:, iu] * npose + blk[:, ju]).ravel())
        keys = np.unique(np.concatenate(keys + [np.arange(npose) * (npose + 1)]))
    else:
        a, b = hidx[e.v0], hidx[e.v1]
        keep = (a >= 0) & (b >= 0)
        i, j = np.minimum(a[keep], b[keep]), np.maximum(a[keep], b[keep])
        keys = np.unique(np.concatenate([i * npose + j, np.arange(npose) * (npose + 1)]))
    return npose, (keys // npose).astype(np.int32), (keys % npose).astype(np.int32)


def main(names):
    assert oracle_py.ref_available(), "oracle/_ref (reference CSparse) not built: make -C oracle"
    path = os.environ.get("CHOL_FLOPS_OUT", os.path.join(ROOT, "profiles", "chol_flops.json"))
    out = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        prob = synth.by_name(name)
        nb, bi, bj = reduced_pattern(prob)
        bdim = prob.pose_dim
        lnz, fl = oracle_py.block_symbolic(nb, bdim, bi, bj, use_ref=True)
        _, st = g2o_amd.symbolic_analyze(nb, bdim, bi, bj)
        out[name] = {
            "workload": prob.name, "n": nb * bdim, "blocks_upper": int(len(bi)),
            "ref_cs_amd": {"nnzL": lnz, "flops": fl},
            "builder_nd": {"nnzL": st["nnzL"], "flops": st["flops"], "supernodes": st["supernodes"],
                           "levels": st["levels"]},
            "source": "tools/chol_flops.py (oracle_block_symbolic over oracle/_ref cs_amd; g2ohip_symbolic_analyze)",
        }
        print(name, json.dumps(out[name]), flush=True)
    json.dump(out, open(path, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or ["C1", "C2", "C3", "C4", "C5"])
