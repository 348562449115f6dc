"""The distributed factorization's cut model (plan_distribution, symbolic.cpp) for a BASELINE config at
N = 2, 4, 8 ranks, on the host (no GPU): per N the cut's slowest rank's subtrees, the shared top, the root all-gather +
x all-reduce, the input exchange, against the replicated factorization with its whole-S all-reduce.
    python tools/dist_model.py C5 [C4 ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

import g2o_amd  # noqa: E402
from g2o_amd import synth  # noqa: E402
from chol_flops import reduced_pattern  # noqa: E402


def main(names):
    out = {}
    for name in names:
        prob = synth.by_name(name)
        nb, bi, bj = reduced_pattern(prob)
        # per pose its observations of free landmarks x the sharded work per observation (dist_cost::OBS_S)
        poses = prob.vertices[0]
        free = poses.fixed == 0
        hidx = np.full(int(poses.ids.max()) + 1, -1, np.int64)
        hidx[poses.ids[free]] = np.arange(int(free.sum()))
        cams = hidx[prob.edges[0].v1]
        pw = np.bincount(cams[cams >= 0], minlength=nb).astype(np.float64) * 0.3e-9
        rows = {}
        for n in (2, 4, 8):
            d, owner = g2o_amd.dist_plan(nb, prob.pose_dim, bi, bj, n, pose_work=pw)
            subtrees = sorted({int(o) for o in owner if o >= 0})
            d["subtree_ranks"] = len(subtrees)
            d["shared_fronts"] = int((owner < 0).sum())
            d["cut_total_s"] = (d["max_rank_subtrees_s"] + d["shared_s"] + d["exchange_s"] + d["input_s"] +
                                d["shard_s"])
            rows[n] = d
            print(f"{name} N={n}: cut {d['cut_total_s'] * 1e3:.3f} ms (slowest rank {d['max_rank_subtrees_s'] * 1e3:.3f}, "
                  f"shared {d['shared_s'] * 1e3:.3f}, exchanges {d['exchange_s'] * 1e3:.3f}, input {d['input_s'] * 1e3:.3f}, "
                  f"sharded work {d['shard_s'] * 1e3:.3f}; "
                  f"{d['subtree_ranks']} ranks own subtrees, {d['shared_fronts']} shared fronts, root all-gather "
                  f"{d['root_allgather_doubles'] / 1e6:.2f} M doubles per rank) vs replicated "
                  f"{d['replicated_s'] * 1e3:.3f} ms; distributed={int(d['distributed'])}", flush=True)
        out[name] = rows
    if os.environ.get("DIST_MODEL_OUT"):
        json.dump(out, open(os.environ["DIST_MODEL_OUT"], "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or ["C5"])
