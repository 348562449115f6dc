"""Measured per-rank factorization time of the distributed factorization on ONE GPU.

For each rank r of N, one process plays rank r (G2OHIP_DIST_SIMULATE=r/N: its own subtrees + the shared top, the
exchanges no-ops) on the full C5 problem and times the factor + solve kernel chains with HIP events; the single-GPU
factorization is timed beside it. The trajectories of the simulated runs are not meaningful (the exchanged parts are
missing); only the kernel chains' durations are. Prints one JSON line.

    python tools/dist_factor_time.py [--config C5] [--ranks 8]
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def one(config, sim):
    code = f"""
import sys, json
sys.path.insert(0, {ROOT!r})
import g2o_amd
from g2o_amd import synth
prob = synth.by_name({config!r})
opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
opt.set_algorithm("lm_hip_fix6_3")
for it in range(2):
    opt.optimize_step(it)
opt.enable_kernel_timing(True)
for it in range(2, 6):
    opt.optimize_step(it)
info = opt.factor_info()
print(json.dumps(dict(factor_ms=opt.kernel_ms("chol_factor"), solve_ms=opt.kernel_ms("chol_solve"), info=info)))
"""
    env = dict(os.environ)
    env.pop("G2OHIP_DIST_SIMULATE", None)
    if sim:
        env["G2OHIP_DIST_SIMULATE"] = sim
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--ranks", type=int, default=8)
    a = ap.parse_args()
    res = {"config": a.config, "ranks": a.ranks, "single": one(a.config, None), "per_rank": []}
    for r in range(a.ranks):
        res["per_rank"].append(one(a.config, f"{r}/{a.ranks}"))
        print(f"rank {r}: factor {res['per_rank'][-1]['factor_ms']:.3f} ms", file=sys.stderr, flush=True)
    res["max_rank_factor_ms"] = max(x["factor_ms"] for x in res["per_rank"])
    res["max_rank_solve_ms"] = max(x["solve_ms"] for x in res["per_rank"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
