"""Measured per-rank factorization time of the distributed factorization on ONE GPU.

For each rank r of N, one process plays rank r (G2OHIP_DIST_SIMULATE=r/N: its own subtrees + the shared top, the
exchanges no-ops) on the full C5 problem and times the factor + solve kernel chains with HIP events; the single-GPU
factorization is timed beside it. The trajectories of the simulated runs are not meaningful (the exchanged parts are
missing); only the kernel chains' durations are. Prints one JSON line.

    python tools/dist_factor_time.py [--config C5] [--ranks 8[,4,2]]

Beside the measured times each run reports the setup's cost model (factor_info: model_rank_subtrees_s + model_shared_s
for the rank, model_single_gpu_s for the replicated factorization, model_exchange_s for the two all-reduces it adds),
the calibration data of engine.hpp's dist_cost constants.
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
    ap.add_argument("--ranks", default="8")
    a = ap.parse_args()
    res = {"config": a.config, "single": one(a.config, None), "by_ranks": {}}
    for n in [int(x) for x in a.ranks.split(",")]:
        d = {"per_rank": []}
        for r in range(n):
            d["per_rank"].append(one(a.config, f"{r}/{n}"))
            i = d["per_rank"][-1]["info"]
            print(f"N={n} rank {r}: factor {d['per_rank'][-1]['factor_ms']:.3f} ms, model "
                  f"{1e3 * (i['model_rank_subtrees_s'] + i['model_shared_s']):.3f} ms (+ exchange "
                  f"{1e3 * i['model_exchange_s']:.3f}; replicated model {1e3 * i['model_single_gpu_s']:.3f})",
                  file=sys.stderr, flush=True)
        d["max_rank_factor_ms"] = max(x["factor_ms"] for x in d["per_rank"])
        d["max_rank_solve_ms"] = max(x["solve_ms"] for x in d["per_rank"])
        res["by_ranks"][str(n)] = d
    print(json.dumps(res))


if __name__ == "__main__":
    main()
