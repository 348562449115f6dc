"""Measured per-rank critical path of the landmark-sharded C5 iteration on ONE GPU.

For N = 2, 4, 8 ranks:
  1. the aligned landmark shards: N engines over the in-process transport build the structure (align_shards places each
     landmark on the rank owning its first-eliminated camera's subtree) and report the landmark ids they hold;
  2. each rank's sharded stages alone: the sub-problem of all cameras + that rank's landmarks runs on the GPU with the
     kernel timers on (linearize, camera pass, Schur rows, back-substitution, chi2, update) — the work that rank does
     between its collectives;
  3. each rank's factorization chain: G2OHIP_DIST_SIMULATE=r/N plays rank r of the aligned cut on the full problem
     (its subtrees + the shared top, exchanges no-ops) and times factor + solve.
Only the collectives are modelled (factor_info: the cut's root all-gather + x all-reduce, the tail all-reduce of the
reduced system). Prints progress on stderr and one JSON object on stdout (profiles/r05_dist_rank_times.json).
    python tools/dist_rank_times.py [--config C5] [--ranks 2,4,8]
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import uuid

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
STAGES = ["linearize", "vreduce", "schur_rows", "backsub", "error", "oplus"]


def shard_ids(config, n):
    sys.path.insert(0, ROOT)
    import g2o_amd
    from g2o_amd import synth
    prob = synth.by_name(config)
    key = uuid.uuid4().hex
    opts = [g2o_amd.SparseOptimizer(0).add_problem(prob) for _ in range(n)]
    for r, o in enumerate(opts):
        o.set_algorithm("lm_hip_fix6_3")
        o.set_comm_local(key, r, n)
    errs = []

    def body(r):
        try:
            opts[r].initialize_optimization()
            opts[r].build_structure()
        except Exception as ex:  # surfaced below
            errs.append(ex)
    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    ids = [o.local_landmark_ids().tolist() for o in opts]
    infos = [o.factor_info() for o in opts]
    for o in opts:
        o.close()
    return ids, infos


def run_child(code, env_extra=None):
    env = dict(os.environ)
    env.pop("G2OHIP_DIST_SIMULATE", None)
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-3000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def shard_stages(config, ids_path, rank):
    code = f"""
import sys, json
sys.path.insert(0, {ROOT!r})
import numpy as np
import g2o_amd
from g2o_amd import synth
ids = json.load(open({ids_path!r}))[{rank}]
prob = synth.landmark_subset(synth.by_name({config!r}), ids, "rank{rank}")
opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
opt.set_algorithm("lm_hip_fix6_3")
for it in range(2):
    opt.optimize_step(it)
opt.enable_kernel_timing(True)
for it in range(2, 5):
    opt.optimize_step(it)
print(json.dumps(dict(landmarks=len(ids), edges=int(prob.num_edges),
                      stages_ms={{k: opt.kernel_ms(k) for k in {STAGES!r}}})))
"""
    return run_child(code)


def factor_chain(config, sim):
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
opt.enable_kernel_timing(True, only="chol_factor")
for it in range(2, 5):
    opt.optimize_step(it)
f = opt.kernel_ms("chol_factor")
opt.enable_kernel_timing(True, only="chol_solve")
for it in range(5, 7):
    opt.optimize_step(it)
print(json.dumps(dict(factor_ms=f, solve_ms=opt.kernel_ms("chol_solve"), info=opt.factor_info())))
"""
    return run_child(code, {"G2OHIP_DIST_SIMULATE": sim} if sim else None)


def solo_rank(config, rank, n):
    """Rank `rank` of `n` as the product runs it: the full problem in one engine that plays that rank alone through the
    timing transport (set_comm_local("solo:...")): its aligned landmark shard, the GLOBAL Schur pattern and task lists,
    its subtrees + the shared top of the distributed factorization, every collective a no-op. Stage and factor / solve
    timers of that engine (the sums are partial, so its LM decisions are not meaningful; the kernels are the rank's)."""
    code = f"""
import sys, json
sys.path.insert(0, {ROOT!r})
import g2o_amd
from g2o_amd import synth
prob = synth.by_name({config!r})
opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
opt.set_algorithm("lm_hip_fix6_3")
opt.set_comm_local("solo:dist_rank_times", {rank}, {n})
def steps(a, b):
    for it in range(a, b):
        try:
            opt.optimize_step(it)
        except Exception:
            pass
steps(0, 2)
opt.enable_kernel_timing(True)
steps(2, 5)
st = {{k: opt.kernel_ms(k) for k in {STAGES!r}}}
opt.enable_kernel_timing(True, only="chol_factor")
steps(5, 8)
f = opt.kernel_ms("chol_factor")
opt.enable_kernel_timing(True, only="chol_solve")
steps(8, 10)
print(json.dumps(dict(landmarks=len(opt.local_landmark_ids()), stages_ms=st, factor_ms=f,
                      solve_ms=opt.kernel_ms("chol_solve"), info=opt.factor_info())))
"""
    return run_child(code)


def main_solo(a):
    """--solo: every rank measured on the product's own sharded engine (timing transport)."""
    res = {"config": a.config, "method": "solo transport: each rank's engine alone on one GPU, collectives no-ops",
           "by_ranks": {}}
    for n in [int(x) for x in a.ranks.split(",")]:
        per = []
        for r in range(n):
            m = solo_rank(a.config, r, n)
            i = m["info"]
            coll_ms = 1e3 * (i["model_exchange_s"] + i["model_input_s"])
            st = sum(m["stages_ms"].values())
            total = st + m["factor_ms"] + m["solve_ms"] + coll_ms
            per.append(dict(rank=r, landmarks=m["landmarks"], stages_ms=m["stages_ms"], factor_ms=m["factor_ms"],
                            solve_ms=m["solve_ms"], collectives_model_ms=coll_ms, total_ms=total,
                            exchange_bytes_per_rank=i["exchange_bytes_per_rank"], owned_fronts=i["owned_fronts"]))
            print(f"N={n} rank {r}: {m['landmarks']} landmarks, stages {st:.3f} ms "
                  f"({', '.join(f'{k} {v:.3f}' for k, v in m['stages_ms'].items())}), factor {m['factor_ms']:.3f} + "
                  f"solve {m['solve_ms']:.3f} ms, collectives (model) {coll_ms:.3f} ms -> {total:.3f} ms",
                  file=sys.stderr, flush=True)
        res["by_ranks"][str(n)] = {"per_rank": per, "max_rank_total_ms": max(p["total_ms"] for p in per),
                                   "max_rank_stages_ms": max(sum(p["stages_ms"].values()) for p in per),
                                   "max_rank_schur_rows_ms": max(p["stages_ms"]["schur_rows"] for p in per),
                                   "max_rank_factor_ms": max(p["factor_ms"] for p in per)}
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--tmp", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--solo", action="store_true", help="measure each rank on the product's sharded engine")
    a = ap.parse_args()
    if a.solo:
        return main_solo(a)
    os.makedirs(a.tmp, exist_ok=True)
    single = factor_chain(a.config, None)
    full = shard_stages_full(a.config, a.tmp)
    print(f"single GPU: factor {single['factor_ms']:.3f} ms, solve {single['solve_ms']:.3f} ms, stages "
          f"{sum(full['stages_ms'].values()):.3f} ms", file=sys.stderr, flush=True)
    res = {"config": a.config, "single_gpu": {"factor": single, "stages": full}, "by_ranks": {}}
    for n in [int(x) for x in a.ranks.split(",")]:
        ids, infos = shard_ids(a.config, n)
        ids_path = os.path.join(a.tmp, f"dist_ids_{a.config}_{n}.json")
        json.dump(ids, open(ids_path, "w"))
        per = []
        for r in range(n):
            st = shard_stages(a.config, ids_path, r)
            fc = factor_chain(a.config, f"{r}/{n}")
            i = fc["info"]
            coll_ms = 1e3 * (i["model_exchange_s"] + i["model_input_s"])
            total = sum(st["stages_ms"].values()) + fc["factor_ms"] + fc["solve_ms"] + coll_ms
            per.append(dict(rank=r, landmarks=st["landmarks"], edges=st["edges"], stages_ms=st["stages_ms"],
                            factor_ms=fc["factor_ms"], solve_ms=fc["solve_ms"], collectives_model_ms=coll_ms,
                            exchange_bytes_per_rank=infos[r]["exchange_bytes_per_rank"],
                            owned_fronts=infos[r]["owned_fronts"], aligned_shards=infos[r]["aligned_shards"],
                            distributed=infos[r]["distributed"], total_ms=total))
            print(f"N={n} rank {r}: {st['landmarks']} landmarks, stages {sum(st['stages_ms'].values()):.3f} ms, factor "
                  f"{fc['factor_ms']:.3f} + solve {fc['solve_ms']:.3f} ms, collectives (model) {coll_ms:.3f} ms -> "
                  f"{total:.3f} ms", file=sys.stderr, flush=True)
        res["by_ranks"][str(n)] = {"per_rank": per, "max_rank_total_ms": max(p["total_ms"] for p in per),
                                   "max_rank_stages_ms": max(sum(p["stages_ms"].values()) for p in per),
                                   "max_rank_factor_ms": max(p["factor_ms"] for p in per)}
    print(json.dumps(res))


def shard_stages_full(config, tmp):
    """The single-GPU reference: the same stage timers on the whole problem."""
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
for it in range(2, 5):
    opt.optimize_step(it)
print(json.dumps(dict(stages_ms={{k: opt.kernel_ms(k) for k in {STAGES!r}}})))
"""
    return run_child(code)


if __name__ == "__main__":
    main()
