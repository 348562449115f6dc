"""Benchmark: LM iterations/sec (+ ms per linear solve) of the MI355X BlockSolver
backend on synthetic BA 1k cameras x 100k points x 1M observations (BASELINE
config C4), with landmarks sharded over N GPUs (RCCL all-reduce of the reduced
camera system) when launched with torch.distributed.run.

A "step" is one SparseOptimizer::optimize loop body = one LM outer iteration
(computeActiveErrors, buildSystem, >=1 trial of setLambda/solve/update/
restoreDiagonal/computeActiveErrors), all device-resident.  Inputs are resident
in HBM before the timed region.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6    # MI355X FP64 vector == FP64 matrix (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); N > 1 without a launcher spawns N ranks itself (default: "
                         "WORLD_SIZE under torch.distributed.run, else 1)")
    ap.add_argument("--dry-run", action="store_true",
                    help="control plane only (rank spawn, gloo barrier, max over ranks, JSON shape): no GPU call")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C4", help="C4 (default, BASELINE metric) or C5/C3/C2/C1; C4R (random covisibility), S2 (BlockSolver_3_2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-iters", type=int, default=6, help="timed oracle LM iterations (after iteration 0)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="OpenMP threads for the CPU baseline (0 = all)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-posegraph", action="store_true", help="skip the C3 (100k-pose SE3) secondary leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (4k x 1M x 10M BA) secondary leg")
    return ap.parse_args()


def make_problem(cfg):
    from g2o_amd import synth
    return synth.by_name(cfg)


def spawn_ranks(n, deadline_s=None):
    """`--gpus N` (N > 1) without a launcher: start N child ranks of this same command line, one process per GPU, with
    the torch.distributed.run environment (RANK / LOCAL_RANK / WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free port), and
    return the worst exit code. Runs before this process makes any HIP call (nothing here loads libg2o_hip.so). Rank
    0's stdout is this process's (it prints the one JSON line); the other ranks print nothing on stdout. If a rank
    fails, the others are terminated (by their own PIDs) so no rank is left waiting in a collective. A wall-clock
    deadline (G2OHIP_BENCH_DEADLINE seconds, default 1800) ends a job whose ranks hang: every rank is killed and the
    exit code is 124. The port is probed by bind-and-close, which can race with another process: a job whose ranks
    all fail within 30 s (the rendezvous) is retried once on a fresh port."""
    import socket
    import subprocess
    if deadline_s is None:
        deadline_s = float(os.environ.get("G2OHIP_BENCH_DEADLINE", "1800"))

    def attempt():
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        procs = []
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                          stdout=None if r == 0 else subprocess.DEVNULL))
        rc = 0
        t0 = time.monotonic()
        pending = set(range(n))
        while pending:
            if time.monotonic() - t0 > deadline_s:
                print(f"bench.py: deadline of {deadline_s:.0f} s passed; killing ranks {sorted(pending)}",
                      file=sys.stderr, flush=True)
                for q in pending:
                    procs[q].kill()
                for q in pending:
                    procs[q].wait()
                return 124, time.monotonic() - t0, False
            for r in sorted(pending):
                c = procs[r].poll()
                if c is None:
                    continue
                pending.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
                    for q in pending:
                        procs[q].terminate()
            time.sleep(0.05)
        return rc, time.monotonic() - t0, all(p.returncode != 0 for p in procs)

    rc, dt, all_failed = attempt()
    if rc != 0 and rc != 124 and all_failed and dt < 30:
        print("bench.py: every rank failed during start-up; retrying once on a fresh port", file=sys.stderr, flush=True)
        rc, _, _ = attempt()
    return rc


def dist_setup(n=None):
    """torch.distributed (gloo, CPU only) is the multi-process control plane: uid broadcast, barriers, max over
    ranks. libg2o_hip.so is loaded BEFORE torch so its HIP runtime and RCCL are /opt/rocm's (ROCm 7.2, the ones it
    was built against) and not the copies torch bundles; torch never touches the GPU here. `n` (the --gpus request)
    must equal the launcher's WORLD_SIZE: the line can never report fewer GPUs than asked for."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if n is not None and n != world:
        raise SystemExit(f"bench.py: --gpus {n} but WORLD_SIZE={world}")
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def allmax(v, world):
    if world <= 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_obj(obj, world):
    """Per-rank records, in rank order (gloo)."""
    if world <= 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def bcast_bytes(b, world):
    if world <= 1:
        return b
    import torch.distributed as dist
    obj = [b]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def cpu_model():
    """lscpu model name + logical CPU count of this host (BASELINE.md asks for both)."""
    model = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    if model is None and os.path.exists("/proc/cpuinfo"):
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    return {"model": model, "nproc": os.cpu_count()}


def _oracle_run(prob, iters, nthreads):
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle_py
    g = oracle_py.OracleGraph(prob)
    cfg = oracle_py.make_config(threads=nthreads, use_ref=True, block_ordering=True)
    n, st = g.optimize(iters + 1, cfg)
    timed = st[1:n]
    if not timed:
        return None, oracle_py
    t = sum(s.timeIteration for s in timed)
    lin = [s.timeLinearSolution / max(s.levenbergIterations, 1) for s in timed]
    return {"value": len(timed) / t, "iterations": len(timed), "ms_per_linear_solve": 1e3 * float(np.median(lin)),
            "chi2": timed[-1].chi2}, oracle_py


def cpu_grant():
    """The CPUs this process is granted (the baseline runs on all of them): the affinity mask, capped by a
    cgroup CPU quota (the GPU box grants a share of a larger host, so os.cpu_count() counts CPUs this job cannot use)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            parts = open(path).read().split()
            if path.endswith("cpu.max") and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif path.endswith("cfs_quota_us") and int(parts[0]) > 0:
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                quota = int(parts[0]) / per
            if quota:
                break
        except (OSError, ValueError, IndexError):
            continue
    cpus = aff if quota is None else max(1, min(aff, int(quota)))
    return {"cpus": cpus, "affinity": aff, "cgroup_quota": quota, "os_cpu_count": os.cpu_count()}


def cpu_baseline(prob, iters, threads, iters_1t=2):
    """The oracle (C++ restatement of BlockSolver + LM) with the reference's own CSparse (oracle/_ref,
    cs_amd block ordering + up-looking LL^T) timed on this host: OpenMP assembly/Schur on all granted
    cores (the reference forces OpenMP, CMakeLists.txt:146) and a 1-thread run; the factorization is
    single-threaded in both, as CSparse is."""
    grant = cpu_grant()
    nthreads = threads or grant["cpus"]
    multi, oracle_py = _oracle_run(prob, iters, nthreads)
    if multi is None:
        return None
    one, _ = _oracle_run(prob, iters_1t, 1)
    return {
        "value": multi["value"],
        "unit": "LM it/s",
        "cores": nthreads,
        "cpu_grant": grant,
        "kind": "port",
        "ms_per_linear_solve": multi["ms_per_linear_solve"],
        "one_thread": one,
        "host": cpu_model(),
        "ref_csparse": bool(oracle_py.ref_available()),
        "sample": f"{multi['iterations']} LM iterations ({nthreads} threads) and {one['iterations'] if one else 0} "
                  f"(1 thread), each after iteration 0, of the same {prob.name} problem: oracle C++ restatement of "
                  f"BlockSolver/Schur/LM with the reference's vendored CSparse 3.1.0 cs_amd(block)+LL^T "
                  f"({'loaded' if oracle_py.ref_available() else 'restated'}), single-threaded factorization as in "
                  f"the reference",
    }


def solver_name(prob):
    if prob.landmark_dim:
        return f"BlockSolver_{prob.pose_dim}_{prob.landmark_dim} + Schur"
    return f"BlockSolver_{prob.pose_dim}_{prob.pose_dim} (no Schur)"


def posegraph_leg(local, steps=5, warmup=1):
    """The metric's second workload (BASELINE config C3: 100k-pose SE3 pose graph, 500k edges,
    BlockSolver_6_6, no Schur), measured the same way on the same GPU: LM it/s, ms/linear-solve and the
    supernodal factorization's MFMA throughput against the FP64 peak."""
    import g2o_amd
    prob = make_problem("C3")
    opt = g2o_amd.SparseOptimizer(local).add_problem(prob)
    opt.set_algorithm("lm_hip_fix6_6")
    it = 0
    for _ in range(max(warmup, 1)):
        opt.optimize_step(it)
        it += 1
    opt.set_stats_level(0)  # (as the main leg: no statistics timings in the timed region)
    t0 = time.perf_counter()
    timed = []
    for _ in range(steps):
        timed.append(opt.optimize_step(it)[1])
        it += 1
    dt = time.perf_counter() - t0  # optimize_step returns after the trial's scalar readback: device idle
    opt.enable_kernel_timing(True, only="chol_factor")
    opt.set_stats_level(2)
    stage_st = []
    for _ in range(2):
        stage_st.append(opt.optimize_step(it)[1])
        it += 1
    fms = opt.kernel_ms("chol_factor")
    own = opt.kernel_flops("chol_factor")
    ref = load_json("chol_flops.json").get("C3", {}).get("ref_cs_amd", {}).get("flops")
    # C3's fronts are dense enough that the executed flops are what the MFMA pipes see: the primary figure is on them,
    # the reference-ordering count (sum c_k^2 of cs_amd) is reported beside it, labelled
    tf = own / (fms * 1e-3) / 1e12 if fms > 0 else 0.0
    tref = ref / (fms * 1e-3) / 1e12 if fms > 0 and ref else None
    lin = [1e3 * s.timeLinearSolution / max(s.levenbergIterations, 1) for s in stage_st]
    return {
        "workload": f"C3: {prob.name} ({prob.num_vertices} poses, {prob.num_edges} edges), {solver_name(prob)}",
        "value": steps / dt,
        "unit": "LM it/s",
        "ms_per_linear_solve": float(np.median(lin)),
        "steps": steps,
        "final_chi2": timed[-1].chi2,
        "factor": with_peaks({"bound": "mfma", "achieved": tf, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                   "frac": tf / PEAK_FP64_TFLOPS, "flops_per_launch": own,
                   "flops_convention": "executed (backend nested-dissection ordering, supernodal)",
                   "ref_order_flops": ref, "ref_order_convention": "reference cs_amd sum c_k^2",
                   "ref_order_achieved": tref,
                   "ref_order_frac": tref / PEAK_FP64_TFLOPS if tref is not None else None,
                   "avg_launch_ms": fms, "traffic": traffic_lookup("C3")("chol_factor")}),
    }


RANK_KEYS = ("distributed", "aligned_shards", "exchange_bytes_per_rank", "local_landmarks", "owned_fronts",
             "shared_fronts", "local_block_doubles", "rs_segment_doubles", "rs_tail_doubles", "root_exchange_doubles",
             "reduce_scatter")


def rank_record(opt, rank, local, stages=None):
    """What one rank saw: its device, the RCCL its communicator was built on, its landmark shard and its share of the
    distributed factorization (factor_info), and optionally its own stage times."""
    fi = opt.factor_info()
    rt = {}
    try:
        import g2o_amd
        rt = g2o_amd.runtime_info()
    except Exception as ex:  # reported, not fatal
        rt = {"error": repr(ex)}
    rec = {"rank": rank, "device": local, "rccl_version": rt.get("rccl_version"), "librccl": rt.get("librccl")}
    rec.update({k: fi.get(k) for k in RANK_KEYS})
    if stages is not None:
        rec["stages_ms_avg"] = stages
    return rec


def c5_leg(local, steps=10, warmup=2, rank=0, world=1):
    """BASELINE config C5 (4k cameras x 1M points x 10M observations), measured like the headline: LM it/s,
    ms/linear-solve, the factorization's time and its stage split. With N > 1 ranks this is the configuration BASELINE
    defines as "landmarks sharded over 8xMI355X": every rank holds all cameras and its landmark shard (aligned with the
    cut of the elimination tree), the reduced camera system meets in RCCL collectives over xGMI
    (block_solver.hpp:340-393 is the loop each shard runs), and the timed region is bracketed by a barrier + device sync
    on every rank, max over ranks."""
    import g2o_amd
    t0 = time.time()
    prob = make_problem("C5")
    gen = time.time() - t0
    opt = g2o_amd.SparseOptimizer(local).add_problem(prob)
    opt.set_algorithm("lm_hip_fix6_3")
    if world > 1:
        uid = g2o_amd.SparseOptimizer.comm_unique_id() if rank == 0 else None
        opt.set_comm(bcast_bytes(uid, world), rank, world)
    t0 = time.time()
    it = 0
    for _ in range(max(warmup, 1)):
        opt.optimize_step(it)
        it += 1
    warm_s = time.time() - t0
    opt.set_stats_level(0)  # (as the main leg: no statistics timings in the timed region)
    barrier(world)
    g2o_amd.device_synchronize(local)
    t0 = time.perf_counter()
    timed = []
    for _ in range(steps):
        timed.append(opt.optimize_step(it)[1])
        it += 1
    g2o_amd.device_synchronize(local)
    barrier(world)
    dt = allmax(time.perf_counter() - t0, world)
    names = ["linearize", "vreduce", "schur_rows", "chol_factor", "chol_solve", "backsub", "error", "oplus"]
    opt.enable_kernel_timing(True)
    opt.set_stats_level(2)
    stage_st = []
    for _ in range(2):
        stage_st.append(opt.optimize_step(it)[1])
        it += 1
    kt = {k: opt.kernel_ms(k) for k in names}
    ranks = allgather_obj(rank_record(opt, rank, local, kt), world)
    rows_bytes = opt.kernel_bytes("schur_rows")
    tr = traffic_lookup("C5") if world == 1 else (lambda *a: None)  # the PMC files are one-GPU measurements
    cf = load_json("chol_flops.json").get("C5", {}).get("ref_cs_amd", {}).get("flops")
    own = opt.kernel_flops("chol_factor")
    fms = kt["chol_factor"]
    lin = [1e3 * s.timeLinearSolution / max(s.levenbergIterations, 1) for s in stage_st]
    out = {
        "workload": f"C5: {prob.name} ({prob.num_vertices} vertices, {prob.num_edges} edges), {solver_name(prob)}, "
                    f"{int(prob.vertices[0].fixed.sum())} fixed cameras, "
                    + ("1 GPU" if world == 1 else f"landmarks sharded over {world} GPUs (RCCL)"),
        "value": steps / dt, "unit": "LM it/s", "n_gpus": world, "scaling": "strong", "steps": steps, "warmup": warmup,
        "ms_per_step": 1e3 * dt / steps, "ms_per_linear_solve": float(np.median(lin)),
        "levenberg_trials": sum(s.levenbergIterations for s in timed), "final_chi2": timed[-1].chi2,
        "stages_ms_avg": kt,
        "factor": with_peaks({"bound": "mfma", "avg_launch_ms": fms, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                              "ref_order_flops": cf, "backend_ordering_flops": own,
                              "achieved": (cf or own) / (fms * 1e-3) / 1e12 if fms > 0 else 0.0,
                              "frac": (cf or own) / (fms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS if fms > 0 else 0.0,
                              "backend_ordering_achieved": own / (fms * 1e-3) / 1e12 if fms > 0 else 0.0,
                              "traffic": tr("chol_factor"), "traffic_fetch_doubled": tr("chol_factor", "bytes_fetch_doubled")}),
        "generate_s": gen, "warmup_incl_structure_s": warm_s,
    }
    if world > 1:
        out["ranks"] = ranks
        out["comm"] = comm_record(ranks, world)
    if kt["schur_rows"] > 0:
        a = rows_bytes / (kt["schur_rows"] * 1e-3) / 1e9
        out["schur_rows"] = with_peaks({"bound": "hbm", "achieved": a, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                        "frac": a / PEAK_HBM_GBS, "algorithmic_bytes_per_launch": rows_bytes,
                                        "avg_launch_ms": kt["schur_rows"], "traffic": tr("schur_rows"),
                                        "traffic_fetch_doubled": tr("schur_rows", "bytes_fetch_doubled")})
    opt.close()
    return out


def comm_record(ranks, world):
    """The transport the ranks actually used: RCCL communicator size and the RCCL build each rank bound to."""
    vers = sorted({r.get("rccl_version") for r in ranks if r.get("rccl_version") is not None})
    return {"transport": "RCCL (ncclCommInitRank, one process per GPU)", "nranks": world, "ranks_reporting": len(ranks),
            "rccl_versions": vers, "librccl": sorted({r.get("librccl") for r in ranks if r.get("librccl")})}


def load_json(name):
    path = os.path.join(HERE, "profiles", name)
    try:
        return json.load(open(path)) if os.path.exists(path) else {}
    except Exception:
        return {}


def traffic_lookup(config):
    """PMC traffic per launch (tools/pmc_traffic.py output) for `config`: G2OHIP_TRAFFIC_JSON_<CONFIG>, else
    G2OHIP_TRAFFIC_JSON, else profiles/traffic_<config>.json, else profiles/traffic.json, whichever exists first and
    was measured on that workload (its _meta.config); null otherwise.
    traffic: the raw PMC bytes (FETCH_SIZE + WRITE_SIZE); traffic_fetch_doubled: with the guide's gfx950 half-count
    correction of FETCH_SIZE, which is exact only for 16-B/lane streaming reads."""
    data = {}
    for path in (os.environ.get(f"G2OHIP_TRAFFIC_JSON_{config}"), os.environ.get("G2OHIP_TRAFFIC_JSON"),
                 os.path.join(HERE, "profiles", f"traffic_{config.lower()}.json"),
                 os.path.join(HERE, "profiles", "traffic.json")):
        if not path or not os.path.exists(path):
            continue
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("_meta", {}).get("config", "C4") == config:
            data = d
            break

    def traffic(k, key="bytes_per_launch"):
        rec = data.get(k)
        if not isinstance(rec, dict):
            return None
        if key == "bytes_per_launch" and "bytes_fetch_doubled" not in rec:  # older file: only the doubled figure
            return (rec["fetch_size_kb_raw"] + rec["write_size_kb"]) * 1024.0
        if key == "bytes_fetch_doubled" and key not in rec:
            return rec.get("bytes_per_launch")
        return rec.get(key)
    return traffic


PEAKS_MEASURED = {}


def with_peaks(d):
    """Every roofline line against both peaks: the spec one (`peak`, `frac`) and the one measured on this GPU in this run
    (g2ohip_measure_peaks: HBM streaming copy, FP64 MFMA issue loop)."""
    if not PEAKS_MEASURED or not isinstance(d, dict):
        return d
    pm = PEAKS_MEASURED["hbm_copy_GBps"] if d.get("unit") == "GB/s" else PEAKS_MEASURED["fp64_mfma_TFps"]
    d["peak_measured"] = pm
    d["frac_measured"] = d["achieved"] / pm if pm > 0 else None
    return d


def stage_bytes(prob):
    """SURVEY.md §8d algorithmic bytes per launch of the assembly and Schur stages (BA configs):
    assembly: per edge 80 B read (meas 16, Omega 24, intrinsics 32, 2 ids 8) + 144 B Hpl written, per point 24 B
    read + 96 B (Hll, b_l) written, per camera 56 B read + 336 B (Hpp block, b_p) written;
    Schur: per point k*144 + 96 B read, 288 B per upper Hschur block written once.
    Omega and the intrinsics are counted once, not per edge, when every edge of the group holds the same record:
    the engine then stores and reads ONE shared record (EdgeData::ue), so those bytes never move."""
    if not prob.landmark_dim:
        return None
    cams, pts = prob.vertices
    es = prob.edges[0]
    ne = es.v0.size
    nc, npt = int((cams.fixed == 0).sum()), pts.ids.size
    info = np.asarray(es.info).reshape(ne, -1)
    par = np.asarray(es.params).reshape(ne, -1) if es.params is not None else None
    shared_info = bool(ne and (info == info[0]).all())
    shared_par = bool(ne and par is not None and (par == par[0]).all())
    per_edge = 16 + 8 + (0 if shared_info else 24) + (0 if shared_par else 32)
    asm = ne * (per_edge + 144) + npt * (24 + 96) + nc * (56 + 336)
    return {"assembly": asm, "schur_read": ne * 144 + npt * 96, "edge_read_bytes": per_edge,
            "shared_records": {"information": shared_info, "intrinsics": shared_par}}


METRIC = "LM iterations/sec + ms/linear-solve, synthetic BA 1k×100k at 1/2/4/8 GPUs"


def dry_run(args):
    """The multi-rank control plane without a GPU (tests/test_dist_cpu.py): ranks, barrier-bracketed max-over-ranks
    timing, per-rank records, and the JSON line's shape with value = null."""
    rank, world, local = dist_setup(args.gpus)
    barrier(world)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    barrier(world)
    dt = allmax(time.perf_counter() - t0, world)
    ranks = allgather_obj({"rank": rank, "device": local, "pid": os.getpid(),
                           "world_size_env": int(os.environ.get("WORLD_SIZE", "1"))}, world)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "LM it/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": 1e3 * dt, "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "none (dry run)",
                          "config": {"workload": f"{args.config} (dry run: no GPU call)",
                                     "parallelism": f"landmark-shard{world}" if world > 1 else "single"},
                          "dry_run": True, "ranks": ranks,
                          "comm": {"transport": "gloo control plane only", "nranks": world}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))  # before any HIP call: the children are the ranks
    if args.dry_run:
        return dry_run(args)
    import g2o_amd
    g2o_amd.lib()  # bind the ROCm 7.2 HIP runtime + RCCL first (dist_setup imports torch)
    rank, world, local = dist_setup(args.gpus)

    t0 = time.time()
    prob = make_problem(args.config)
    gen_s = time.time() - t0
    opt = g2o_amd.SparseOptimizer(local).add_problem(prob)
    pd, ldim = prob.pose_dim, prob.landmark_dim
    opt.set_algorithm(f"lm_hip_fix{pd}_{ldim}" if ldim else f"lm_hip_fix{pd}_{pd}")
    if world > 1:
        uid = g2o_amd.SparseOptimizer.comm_unique_id() if rank == 0 else None
        uid = bcast_bytes(uid, world)
        opt.set_comm(uid, rank, world)
    # device-wide synchronize in the product's own HIP runtime (the product does not use torch's)
    def sync():
        g2o_amd.device_synchronize(local)

    # warmup: iteration 0 builds the structure (symbolic analysis) and lambda0
    t0 = time.time()
    it = 0
    for _ in range(max(args.warmup, 1)):
        opt.optimize_step(it)
        it += 1
    warm_s = time.time() - t0
    # roofline kernel: the dominant dispatch chain, the supernodal factorization of the reduced system
    # (60 % of the C4 step), timed with HIP events on the engine's stream inside the timed region (only it:
    # every timed class adds two event records per launch to the stream)
    dom = "chol_factor"
    if not args.no_kernel_timing:
        opt.enable_kernel_timing(True, only=dom)
    # no G2OBatchStatistics timings in the timed region (each is a pair of event records per trial on the stream, a few
    # us of idle GPU each; the reference collects none by default): ms/linear-solve comes from the stage iterations below
    opt.set_stats_level(0)
    barrier(world)
    sync()
    t0 = time.perf_counter()
    timed = []
    for _ in range(args.steps):
        r, st = opt.optimize_step(it)
        timed.append(st)
        it += 1
    sync()
    barrier(world)
    dt = time.perf_counter() - t0
    dt = allmax(dt, world)
    value = args.steps / dt
    trials = sum(s.levenbergIterations for s in timed)
    avg_ms = opt.kernel_ms(dom)
    launches = opt.kernel_count(dom)

    # stage breakdown: two more (untimed) iterations with every kernel class and stage timer on
    names = ["linearize", "vreduce", "schur_dinv", "schur_diag", "schur_rows", "chol_factor", "chol_solve", "backsub",
             "error", "oplus"]
    if not args.no_kernel_timing:
        opt.enable_kernel_timing(True)
    opt.set_stats_level(2)
    stage_st = []
    for _ in range(2):
        stage_st.append(opt.optimize_step(it)[1])
        it += 1
    lin_ms = [1e3 * s.timeLinearSolution / max(s.levenbergIterations, 1) for s in stage_st]
    kt = {k: {"avg_ms": opt.kernel_ms(k), "count": opt.kernel_count(k)} for k in names}
    finfo = opt.factor_info()
    ranks = allgather_obj(rank_record(opt, rank, local, {k: v["avg_ms"] for k, v in kt.items()}), world)
    try:  # after the timed region: ~1 s of streaming copy and MFMA / VALU issue loops
        PEAKS_MEASURED.update(g2o_amd.measure_peaks(local))
    except Exception as ex:  # reported, not fatal
        PEAKS_MEASURED["error"] = repr(ex)

    # algorithmic flops of the factorization: sum_k c_k^2 under the REFERENCE ordering (cs_amd on the block
    # pattern), from tools/chol_flops.py (oracle/_ref, committed JSON); the backend's own
    # nested-dissection ordering count beside it
    cf = load_json("chol_flops.json").get(args.config, {})
    ref_flops = cf.get("ref_cs_amd", {}).get("flops")
    own_flops = finfo["flops"]
    traffic = traffic_lookup(args.config)

    flops = ref_flops if ref_flops else own_flops
    achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    roofline = {
        "kernel": dom,
        "bound": "mfma",
        "achieved": achieved,
        "peak": PEAK_FP64_TFLOPS,
        "unit": "TFLOP/s",
        "frac": achieved / PEAK_FP64_TFLOPS,
        "traffic": traffic(dom),
        "traffic_fetch_doubled": traffic(dom, "bytes_fetch_doubled"),
        "algorithmic_flops_per_launch": flops,
        "flops_convention": ("sum_k c_k^2 of the reference cs_amd block ordering (tools/chol_flops.py)" if ref_flops
                             else "backend ordering (reference count missing for this config)"),
        "backend_ordering_flops": own_flops,
        "backend_ordering_frac": own_flops / (avg_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS if avg_ms > 0 else 0.0,
        "avg_launch_ms": avg_ms,
        "launches_timed": launches,
    }
    secondary = []
    if prob.landmark_dim:
        sb = stage_bytes(prob)
        rows_bytes = opt.kernel_bytes("schur_rows")
        ms_rows = kt["schur_rows"]["avg_ms"]
        if ms_rows > 0:
            a = rows_bytes / (ms_rows * 1e-3) / 1e9
            secondary.append({"kernel": "schur_rows", "bound": "hbm", "achieved": a, "peak": PEAK_HBM_GBS,
                              "unit": "GB/s", "frac": a / PEAK_HBM_GBS, "traffic": traffic("schur_rows"),
                              "traffic_fetch_doubled": traffic("schur_rows", "bytes_fetch_doubled"),
                              "algorithmic_bytes_per_launch": rows_bytes, "avg_launch_ms": ms_rows})
        nsblk = cf.get("blocks_upper")
        split = kt["schur_diag"]["count"] == 0  # Schur split formed at assembly (the LM loop's first trials)
        if not split:
            ms_asm = kt["linearize"]["avg_ms"] + kt["vreduce"]["avg_ms"]
            if ms_asm > 0:
                a = sb["assembly"] / (ms_asm * 1e-3) / 1e9
                tr = [traffic(k) for k in ("linearize", "vreduce")]
                secondary.append({"kernel": "assembly (linearize + vertex reductions)", "bound": "hbm", "achieved": a,
                                  "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": a / PEAK_HBM_GBS,
                                  "traffic": sum(tr) if all(t is not None for t in tr) else None,
                                  "algorithmic_bytes_per_launch": sb["assembly"], "avg_launch_ms": ms_asm})
            ms_sch = kt["schur_dinv"]["avg_ms"] + kt["schur_diag"]["avg_ms"] + kt["schur_rows"]["avg_ms"]
            if ms_sch > 0 and nsblk:
                by = sb["schur_read"] + 288 * nsblk
                a = by / (ms_sch * 1e-3) / 1e9
                tr = [traffic(k) for k in ("schur_dinv", "schur_diag", "schur_rows")]
                secondary.append({"kernel": "schur stage (dinv + diag + rows)", "bound": "hbm", "achieved": a,
                                  "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": a / PEAK_HBM_GBS,
                                  "traffic": sum(tr) if all(t is not None for t in tr) else None,
                                  "algorithmic_bytes_per_launch": by, "avg_launch_ms": ms_sch})
        else:
            # the landmark pass and the diagonal Schur terms run inside the assembly kernels: one line for the
            # whole assembly + Schur stage against the sum of SURVEY 8d's algorithmic bytes of both stages
            ms_as = kt["linearize"]["avg_ms"] + kt["vreduce"]["avg_ms"] + kt["schur_rows"]["avg_ms"]
            if ms_as > 0 and nsblk:
                by = sb["assembly"] + sb["schur_read"] + 288 * nsblk
                a = by / (ms_as * 1e-3) / 1e9
                tr = [traffic(k) for k in ("linearize", "vreduce", "schur_rows")]
                td = [traffic(k, "bytes_fetch_doubled") for k in ("linearize", "vreduce", "schur_rows")]
                secondary.append({"kernel": "assembly + schur (split at assembly: linearize, camera pass, rows)",
                                  "bound": "hbm", "achieved": a, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                  "frac": a / PEAK_HBM_GBS,
                                  "traffic": sum(tr) if all(t is not None for t in tr) else None,
                                  "traffic_fetch_doubled": sum(td) if all(t is not None for t in td) else None,
                                  "edge_read_bytes": sb["edge_read_bytes"], "shared_records": sb["shared_records"],
                                  "algorithmic_bytes_per_launch": by, "avg_launch_ms": ms_as})
    runtime = g2o_amd.runtime_info()
    runtime["mapped"] = sorted({ln.split()[-1] for ln in open("/proc/self/maps")
                                if ("libamdhip64" in ln or "librccl" in ln) and "/" in ln})
    fixed = ""
    if prob.landmark_dim:
        fixed = f", {int(prob.vertices[0].fixed.sum())} fixed cameras (gauge + monocular scale; ba_demo.cpp fixes 1)"
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "LM it/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps,
        "ms_per_linear_solve": float(np.median(lin_ms)),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (numpy Philox seed 20261015, BAL-style recipe of ba_demo.cpp; SURVEY.md 8d)",
        "config": {
            "workload": f"{args.config}: {prob.name} ({prob.num_vertices} vertices, {prob.num_edges} edges), "
                        f"{solver_name(prob)}{fixed}" + (f", landmarks sharded over {world} GPU(s)" if prob.landmark_dim else ""),
            "levenberg_trials": trials,
            "final_chi2": timed[-1].chi2 if timed else None,
            "parallelism": f"landmark-shard{world}" if world > 1 else "single",
        },
        "stages_ms_avg": {k: v["avg_ms"] for k, v in kt.items()},  # 2 extra untimed iterations
        "roofline": with_peaks(roofline),
        "roofline_secondary": [with_peaks(d) for d in secondary],
        "peaks": {"spec": {"hbm_GBps": PEAK_HBM_GBS, "fp64_TFps": PEAK_FP64_TFLOPS,
                           "source": "MI355X_MICROARCH.md (spec)"},
                  "measured": dict(PEAKS_MEASURED, source="g2ohip_measure_peaks on this GPU, this run")},
        "factor": finfo,
        "setup_s": {"generate": gen_s, "warmup_incl_structure": warm_s},
        "runtime": runtime,
    }
    if rank == 0 and world == 1 and not args.no_posegraph and args.config == "C4":
        try:
            out["pose_graph"] = posegraph_leg(local)
        except Exception as ex:  # reported, not fatal
            out["pose_graph"] = {"error": repr(ex)}
    if world > 1:
        out["ranks"] = ranks
        out["comm"] = comm_record(ranks, world)
    if not args.no_c5 and args.config == "C4":
        # every rank: at N > 1 the C5 leg is the landmark-sharded multi-GPU configuration (its collectives need all)
        opt.close()
        if world == 1:
            try:
                out["c5"] = c5_leg(local)
            except Exception as ex:  # reported, not fatal
                out["c5"] = {"error": repr(ex)}
        else:  # a rank failing inside collectives cannot be reported around: let the launcher see it
            out["c5"] = c5_leg(local, rank=rank, world=world)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(prob, args.cpu_iters, args.cpu_threads)
        except Exception as ex:  # reported, not fatal
            out["cpu_baseline"] = {"error": repr(ex)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
