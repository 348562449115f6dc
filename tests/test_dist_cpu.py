"""world_size-2 gloo tests of the multi-rank path on CPU (no GPU).

* bench.py's control plane (uid broadcast, barrier, max-over-ranks timing) over gloo.
* The landmark-sharding decomposition the device engine relies on: the Schur complements of the
  landmark shards, each built by the oracle on its own sub-problem and summed across ranks with
  a gloo all-reduce (the RCCL all-reduce's stand-in), equal the full reduced camera system —
  once the per-shard lambda on the camera diagonal (added on rank 0 only by the engine) is
  accounted for.  Same for chi2 (sum of shard chi2s).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

LAM = 1e-3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch

    import bench
    import oracle_py
    from g2o_amd import synth

    r, w, loc = bench.dist_setup(world)
    assert (r, w, loc) == (rank, world, rank)
    uid = bench.bcast_bytes(bytes([7] * 128) if rank == 0 else None, w)
    assert uid == bytes([7] * 128)
    bench.barrier(w)
    assert bench.allmax(float(rank + 1), w) == float(world)

    prob = synth.by_name("C4", "small")
    sub = synth.landmark_shard(prob, rank, world)
    g = oracle_py.OracleGraph(sub)
    st = g.stage(LAM)
    H = torch.from_numpy(st["Hschur"].copy())
    b = torch.from_numpy(st["bschur"].copy())
    c = torch.tensor([g.chi2()], dtype=torch.float64)
    for t in (H, b, c):
        dist.all_reduce(t)
    if rank == 0:
        np.savez(os.path.join(outdir, "sum.npz"), H=H.numpy(), b=b.numpy(), c=c.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_landmark_shard_reduction(oracle, tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from g2o_amd import synth
    prob = synth.by_name("C4", "small")
    full = oracle.OracleGraph(prob)
    ref = full.stage(LAM)
    got = np.load(tmp_path / "sum.npz")
    H = got["H"] - (world - 1) * LAM * np.eye(ref["np"])  # lambda once, not once per shard
    assert np.linalg.norm(H - ref["Hschur"]) <= 1e-12 * np.linalg.norm(ref["Hschur"])
    assert np.linalg.norm(got["b"] - ref["bschur"]) <= 1e-12 * np.linalg.norm(ref["bschur"])
    assert abs(got["c"][0] - full.chi2()) <= 1e-12 * full.chi2()


def test_landmark_shard_partition():
    from g2o_amd import synth
    prob = synth.by_name("C4", "small")
    for n in (1, 2, 3, 8):
        subs = [synth.landmark_shard(prob, r, n) for r in range(n)]
        assert sum(s.num_edges for s in subs) == prob.num_edges
        ids = np.concatenate([s.vertices[1].ids for s in subs])
        assert np.array_equal(ids, prob.vertices[1].ids)


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


def test_bench_spawns_ranks_dry_run():
    """`bench.py --gpus 2` without a launcher starts two ranks itself (before any HIP call) and the line reports
    n_gpus 2 with one record per rank; --dry-run stops before the GPU."""
    p, out = _run_bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out is not None and out["dry_run"] is True
    assert out["n_gpus"] == 2
    assert [r["rank"] for r in out["ranks"]] == [0, 1]
    assert [r["device"] for r in out["ranks"]] == [0, 1]
    assert len({r["pid"] for r in out["ranks"]}) == 2
    assert all(r["world_size_env"] == 2 for r in out["ranks"])
    assert out["config"]["parallelism"] == "landmark-shard2"
    assert out["ms_per_step"] >= 20.0  # max over ranks: rank 1 sleeps 20 ms inside the bracketed region
    for k in ("metric", "unit", "steps", "warmup", "higher_is_better", "scaling", "vs_baseline", "dtype", "data"):
        assert k in out
    assert out["steps"] == 3 and out["warmup"] == 1


def test_bench_single_rank_dry_run():
    p, out = _run_bench(["--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["n_gpus"] == 1 and len(out["ranks"]) == 1


def test_bench_refuses_world_mismatch():
    """Under a launcher whose WORLD_SIZE differs from --gpus the bench refuses instead of reporting the wrong N."""
    p, out = _run_bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and out is None
    assert "WORLD_SIZE=1" in p.stderr
