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
