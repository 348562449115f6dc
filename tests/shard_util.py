"""Shared helper of the sharded tests: the whole state of a landmark-sharded run gathered from its ranks."""
import numpy as np


def gather_sharded_state(prob, opts):
    """Cameras from rank 0 (identical on every rank), each free landmark from the rank whose shard holds it
    (g2ohip_local_landmarks: the shards follow the distributed factorization's cut, or are contiguous ranges of the
    landmark order). Returns (state, per-rank states); checks that no landmark is held twice."""
    C = prob.vertices[0].ids.size
    ids = np.asarray(prob.vertices[1].ids)
    order = np.argsort(ids, kind="stable")
    states = [o.minimal_state() for o in opts]
    out = states[0].copy()
    seen = np.zeros(ids.size, np.int32)
    for r, o in enumerate(opts):
        lid = o.local_landmark_ids()
        k = order[np.searchsorted(ids, lid, sorter=order)]
        assert np.array_equal(ids[k], lid), "unknown landmark id in a shard"
        seen[k] += 1
        rows = (6 * C + 3 * k[:, None] + np.arange(3)[None, :]).ravel()
        out[rows] = states[r][rows]
    assert seen.max(initial=0) <= 1, "a landmark held by two shards"
    return out, states
