"""Full-size BASELINE fixtures (C2, C3, C4, C5, and C4R: C4 with random covisibility, a dense reduced camera system)
for the -m gpu parity tests.

Every fixture of a config bench.py times covers exactly the iterations it runs: C4 30 (iteration 0 with the
structure, then 29 more: the driver runs --warmup 5 --steps 20, the default is 5 + 30 minus the untimed stage
iterations), C3 8 (posegraph_leg: 1 warmup + 5 timed + 2 factor-timer iterations), C5 14 (c5_leg: 2 warmup + 10
timed + 2 stage-timer iterations); C2 6, C4R 3.

Run in the development container, where oracle/_ref (the reference's vendored CSparse compiled
from /root/reference) is available.  Each fixture is data only: the synth recipe, the oracle's LM
trajectory (chi2 / lambda / trials per iteration, reference CSparse cs_amd block ordering +
cs_chol) and the final minimal state (C2, C3: the whole state; C5: the cameras, a fixed stride of
the points and per-chunk sums of all point coordinates, to keep the file small).

    python tests/golden/make_fullsize.py C2 C3 C4 C5 C4R
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_py  # noqa: E402
from g2o_amd import synth  # noqa: E402

# name -> LM iterations recorded
ITERS = {"C2": 6, "C3": 8, "C4": 30, "C5": 14, "C4R": 3}
C5_POINT_STRIDE = 97      # every 97th point's coordinates stored exactly
C5_CHUNK = 4096           # per-chunk sums of the point block of the minimal state


def compact_state(name, prob, state):
    if name != "C5":
        return {"state": state}
    ncam = prob.vertices[0].ids.size
    cams = state[: 6 * ncam]
    pts = state[6 * ncam:].reshape(-1, 3)
    nch = (pts.shape[0] + C5_CHUNK - 1) // C5_CHUNK
    sums = np.array([pts[c * C5_CHUNK:(c + 1) * C5_CHUNK].sum(axis=0) for c in range(nch)])
    return {"cams": cams, "pts_strided": pts[::C5_POINT_STRIDE].copy(), "pts_chunk_sums": sums,
            "stride": np.array(C5_POINT_STRIDE), "chunk": np.array(C5_CHUNK)}


def make(name, threads):
    assert oracle_py.ref_available(), "build oracle/_ref first (make -C oracle)"
    t0 = time.time()
    prob = synth.by_name(name)
    g = oracle_py.OracleGraph(prob)
    chi0 = g.chi2()
    iters = ITERS[name]
    n, st = g.optimize(iters, oracle_py.make_config(threads=threads, use_ref=True, block_ordering=True))
    state = g.minimal_state()
    np.savez_compressed(
        os.path.join(HERE, f"{name.lower()}_full.npz"),
        config=np.array(name), seed=np.array(synth.SEED), iterations=np.array(n), chi2_0=np.array(chi0),
        chi2=np.array([s.chi2 for s in st[:n]]), lam=np.array([s.lambda_ for s in st[:n]]),
        trials=np.array([s.levenbergIterations for s in st[:n]]), state_norm=np.array(np.linalg.norm(state)),
        state_len=np.array(state.size), **compact_state(name, prob, state))
    print(name, "iters", n, "chi2_0", chi0, "chi2", [s.chi2 for s in st[:n]],
          "trials", [s.levenbergIterations for s in st[:n]],
          "t_iter", [round(s.timeIteration, 2) for s in st[:n]], "total_s", round(time.time() - t0, 1), flush=True)


if __name__ == "__main__":
    for nm in sys.argv[1:] or ["C2", "C3", "C4", "C5"]:
        make(nm, threads=int(os.environ.get("ORACLE_THREADS", "8")))
