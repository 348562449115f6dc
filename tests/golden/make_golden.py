"""Generate the golden fixtures in tests/golden/ (run in the development container, where
oracle/_ref — the reference's vendored CSparse compiled from /root/reference — is available).

Fixtures are data only: the problem recipe (synth.py call + seed), the oracle's LM trajectory
(chi2 / lambda / trials per iteration) and final minimal state computed with the REFERENCE CSparse
(cs_amd block ordering + cs_chol), and reference-CSparse solutions of small SPD systems.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle_py  # noqa: E402
from g2o_amd import synth  # noqa: E402

# (name, synth call, LM iterations)
CASES = [
    ("ba_tiny", "ba(12, 200, 5, 8)", 6),
    ("sphere_tiny", "sphere(6, 6)", 6),
    ("se2_tiny", "se2_grid(200)", 6),
    ("sphere_lap2_tiny", "sphere(8, 8, extra_lap2=True)", 6),
]


def make_trajectories():
    assert oracle_py.ref_available(), "build oracle/_ref first (make -C oracle)"
    for name, call, iters in CASES:
        prob = eval("synth." + call)
        g = oracle_py.OracleGraph(prob)
        chi0 = g.chi2()
        n, st = g.optimize(iters, oracle_py.make_config(threads=1, use_ref=True, block_ordering=True))
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"),
            recipe=np.array(call), seed=np.array(synth.SEED), iterations=np.array(n), chi2_0=np.array(chi0),
            chi2=np.array([s.chi2 for s in st[:n]]), lam=np.array([s.lambda_ for s in st[:n]]),
            trials=np.array([s.levenbergIterations for s in st[:n]]), state=g.minimal_state())
        print(name, n, chi0, st[n - 1].chi2)


def make_ccs():
    rng = np.random.default_rng(11)
    out = {}
    for k, (n, dens) in enumerate([(1, 1.0), (6, 0.5), (30, 0.15), (120, 0.05)]):
        A = np.zeros((n, n))
        m = rng.random((n, n)) < dens
        A[m] = rng.standard_normal(m.sum())
        A = A @ A.T + n * np.eye(n)
        Ap, Ai, Ax = [0], [], []
        for j in range(n):
            rows = np.nonzero(A[: j + 1, j])[0]
            Ai += rows.tolist()
            Ax += A[rows, j].tolist()
            Ap.append(len(Ai))
        b = rng.standard_normal(n)
        ok, x = oracle_py.ccs_cholsol(n, np.array(Ap), np.array(Ai), np.array(Ax), b, mode=2)  # reference cs_cholsol
        assert ok == 1
        out.update({f"n{k}": np.array(n), f"Ap{k}": np.array(Ap), f"Ai{k}": np.array(Ai), f"Ax{k}": np.array(Ax),
                    f"b{k}": b, f"x{k}": x})
    np.savez_compressed(os.path.join(HERE, "csparse_cholsol.npz"), count=np.array(4), **out)


if __name__ == "__main__":
    make_trajectories()
    make_ccs()
    json.dump({"generator": "tests/golden/make_golden.py", "seed": synth.SEED,
               "cases": [c[0] for c in CASES] + ["csparse_cholsol"]},
              open(os.path.join(HERE, "MANIFEST.json"), "w"), indent=1)
