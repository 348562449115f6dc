"""Dev measurement: C4 with random covisibility (SURVEY.md §8d "covis=random": every point seen by 10 of all 1000
cameras, so the reduced camera system is dense, 6000 x 6000). Stage times per LM iteration and the factor schedule.
    python tools/time_dense.py [CAMERAS [POINTS [ITERS]]]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import g2o_amd  # noqa: E402
from g2o_amd import synth  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
P = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
prob = synth.ba(C, P, window=C)
opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
t = time.perf_counter()
opt.optimize(1)
warm = time.perf_counter() - t
opt.enable_kernel_timing(True)
t = time.perf_counter()
n, st = opt.optimize(iters)
dt = time.perf_counter() - t
names = ["linearize", "vreduce", "schur_dinv", "schur_diag", "schur_rows", "chol_factor", "chol_solve", "backsub"]
trials = sum(s.levenbergIterations for s in st)
out = {"workload": prob.name, "iters": n, "trials": trials, "s_per_iter": dt / max(n, 1), "warmup_s": warm,
       "chi2": st[-1].chi2 if st else None,
       "ms_per_trial": {k: opt.kernel_ms(k) / max(opt.kernel_count(k), 1) for k in names},
       "factor": opt.factor_info()}
print(json.dumps(out))
