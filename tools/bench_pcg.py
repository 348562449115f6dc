"""Dev measurement: LM with the GPU iterative linear solvers — g2o's block-Jacobi PCG on S (lm_pcg6_3) and the
fork's matrix-free CGLS on J (lm_pcg6_3_eigen) — vs the Cholesky (lm_hip_fix6_3) on a BASELINE config.
Not the bench.py contract line; prints one JSON line per algorithm.
    python tools/bench_pcg.py [CONFIG [ITERS [ALGO...]]]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import g2o_amd  # noqa: E402
from g2o_amd import synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
prob = synth.by_name(name)
algos = sys.argv[3:] or ["lm_hip_fix6_3", "lm_pcg6_3", "lm_pcg6_3_eigen"]
for algo in algos:
    opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
    opt.set_algorithm(algo)
    opt.initialize_optimization()
    opt.optimize_step(0)  # iteration 0: structure, symbolic analysis, λ init (untimed)
    st = []
    t = time.perf_counter()
    for i in range(1, iters + 1):
        st.append(opt.optimize_step(i)[1])
    dt = time.perf_counter() - t
    print(json.dumps({"config": name, "algorithm": algo, "iterations": iters,
                      "levenberg_trials": int(sum(s.levenbergIterations for s in st)),
                      "ms_per_iteration": 1e3 * dt / iters, "final_chi2": st[-1].chi2,
                      "linear_iterations_last_solve": opt.linear_iterations() if algo != "lm_hip_fix6_3" else None}),
          flush=True)
    opt.close()
