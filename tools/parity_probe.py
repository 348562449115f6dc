import sys, time, os
R = __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, R + '/oracle')
import numpy as np
import g2o_amd, oracle_py
from g2o_amd import synth
def cmp(name, prob, iters=5):
    opt = g2o_amd.SparseOptimizer(0).add_problem(prob)
    c0 = opt.chi2()
    t=time.time(); n, st = opt.optimize(iters); dt=time.time()-t
    ref = oracle_py.OracleGraph(prob); nr, sr = ref.optimize(iters, oracle_py.make_config(threads=8))
    xg, xr = opt.minimal_state(), ref.minimal_state()
    rel = np.linalg.norm(xg-xr)/np.linalg.norm(xr)
    print(name, "chi0 %.8g"%c0, "gpu", [("%.10g"%s.chi2) for s in st], "\n   ref", [("%.10g"%s.chi2) for s in sr], "rel state %.2e"%rel, "t %.3f"%dt, flush=True)
print(g2o_amd.lib().g2ohip_version())
cmp("BA tiny", synth.ba(24, 600, 6, 12), 3)
cmp("C4s", synth.by_name("C4","small"))
cmp("C1s", synth.by_name("C1","small"))
cmp("C2s", synth.by_name("C2","small"))
cmp("C3s", synth.by_name("C3","small"))
cmp("C1", synth.by_name("C1"), 5)
