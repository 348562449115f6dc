"""Dev measurement (§8f rank 2, the .g2o loader at scale): write a BASELINE config as a .g2o file through
g2ohip_save_g2o, read it back with g2ohip_load_g2o (the parallel chunked parser) and time both, checking the
vertex / edge counts and chi2 of the reloaded graph.   python tools/time_loader.py [CONFIG [PATH]]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import g2o_amd  # noqa: E402
from g2o_amd import synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C5"
path = sys.argv[2] if len(sys.argv) > 2 else "/tmp/g2ohip_%s.g2o" % name
t = time.perf_counter()
prob = synth.by_name(name)
gen_s = time.perf_counter() - t
a = g2o_amd.SparseOptimizer(0).add_problem(prob)
t = time.perf_counter()
a.save(path)
save_s = time.perf_counter() - t
size = os.path.getsize(path)
chi_a = a.chi2()
nv, ne = a.num_vertices(), a.num_edges()
a.close()
b = g2o_amd.SparseOptimizer(0)
t = time.perf_counter()
b.load(path, marginalize_xyz=True)
load_s = time.perf_counter() - t
ok = (b.num_vertices(), b.num_edges()) == (nv, ne)
chi_b = b.chi2()
print(json.dumps({"config": name, "file_bytes": size, "vertices": nv, "edges": ne, "generate_s": gen_s,
                  "save_s": save_s, "load_s": load_s, "load_MB_per_s": size / 1e6 / load_s,
                  "counts_match": ok, "chi2_written": chi_a, "chi2_reloaded": chi_b,
                  "cpus": os.cpu_count()}))
os.remove(path)
