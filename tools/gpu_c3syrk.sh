#!/bin/bash
# Dev: C3 kernel trace; per k_syrk launch its workgroup count and duration (tail-effect analysis)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/c3tr
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3tr -o run -- python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-posegraph > gpurun_out/c3tr.json 2> gpurun_out/c3tr.err || { echo FAIL; tail -5 gpurun_out/c3tr.err; exit 1; }
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/c3tr/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# last factorization: from the last k_chol_scatter / k_vec_init to the next k_bwd_gemv
idx = [i for i, r in enumerate(rows) if "k_vec_init" in r["Kernel_Name"]]
a = idx[-1]
b = next(i for i in range(a, len(rows)) if "k_bwd_gemv" in rows[i]["Kernel_Name"])
seg = rows[a:b]
tot = collections.defaultdict(float)
hist = []
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("g2ohip::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[n] += d
    if n.startswith("k_syrk"):
        wg = int(r.get("Grid_Size", r.get("Grid_Size_X", 0))) // int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 256)))
        hist.append((wg, d))
print({k: round(v) for k, v in tot.items()}, "span us", (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3)
hist.sort(key=lambda x: -x[1])
print("k_syrk launches", len(hist), "total us", round(sum(d for _, d in hist)))
for wg, d in hist[:40]:
    print("  wg %6d  us %8.1f  rounds %.2f" % (wg, d, wg / 1024))
PY
