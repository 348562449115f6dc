#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "G2OHIP_SYRK_SPLIT=0" "G2OHIP_SYRK_SPLIT=1"; do
rm -rf gpurun_out/sptr
env $e timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sptr -o run -- python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-posegraph > gpurun_out/sptr.json 2> gpurun_out/sptr.err || { echo FAIL; tail -5 gpurun_out/sptr.err; exit 1; }
echo "== $e"
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/sptr/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_vec_init" in r["Kernel_Name"]]
a = idx[-1]
b = next(i for i in range(a, len(rows)) if "k_bwd_gemv" in rows[i]["Kernel_Name"])
seg = rows[a:b]
tot = collections.defaultdict(float)
for i, r in enumerate(seg):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("g2ohip::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[n] += d
    if "split" in n or "reduce" in n or (n.startswith("k_syrk") and d > 400):
        wg = int(r.get("Grid_Size", 0)) // 256
        print("  %-16s wg %6d us %8.1f" % (n, wg, d))
print({k: round(v) for k, v in tot.items()}, "span us", (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3)
PY
done
