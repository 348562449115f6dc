#!/bin/bash
# Dev A/B on the dense-front schedule: C4R (random covisibility, one 5982-column front) per env setting,
# factor ms and the kernel-time split of one rocprofv3-traced run.   bash tools/ab_dense.sh "A=1" "B=2" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for envs in "$@"; do
  k=$((k+1))
  rm -rf gpurun_out/dn$k
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dn$k -o run -- python bench.py --config C4R --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/dn$k.json 2> gpurun_out/dn$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/dn$k.err; exit 1; }
  python - "$envs" "$k" <<'PY'
import csv, json, sys
envs, k = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/dn{k}.json"))
s = d["stages_ms_avg"]
rows = list(csv.DictReader(open(f"gpurun_out/dn{k}/run_kernel_stats.csv")))
top = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:6]
print("==", envs, "it/s %.1f factor %.3f solve %.3f" % (d["value"], s["chol_factor"], s["chol_solve"]))
for r in top:
    print("   %-40s calls %6s total %8.2f ms avg %7.1f us" % (r["Name"][:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
PY
done
