#!/bin/bash
# Dev: LDS / issue counters of the Schur row pass (C4 bench, k_schur_rows only), one PMC pass per counter group
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z_]*LDS[A-Z_]*\|SQ_WAVE_CYCLES\|SQ_BUSY_CYCLES\|SQ_WAIT_INST_ANY\|SQ_INSTS_VALU\b" gpurun_out/counters_list.txt | sort -u | head -40
k=0
for grp in "$@"; do
  k=$((k+1))
  rm -rf gpurun_out/pmcs$k
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_schur_rows" --output-format csv -d gpurun_out/pmcs$k -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 --no-kernel-timing > gpurun_out/pmcs$k.log 2>&1 || { echo PMC_FAIL "$grp"; tail -5 gpurun_out/pmcs$k.log; exit 1; }
  python - "$k" <<'PY'
import csv, glob, sys, collections
k = sys.argv[1]
f = glob.glob(f"gpurun_out/pmcs{k}/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
acc = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
disp = len(set(r["Dispatch_Id"] for r in rows))
print({c: round(v / disp) for c, v in acc.items()}, "dispatches", disp)
PY
done
