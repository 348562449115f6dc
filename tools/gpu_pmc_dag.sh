#!/bin/bash
# SQ counters of the tile-DAG factor and its sequential backward solve (one pass, one bench run)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pmcdag}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU --kernel-include-regex "k_dag|k_bwd_seq|k_step" --output-format csv -d gpurun_out/${TAG} -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 --no-kernel-timing > gpurun_out/${TAG}.log 2>&1 || { tail -20 gpurun_out/${TAG}.log; exit 1; }
python - <<PY
import csv, glob, collections
f = glob.glob('gpurun_out/${TAG}/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name'].split('(')[0].replace('g2ohip::', '').replace('void ', '')
    agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, d in agg.items():
    print(n, {k: round(sum(v) / len(v)) for k, v in sorted(d.items())})
PY
