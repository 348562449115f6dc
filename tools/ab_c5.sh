#!/bin/bash
# Dev A/B at C5: profiled short C5 bench per env setting ("A=1 B=2" per argument); it/s and the per-level factor breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for envs in "$@"; do
  k=$((k+1))
  rm -rf gpurun_out/abc5_$k
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abc5_$k -o run -- python bench.py --config C5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/abc5_$k.json 2> gpurun_out/abc5_$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/abc5_$k.err; exit 1; }
  echo "== $envs"; python -c "import json; d=json.load(open('gpurun_out/abc5_$k.json')); print('it/s', round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms_avg'].items()})"
  python tools/factor_levels.py gpurun_out/abc5_$k/run_kernel_trace.csv
done
