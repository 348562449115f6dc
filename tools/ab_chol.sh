#!/bin/bash
# Dev A/B: profiled C4 bench per env setting ("A=1 B=2" per argument); it/s and the per-level factor breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for envs in "$@"; do
  k=$((k+1))
  rm -rf gpurun_out/ab$k
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab$k -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-posegraph > gpurun_out/ab$k.json 2> gpurun_out/ab$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/ab$k.err; exit 1; }
  echo "== $envs"; python -c "import json; d=json.load(open('gpurun_out/ab$k.json')); print('it/s', round(d['value'],1))"
  python tools/factor_levels.py gpurun_out/ab$k/run_kernel_trace.csv
done
