#!/bin/bash
# Dev: profiled C4 bench under an env setting; prints one iteration's kernel timeline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for envs in "$@"; do
  k=$((k+1))
  rm -rf gpurun_out/pe$k
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pe$k -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/pe$k.json 2> gpurun_out/pe$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/pe$k.err; exit 1; }
  echo "== $envs"; python -c "import json; d=json.load(open('gpurun_out/pe$k.json')); print('it/s', round(d['value'],1))"
  python tools/iter_trace.py gpurun_out/pe$k/run_kernel_trace.csv
done
