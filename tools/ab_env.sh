#!/bin/bash
# Dev A/B: bench.py C4 under env settings given as arguments ("VAR=val VAR2=val" per run)
set -o pipefail
mkdir -p gpurun_out
k=0
for envs in "$@"; do
  k=$((k+1))
  env $envs timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_env_$k.json 2>gpurun_out/ab_env_$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/ab_env_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_env_$k.json')); print('$envs', round(d['value'],1), 'it/s', {k: round(v*1e3,1) for k,v in d['stages_ms_avg'].items() if k.startswith('chol')})"
done
