#!/bin/bash
# Dev A/B: bench.py (CONFIG, default C4) under env settings given as arguments ("VAR=val VAR2=val" per run), all stages
set -o pipefail
mkdir -p gpurun_out
CFG=${CONFIG:-C4}
k=0
for envs in "$@"; do
  k=$((k+1))
  env $envs timeout -k 10 180 python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-posegraph > gpurun_out/ab_st_$k.json 2>gpurun_out/ab_st_$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/ab_st_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_st_$k.json')); print('$CFG $envs', round(d['value'],1), 'it/s', {k: round(v*1e3,1) for k,v in d['stages_ms_avg'].items() if v > 0})"
done
