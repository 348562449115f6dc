#!/bin/bash
# Dev A/B: one bench line (C4 + the C5 leg) per env setting, printing LM it/s and the factor / Schur stage times.
#   bash tools/gpu_envab.sh "X=0" "G2OHIP_CHOL_FUSED_MAX=256" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
k=0
for e in "$@"; do
  k=$((k+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-posegraph > gpurun_out/ab_env$k.json 2> gpurun_out/ab_env$k.err || { echo BENCH_FAIL "$e"; tail -5 gpurun_out/ab_env$k.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab_env$k.json')); c=d.get('c5',{}); s=d['stages_ms_avg']; t=c.get('stages_ms_avg',{})
print('%-40s C4 %6.1f it/s factor %5.1f solve %5.1f | C5 %6.1f it/s factor %6.1f solve %5.1f' % ('$e', d['value'], s['chol_factor']*1e3, s['chol_solve']*1e3, c.get('value',0), t.get('chol_factor',0)*1e3, t.get('chol_solve',0)*1e3))"
done
