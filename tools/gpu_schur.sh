#!/bin/bash
# Dev: Schur split parity tests, then the C4 + C5 bench stage times per env setting (k_schur_rows variants)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G2OHIP_SCHUR_RS=${TEST_RS:-3} timeout -k 10 400 python -u -m pytest tests/test_gpu_schur_split.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -k "not factor_schedules and not full_size" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sch_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/sch_tests.log; exit 1; }
tail -1 gpurun_out/sch_tests.log
k=0
for e in "$@"; do
  k=$((k+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-posegraph > gpurun_out/sb$k.json 2> gpurun_out/sb$k.err || { echo BENCH_FAIL "$e"; tail -5 gpurun_out/sb$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sb$k.json')); c=d.get('c5',{}); print('$e', 'C4 it/s', round(d['value'],1), 'schur_rows', round(d['stages_ms_avg']['schur_rows']*1e3,1), '| C5 it/s', round(c.get('value',0),1), 'schur_rows', round(c.get('stages_ms_avg',{}).get('schur_rows',0)*1e3,1))"
done
