#!/bin/bash
# Dev: parity of the factor schedules (pytest -k expression, default the parity + marginals files), then per env setting a
# profiled C4 bench (per-level factor breakdown) and the C5 leg's LM it/s.
#   bash tools/gpu_w64.sh "G2OHIP_CHOL_W64=0" "G2OHIP_CHOL_W64=1"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_parity.py tests/test_gpu_marginals.py}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w64_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/w64_tests.log; exit 1; }
tail -2 gpurun_out/w64_tests.log
k=0
for envs in "$@"; do
  k=$((k+1))
  rm -rf gpurun_out/w$k
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/w$k -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 > gpurun_out/w$k.json 2> gpurun_out/w$k.err || { echo FAIL "$envs"; tail -5 gpurun_out/w$k.err; exit 1; }
  echo "== $envs"; python -c "import json; d=json.load(open('gpurun_out/w$k.json')); print('C4 it/s (traced)', round(d['value'],1), {k: round(v*1e3,1) for k,v in d['stages_ms_avg'].items()})"
  python tools/factor_levels.py gpurun_out/w$k/run_kernel_trace.csv
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-posegraph > gpurun_out/wb$k.json 2> gpurun_out/wb$k.err || { echo BENCH_FAIL "$envs"; tail -5 gpurun_out/wb$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/wb$k.json')); c=d.get('c5',{}); print('C4 it/s', round(d['value'],1), 'factor', round(d['stages_ms_avg']['chol_factor']*1e3,1), '| C5 it/s', c.get('value'), {k: round(v*1e3,1) for k,v in c.get('stages_ms_avg',{}).items()})"
done
