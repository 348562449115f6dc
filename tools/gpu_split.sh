#!/bin/bash
# Dev: C3 trajectory + factor schedule tests with the split-K contribution passes, then the C3 factor time per setting
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread -k "c3 or C3 or linear_residual or random_cov or factor_schedules" > gpurun_out/split_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-c5 --no-posegraph > gpurun_out/split_b.json 2> gpurun_out/split_b.err || { echo BENCH_FAIL; tail -5 gpurun_out/split_b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/split_b.json')); s=d['stages_ms_avg']; print('$e', 'C3 it/s %.2f factor %.2f ms' % (d['value'], s['chol_factor']), 'split ops', d['factor'].get('split_syrk_ops'))"
done
