#!/bin/bash
# Quick GPU iteration: parity probe -> GPU test suite -> profiled C4 bench (kernel trace + stats).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u gpurun_probe.py > $O/probe.log 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe.log; exit 1; }
echo PROBE_OK
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-posegraph ${BENCH_ARGS} > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -20 $O/bench_prof.err; exit 1; }
echo PROF_OK
python -c "
import json; d=json.load(open('$O/bench_prof.json')); print('it/s', round(d['value'],1), 'ms/lin', round(d['ms_per_linear_solve'],3)); print({k: round(v,4) for k,v in d['stages_ms_avg'].items()}); r=d['roofline']; print('roofline', r['kernel'], round(r['achieved'],1), round(r['frac'],4))"
python tools_profsum.py $O/prof/run_kernel_stats.csv 14
