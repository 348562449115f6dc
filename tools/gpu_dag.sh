#!/bin/bash
# tile-DAG factorization check: schedule parity on small configs, then C4/C5 full, then a short C4 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dag}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "factor_schedules" -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_sched.log 2>&1; rc=$?
tail -25 gpurun_out/${TAG}_sched.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_marginals.py tests/test_gpu_solver_contract.py tests/test_host.py -x -v --timeout 300 --timeout-method thread -k "not sharded_8" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-posegraph --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('C4', round(d['value'],1), 'factor', d['roofline']['avg_launch_ms'], d['stages_ms_avg'], d['factor'], json.dumps(d.get('c5'))[:800])"
