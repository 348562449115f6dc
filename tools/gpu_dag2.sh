#!/bin/bash
# remaining checks after gpu_dag.sh: contract tests from the round trip on, then a C4 bench (+ C5 leg)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dagb}
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver_contract.py tests/test_host.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -6 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-posegraph --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('C4', round(d['value'],1), 'factor', d['roofline']['avg_launch_ms'], d['stages_ms_avg'], d['factor'], d['runtime'], json.dumps(d.get('c5'))[:900])"
