#!/bin/bash
# quick GPU check after a kernel change: the -m gpu suite (minus PCG) + a C4 bench line (no CPU baseline)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-posegraph --no-c5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('C4', round(d['value'],1), 'LM it/s', {k: round(v*1e3,1) for k,v in d['stages_ms_avg'].items()})"
timeout -k 10 300 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.err || { echo BENCH_C5_FAIL; tail -20 gpurun_out/${TAG}_bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_c5.json')); print('C5', round(d['value'],1), 'LM it/s', {k: round(v*1e3,1) for k,v in d['stages_ms_avg'].items()})"
