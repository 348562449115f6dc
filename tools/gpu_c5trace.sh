#!/bin/bash
# C5 kernel trace (one short bench run) + the RCCL binding test + factor parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_parity.py > gpurun_out/c5tr_tests.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5tr -o run -- python bench.py --config C5 --steps 4 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 > gpurun_out/c5tr.json 2> gpurun_out/c5tr.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-posegraph > gpurun_out/c4b.json 2> gpurun_out/c4b.err
rc=$?; tail -3 gpurun_out/c5tr_tests.log; cut -c1-300 gpurun_out/c5tr.json; cut -c1-300 gpurun_out/c4b.json; exit $rc
