#!/bin/bash
# one GPU session: parity probe -> profiled bench -> gpu test suite (stops at the first failure)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python gpurun_probe.py > gpurun_out/probe.log 2>&1 || { echo PROBE_FAIL $?; exit 1; }
echo PROBE_OK
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo PROF_FAIL $?; exit 1; }
echo PROF_OK
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL $?; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
tail -3 gpurun_out/pytest_gpu.log
