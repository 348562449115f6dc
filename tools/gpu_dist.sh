#!/bin/bash
# distributed factorization: sharded tests (LocalComm ranks on one GPU), then the C5 8-rank full-size test
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dist}
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_sharded.log 2>&1; rc=$?
tail -14 gpurun_out/${TAG}_sharded.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_sharded.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "sharded_8" -x -v -s --timeout 500 --timeout-method thread > gpurun_out/${TAG}_c5s.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_c5s.log
exit $rc
