#!/bin/bash
# run selected GPU test files: bash tools/gpu_tests_sel.sh TAG test_file...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
ARGS=""
for f in "$@"; do ARGS="$ARGS tests/$f"; done
timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -25 gpurun_out/${TAG}_pytest.log; exit $rc
