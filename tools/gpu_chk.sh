#!/bin/bash
# Dev: quick parity subset + one profiled C4 A/B run.  bash tools/gpu_chk.sh TAG "ENV..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_marginals.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not full and not c4_full" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
bash tools/ab_chol.sh "$@"
