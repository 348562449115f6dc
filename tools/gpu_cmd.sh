set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r04aj
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
