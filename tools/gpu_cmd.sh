set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r04ao
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/${T}_smoke.log; exit 1; }
cat $O/${T}_smoke.log
