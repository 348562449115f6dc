set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/r04i_sharded.log 2>&1 || { echo SHARDED_FAIL; tail -40 $O/r04i_sharded.log; exit 1; }
tail -3 $O/r04i_sharded.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s -k "sharded" --timeout 800 --timeout-method thread > $O/r04i_c5_8ranks.log 2>&1 || { echo FULL8_FAIL; tail -40 $O/r04i_c5_8ranks.log; exit 1; }
grep -E "rank [0-9]:|passed|failed" $O/r04i_c5_8ranks.log | tail -12
