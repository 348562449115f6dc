set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -k "not sharded_8" --timeout 600 --timeout-method thread > $O/r04r_tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/r04r_tests.log; exit 1; }
tail -2 $O/r04r_tests.log
bash tools/gpu_ab.sh r04r "C4 - -" "C5 - --steps 6" "C3 - --steps 3 --warmup 1"
