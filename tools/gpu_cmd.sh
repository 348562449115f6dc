set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_marginals.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04k_tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/r04k_tests.log; exit 1; }
tail -2 $O/r04k_tests.log
bash tools/gpu_ab.sh r04k "C3 - G2OHIP_EA_BIG=1024 G2OHIP_EA_BIG=512 - --steps 3 --warmup 1"
