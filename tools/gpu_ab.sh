set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_schur_split.py tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04f_schur3_tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/r04f_schur3_tests.log; exit 1; }
tail -2 $O/r04f_schur3_tests.log
timeout -k 10 300 python tools/ab_bench.py C4 - G2OHIP_SCHUR_PIPE=0 - G2OHIP_SCHUR_PIPE=0 > $O/r04f_ab_c4_pipe.log 2>&1 || { echo AB4_FAIL; tail -20 $O/r04f_ab_c4_pipe.log; exit 1; }
cat $O/r04f_ab_c4_pipe.log
timeout -k 10 400 python tools/ab_bench.py C5 - G2OHIP_SCHUR_PIPE=0 --steps 6 > $O/r04f_ab_c5_pipe.log 2>&1 || { echo AB5_FAIL; tail -20 $O/r04f_ab_c5_pipe.log; exit 1; }
cat $O/r04f_ab_c5_pipe.log
