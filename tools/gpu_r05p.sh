# Schur rows (Kt records): column half per wave (uniform branch); parity tests, A/B against the previous library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipe_bitwise or schur or split or c4_bench or c5_bench or sharded" > $O/r05p_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05p_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05p_ab "C4 - $B - $B --steps 20 --warmup 3" "C5 - $B - $B --steps 8 --warmup 2"
