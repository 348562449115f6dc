# extend-add block-0 task: the first child group's records read with the block (one round trip off each level's
# chain): parity subset, A/B C4 / C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "factor_schedules or c4_bench or c5_bench or sharded or csparse or marginals or extend" > $O/r05z7_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z7_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05z7_ab "C4 - $B - $B - $B --steps 20 --warmup 3" "C5 - $B - $B --steps 8 --warmup 2" || exit 1
