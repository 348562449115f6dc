# camera pass gathers one packed [U | c] landmark record (80 B) instead of the U and c arrays: parity subset, A/B vs the
# previous library (C5: the recomputing camera pass; C4 uses the Kt records and is unchanged by design)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "split or c5 or c4_bench or sharded or assembly or schur or backsub or dist" > $O/r05z3_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z3_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05z3_ab "C5 - $B - $B --steps 8 --warmup 2" "C4 - $B --steps 20 --warmup 3" || exit 1
