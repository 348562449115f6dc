# chi2 / scale partial sums: the loads of four edges (and of a thread's sixteen scale terms) in flight together instead
# of one guarded round trip per term: parity subset, A/B C4 / C5 / C3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_bench or c5_bench or c3_bench or robust or lm or chi2 or gn or pcg or fixed" > $O/r05z6_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z6_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05z6_ab "C4 - $B - $B --steps 20 --warmup 3" "C5 - $B - $B --steps 8 --warmup 2" "C3 - $B --steps 3 --warmup 1" || exit 1
