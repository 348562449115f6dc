# camera pass from the Kt records (C4): record and landmark indices read ahead (software pipeline): parity subset, A/B
# against the linearize-only library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "split or c4 or assembly or robust or fixed" > $O/r05z5_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z5_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_lin.so
bash tools/gpu_ab.sh r05z5_ab "C4 - $B - $B - $B --steps 20 --warmup 3" || exit 1
