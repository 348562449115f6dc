# backward-solve columns in chunks sized to the rows left (1024 / 512 / 256 / 128 / 64 rows per chunk, every load of a
# chunk in flight): parity subset, A/B against the previous library on C3 / C4 / C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "factor_schedules or c5_bench or c4_bench or c3_bench or sharded or csparse or marginals" > $O/r05z2_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z2_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05z2_ab "C3 - $B - $B --steps 3 --warmup 1" "C4 - $B - $B --steps 20 --warmup 3" "C5 - $B - $B --steps 8 --warmup 2" || exit 1
