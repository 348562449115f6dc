# GemmNTd: C tile prefetched before the K loop; ubench, parity subset, A/B against the previous library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 120 ./tools/ubench_gemm 4096 2048 > $O/r05o_ubench_4096.log 2>&1 && grep -E "check d|k16s2o4|k32s2" $O/r05o_ubench_4096.log || exit 1
timeout -k 10 120 ./tools/ubench_gemm 1152 384 > $O/r05o_ubench_1152.log 2>&1 && grep -E "k16s2o4|k32s2" $O/r05o_ubench_1152.log || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "factor_schedules or c5_bench or c4_bench or c3_bench" > $O/r05o_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05o_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
P=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_pre.so
bash tools/gpu_ab.sh r05o_ab "C3 - $B $P - $B $P --steps 3 --warmup 1" "C5 - $B $P - $B --steps 8 --warmup 2" "C4 - $B $P - $B --steps 20 --warmup 3"
