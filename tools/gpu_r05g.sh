# single-path GemmNTd chunk loop + two-panel lag v2: GEMM ubench, parity subset, A/B, C4 per-level split
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 120 ./tools/ubench_gemm 4096 2048 > $O/r05g_ubench_gemm_4096.log 2>&1 && grep -E "check d|k16s2o4|k32s2|d128x64w8 |rocblas" $O/r05g_ubench_gemm_4096.log || { echo UBENCH_FAIL; tail -5 $O/r05g_ubench_gemm_4096.log; exit 1; }
timeout -k 10 120 ./tools/ubench_gemm 1152 384 > $O/r05g_ubench_gemm_1152.log 2>&1 && grep -E "k16s2o4|k32s2" $O/r05g_ubench_gemm_1152.log || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "factor_schedules or c5_bench or c4_bench or c3_bench" > $O/r05g_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05g_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r05g_ab "C4 - G2OHIP_CHOL_LAG2=0 - G2OHIP_CHOL_LAG2=0 --steps 20 --warmup 3" "C5 - G2OHIP_CHOL_LAG2=0 - --steps 8 --warmup 2" "C3 - --steps 3 --warmup 1" || exit 1
for L2 in 1 0; do
  D=$O/r05g_C4_lag2_$L2
  G2OHIP_CHOL_LAG2=$L2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL $L2; tail -5 $D.err; exit 1; }
  F=$(find $D -name '*kernel_trace.csv' | head -1)
  echo "== C4 LAG2=$L2"; python tools/factor_levels.py $F | head -4
done
