set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_schur_split.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_blocksolver_3_2.py "tests/test_gpu_fullsize.py::test_c4_bench_sequence" "tests/test_gpu_fullsize.py::test_c5_bench_sequence" -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04d_pytest_schur2.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/r04d_pytest_schur2.log; exit 1; }
tail -2 $O/r04d_pytest_schur2.log
timeout -k 10 500 python tools/ab_bench.py C4 - G2OHIP_SCHUR_V=1 G2OHIP_SCHUR_SB=64 - G2OHIP_CHOL_BLOCK_MIN=256 G2OHIP_CHOL_LAG_FUSED_MIN=100000 G2OHIP_CHOL_FUSED_MAX=1024 --steps 20 --warmup 3 > $O/ab_c4s.log 2>&1; cat $O/ab_c4s.log
timeout -k 10 300 python tools/ab_bench.py C5 - G2OHIP_SCHUR_V=1 G2OHIP_SCHUR_SB=64 --steps 6 --warmup 2 > $O/ab_c5s.log 2>&1; cat $O/ab_c5s.log
timeout -k 10 200 python tools/time_loader.py C5 > $O/r04_loader_c5.json 2> $O/r04_loader_c5.err; cat $O/r04_loader_c5.json
