# Schur rows PIPE 2 (two staged batches in flight): bitwise / split / schedule tests, then A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipe_bitwise or schur_rows_pipe2 or split_stage or split_fixed or c4_bench or c5_bench" > $O/r05k_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -3 $O/r05k_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r05k_ab "C4 - G2OHIP_SCHUR_PIPE=2,G2OHIP_SCHUR_SB_KX=128 G2OHIP_SCHUR_SB_KX=128 - G2OHIP_SCHUR_PIPE=2,G2OHIP_SCHUR_SB_KX=128 --steps 20 --warmup 3" "C5 - G2OHIP_SCHUR_PIPE=2,G2OHIP_SCHUR_SB_KX=128 G2OHIP_SCHUR_SB_KX=128 - G2OHIP_SCHUR_PIPE=2,G2OHIP_SCHUR_SB_KX=128 --steps 8 --warmup 2"
