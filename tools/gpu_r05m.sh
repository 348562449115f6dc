# Schur rows: strided observation walk over a row's batches (slot balance): parity, A/B, dev mode split
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pipe_bitwise or schur or split or c4_bench or c5_bench or sharded or ba_" > $O/r05m_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -3 $O/r05m_tests.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab.sh r05m_ab "C4 - G2OHIP_SCHUR_ORDER=0 - G2OHIP_SCHUR_ORDER=0 --steps 20 --warmup 3" "C5 - G2OHIP_SCHUR_ORDER=0 - --steps 8 --warmup 2"
