set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
T=r04ac
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1 || { echo TEST_FAIL; tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/${T}_trace -o run -- python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $O/${T}_trace.json 2> $O/${T}_trace.err || { echo TRACE_FAIL; exit 1; }
bash tools/gpu_ab.sh ${T} "C4 - G2OHIP_SCATTER_BLOCKS=0 - G2OHIP_SCATTER_BLOCKS=0" "C5 - G2OHIP_SCATTER_BLOCKS=0 --steps 6" "C3 - G2OHIP_SCATTER_BLOCKS=0 --steps 3 --warmup 1"
