# timing events without the system-scope fence (G2OHIP_EVENT_FENCE=1: default events) + camera pass / backsub_j
# software-pipelined index loads: full GPU suite, A/B, C4 gaps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05x_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05x_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05x_ab "C4 - $B G2OHIP_EVENT_FENCE=1 - $B --steps 20 --warmup 3" "C5 - $B G2OHIP_EVENT_FENCE=1 - $B --steps 8 --warmup 2" || exit 1
D=$O/r05x_C4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL; tail -5 $D.err; exit 1; }
F=$(find $D -name '*kernel_trace.csv' | head -1)
python tools/iter_gaps.py $F | tail -12
