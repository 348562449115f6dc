# the factor's roofline timer on its first / last launches (hipExtLaunchKernel start / stop events, no marker packets):
# full GPU suite, A/B, and the rocprofv3 factor time against the bench line's HIP-event time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/r05z8_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05z8_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05z8_ab "C4 - $B G2OHIP_EVENT_FENCE=1 - $B --steps 20 --warmup 3" "C5 - $B - $B --steps 8 --warmup 2" "C3 - $B --steps 3 --warmup 1" || exit 1
D=$O/r05z8_prof_C4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python bench.py --config C4 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL; tail -5 $D.err; exit 1; }
python -c "import json; d=json.load(open('$D.json')); print('events factor ms', d['roofline']['avg_launch_ms'], 'value', d['value'])"
