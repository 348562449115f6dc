# decision readback by a polled sequence number + backward-solve kernels with 16 rows per lane in flight + timed regions at
# stats level 0: full GPU suite, A/B (base lib = previous commit, its bench timed region still at stats level 1), bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05y_tests.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -2 $O/r05y_tests.log
[ $rc -eq 0 ] || exit 1
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
bash tools/gpu_ab.sh r05y_ab "C4 - $B G2OHIP_EVENT_FENCE=1 - $B --steps 20 --warmup 3" "C5 - $B - $B --steps 8 --warmup 2" "C3 - $B --steps 3 --warmup 1" || exit 1
timeout -k 10 600 python bench.py > $O/r05y_bench.json 2> $O/r05y_bench.err || { echo BENCH_FAIL; tail -5 $O/r05y_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/r05y_bench.json')); print(d['value'], d['ms_per_step'], d['ms_per_linear_solve'], d['roofline']['achieved'], d.get('c5',{}).get('value'), d.get('posegraph',{}).get('value'))"
