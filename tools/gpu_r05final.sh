# round-5 final state: full GPU suite, smoke, the bench line (C4 + C3 + C5 legs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/r05f_pytest_gpu.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -3 $O/r05f_pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05f_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/r05f_smoke.log; exit 1; }
cat $O/r05f_smoke.log
timeout -k 10 900 python bench.py > $O/r05f_bench.json 2> $O/r05f_bench.err || { echo BENCH_FAIL; tail -20 $O/r05f_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/r05f_bench.json'));print('C4',d['value'],'factor',d['roofline']['avg_launch_ms'],'C5',d['c5']['value'],'C3',d['pose_graph']['value'])"
