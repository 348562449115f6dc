# round-5 closing state (final): full GPU suite, smoke, the bench line, per-config kernel stats of the bench legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/r05zg_pytest_gpu.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -3 $O/r05zg_pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05zg_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/r05zg_smoke.log; exit 1; }
tail -3 $O/r05zg_smoke.log
timeout -k 10 900 python bench.py > $O/r05zg_bench.json 2> $O/r05zg_bench.err || { echo BENCH_FAIL; tail -20 $O/r05zg_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/r05zg_bench.json'));print('C4',d['value'],'factor',d['roofline']['avg_launch_ms'],'C5',d['c5']['value'],'C3',d['pose_graph']['value'])"
for C in C4 C5 C3; do
  D=$O/r05zg_prof_$C
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python bench.py --config $C --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL $C; tail -5 $D.err; exit 1; }
done
echo PROF_OK
