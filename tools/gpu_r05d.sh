# round-5 session: full GPU tests + smoke, the bench line, then the per-rank C5 critical path
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05d_pytest_gpu.log 2>&1; rc=$?; echo TESTS_RC=$rc; tail -3 gpurun_out/r05d_pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05d_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/r05d_smoke.log; exit 1; }
tail -1 gpurun_out/r05d_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err || { echo BENCH_FAIL; tail -5 gpurun_out/r05d_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r05d_bench.json')); print('C4', d['value'], 'factor', d['roofline']['avg_launch_ms'], 'C5', d['c5']['value'], 'C3', d['pose_graph']['value'])"
timeout -k 10 900 python -u tools/dist_rank_times.py --config C5 --ranks 2,4,8 > gpurun_out/r05d_dist_rank_times.json 2> gpurun_out/r05d_dist_rank_times.log || { echo DIST_FAIL; tail -20 gpurun_out/r05d_dist_rank_times.log; exit 1; }
tail -20 gpurun_out/r05d_dist_rank_times.log
