#!/bin/bash
# One GPU session: parity probe -> profiled bench (kernel trace + stats) -> PMC traffic passes ->
# plain bench (with the measured traffic) -> gpu test suite. Stops at the first failure.
# Usage: bash gpu_session.sh [TAG]   (outputs under gpurun_out/, TAG names the round)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u gpurun_probe.py > $O/probe.log 2>&1 || { echo PROBE_FAIL; tail -20 $O/probe.log; exit 1; }
echo PROBE_OK
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-posegraph > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -20 $O/bench_prof.err; exit 1; }
echo PROF_OK
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_schur|k_linearize|k_backsub|k_vertex_reduce' --output-format csv -d $O/pmc_fetch -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-kernel-timing > $O/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_schur|k_linearize|k_backsub|k_vertex_reduce' --output-format csv -d $O/pmc_write -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-kernel-timing > $O/pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; tail -20 $O/pmc_write.log; exit 1; }
python tools/pmc_traffic.py $O/traffic_$TAG.json $O/pmc_fetch $O/pmc_write > $O/traffic.log 2>&1 || { echo TRAFFIC_PARSE_FAIL; cat $O/traffic.log; }
echo PMC_OK
G2OHIP_TRAFFIC_JSON=$O/traffic_$TAG.json timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCH_FAIL; tail -20 $O/bench_$TAG.err; exit 1; }
echo BENCH_OK
cat $O/bench_$TAG.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
echo PYTEST_OK
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
echo SMOKE_OK
cat $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc3 -o run -- python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3prof.json 2> $O/bench_c3prof.err || { echo PROF_C3_FAIL; tail -20 $O/bench_c3prof.err; exit 1; }
echo PROF_C3_OK
