#!/bin/bash
# GPU session on the MI355X box (run through gpurun). Stages, each under its own time limit, stop at the first
# failure:
#   test   parity probe -> pytest -m gpu (incl. full-size C2/C3/C5) -> smoke
#   prof   rocprofv3 kernel trace + stats of the C4 bench, PMC FETCH_SIZE / WRITE_SIZE passes -> traffic JSON
#   bench  bench.py (C4, with the measured traffic) and the C5 leg
# Usage: bash gpu_session.sh TAG STAGE...   (outputs under gpurun_out/, TAG names the round)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
shift
O=gpurun_out
mkdir -p $O
for STAGE in "$@"; do
case $STAGE in
test)
  timeout -k 10 300 python -u tools/parity_probe.py > $O/${TAG}_probe.log 2>&1 || { echo PROBE_FAIL; tail -20 $O/${TAG}_probe.log; exit 1; }
  echo PROBE_OK
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > $O/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/${TAG}_pytest_gpu.log; exit 1; }
  echo PYTEST_OK
  tail -3 $O/${TAG}_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/${TAG}_smoke.log; exit 1; }
  echo SMOKE_OK
  ;;
prof)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 > $O/${TAG}_bench_prof.json 2> $O/${TAG}_bench_prof.err || { echo PROF_FAIL; tail -20 $O/${TAG}_bench_prof.err; exit 1; }
  echo PROF_OK
  RX='k_schur|k_linearize|k_backsub|k_vertex_reduce|k_cam_assemble|k_lm_fixup|k_zero_ranges|k_chol_scatter|k_vec_init|k_extend_add|k_step|k_syrk|k_permute'
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/${TAG}_pmc_fetch -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 --no-kernel-timing > $O/${TAG}_pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; tail -20 $O/${TAG}_pmc_fetch.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/${TAG}_pmc_write -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 --no-kernel-timing > $O/${TAG}_pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; tail -20 $O/${TAG}_pmc_write.log; exit 1; }
  python tools/pmc_traffic.py $O/${TAG}_traffic.json $O/${TAG}_pmc_fetch $O/${TAG}_pmc_write > $O/${TAG}_traffic.log 2>&1 || { echo TRAFFIC_PARSE_FAIL; cat $O/${TAG}_traffic.log; }
  echo PMC_OK
  ;;
bench)
  TJ=$O/${TAG}_traffic.json
  [ -f $TJ ] || TJ=profiles/traffic.json
  G2OHIP_TRAFFIC_JSON=$TJ timeout -k 10 900 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo BENCH_FAIL; tail -20 $O/${TAG}_bench.err; exit 1; }
  echo BENCH_OK
  cat $O/${TAG}_bench.json
  timeout -k 10 600 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench_c5.json 2> $O/${TAG}_bench_c5.err || { echo BENCH_C5_FAIL; tail -20 $O/${TAG}_bench_c5.err; exit 1; }
  echo BENCH_C5_OK
  ;;
esac
done
