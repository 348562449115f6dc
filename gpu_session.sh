#!/bin/bash
# GPU session on the MI355X box (run through gpurun). Stages, each under its own time limit, stop at the first
# failure:
#   test   parity probe -> pytest -m gpu (incl. full-size C2/C3/C5) -> smoke
#   prof / prof5 / prof3   rocprofv3 kernel trace + stats of the C4 / C5 / C3 bench, PMC FETCH_SIZE / WRITE_SIZE passes
#          -> traffic JSON (keyed by _meta.config)
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
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/${TAG}_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/${TAG}_pytest_gpu.log; exit 1; }
  echo PYTEST_OK
  tail -3 $O/${TAG}_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/${TAG}_smoke.log; exit 1; }
  echo SMOKE_OK
  ;;
prof|prof5|prof3)
  # rocprofv3 kernel trace + stats of one config's bench run, then the PMC FETCH_SIZE / WRITE_SIZE passes -> traffic JSON
  case $STAGE in prof) CF=C4; ST=10;; prof5) CF=C5; ST=4;; prof3) CF=C3; ST=2;; esac
  CL=$(echo $CF | tr 'A-Z' 'a-z')
  BA="--config $CF --no-cpu-baseline --no-posegraph --no-c5"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof_$CL -o run -- python bench.py --steps $ST --warmup 2 $BA > $O/${TAG}_bench_prof_$CL.json 2> $O/${TAG}_bench_prof_$CL.err || { echo PROF_FAIL $CF; tail -20 $O/${TAG}_bench_prof_$CL.err; exit 1; }
  echo PROF_OK $CF
  RX='k_schur|k_linearize|k_backsub|k_vertex_reduce|k_cam_assemble|k_lm_fixup|k_zero_ranges|k_chol_scatter|k_vec_init|k_extend_add|k_step|k_syrk|k_permute'
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/${TAG}_pmc_fetch_$CL -o run -- python bench.py --steps 2 --warmup 1 $BA --no-kernel-timing > $O/${TAG}_pmc_fetch_$CL.log 2>&1 || { echo PMC_FETCH_FAIL; tail -20 $O/${TAG}_pmc_fetch_$CL.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/${TAG}_pmc_write_$CL -o run -- python bench.py --steps 2 --warmup 1 $BA --no-kernel-timing > $O/${TAG}_pmc_write_$CL.log 2>&1 || { echo PMC_WRITE_FAIL; tail -20 $O/${TAG}_pmc_write_$CL.log; exit 1; }
  G2OHIP_TRAFFIC_CONFIG=$CF python tools/pmc_traffic.py $O/${TAG}_traffic_$CL.json $O/${TAG}_pmc_fetch_$CL $O/${TAG}_pmc_write_$CL > $O/${TAG}_traffic_$CL.log 2>&1 || { echo TRAFFIC_PARSE_FAIL; cat $O/${TAG}_traffic_$CL.log; }
  echo PMC_OK $CF
  ;;
bench)
  # traffic files of this session's prof stages (when run), else the committed profiles/traffic_<config>.json
  for CL in c4 c5 c3; do
    CU=$(echo $CL | tr 'a-z' 'A-Z')
    [ -f $O/${TAG}_traffic_$CL.json ] && export G2OHIP_TRAFFIC_JSON_$CU=$O/${TAG}_traffic_$CL.json
  done
  timeout -k 10 900 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo BENCH_FAIL; tail -20 $O/${TAG}_bench.err; exit 1; }
  echo BENCH_OK
  cat $O/${TAG}_bench.json
  timeout -k 10 600 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench_c5.json 2> $O/${TAG}_bench_c5.err || { echo BENCH_C5_FAIL; tail -20 $O/${TAG}_bench_c5.err; exit 1; }
  echo BENCH_C5_OK
  ;;
esac
done
