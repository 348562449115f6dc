#!/bin/bash
# GPU session on the MI355X box (run through gpurun). Stages, each under its own time limit, stop at the first
# failure:
#   test     parity probe -> pytest -m gpu (incl. full-size C2/C3/C5) -> smoke
#   suite    pytest -m gpu (PYTEST_K selects) without the probe; smoke
#   prof / prof5 / prof3   rocprofv3 kernel trace + stats of the C4 / C5 / C3 bench, PMC FETCH_SIZE / WRITE_SIZE passes
#            -> traffic JSON (keyed by _meta.config)
#   kstats   rocprofv3 kernel trace + stats of the C4, C5 and C3 bench legs (no PMC) and their factor level splits
#   bench    bench.py (C4, with the measured traffic) and the C5 leg
#   line     bench.py alone (the driver's default line)
#   ab       tools/ab_bench.py over the "CONFIG SETTINGS..." specs in $AB_SPECS (one per line), one process each
#   phases   tools/phase_probe.py on the phase build (make -C g2o_amd phases beforehand, on the CPU)
#   dist     tools/dist_rank_times.py (per-rank sharded stages + factor chains at N = 2 / 4 / 8 on one GPU)
# Usage: bash gpu_session.sh TAG STAGE...   (outputs under gpurun_out/, TAG names the run)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r06}
shift
O=gpurun_out
mkdir -p $O
for STAGE in "$@"; do
case $STAGE in
test)
  timeout -k 10 300 python -u tools/parity_probe.py > $O/${TAG}_probe.log 2>&1 || { echo PROBE_FAIL; tail -20 $O/${TAG}_probe.log; exit 1; }
  echo PROBE_OK
  ;&
suite)
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
kstats)
  for CF in ${KSTATS_CONFIGS:-C4 C5 C3}; do
    D=$O/${TAG}_prof_$CF
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python bench.py --config $CF --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL $CF; tail -5 $D.err; exit 1; }
    T=$(find $D -name '*kernel_trace.csv' | head -1)
    [ -n "$T" ] && python tools/factor_levels.py $T > $O/${TAG}_$(echo $CF | tr 'A-Z' 'a-z')_factor_levels.txt 2>&1
    echo KSTATS_OK $CF
  done
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
line)
  timeout -k 10 900 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo BENCH_FAIL; tail -20 $O/${TAG}_bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_bench.json'));print('C4',d['value'],'factor',d['roofline']['avg_launch_ms'],'C5',d['c5']['value'],'C3',d['pose_graph']['value'])"
  ;;
ab)
  i=0
  while IFS= read -r spec; do
    [ -z "$spec" ] && continue
    i=$((i+1))
    timeout -k 10 400 python tools/ab_bench.py $spec > $O/${TAG}_ab_$i.log 2>&1 || { echo AB_FAIL $spec; tail -20 $O/${TAG}_ab_$i.log; exit 1; }
    cat $O/${TAG}_ab_$i.log
  done <<< "$AB_SPECS"
  ;;
phases)
  G2OHIP_LIB=g2o_amd/libg2o_hip_phases.so timeout -k 10 300 python -u tools/phase_probe.py ${PHASE_CONFIG:-C4} > $O/${TAG}_phases.log 2>&1 || { echo PHASES_FAIL; tail -20 $O/${TAG}_phases.log; exit 1; }
  echo PHASES_OK
  ;;
dist)
  timeout -k 10 900 python -u tools/dist_rank_times.py $O/${TAG}_dist_rank_times.json > $O/${TAG}_dist_rank_times.log 2>&1 || { echo DIST_FAIL; tail -20 $O/${TAG}_dist_rank_times.log; exit 1; }
  echo DIST_OK
  tail -12 $O/${TAG}_dist_rank_times.log
  ;;
*)
  echo "unknown stage $STAGE"; exit 2
  ;;
esac
done
