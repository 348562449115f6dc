#!/bin/bash
# Round artifacts after the tests: kernel stats (C4 short bench, C5 leg alone), the PMC FETCH_SIZE / WRITE_SIZE passes
# over the C4 short bench (-> traffic JSON for bench.py's `traffic`), and the .g2o writer/loader at C5.
#   bash tools/gpu_profiles.sh TAG      (outputs under gpurun_out/TAG_*)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
O=gpurun_out/${TAG}
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-posegraph --no-c5 > $O/c4_bench.json 2> $O/c4_bench.err || { echo C4_PROF_FAIL; tail -20 $O/c4_bench.err; exit 1; }
echo C4_PROF_OK
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_bench.json 2> $O/c5_bench.err || { echo C5_PROF_FAIL; tail -20 $O/c5_bench.err; exit 1; }
echo C5_PROF_OK
k=0
for P in FETCH_SIZE WRITE_SIZE; do
  k=$((k+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$P -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 --no-kernel-timing > $O/pmc_$P.log 2>&1 || { echo PMC_FAIL $P; tail -5 $O/pmc_$P.log; exit 1; }
  echo PMC_OK $P
done
python tools/pmc_traffic.py $O/traffic.json $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE || exit 1
timeout -k 10 300 python tools/time_loader.py C5 > $O/loader_c5.json 2> $O/loader_c5.err || { echo LOADER_FAIL; tail -5 $O/loader_c5.err; exit 1; }
cat $O/loader_c5.json
