# round-5 closing state (late): PMC FETCH_SIZE / WRITE_SIZE passes of the C4 and C5 bench legs (separate passes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for C in C4 C5; do
  for K in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $K -d $O/r05zf_pmc_${C}_$K -o run --output-format csv -- python bench.py --config $C --steps 3 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 > $O/r05zf_pmc_${C}_$K.json 2> $O/r05zf_pmc_${C}_$K.err || { echo PMC_FAIL $C $K; tail -5 $O/r05zf_pmc_${C}_$K.err; exit 1; }
  done
  G2OHIP_TRAFFIC_CONFIG=$C python tools/pmc_traffic.py $O/r05zf_traffic_$(echo $C | tr A-Z a-z).json $O/r05zf_pmc_${C}_FETCH_SIZE $O/r05zf_pmc_${C}_WRITE_SIZE || exit 1
done
echo PMC_OK
