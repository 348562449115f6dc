# per-level factor split (rocprofv3 kernel trace) with the two-panel lag on / off, C4 and C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for CF in C4 C5; do
  for L2 in 1 0; do
    D=$O/r05f_${CF}_lag2_$L2
    G2OHIP_CHOL_LAG2=$L2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python bench.py --config $CF --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL $CF $L2; tail -5 $D.err; exit 1; }
    F=$(find $D -name '*kernel_trace.csv' | head -1)
    echo "== $CF LAG2=$L2"; python tools/factor_levels.py $F | tee $O/r05f_${CF}_lag2_${L2}_levels.txt
  done
done
