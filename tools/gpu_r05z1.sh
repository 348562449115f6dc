# decision polling vs adaptive-width backward-solve chunks (current) vs base: C3 and C4, per-kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_base.so
P=G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_poll.so
bash tools/gpu_ab.sh r05z1_ab "C3 - $B $P - $B $P --steps 3 --warmup 1" "C4 - $B $P - $B $P --steps 20 --warmup 3" || exit 1
for L in base poll; do
  D=$O/r05z1_C3_$L
  G2OHIP_LIB=/root/repo/g2o_amd/libg2o_hip_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL; tail -5 $D.err; exit 1; }
done
D=$O/r05z1_C3_cur
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python bench.py --config C3 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL; tail -5 $D.err; exit 1; }
for L in base poll cur; do F=$(find $O/r05z1_C3_$L -name '*kernel_stats.csv' | head -1); echo "== $L"; grep -E "bwd|permute|backsub" $F | cut -d, -f1-4; done
