# level shapes (G2OHIP_PRINT_LEVELS) for C4 / C5 and the C5 factor level split
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
G2OHIP_PRINT_LEVELS=1 timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $O/r05v_c4.json 2> $O/r05v_c4_levels.txt || { echo FAIL_C4; tail -5 $O/r05v_c4_levels.txt; exit 1; }
grep "^level" $O/r05v_c4_levels.txt | head -20
D=$O/r05v_C5
G2OHIP_PRINT_LEVELS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL; tail -5 $D.err; exit 1; }
grep "^level" $D.err | head -20
F=$(find $D -name '*kernel_trace.csv' | head -1)
python tools/factor_levels.py $F
bash tools/gpu_ab.sh r05v_ab "C4 - HIP_FORCE_DEV_KERNARG=1 HIP_FORCE_DEV_KERNARG=0 --steps 20 --warmup 3" || exit 1
