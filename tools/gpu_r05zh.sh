# final committed state: the bench line and the C4 leg's kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python bench.py > $O/r05zh_bench.json 2> $O/r05zh_bench.err || { echo BENCH_FAIL; tail -20 $O/r05zh_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/r05zh_bench.json'));print('C4',d['value'],'factor',d['roofline']['avg_launch_ms'],'C5',d['c5']['value'],'C3',d['pose_graph']['value'])"
D=$O/r05zh_prof_C4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python bench.py --config C4 --no-cpu-baseline --no-posegraph --no-c5 > $D.json 2> $D.err || { echo PROF_FAIL; tail -5 $D.err; exit 1; }
echo PROF_OK
