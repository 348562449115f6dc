# C5 PMC traffic per kernel (FETCH_SIZE / WRITE_SIZE passes) + kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/r05w_fetch -o run --output-format csv -- python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $O/r05w_f.json 2> $O/r05w_f.err || { echo FAIL_F; tail -5 $O/r05w_f.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/r05w_write -o run --output-format csv -- python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $O/r05w_w.json 2> $O/r05w_w.err || { echo FAIL_W; tail -5 $O/r05w_w.err; exit 1; }
python tools/pmc_traffic.py $O/r05w_traffic_c5.json $O/r05w_fetch $O/r05w_write && cat $O/r05w_traffic_c5.json | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['bytes_per_launch']/1e6,1), round(v['bytes_fetch_doubled']/1e6,1)) for k,v in d.items() if k!='_meta']"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r05w_stats -o run --output-format csv -- python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > $O/r05w_s.json 2> $O/r05w_s.err || { echo FAIL_S; exit 1; }
F=$(find $O/r05w_stats -name '*kernel_stats.csv' | head -1); head -30 $F | cut -d, -f1-6
