#!/bin/bash
# kernel trace of a short C4 bench: per-kernel stats + the trace CSV (for tools/factor_levels.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pq}
shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-posegraph --no-c5 "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -c1-200
