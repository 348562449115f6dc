#!/bin/bash
# C5 kernel trace with the big-panel (blocked) schedule forced on every level (dev A/B of the factor schedules)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
G2OHIP_CHOL_WIDE_FRONTS=${WF:-4} timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/c5wide -o run -- python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-posegraph --no-c5 > gpurun_out/c5wide.json 2> gpurun_out/c5wide.err
