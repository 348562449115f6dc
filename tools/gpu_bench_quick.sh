#!/bin/bash
# Dev: parity subset (-k expression) then one C4 bench line per env setting, with the stage times.
#   bash tools/gpu_bench_quick.sh "C4" "X=0" "VAR=1"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
K=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "$K" > gpurun_out/q_tests.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for e in "$@"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-posegraph > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { echo BENCH_FAIL; tail -5 gpurun_out/q_bench.err; exit 1; }
  python - "$e" <<'PY'
import json, sys
d = json.load(open("gpurun_out/q_bench.json")); s = d["stages_ms_avg"]
print(sys.argv[1], "it/s %.1f" % d["value"], " ".join("%s %.1f" % (k, v * 1e3) for k, v in s.items()))
PY
done
