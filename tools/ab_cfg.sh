#!/bin/bash
# Dev A/B: one bench config per env setting, LM it/s and the factor / solve stage times.
#   bash tools/ab_cfg.sh CONFIG STEPS "A=1" "B=2" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=$1; STEPS=$2; shift 2
for envs in "$@"; do
  env $envs timeout -k 10 400 python bench.py --config $CFG --steps $STEPS --warmup 2 --no-cpu-baseline --no-posegraph > gpurun_out/abc.json 2> gpurun_out/abc.err || { echo FAIL "$envs"; tail -5 gpurun_out/abc.err; exit 1; }
  python - "$CFG" "$envs" <<'PY'
import json, sys
d = json.load(open("gpurun_out/abc.json")); s = d["stages_ms_avg"]
print(sys.argv[1], sys.argv[2], "it/s %.2f factor %.3f solve %.3f" % (d["value"], s["chol_factor"], s["chol_solve"]))
PY
done
