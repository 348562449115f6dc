#!/bin/bash
# C3 (100k-pose SE3 pose graph) A/B of Cholesky schedule knobs: runs bench.py --config C3 once per
# "VAR=value ..." argument (empty string = defaults); prints it/s and factor ms per run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 240 python bench.py --config ${CFG:-C3} --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > $O/c3_ab_$i.json 2> $O/c3_ab_$i.err || { echo "FAIL [$envs]"; tail -20 $O/c3_ab_$i.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/c3_ab_$i.json')); s=d['stages_ms_avg']
print('[$envs]', 'it/s %.2f' % d['value'], 'ms/lin %.3f' % d['ms_per_linear_solve'], 'factor %.3f' % s['chol_factor'], 'solve %.3f' % s['chol_solve'], 'chi2 %.10g' % d['config']['final_chi2'])"
done
