#!/bin/bash
# per-rank factor times of the distributed factorization (one GPU plays each rank in turn) + the cost model beside them
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in ${CONFIGS:-C4 C5}; do
  timeout -k 10 900 python -u tools/dist_factor_time.py --config $C --ranks ${RANKS:-2,4,8} > gpurun_out/dist_factor_$C.json 2> gpurun_out/dist_factor_$C.err || { tail -12 gpurun_out/dist_factor_$C.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/dist_factor_$C.json')); s=d['single']; print('$C single', round(s['factor_ms'],3)); [print('$C N', n, 'max rank', round(v['max_rank_factor_ms'],3), [round(x['factor_ms'],3) for x in v['per_rank']]) for n, v in d['by_ranks'].items()]"
  grep "N=" gpurun_out/dist_factor_$C.err | head -20
done
