#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/dist_factor_time.py --config C5 --ranks 8 > gpurun_out/dist_factor_c5.json 2> gpurun_out/dist_factor_c5.err; rc=$?
tail -12 gpurun_out/dist_factor_c5.err
python -c "import json; d=json.load(open('gpurun_out/dist_factor_c5.json')); print('single', d['single']['factor_ms'], d['single']['solve_ms'], 'max rank', d['max_rank_factor_ms'], d['max_rank_solve_ms']); print([round(x['factor_ms'],3) for x in d['per_rank']]); print(d['per_rank'][0]['info'])"
exit $rc
