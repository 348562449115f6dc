#!/bin/bash
# schedule parity (small configs), C4 full parity + residuals, a kernel trace of a short C4 bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-dag3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "factor_schedules or c4_full or stage_reduced" -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_sched.log 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_sched.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_sched.log | head -20; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "c4_bench or residual" -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_full.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_full.log | head -20; exit $rc; }
bash tools/gpu_prof_quick.sh ${TAG}p > /dev/null || exit 1
python - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/${TAG}p_prof/run_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'k_vec_init' in r['Kernel_Name']]
a=idx[-1]; t0=int(rows[a]['Start_Timestamp'])
for r in rows[a:a+80]:
    nm=r['Kernel_Name'].split('(')[0].replace('g2ohip::','').replace('void ','')
    s=(int(r['Start_Timestamp'])-t0)/1e3; d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    print(f"{s:8.1f} {d:7.1f} {nm[:40]}")
    if 'k_backsub' in nm: break
PY
python -c "import json; d=json.load(open('gpurun_out/${TAG}p_bench.json')); print('C4', round(d['value'],1), 'factor', d['roofline']['avg_launch_ms'], d['stages_ms_avg'])"
