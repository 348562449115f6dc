#!/bin/bash
# Dev: one C4 kernel trace; per-level factor breakdown and the k_step durations in launch order.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/tr
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-posegraph > gpurun_out/tr.json 2> gpurun_out/tr.err || { echo FAIL; tail -5 gpurun_out/tr.err; exit 1; }
python tools/factor_levels.py gpurun_out/tr/run_kernel_trace.csv
python - <<'PY'
import csv
rows = sorted(csv.DictReader(open('gpurun_out/tr/run_kernel_trace.csv')), key=lambda r: int(r['Start_Timestamp']))
sc = [i for i, r in enumerate(rows) if 'k_chol_scatter' in r['Kernel_Name']]
a = sc[-2]
b = next(i for i in range(a, len(rows)) if 'k_bwd_gemv' in rows[i]['Kernel_Name'])
prev = None
out = []
for r in rows[a:b]:
    n = r['Kernel_Name'].split('(')[0].replace('g2ohip::', '').replace('void ', '')
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    out.append('%-28s dur %6.1f  gap %5.1f  grid %s' % (n[:28], (e - s) / 1e3, gap, int(r['Grid_Size_X'])//256))
    prev = e
print('\n'.join(out))
PY
