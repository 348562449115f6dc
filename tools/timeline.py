"""Dev helper: per-LM-iteration GPU busy time vs span from a rocprofv3 kernel trace, largest gaps."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_linearize' in r['Kernel_Name']]
for a, b in zip(idx[-4:-1], idx[-3:]):
    seg = rows[a:b]
    t0 = int(seg[0]['Start_Timestamp'])
    t1 = int(rows[b]['Start_Timestamp'])
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seg)
    gaps = []
    for x, y in zip(seg, seg[1:] + [rows[b]]):
        gaps.append((int(y['Start_Timestamp']) - int(x['End_Timestamp']), x['Kernel_Name'][:34], y['Kernel_Name'][:34]))
    gsum = sum(g[0] for g in gaps)
    gaps.sort(reverse=True)
    print('span %.1f us busy %.1f us gaps %.1f us launches %d' % ((t1 - t0) / 1e3, busy / 1e3, gsum / 1e3, len(seg)))
    for g in gaps[:5]:
        print('   gap %.1f us after %s before %s' % (g[0] / 1e3, g[1], g[2]))
