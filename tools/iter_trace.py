"""Dev helper: kernel durations (us) of one LM iteration from a rocprofv3 kernel trace, in order."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_linearize' in r['Kernel_Name']]
a, b = idx[-3], idx[-2]
out = []
for r in rows[a:b]:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('g2ohip::', '').replace('k_', '')
    out.append('%s:%.1f' % (n[:14], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
print(' '.join(out))
tot = {}
for r in rows[a:b]:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('g2ohip::', '')
    tot[n] = tot.get(n, 0) + (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
print({k: round(v, 1) for k, v in sorted(tot.items(), key=lambda x: -x[1])})
print('span %.1f us' % ((int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1e3))
