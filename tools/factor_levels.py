"""Dev helper: split one Cholesky factorization of a rocprofv3 kernel trace into tree levels (each level starts
with its k_extend_add) and report per level the time in each kernel class, launch count and the span."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
sc = [i for i, r in enumerate(rows) if 'k_chol_scatter' in r['Kernel_Name'] or 'k_vec_init' in r['Kernel_Name']]
a = sc[-2]
b = next(i for i in range(a, len(rows)) if 'k_bwd_gemv' in rows[i]['Kernel_Name'])
seg = rows[a + 1:b]
levels, cur = [], None
for r in seg:
    name = r['Kernel_Name'].split('(')[0].replace('g2ohip::', '').replace('void ', '').split('<')[0]
    if cur is None or (name == 'k_extend_add' and cur['has_ea']):
        cur = {'k': collections.defaultdict(float), 'n': collections.Counter(), 't0': int(r['Start_Timestamp']), 'has_ea': False}
        levels.append(cur)
    if name == 'k_extend_add':
        cur['has_ea'] = True
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cur['k'][name] += d
    cur['n'][name] += 1
    if name == 'k_step':
        cur.setdefault('steps', []).append(d)
    cur['t1'] = int(r['End_Timestamp'])
tot = collections.defaultdict(float)
for l, c in enumerate(levels):
    span = (c['t1'] - c['t0']) / 1e3
    parts = '  '.join('%s %.0f(%d)' % (k[2:], v, c['n'][k]) for k, v in sorted(c['k'].items()))
    print('lev %2d span %8.0f us  %s' % (l, span, parts))
    if c.get('steps'):
        print('        k_step us: ' + ' '.join('%.1f' % v for v in c['steps']))
    for k, v in c['k'].items():
        tot[k] += v
print('total', {k: round(v) for k, v in tot.items()}, 'span %.0f us' % ((int(seg[-1]['End_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3))
