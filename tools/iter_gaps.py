"""Dev helper: GPU idle gaps in a rocprofv3 kernel trace (--kernel-trace --output-format csv): every gap longer than
a threshold between one dispatch's end and the next one's start, with the kernels on either side, and the totals per
LM iteration (an iteration starts at each k_copy_multi = push()).   python tools/iter_gaps.py TRACE.csv [MIN_US]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
rows.sort(key=lambda r: int(r['Start_Timestamp']))


def short(n):
    return n.split('(')[0].replace('void ', '').replace('g2ohip::', '')[:40]


starts = [i for i, r in enumerate(rows) if 'k_copy_multi' in r['Kernel_Name']]
for a, b in zip(starts[-6:-1], starts[-5:]):
    seg = rows[a:b]
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seg) / 1e3
    period = (int(rows[b]['Start_Timestamp']) - int(seg[0]['Start_Timestamp'])) / 1e3
    gaps = []
    for x, y in zip(seg, seg[1:] + [rows[b]]):
        g = (int(y['Start_Timestamp']) - int(x['End_Timestamp'])) / 1e3
        if g > thr:
            gaps.append((round(g, 1), short(x['Kernel_Name']), short(y['Kernel_Name'])))
    print(f"period {period:.1f} us, busy {busy:.1f} us, {len(seg)} dispatches, gaps > {thr} us: {sum(g[0] for g in gaps):.1f}")
    for g in sorted(gaps, reverse=True)[:8]:
        print("   ", g)
