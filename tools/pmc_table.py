"""Dev: per-kernel mean of every collected counter from tools/pmc_diag.sh passes."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("g2ohip::", "")
        vals[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in sorted(vals.items()):
    print(n)
    for c, v in sorted(cs.items()):
        print("   %-34s %14.4g" % (c, sum(v) / len(v)))
