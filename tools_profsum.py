"""Summarise a rocprofv3 kernel_stats.csv (dev helper)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print(r['Name'][:58].ljust(58), r['Calls'].rjust(5), '%10.1f us tot' % (float(r['TotalDurationNs'])/1e3), '%9.2f us avg' % (float(r['AverageNs'])/1e3), r['Percentage'][:5])
