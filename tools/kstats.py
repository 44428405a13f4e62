#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for r in rows[:n]:
    name = r["Name"]
    name = name.replace("void ", "").split("(")[0][:60]
    print(f"{name:60s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} us {float(r['Percentage']):6.2f}%")
