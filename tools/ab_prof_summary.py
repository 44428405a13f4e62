#!/usr/bin/env python3
"""Average kernel durations per variant from gpurun_out/abp/<variant>_<round>/**/k_kernel_stats.csv."""
import collections
import csv
import glob
import os
import statistics

res = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob("gpurun_out/abp/*/**/k_kernel_stats.csv", recursive=True):
    var = os.path.relpath(p, "gpurun_out/abp").split(os.sep)[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(p)):
        name = r["Name"].replace("void ", "").split("(")[0]
        if "render" in name or "preprocess" in name or "tile" in name:
            res[var][name[:40]].append(float(r["AverageNs"]) / 1e3)
for var, ks in sorted(res.items()):
    print(var)
    for k, v in sorted(ks.items()):
        print(f"   {k:40s} {statistics.median(v):8.2f} us  (n={len(v)})")
