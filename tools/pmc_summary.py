#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel, counters averaged per dispatch."""
import collections
import csv
import sys


def summarize(path, width=46):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"][:width]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    out = {}
    for k, v in agg.items():
        n = len(cnt[k])
        out[k] = {c: x / n for c, x in v.items()}
        out[k]["_dispatches"] = n
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for k, v in summarize(p).items():
            print(p.split("/")[-2], k, {c: round(x) for c, x in v.items()})
