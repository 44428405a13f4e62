#!/usr/bin/env python3
"""Per-launch sums of arbitrary rocprofv3 --pmc counters for the rasterizer
kernels (any number of counter_collection.csv files, one per pass), printed
as JSON per kernel and per camera.

    python tools/pmc_generic.py CAMS pass1/..._counter_collection.csv [pass2/...]
"""
import collections
import csv
import json
import sys

from pmc_traffic import STAGE_OF


def main():
    cams = int(sys.argv[1])
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in sys.argv[2:]:
        for r in csv.DictReader(open(path)):
            for key in STAGE_OF:
                if key in r["Kernel_Name"]:
                    tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[key][r["Counter_Name"]].add(r["Dispatch_Id"])
    out = {k: {c: round(v / len(disp[k][c]) / cams) for c, v in sorted(d.items())} for k, d in tot.items()}
    print(json.dumps({"per": "camera", "cams_per_launch": cams, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
