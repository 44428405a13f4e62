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

from pmc_traffic import per_rep


def main():
    cams = int(sys.argv[1])
    tot = collections.defaultdict(dict)
    for path in sys.argv[2:]:
        with open(path) as f:
            rows = list(csv.DictReader(f))
        for c in sorted({r["Counter_Name"] for r in rows}):
            for (_, key), v in per_rep(rows, c).items():  # refuses uneven launches
                tot[key][c] = v
    out = {k: {c: round(v / cams) for c, v in sorted(d.items())} for k, d in tot.items()}
    print(json.dumps({"per": "camera", "cams_per_launch": cams, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
