#!/usr/bin/env python3
"""Effective GPU clock per kernel from one rocprofv3 run with
`--pmc GRBM_GUI_ACTIVE --kernel-trace`: the counter's cycles of the dispatch
over its duration in the kernel trace.  GRBM_GUI_ACTIVE is summed over the
XCDs (divide by `xcds`); reported per kernel name and grid shape as the
median MHz over the dispatches, next to the 2400 MHz peak the issue
roofline assumes.

    python tools/pmc_clock.py <counter_collection.csv> <kernel_trace.csv> [xcds=8]
"""
import collections
import csv
import json
import statistics
import sys


def main():
    cnt, trace = sys.argv[1], sys.argv[2]
    xcds = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    cyc = collections.defaultdict(float)
    for r in csv.DictReader(open(cnt)):
        if r["Counter_Name"].startswith("GRBM_GUI_ACTIVE"):
            cyc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        d = r["Dispatch_Id"]
        if d not in cyc:
            continue
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if ns < 20_000:  # short launches: ramp noise
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = f"{name} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}"
        out[key].append(cyc[d] / xcds / ns * 1e3)  # MHz
    res = {k: {"dispatches": len(v), "median_MHz": round(statistics.median(v), 1),
               "min_MHz": round(min(v), 1), "max_MHz": round(max(v), 1)} for k, v in out.items()}
    print(json.dumps(dict(sorted(res.items(), key=lambda kv: -kv[1]["dispatches"])), indent=1))


if __name__ == "__main__":
    main()
