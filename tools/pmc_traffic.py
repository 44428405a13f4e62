#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs
(separate passes), corrected as MI355X_MICROARCH.md prescribes for gfx950:
FETCH_SIZE counts half the bytes of wide coalesced reads -> x2.  Writes the
per-stage bytes to profiles/pmc_traffic.json for bench.py's roofline.traffic.

    python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv [CAMS]

CAMS = cameras per launch of the profiled program (tools/batch_steps.py: 27);
the file keeps bytes per camera (bench.py multiplies by its cameras per launch).
"""
import collections
import csv
import json
import os
import sys

STAGE_OF = {"preprocess_fwd": "preprocess", "tile_hist_kernel<false>": "scan", "tile_rowscan": "scan",
            "tile_offsets": "scan", "tile_hist_kernel<true>": "duplicate", "tile_bucket": "duplicate",
            "tile_order": "ranges", "tile_sort": "sort",
            "render_fwd": "render_fwd", "render_bwd": "render_bwd", "preprocess_bwd": "preprocess_bwd"}


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for key, stage in STAGE_OF.items():
            if key in name:
                tot[(stage, key)] += float(r["Counter_Value"])
                disp[(stage, key)].add(r["Dispatch_Id"])
    return {k: tot[k] / len(disp[k]) for k in tot}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    stages = collections.defaultdict(float)
    detail = {}
    for k in set(fetch) | set(write):
        fb = 2.0 * fetch.get(k, 0.0) * 1024.0  # KB -> B, gfx950 x2 correction
        wb = write.get(k, 0.0) * 1024.0
        stages[k[0]] += fb + wb
        detail[k[1]] = {"fetch_bytes_x2": fb, "write_bytes": wb}
    cams = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    out = {"bytes_per_camera": {k: int(v / cams) for k, v in stages.items()},
           "bytes_per_launch": {k: int(v) for k, v in stages.items()}, "cams_per_launch": cams, "kernels": detail,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes), FETCH_SIZE x2 "
                     "(gfx950 correction), KB -> bytes; tools/batch_steps.py (300k Gaussians, "
                     f"{cams} cameras 800x800 per launch, F = 32)"}
    wl = os.environ.get("PMC_WORKLOAD")
    if wl:
        out["workload"] = json.loads(wl)
    path = os.environ.get("PMC_TRAFFIC_OUT") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out["bytes_per_launch"]))


if __name__ == "__main__":
    main()
