#!/usr/bin/env python3
"""Per-launch instruction counts (rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA
SQ_INSTS_SALU SQ_WAVES) of the rasterizer kernels -> profiles/pmc_valu.json,
used by bench.py for the VALU-issue view of the blend kernels' roofline."""
import collections
import csv
import json
import os
import sys

from pmc_traffic import STAGE_OF


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        for key, stage in STAGE_OF.items():
            if key in r["Kernel_Name"]:
                tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[key].add(r["Dispatch_Id"])
    cams = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    out = {"kernels": {k: {c: round(v / len(disp[k]) / cams) for c, v in d.items()} for k, d in tot.items()},
           "per": "camera", "cams_per_launch": cams,
           "method": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES; per launch / cameras "
                     f"per launch; tools/batch_steps.py ({cams} cameras per launch)"}
    wl = os.environ.get("PMC_WORKLOAD")
    if wl:
        out["workload"] = json.loads(wl)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "pmc_valu.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out["kernels"]))


if __name__ == "__main__":
    main()
