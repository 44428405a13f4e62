#!/usr/bin/env python3
"""Per-launch instruction counts (rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA
SQ_INSTS_SALU SQ_WAVES) of the rasterizer kernels -> profiles/pmc_valu.json,
used by bench.py for the VALU-issue view of the blend kernels' roofline."""
import collections
import csv
import json
import os
import sys

from pmc_traffic import per_rep


def main():
    with open(sys.argv[1]) as f:
        rows = list(csv.DictReader(f))
    tot = collections.defaultdict(dict)
    for c in sorted({r["Counter_Name"] for r in rows}):
        for (_, key), v in per_rep(rows, c).items():  # refuses uneven launches
            tot[key][c] = v
    cams = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    out = {"kernels": {k: {c: round(v / cams) for c, v in d.items()} for k, d in tot.items()},
           "per": "camera", "cams_per_launch": cams,
           "method": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES; per rep (one launch "
                     f"per stage) / cameras per launch; tools/batch_steps.py ({cams} cameras per launch, "
                     "two-phase forward, reps checked equal: pmc_traffic.per_rep)"}
    wl = os.environ.get("PMC_WORKLOAD")
    if wl:
        out["workload"] = json.loads(wl)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                        "pmc_valu.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out["kernels"]))


if __name__ == "__main__":
    main()
