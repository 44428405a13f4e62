#!/usr/bin/env python3
"""Summarise tools/gpu_pmc_variants.sh: render_bwd / render_fwd HBM bytes per
27-camera launch (FETCH x2 + WRITE) per build variant, next to the product.

    python tools/pmc_variants_summary.py gpurun_out/<TAG>
"""
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    rows = {}
    for p in sorted(glob.glob(os.path.join(d, "traffic_*.json"))):
        n = os.path.basename(p)[len("traffic_"):-len(".json")]
        t = json.load(open(p))
        k = t["kernels"]
        rows[n] = {s: {"fetch_x2_GB": round(v["fetch_bytes_x2"] / 1e9, 3), "write_GB": round(v["write_bytes"] / 1e9, 3)}
                   for s, v in k.items() if s in ("render_bwd", "render_fwd")}
    print(json.dumps(rows, indent=1))
    json.dump(rows, open(os.path.join(d, "traffic_summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
