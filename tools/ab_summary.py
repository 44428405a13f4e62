#!/usr/bin/env python3
"""Median blend-kernel times per variant from gpurun_out/ab_lib.jsonl."""
import collections
import json
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_lib.jsonl"
res = collections.defaultdict(lambda: collections.defaultdict(list))
v = None
for line in open(path):
    if line.startswith("variant="):
        v = line.strip().split("=", 1)[1] or "product"
        continue
    d = json.loads(line)
    for k, t in d["stages_ms_per_cam"].items():
        res[(v, d["F"])][k].append(t)
    res[(v, d["F"])]["total"].append(d["total_ms_per_cam"])
for (v, F), st in res.items():
    print(f"{v:16s} F={F:2d} " + " ".join(f"{k}={statistics.median(x):.4f}" for k, x in st.items()
                                           if k in ("render_fwd", "render_bwd", "total")) + f" (n={len(st['total'])})")
