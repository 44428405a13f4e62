#!/usr/bin/env python3
"""One line per (config, compat) of tools/parity_errors.py output: image
errors and the worst gradient relative L2 next to the fp32 envelope."""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    fe = d.get("feature", {})
    g = d["grad_rel_l2"]
    worst = max(g, key=lambda k: g[k]["gpu"]) if g else None
    ratio = max((v["gpu"] / max(v["envelope"], 1e-12) for v in g.values()), default=0.0)
    print(f"{json.dumps(d['cfg']):45s} {d['compat'][:3]} color max {d['color']['max']:.1e} "
          f"w1e-5 {d['color']['within_1e5']:.4f} | feat max {fe.get('max', 0):.1e} w1e-5 {fe.get('within_1e5', 1):.4f} "
          f"| grad worst {worst} {g[worst]['gpu'] if worst else 0:.1e} (env {g[worst]['envelope'] if worst else 0:.1e}) "
          f"max gpu/env {ratio:.1f}")
