#!/usr/bin/env python3
"""Memory-side float-atomic requests per launch from a rocprofv3
--pmc TCC_EA0_ATOMIC_sum run (each request = one 64-B atomic segment,
MI355X_MICROARCH.md "Global float atomics"), per camera, written to
profiles/pmc_atomic.json for bench.py's roofline.atomics view.

    python tools/pmc_atomic.py ATOMIC_counter_collection.csv [CAMS]
"""
import csv
import json
import os
import sys

from pmc_traffic import per_rep

KERNELS = {"render_bwd": "render_bwd", "render_fwd": "render_fwd", "preprocess_bwd": "preprocess_bwd"}


def main():
    with open(sys.argv[1]) as f:
        tot = {stage: v for (stage, _), v in per_rep(csv.DictReader(f), lambda c: c.startswith("TCC_EA0_ATOMIC"),
                                                     stages=KERNELS).items()}
    cams = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    out = {"requests_per_camera": {k: int(tot[k] / cams) for k in tot},
           "bytes_per_request": 64, "cams_per_launch": cams,
           "method": "rocprofv3 --pmc TCC_EA0_ATOMIC_sum on tools/batch_steps.py (27-camera launches), "
                     "per launch / cameras per launch"}
    wl = os.environ.get("PMC_WORKLOAD")
    if wl:
        out["workload"] = json.loads(wl)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_atomic.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
