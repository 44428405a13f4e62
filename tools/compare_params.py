#!/usr/bin/env python3
"""Compare parameter dumps of bench.py runs (--dump-params): the run under
test against a reference run and a repeat of the reference (the noise floor
of float-atomic summation order).  Prints per tensor the mean / max absolute
difference and exits non-zero if the tested run's mean difference exceeds
max(3 x the floor, 1e-7).

    python tools/compare_params.py test.npz ref.npz ref_repeat.npz
"""
import json
import sys

import numpy as np


def main():
    t, a, b = (np.load(p) for p in sys.argv[1:4])
    out, ok = {}, True
    for k in a.files:
        d = np.abs(t[k].astype(np.float64) - a[k])
        f = np.abs(b[k].astype(np.float64) - a[k])
        out[k] = {"mean": float(d.mean()), "max": float(d.max()), "floor_mean": float(f.mean()),
                  "floor_max": float(f.max())}
        ok &= out[k]["mean"] <= max(3 * out[k]["floor_mean"], 1e-7)
    print(json.dumps(out, indent=1))
    print("OK" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
