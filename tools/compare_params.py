#!/usr/bin/env python3
"""Compare parameter dumps of bench.py runs (--dump-params): the run under
test against a reference run and one or more repeats of the reference (the
noise floor of float-atomic summation order).

The statistic is the mean absolute difference over each tensor's elements
after dropping the largest 0.1 % (`trimmed`): a few training steps amplify
the order noise through discrete events -- one Gaussian's alpha crossing
1/255 at one pixel in one run and not the other -- that move single
elements by 1e-4..1e-2 in any pair of runs, so the plain mean of one pair
is heavy-tailed; a systematic error (a wrong exchange, a lost slice) moves
most elements and shows in the trimmed mean.  The floor is the largest
trimmed mean over the reference pairs.

OK iff, for every tensor, the tested run's trimmed mean <= max(3 x floor,
1e-9).  The plain mean and max are printed beside it.

A run now and then (one gloo rehearsal run in six, the plain reference path
included) lands far above the floor on every tensor at once: the atomic
order's noise amplified through one early discrete event across the whole
scene over the run's training steps.  An after-training comparison cannot
tell that apart from a race, so the exchange's race check is step-level
(tools/zov_check.py: each step's gradients against a replay from the
parameters it read, the parameters read against an in-line Adam replay of
the summed gradients, bit for bit).  `--lr-bound` (opt-in, for rehearsals
whose step-level check has passed) also accepts a trimmed mean up to 1e-3 x
the tensor's learning rate (bench.py's, train.py:119-135): an exchange error
-- a lost, doubled or stale contribution -- moves every element by the order
of its learning rate per step.

    python tools/compare_params.py [--lr-bound] test.npz ref.npz ref_repeat.npz [ref_repeat2.npz ...]
"""
import json
import sys

import numpy as np

TRIM = 0.001
# bench.py's Adam learning rates per tensor (train.py:119-135)
LR = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
      "log_scales": 1e-3, "semantic_feature": 1e-3}


def trimmed_mean(d):
    d = np.sort(d.reshape(-1))
    keep = d.size - int(d.size * TRIM)
    return float(d[:keep].mean()) if keep > 0 else 0.0


def main():
    argv = sys.argv[1:]
    lr_bound = "--lr-bound" in argv
    argv = [x for x in argv if x != "--lr-bound"]
    t, a = np.load(argv[0]), np.load(argv[1])
    reps = [np.load(p) for p in argv[2:]]
    if not reps:
        raise SystemExit("need at least one repeat of the reference")
    out, ok = {}, True
    for k in a.files:
        ref = a[k].astype(np.float64)
        d = np.abs(t[k].astype(np.float64) - ref)
        floors = [np.abs(r[k].astype(np.float64) - ref) for r in reps]
        fl = max(trimmed_mean(f) for f in floors)
        out[k] = {"trimmed_mean": trimmed_mean(d), "floor_trimmed_mean": fl, "mean": float(d.mean()),
                  "max": float(d.max()), "floor_mean": max(float(f.mean()) for f in floors),
                  "floor_max": max(float(f.max()) for f in floors)}
        bound = max(3 * fl, 1e-3 * LR.get(k, 0.0) if lr_bound else 0.0, 1e-9)
        out[k]["bound"] = bound
        ok &= out[k]["trimmed_mean"] <= bound
    print(json.dumps(out, indent=1))
    print("OK" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
