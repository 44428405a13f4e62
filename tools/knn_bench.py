#!/usr/bin/env python3
"""k-NN timing at the reference's call shapes: k = 3 (initial scales,
train.py:95) and k = 20 (neighbour graph, train.py:316-326) on clustered
synthetic clouds.  JSON lines.

    python tools/knn_bench.py --n 300000 --reps 5
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd.knn import knn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[100000, 300000, 1000000])
    ap.add_argument("--k", type=int, nargs="+", default=[3, 20])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    for n in a.n:
        g = np.random.default_rng(0)
        c = g.random((64, 3)) * 4
        p = (c[g.integers(0, 64, n)] + g.normal(0, 0.05, (n, 3))).astype(np.float32)
        pts = torch.from_numpy(p).cuda()
        for k in a.k:
            knn(pts, k)
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.reps):
                knn(pts, k)
            s1.record()
            torch.cuda.synchronize()
            print(json.dumps({"N": n, "k": k, "ms": round(s0.elapsed_time(s1) / a.reps, 3)}), flush=True)


if __name__ == "__main__":
    main()
