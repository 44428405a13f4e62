#!/usr/bin/env python3
"""bench.py with the host's time split: time spent inside gs_forward_plan
(which ends with the plan's device->host read, i.e. waits for the GPU) vs the
rest of the step on the host.  Prints one extra JSON line after bench's."""
import atexit
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd import _lib  # noqa: E402

L = _lib.load()
acc = {"plan_s": 0.0, "plan_calls": 0, "bwd_s": 0.0, "bwd_calls": 0, "render_s": 0.0}
for name, key in (("gs_forward_plan", "plan"), ("gs_backward", "bwd"), ("gs_forward_render", "render")):
    orig = getattr(L, name)

    def wrap(*a, _orig=orig, _key=key):
        t0 = time.perf_counter()
        r = _orig(*a)
        acc[_key + "_s"] += time.perf_counter() - t0
        if _key + "_calls" in acc:
            acc[_key + "_calls"] += 1
        return r
    setattr(L, name, wrap)

atexit.register(lambda: print(json.dumps({k: round(v, 4) if isinstance(v, float) else v for k, v in acc.items()}),
                              flush=True))
t_start = time.perf_counter()
import bench  # noqa: E402

bench.main()
acc["wall_s"] = time.perf_counter() - t_start
