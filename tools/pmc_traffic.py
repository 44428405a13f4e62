#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs
(separate passes), corrected as MI355X_MICROARCH.md prescribes for gfx950:
FETCH_SIZE counts half the bytes of wide coalesced reads -> x2.  Writes the
per-stage bytes to profiles/pmc_traffic.json for bench.py's roofline.traffic.

    python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv [CAMS]

CAMS = cameras per launch of the profiled program (tools/batch_steps.py: 27);
the file keeps bytes per camera (bench.py multiplies by its cameras per launch).
"""
import collections
import csv
import json
import os
import sys

STAGE_OF = {"preprocess_fwd": "preprocess", "tile_hist_kernel<false>": "scan", "tile_rowscan": "scan",
            "tile_offsets": "scan", "tile_hist_kernel<true>": "duplicate", "tile_bucket": "duplicate",
            "tile_order": "ranges", "tile_sort": "sort",
            "render_fwd": "render_fwd", "render_bwd": "render_bwd", "preprocess_bwd": "preprocess_bwd"}


# The counted program runs the same batch forward + backward REPS times
# (tools/batch_steps.py --reps, two-phase forward): every kernel's dispatches
# fall into REPS equal groups of equal work.  A group count that does not
# divide, or a group with less work than the others (e.g. a sync-free
# forward's first call, which renders every camera empty and retries), means
# the counts are not of the workload they claim, and the tools refuse them.
REPS = int(os.environ.get("PMC_REPS", "2"))
TOL = float(os.environ.get("PMC_TOL", "0.2"))


class UnevenLaunches(ValueError):
    """A kernel's dispatches do not split into equal reps of equal work."""


def per_rep(rows, counter, reps=None, tol=None, stages=None):
    """{(stage, kernel key): counter sum per rep} over csv rows (dicts) whose
    Counter_Name satisfies `counter` (a name or a predicate); raises
    UnevenLaunches when a kernel's dispatches are not `reps` groups (in
    dispatch order) of equal work within `tol`."""
    reps = REPS if reps is None else int(reps)
    tol = TOL if tol is None else float(tol)
    stages = STAGE_OF if stages is None else stages
    match = counter if callable(counter) else (lambda c: c == counter)
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if not match(r["Counter_Name"]):
            continue
        name = r["Kernel_Name"]
        for key, stage in stages.items():
            if key in name:
                vals[(stage, key)][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for k, d in vals.items():
        ids = sorted(d)
        if len(ids) % reps:
            raise UnevenLaunches(f"{k[1]}: {len(ids)} dispatches for {reps} reps (a retried or extra launch)")
        m = len(ids) // reps
        sums = [sum(d[i] for i in ids[j * m:(j + 1) * m]) for j in range(reps)]
        hi = max(sums)
        if hi > 0 and min(sums) < (1.0 - tol) * hi:
            raise UnevenLaunches(f"{k[1]}: per-rep work {[round(x) for x in sums]} differs by more than "
                                 f"{tol:.0%} (an empty or partial launch)")
        out[k] = sum(sums) / reps
    return out


def per_kernel(path, counter):
    """Per rep (= per launch of each stage) sums of one counter."""
    with open(path) as f:
        return per_rep(csv.DictReader(f), counter)


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    stages = collections.defaultdict(float)
    detail = {}
    for k in set(fetch) | set(write):
        fb = 2.0 * fetch.get(k, 0.0) * 1024.0  # KB -> B, gfx950 x2 correction
        wb = write.get(k, 0.0) * 1024.0
        stages[k[0]] += fb + wb
        detail[k[1]] = {"fetch_bytes_x2": fb, "write_bytes": wb}
    cams = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    out = {"bytes_per_camera": {k: int(v / cams) for k, v in stages.items()},
           "bytes_per_launch": {k: int(v) for k, v in stages.items()}, "cams_per_launch": cams, "kernels": detail,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes), FETCH_SIZE x2 "
                     "(gfx950 correction), KB -> bytes; tools/batch_steps.py (300k Gaussians, "
                     f"{cams} cameras 800x800 per launch, F = 32)"}
    wl = os.environ.get("PMC_WORKLOAD")
    if wl:
        out["workload"] = json.loads(wl)
    path = os.environ.get("PMC_TRAFFIC_OUT") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out["bytes_per_launch"]))


if __name__ == "__main__":
    main()
