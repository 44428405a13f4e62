#!/usr/bin/env python3
"""One training step of a rocprofv3 kernel trace, kernel by kernel: start
offset, duration, name, and the step's span vs summed kernel time (the host
gaps).  The step is delimited by consecutive launches of the batch render_bwd
of the given camera count.

    python tools/step_trace.py <kernel_trace.csv> CAMS [TILES=2500] [STEP_INDEX=10]
"""
import csv
import sys


def main():
    path, cams = sys.argv[1], int(sys.argv[2])
    tiles = int(sys.argv[3]) if len(sys.argv) > 3 else 2500
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    big = [i for i, r in enumerate(rows) if "render_bwd" in r["Kernel_Name"]
           and int(r["Grid_Size_X"]) == cams * tiles * 4 * 64]
    i0, i1 = big[k], big[k + 1]
    t0 = int(rows[i0]["End_Timestamp"])
    t1 = int(rows[i1]["End_Timestamp"])
    busy, prev_end = 0, t0
    for r in rows[i0 + 1:i1 + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        gap = (s - prev_end) / 1e3
        prev_end = e
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} gap {gap:6.1f}  {r['Kernel_Name'][:80]}")
    print(f"span {(t1 - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, {i1 - i0} launches")


if __name__ == "__main__":
    main()
