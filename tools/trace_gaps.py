#!/usr/bin/env python3
"""Idle gaps of a batch bench step in a rocprofv3 kernel trace: steps
delimited by the render_bwd launches of the batch grid (cams x tiles x 4
workgroups of 64 threads; other-mode single-camera steps are skipped), the
median span and idle time per step, and the median gap before each kernel.

    python tools/trace_gaps.py <kernel_trace.csv> <cameras> [tiles=2500]
"""
import csv
import statistics
import sys


def main():
    path, cams = sys.argv[1], int(sys.argv[2])
    tiles = int(sys.argv[3]) if len(sys.argv) > 3 else 2500
    grid = cams * tiles * 4 * 64
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    big = [i for i, r in enumerate(rows) if "render_bwd_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == grid]
    spans, idles, gaps = [], [], {}
    for a, b in zip(big[:-1], big[1:]):
        seg = rows[a + 1:b + 1]
        if any("render_fwd" in r["Kernel_Name"] and int(r["Grid_Size_X"]) != grid for r in seg):
            continue  # another mode's launches in between
        t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
        busy, prev = 0, t0
        for r in seg:
            s, e = max(int(r["Start_Timestamp"]), prev), int(r["End_Timestamp"])
            gaps.setdefault(r["Kernel_Name"].split("(")[0][-45:], []).append(max(0, int(r["Start_Timestamp"]) - prev) / 1e3)
            busy += max(0, e - s)
            prev = max(prev, e)
        spans.append((t1 - t0) / 1e3)
        idles.append((t1 - t0 - busy) / 1e3)
    print(f"steps {len(spans)}: span median {statistics.median(spans):.1f} us, idle median {statistics.median(idles):.1f} us")
    for k, v in gaps.items():
        m = statistics.median(v)
        if m > 0.3:
            print(f"  gap before {k}: {m:.1f} us")


if __name__ == "__main__":
    main()
