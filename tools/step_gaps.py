#!/usr/bin/env python3
"""Per-step GPU timeline of a rocprofv3 kernel trace of a batch bench run:
steps delimited by the render_bwd launches with the largest grid (the timed
batch), each step's span, summed kernel time and idle gaps, and one step
kernel by kernel.  Works for window splits (any grid).

    python tools/step_gaps.py <kernel_trace.csv> [STEP_INDEX=-5]
"""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else -5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    bwd = [i for i, r in enumerate(rows) if "render_bwd_kernel" in r["Kernel_Name"]]
    grid = collections.Counter(int(rows[i]["Grid_Size_X"]) for i in bwd).most_common(1)[0][0]
    big = [i for i in bwd if int(rows[i]["Grid_Size_X"]) == grid]
    spans, busys = [], []
    for a, b in zip(big[:-1], big[1:]):
        t0, t1 = int(rows[a]["End_Timestamp"]), int(rows[b]["End_Timestamp"])
        busy, prev = 0, t0
        for r in rows[a + 1:b + 1]:
            s, e = max(int(r["Start_Timestamp"]), prev), int(r["End_Timestamp"])
            busy += max(0, e - s)
            prev = max(prev, e)
        spans.append((t1 - t0) / 1e3)
        busys.append(busy / 1e3)
    tail = slice(len(spans) // 2, None)
    print(f"steps {len(spans)}; last half: span median {statistics.median(spans[tail]):.1f} us, "
          f"busy median {statistics.median(busys[tail]):.1f} us, idle median "
          f"{statistics.median([s - b for s, b in zip(spans[tail], busys[tail])]):.1f} us")
    a, b = big[k - 1], big[k]
    t0 = int(rows[a]["End_Timestamp"])
    prev = t0
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f}  "
              f"{r['Kernel_Name'][:70]} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}")
        prev = max(prev, e)


if __name__ == "__main__":
    main()
