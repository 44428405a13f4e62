#!/usr/bin/env python3
"""GPU busy fraction (union of kernel intervals) over the last N render_bwd
launches' window of a rocprofv3 kernel trace, and the largest idle gaps."""
import csv
import sys

path = sys.argv[1]
ncam = int(sys.argv[2]) if len(sys.argv) > 2 else 81
rows = list(csv.DictReader(open(path)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows)
bw = [i for i, x in enumerate(iv) if "render_bwd" in x[2]]
start, end = iv[bw[-ncam]][0], iv[bw[-1]][1]
busy, gaps, cur_s, cur_e = 0, [], None, None
for s, e, n in iv:
    if e < start or s > end:
        continue
    s, e = max(s, start), min(e, end)
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
gaps.sort(reverse=True)
print(f"window {(end - start) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms ({busy / (end - start):.3f}), "
      f"idle gaps {len(gaps)}, total {sum(g for g, _ in gaps) / 1e6:.3f} ms")
print("largest gaps (us, next kernel):", [(round(g / 1e3, 1), n) for g, n in gaps[:8]])
