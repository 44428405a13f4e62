"""Per-kernel launch durations from a rocprofv3 kernel trace, split by grid
shape (the bench times the camera batch and the per-camera drop-in in one
process, so the --stats averages mix both).  Usage:
  python tools/kernel_split.py <kernel_trace.csv> [out.json]"""
import collections
import csv
import json
import sys


def split(path):
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = f"{name} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
        g[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {k: {"launches": len(v), "avg_us": round(sum(v) / len(v), 2), "total_us": round(sum(v), 1)}
           for k, v in g.items()}
    return dict(sorted(out.items(), key=lambda kv: -kv[1]["total_us"]))


if __name__ == "__main__":
    d = split(sys.argv[1])
    s = json.dumps({"source": sys.argv[1], "kernels": d}, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")
    for k, v in list(d.items())[:16]:
        print(f"{v['avg_us']:10.1f} us x {v['launches']:5d}  {k}")
