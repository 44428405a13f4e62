#!/usr/bin/env python3
"""Print basic blocks of one kernel in a hipcc -S listing: label, #VALU, #SALU,
#LDS, #VMEM, #MFMA, branch targets (for inner-loop instruction counting)."""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if (l.startswith("_Z") and pat in l.split(":")[0] and ":" in l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
blocks = []
cur = ["entry", dict(v=0, s=0, l=0, m=0, x=0, o=0), []]
for l in lines[start + 1:end]:
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        m = re.match(r"^(\.LBB\S+):", t)
        if m:
            blocks.append(cur)
            cur = [m.group(1), dict(v=0, s=0, l=0, m=0, x=0, o=0), []]
        continue
    op = t.split()[0]
    c = cur[1]
    if op.startswith("v_mfma"):
        c["x"] += 1
    elif op.startswith("v_"):
        c["v"] += 1
    elif op.startswith("s_cbranch") or op.startswith("s_branch"):
        cur[2].append(t.split()[1])
        c["s"] += 1
    elif op.startswith("s_"):
        c["s"] += 1
    elif op.startswith("ds_"):
        c["l"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        c["m"] += 1
    else:
        c["o"] += 1
blocks.append(cur)
for name, c, br in blocks:
    print(f"{name:14s} valu={c['v']:4d} salu={c['s']:3d} lds={c['l']:3d} vmem={c['m']:3d} "
          f"mfma={c['x']:3d} -> {','.join(br)}")
