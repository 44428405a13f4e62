#!/usr/bin/env python3
"""Per-kernel register / occupancy summary of a hipcc -S listing."""
import re
import sys

cur = None
rows = {}
for line in open(sys.argv[1]):
    m = re.match(r"^(_Z\S+):", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.match(r"^; (TotalNumVgprs|NumVgprs|Occupancy|ScratchSize|LDSByteSize): (\d+)", line)
    if m and cur:
        rows[cur].setdefault(m.group(1), int(m.group(2)))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in rows.items():
    if pat in k:
        name = re.sub(r"EEEv.*", "", k.replace("_ZN2gs", ""))
        print(f"{name:40s} vgpr={v.get('NumVgprs')} total={v.get('TotalNumVgprs')} occ={v.get('Occupancy')} "
              f"scratch={v.get('ScratchSize')} lds={v.get('LDSByteSize')}")
