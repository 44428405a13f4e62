#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter CSVs (any number of passes
over the same workload): counters averaged per launch for every kernel name
(template arguments included), and the wave-cycle split when the pass holds
SQ_WAVE_CYCLES with SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / SQ_WAIT_INST_ANY
(disjoint buckets: issuing, parked at s_waitcnt or a barrier, issue-stalled).

    python tools/pmc_split.py <counter_collection.csv> [...]
"""
import collections
import csv
import json
import sys


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            c = r["Counter_Name"]
            tot[name][c] += float(r["Counter_Value"])
            # dispatch ids restart in every profiled process: a counter
            # collected in two passes has twice the launches
            disp[name][c].add((path, r["Dispatch_Id"]))
    out = {}
    for name, d in sorted(tot.items()):
        per = {c: v / max(1, len(disp[name][c])) for c, v in d.items()}
        row = {c: round(v) for c, v in sorted(per.items())}
        wc = per.get("SQ_WAVE_CYCLES")
        if wc:
            for k, lab in (("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_WAIT_ANY", "parked"),
                           ("SQ_WAIT_INST_ANY", "issue_stalled"), ("SQ_WAIT_INST_LDS", "lds_issue_stalled")):
                if k in per:
                    row[f"frac_{lab}"] = round(per[k] / wc, 3)
        if per.get("SQ_WAVES"):
            row["valu_per_wave"] = round(per.get("SQ_INSTS_VALU", 0) / per["SQ_WAVES"], 1)
            row["lds_per_wave"] = round(per.get("SQ_INSTS_LDS", 0) / per["SQ_WAVES"], 1)
        if per.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict_frac"] = round(per.get("SQ_LDS_BANK_CONFLICT", 0) / per["SQ_LDS_IDX_ACTIVE"], 3)
        row["launches"] = max(len(s) for s in disp[name].values())
        out[name] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
