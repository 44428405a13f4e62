#!/usr/bin/env python3
"""Neighbour-loss kernel summary from rocprofv3 stats + FETCH/WRITE PMC
passes (gfx950 FETCH x2 correction, MI355X_MICROARCH.md): per kernel average
duration, algorithmic bytes (N, K given), PMC bytes, achieved GB/s.

    python tools/nb_prof_summary.py gpurun_out/nbprof/nb_kernel_stats.csv \
        gpurun_out/nbpmcF/pmc_counter_collection.csv gpurun_out/nbpmcW/pmc_counter_collection.csv --n 150000 --k 20
"""
import argparse
import collections
import csv
import json
import re


def algo_bytes(name, N, K):
    NK = N * K
    if "nb_prep" in name:            # fg_rot + prev_inv in, rel_rot (16 B) + rotation record (48 B) out
        return N * (16 + 16 + 64)
    if "nb_fwd" in name:             # nbr, w, dist, prev_offset + own record/pts per Gaussian
        return NK * (8 + 4 + 4 + 12) + N * (64 + 12)
    if "nb_bwd" in name:             # same reads + rev_pos + 32-B pair record + 32-B own record
        return NK * (8 + 4 + 4 + 12 + 4 + 32) + N * (64 + 12 + 32)
    if "nb_gather" in name:          # pair records (reverse order) + rev_ptr + own record + prev_inv + grads out
        return NK * 32 + N * (4 + 32 + 16 + 12 + 16)
    return None


def short(name):
    m = re.search(r"(nb_[a-z_]+kernel)", name)
    return m.group(1) if m else None


def pmc(path, counter):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        if k:
            tot[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: tot[k] / len(disp[k]) * 1024.0 for k in tot}  # KB -> B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--k", type=int, required=True)
    a = ap.parse_args()
    fetch, write = pmc(a.fetch, "FETCH_SIZE"), pmc(a.write, "WRITE_SIZE")
    out = {}
    for r in csv.DictReader(open(a.stats)):
        k = short(r["Name"])
        if not k:
            continue
        us = float(r["AverageNs"]) / 1000.0
        ab = algo_bytes(k, a.n, a.k)
        traffic = (2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)) if k in fetch else None
        out[k] = {"avg_us": round(us, 2), "calls": int(r["Calls"]),
                  "algo_MB": round(ab / 1e6, 2) if ab else None,
                  "achieved_GBs": round(ab / us / 1e3, 1) if ab else None,
                  "frac_of_8TBs": round(ab / us / 1e3 / 8000.0, 3) if ab else None,
                  "pmc_MB": round(traffic / 1e6, 2) if traffic else None}
    print(json.dumps({"N": a.n, "K": a.k, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
