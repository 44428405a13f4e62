"""The analysis tools the round's GPU evidence rests on, on synthetic inputs:
tools/compare_params.py (the exchange rehearsals' verdict),
tools/split_predict.py (the configs[3] prediction) and tools/pmc_split.py (the
binning kernels' PMC summary)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    return subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True)


def test_compare_params_tolerates_order_noise_and_flips_but_not_a_systematic_error(tmp_path):
    rng = np.random.default_rng(0)
    base = rng.standard_normal(200_000).astype(np.float32)

    def run_like():
        x = base + rng.standard_normal(base.size).astype(np.float32) * 1e-8
        x[rng.integers(0, base.size, 40)] += 1e-3  # discrete alpha-threshold flips
        return x
    paths = {}
    for name in ("ref_a", "ref_b", "ref_c", "ok"):
        paths[name] = str(tmp_path / f"{name}.npz")
        np.savez(paths[name], p=run_like())
    bad = run_like()
    bad[::2] += 1e-6  # half the elements off: a lost contribution
    paths["bad"] = str(tmp_path / "bad.npz")
    np.savez(paths["bad"], p=bad)
    refs = [paths["ref_a"], paths["ref_b"], paths["ref_c"]]
    ok = _run(["tools/compare_params.py", paths["ok"]] + refs)
    assert ok.returncode == 0 and ok.stdout.strip().endswith("OK"), ok.stdout + ok.stderr
    bad_r = _run(["tools/compare_params.py", paths["bad"]] + refs)
    assert bad_r.returncode == 1 and bad_r.stdout.strip().endswith("MISMATCH"), bad_r.stdout + bad_r.stderr


def test_split_predict_takes_the_slowest_rank_and_the_exposed_exchange(tmp_path):
    full = {"ms_per_step": 9.0, "config": {"workload": "300k Gaussians x 27 cams"}}
    fp = tmp_path / "full.json"
    fp.write_text(json.dumps(full))
    proxies = []
    for r in range(8):
        for rep, ms in enumerate((1.30 + 0.01 * r, 1.31 + 0.01 * r)):
            d = {"ms_per_step": ms, "config": {"workload": f"rank {r} of 8 of 300k Gaussians x 27 cams split"},
                 "stages_ms_per_step": {"preprocess": 0.06, "scan": 0.05, "duplicate": 0.05, "sort": 0.08,
                                        "ranges": 0.01}}
            p = tmp_path / f"p{r}_{rep}.json"
            p.write_text(json.dumps(d))
            proxies.append(str(p))
    out = _run(["tools/split_predict.py", str(fp)] + proxies)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert d["slowest_rank"] == 7 and abs(d["slowest_rank_ms"] - 1.375) < 1e-9
    pr = d["predictions"]["300GB/s overlapped"]
    # geometry ring all-reduce of 300k x 14 fp32 at 300 GB/s, 8 ranks
    geo = 2 * 7 / 8 * 300_000 * 14 * 4 / 300e9 * 1e3
    assert abs(pr["geometry_allreduce_ms"] - round(geo, 3)) < 1e-9
    assert abs(pr["step_ms"] - round(1.375 + pr["exposed_ms"], 4)) < 1e-4
    assert abs(pr["speedup_vs_1gpu"] - round(9.0 / pr["step_ms"], 3)) < 1e-3


def test_compare_params_bounds_by_the_learning_rate(tmp_path):
    # a chaotic run far above the floor but far below one update, and an
    # exchange error of one update per element
    rng = np.random.default_rng(1)
    base = rng.standard_normal(100_000).astype(np.float32)

    def run_like(shift=0.0):
        return {"means3D": base + rng.standard_normal(base.size).astype(np.float32) * 1e-11 + shift}
    paths = {}
    for name, shift in (("a", 0.0), ("b", 0.0), ("c", 0.0), ("chaos", 5e-8), ("error", 1.6e-4)):
        paths[name] = str(tmp_path / f"{name}.npz")
        np.savez(paths[name], **run_like(shift))
    refs = [paths["a"], paths["b"], paths["c"]]
    # strict by default (3 x floor); the lr-scaled bound only when asked for
    assert _run(["tools/compare_params.py", paths["chaos"]] + refs).returncode == 1
    assert _run(["tools/compare_params.py", "--lr-bound", paths["chaos"]] + refs).returncode == 0
    assert _run(["tools/compare_params.py", "--lr-bound", paths["error"]] + refs).returncode == 1


def test_pmc_split_averages_per_launch_and_splits_wave_cycles(tmp_path):
    # two passes over the same two launches of one kernel, as rocprofv3 writes them
    hdr = "Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n"
    k = "void gs::tile_sort_kernel<256, 10, 8>(gs::TileArgs, gs::CamBatch, int, int, int, int)"
    p1 = tmp_path / "p1.csv"
    p1.write_text(hdr + "".join(f'{d},"{k}",{c},{v}\n' for d in (1, 2) for c, v in
                                (("SQ_WAVE_CYCLES", 1000), ("SQ_ACTIVE_INST_ANY", 200), ("SQ_WAIT_ANY", 700),
                                 ("SQ_WAIT_INST_ANY", 100), ("SQ_WAVES", 10), ("SQ_INSTS_VALU", 2770),
                                 ("SQ_INSTS_LDS", 660))))
    p2 = tmp_path / "p2.csv"
    p2.write_text(hdr + "".join(f'{d},"{k}",{c},{v}\n' for d in (1, 2) for c, v in
                                (("SQ_LDS_BANK_CONFLICT", 35), ("SQ_LDS_IDX_ACTIVE", 100))))
    r = _run(["tools/pmc_split.py", str(p1), str(p2)])
    assert r.returncode == 0, r.stderr
    row = json.loads(r.stdout)["gs::tile_sort_kernel<256, 10, 8>"]
    assert row["SQ_WAVE_CYCLES"] == 1000 and row["launches"] == 2
    assert (row["frac_issuing"], row["frac_parked"], row["frac_issue_stalled"]) == (0.2, 0.7, 0.1)
    assert row["valu_per_wave"] == 277.0 and row["lds_per_wave"] == 66.0 and row["lds_conflict_frac"] == 0.35


def _pmc_csv(path, rows):
    import csv
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, k, c, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": c, "Counter_Value": v})


def test_pmc_tools_refuse_an_empty_or_extra_launch(tmp_path):
    """tools/pmc_*.py count per rep of the profiled program (two reps of one
    launch per stage): a render_fwd launch that rendered nothing (the
    sync-free forward's first call, which retries) or an extra dispatch is
    refused instead of diluting the per-launch average."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic as T
    good = [(1, "render_fwd_kernel<32, 0>", "SQ_INSTS_VALU", 900.0), (2, "render_bwd_kernel<32, 0>", "SQ_INSTS_VALU", 50.0),
            (3, "tile_sort_kernel<256>", "SQ_INSTS_VALU", 7.0), (4, "tile_sort_kernel<512>", "SQ_INSTS_VALU", 3.0),
            (5, "render_fwd_kernel<32, 0>", "SQ_INSTS_VALU", 910.0), (6, "render_bwd_kernel<32, 0>", "SQ_INSTS_VALU", 50.0),
            (7, "tile_sort_kernel<256>", "SQ_INSTS_VALU", 7.0), (8, "tile_sort_kernel<512>", "SQ_INSTS_VALU", 3.0)]
    rows = [dict(Dispatch_Id=d, Kernel_Name=k, Counter_Name=c, Counter_Value=v) for d, k, c, v in good]
    out = T.per_rep(rows, "SQ_INSTS_VALU", reps=2)
    assert out[("render_fwd", "render_fwd")] == 905.0
    assert out[("sort", "tile_sort")] == 10.0  # both class launches of a rep summed
    # one empty forward (3 dispatches for 2 reps) and one light rep
    import pytest
    with pytest.raises(T.UnevenLaunches):
        T.per_rep(rows + [dict(Dispatch_Id=9, Kernel_Name="render_fwd_kernel<32, 0>", Counter_Name="SQ_INSTS_VALU",
                               Counter_Value=0.0)], "SQ_INSTS_VALU", reps=2)
    light = [dict(r) for r in rows]
    light[0]["Counter_Value"] = 0.0
    with pytest.raises(T.UnevenLaunches):
        T.per_rep(light, "SQ_INSTS_VALU", reps=2)
    # the command-line tool exits non-zero on such a file
    p = str(tmp_path / "c.csv")
    _pmc_csv(p, [(0, "render_fwd_kernel<32, 0>", "SQ_INSTS_VALU", 0.0)] + good)
    r = subprocess.run([sys.executable, "pmc_generic.py", "27", p], cwd=os.path.join(ROOT, "tools"),
                       capture_output=True, text=True)
    assert r.returncode != 0 and "UnevenLaunches" in r.stderr, r.stdout + r.stderr
    _pmc_csv(p, good)
    r = subprocess.run([sys.executable, "pmc_generic.py", "1", p], cwd=os.path.join(ROOT, "tools"),
                       capture_output=True, text=True)
    assert r.returncode == 0 and json.loads(r.stdout)["kernels"]["render_fwd"]["SQ_INSTS_VALU"] == 905, r.stderr
