"""bench.py's roofline bookkeeping on the host (no GPU): the byte model per
compat mode, the PMC summaries attached only to their own workload, and the
derived fractions physically possible for the committed counts at the
bench's own measured launch times (derived views copied from
another workload printed atomics 1.149 / issue 1.056 on configs[1])."""
from __future__ import annotations

import json
import os

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_mode_backward_reads_no_feature_rows():
    kw = dict(L=1_000_000, Pv=200_000, P=300_000, W=800, H=800, F=32, cams=27)
    ref, fixed = bench.stage_bytes(compat="reference", **kw), bench.stage_bytes(compat="fixed", **kw)
    assert fixed["render_bwd"] - ref["render_bwd"] == 4 * 32 * kw["L"]
    for k in ref:
        if k != "render_bwd":
            assert ref[k] == fixed[k], k
    # per-launch inputs are shared by the launch's cameras
    one = bench.stage_bytes(compat="reference", **dict(kw, cams=1))
    assert one["preprocess"] > ref["preprocess"] and one["preprocess_bwd"] > ref["preprocess_bwd"]


def test_pmc_summaries_attach_to_their_own_workload_only():
    with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as f:
        wl = json.load(f)["workload"]
    got = bench.pmc_for(wl)
    assert set(got) == {"traffic", "valu", "atomic"}, "the committed PMC files must share one workload"
    for change in ({"gaussians": 100_000}, {"cams_per_launch": 4}, {"features": 0}, {"width": 1920}):
        assert bench.pmc_for(dict(wl, **change)) == {}, change


@pytest.mark.parametrize("stage", ["render_bwd", "render_fwd"])
def test_committed_counts_give_possible_fractions(stage):
    """The committed per-camera counts at the committed bench line's own
    live launch time: every derived fraction in (0, 1]."""
    with open(os.path.join(REPO, "profiles", "pmc_traffic.json")) as f:
        wl = json.load(f)["workload"]
    pmc = bench.pmc_for(wl)
    with open(os.path.join(REPO, "profiles", "r04y", "bench.json")) as f:
        line = json.load(f)
    ms = line["stages_ms_per_step"][stage]
    cams = wl["cams_per_launch"]
    iv = bench.issue_view(pmc, stage, ms, cams)
    assert iv is not None and 0 < iv["frac"] <= 1.0, iv
    av = bench.atomic_view(pmc, stage, ms, cams)
    if stage == "render_bwd":
        assert av is not None and 0 < av["frac"] <= 1.0, av
    else:
        assert av is None  # the forward issues no float atomics
    table = bench.stage_table(line["stages_ms_per_step"], {stage: 1e9 / cams}, pmc, cams)
    assert 0 < table[stage]["hbm_frac"] <= 1.0


def test_committed_bench_line_has_no_fraction_above_one():
    def fracs(o):
        if isinstance(o, dict):
            for k, v in o.items():
                if k.endswith("frac") and isinstance(v, (int, float)):
                    yield k, v
                yield from fracs(v)
    for path in ("r04m/bench.json", "r04m/bench_under_rocprof.json", "r04s/bench.json", "r04s/bench_under_rocprof.json", "r04y/bench.json", "r04y/bench_under_rocprof.json"):
        with open(os.path.join(REPO, "profiles", path)) as f:
            line = json.load(f)
        for k, v in fracs(line["roofline"]):
            assert 0 <= v <= 1.0, (path, k, v)


@pytest.mark.parametrize("world", [1, 2, 8])
def test_other_mode_is_the_same_on_every_rank_of_a_split(world):
    # the ranks of a split differ in whether they hold a tile window; the
    # comparison's steps hold collectives, so the decision may not depend on it
    # (a weak-scaling rank holds whole cameras only; at one rank a split
    # is whole cameras too)
    if world > 1:
        got = {bench.other_mode("batch", w, True, world) for w in (False, True)}
        assert got == {None}, got
    assert bench.other_mode("batch", False, False, world) == "percam"
    assert bench.other_mode("percam", False, False, world) == "batch"
    assert bench.other_mode("batch", False, False, world, enabled=False) is None
    assert bench.other_mode("batch", False, True, 1) == "percam"  # one rank: whole cameras
