#!/usr/bin/env python3
"""What independent sub-strip survivor lists inside one blend wave could
save: from a tools/strip_survey_dump.py export of a bench
camera, per 8x8 strip of the forward

  * the wave's walk: entries up to the last pixel's stop (the reference's
    T * (1 - alpha) < 1e-4 saturation, forward.cu:353-362; the list end for a
    pixel that never saturates),
  * survivors: walked entries with at least one strip pixel at alpha >= 1/255
    and power <= 0 (the any-pixel form of strip_culled),
  * blended (Gaussian, pixel) pairs,

and the same with the strip's 64 lanes split into G independent groups
(2 = 8x4 halves, 4 = 4x4 quarters), each group walking its own survivor list:
the wave then iterates max over its groups, each group stopping at its own
pixels' saturation.  The backward's walks are bounded by n_contrib instead
(the strip's longest last-contributor index, `smax`).

    python tools/quad_survey.py gpurun_out/strip_survey.npz
"""
import json
import sys

import numpy as np

TILE, W, H = 16, 800, 800


def groups(kind):
    yy, xx = np.mgrid[0:8, 0:8]
    if kind == 1:
        return np.zeros(64, int)
    if kind == 2:
        return (yy // 4).reshape(-1)
    return ((yy // 4) * 2 + xx // 4).reshape(-1)


def main():
    d = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/strip_survey.npz")
    m, co, pl, rg, nc = d["means2D"], d["conic_opacity"], d["point_list"], d["ranges"].reshape(-1, 2), d["n_contrib"]
    gx, gy = (W + TILE - 1) // TILE, (H + TILE - 1) // TILE
    yy, xx = np.mgrid[0:TILE, 0:TILE]
    # the tile's 256 pixels in strip-major order: strip s = (row // 8) * 2 + col // 8, lane = strip pixel
    order = np.argsort(((yy // 8) * 2 + xx // 8).reshape(-1) * 64 + ((yy % 8) * 8 + xx % 8).reshape(-1), kind="stable")
    px0 = xx.reshape(-1)[order].astype(np.float32)
    py0 = yy.reshape(-1)[order].astype(np.float32)
    G = {k: groups(k) for k in (1, 2, 4)}
    tot = {f"{d_}_{k}": 0 for d_ in ("fwd", "bwd") for k in (1, 2, 4)}
    pairs_f = pairs_b = 0
    slots_f = {k: 0 for k in (1, 2, 4)}
    for t in range(gx * gy):
        a, b = int(rg[t, 0]), int(rg[t, 1])
        if b <= a:
            continue
        g = pl[a:b]
        tx, ty = (t % gx) * TILE, (t // gx) * TILE
        px, py = tx + px0, ty + py0
        inside = (px < W) & (py < H)
        dx = m[g, 0][:, None] - px[None, :]
        dy = m[g, 1][:, None] - py[None, :]
        power = -0.5 * (co[g, 0][:, None] * dx * dx + co[g, 2][:, None] * dy * dy) - co[g, 1][:, None] * dx * dy
        al = np.minimum(0.99, co[g, 3][:, None] * np.exp(power))
        ok = (power <= 0) & (al >= 1.0 / 255) & inside[None, :]
        n = b - a
        Tn = np.cumprod(np.where(ok, 1 - al, 1.0), axis=0)
        stop = ok & (Tn < 1e-4)
        first = np.where(stop.any(0), stop.argmax(0), n)          # entry at which the pixel is done
        walk_f = np.minimum(first + 1, n)                          # entries the pixel evaluates
        idx = np.arange(n)[:, None]
        blend_f = ok & (idx < first[None, :])
        pairs_f += int(blend_f.sum())
        pidx = (py.astype(int).clip(0, H - 1) * W + px.astype(int).clip(0, W - 1))
        ncp = np.where(inside, nc[pidx].astype(np.int64), 0)
        pairs_b += int((ok & (idx < ncp[None, :])).sum())
        for s in range(4):
            sl = slice(64 * s, 64 * s + 64)
            oks, wf, nb_ = ok[:, sl], walk_f[sl], ncp[sl]
            for k in (1, 2, 4):
                itf = itb = 0
                for q in range(k):
                    lanes = G[k] == q
                    surv = oks[:, lanes].any(1)
                    ef = int(wf[lanes].max()) if lanes.any() else 0
                    eb = int(nb_[lanes].max())
                    itf = max(itf, int(surv[:ef].sum()))
                    itb = max(itb, int(surv[:eb].sum()))
                    slots_f[k] += int(surv[:ef].sum()) * int(lanes.sum())
                tot[f"fwd_{k}"] += itf
                tot[f"bwd_{k}"] += itb
    out = {"blended_pairs_fwd": pairs_f, "blended_pairs_bwd": pairs_b,
           "wave_iterations": tot,
           "fwd_iterations_vs_8x8": {k: tot[f"fwd_{k}"] / tot["fwd_1"] for k in (2, 4)},
           "bwd_iterations_vs_8x8": {k: tot[f"bwd_{k}"] / tot["bwd_1"] for k in (2, 4)},
           "fwd_busy_lane_slots": slots_f,
           "fwd_pair_utilisation_8x8": pairs_f / (64 * tot["fwd_1"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
