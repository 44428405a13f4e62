"""Where the full-size gradient differences (HIP vs oracle) come from:
per-gradient relative L2 HIP vs oracle, HIP vs HIP (a second backward: fp32
atomics reorder), and how concentrated the squared error is (share of the
top 10 / 100 / 1000 Gaussians).  GPU box only; the oracle is the checker."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests import _harness as H  # noqa: E402
from tests.test_gpu_parity import GRAD_NAMES  # noqa: E402


def main():
    compat = sys.argv[1] if len(sys.argv) > 1 else "reference"
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 300_000
    F = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    inp = H.scene(P=P, F=F, W=800, H=800, scale_mult=1.0)
    g = H.gpu_forward(inp, compat)
    o = H.oracle_forward(inp, compat)
    grads = H.upstream_grads(800, 800, F)
    gb = H.gpu_backward(inp, g, grads, compat)
    gb2 = H.gpu_backward(inp, g, grads, compat)
    ob = H.oracle_backward(inp, o, grads, compat)
    radii = o[5]
    # pixels whose last contributor differs (a flipped alpha / termination
    # decision) and whether the worst Gaussians' footprints cover them
    st_g = H.export_state(P, 800, 800, g)
    st_o = o[6]
    # n_contrib is a position in the (pruned) GPU list: compare the last
    # contributor as a Gaussian id, as tests/_harness.check_tile_lists does
    rg = st_g["ranges"].reshape(-1, 2).astype(np.int64)
    ro = np.asarray(st_o.ranges, np.int64).reshape(-1, 2)
    pg, po = st_g["point_list"].astype(np.int64), np.asarray(st_o.point_list, np.int64)
    n_g, n_o = st_g["n_contrib"].astype(np.int64), np.asarray(st_o.n_contrib, np.int64)
    pix = np.arange(800 * 800)
    tile = (pix // 800 // 16) * 50 + (pix % 800) // 16
    gid_g = np.where(n_g > 0, pg[np.clip(rg[tile, 0] + n_g - 1, 0, len(pg) - 1)], -1)
    gid_o = np.where(n_o > 0, po[np.clip(ro[tile, 0] + n_o - 1, 0, len(po) - 1)], -1)
    nd = np.nonzero(gid_g != gid_o)[0]
    px, py = (nd % 800).astype(np.float64), (nd // 800).astype(np.float64)
    m2 = np.asarray(st_o.means2D, np.float64)
    print(json.dumps(dict(compat=compat, n_contrib_diff_pixels=int(nd.size))), flush=True)

    def covers(i):
        d = np.hypot(px - m2[i, 0], py - m2[i, 1])
        return int((d <= radii[i]).sum())
    for name, a, a2, b in zip(GRAD_NAMES, gb, gb2, ob):
        if b.size == 0 or not np.any(b):
            continue
        a64, b64 = a.reshape(P, -1).astype(np.float64), b.reshape(P, -1).astype(np.float64)
        e = ((a64 - b64) ** 2).sum(1)
        order = np.argsort(-e)
        tot = e.sum()
        mag = (b64 ** 2).sum(1)
        rec = dict(grad=name, rel_l2=H.rel_l2(a, b), rel_l2_hip_rerun=H.rel_l2(a, a2),
                   top_share={k: float(e[order[:k]].sum() / tot) for k in (10, 100, 1000)},
                   rel_l2_without_top100=float(np.sqrt(e[order[100:]].sum() / mag[order[100:]].sum())),
                   top5=[dict(id=int(i), err=float(np.sqrt(e[i])), norm=float(np.sqrt(mag[i])),
                              radius=int(radii[i]), diff_pixels_covered=covers(i)) for i in order[:5]],
                   random5_diff_pixels_covered=[covers(i) for i in np.random.default_rng(0).choice(
                       np.nonzero(radii > 0)[0], 5)])
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
