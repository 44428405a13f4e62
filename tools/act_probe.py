#!/usr/bin/env python3
"""Which fp32 operation order reproduces torch's F.normalize (p = 2, dim = 1)
on the GPU bit for bit?  Candidate orders of the 4-element squared norm are
evaluated on the host (fma emulated in float64: a float32 product is exact
there) and compared with torch's GPU result; also torch.exp and
torch.sigmoid against correctly rounded host values.  Used to pick the
order of act_norm (gs_preprocess.hip, GS_FLAG_ACTIVATE).

    python tools/act_probe.py
"""
import json

import numpy as np
import torch


def f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def fma(a, b, c):
    return f32(a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64))


def main():
    g = torch.Generator().manual_seed(0)
    q = torch.randn(400000, 4, generator=g) * torch.exp(0.6 * torch.randn(400000, 1, generator=g))
    ref = torch.nn.functional.normalize(q.cuda()).cpu().numpy()
    x, y, z, w = (q[:, i].numpy() for i in range(4))
    sq = lambda a: f32(a.astype(np.float64) ** 2)  # noqa: E731
    cands = {
        "seq_round ((x2+y2)+z2)+w2": f32(f32(f32(sq(x) + sq(y)) + sq(z)) + sq(w)),
        "seq_fma fma(w,w,fma(z,z,fma(y,y,x2)))": fma(w, w, fma(z, z, fma(y, y, sq(x)))),
        "pair_round (x2+y2)+(z2+w2)": f32(f32(sq(x) + sq(y)) + f32(sq(z) + sq(w))),
        "pair_fma fma(y,y,x2)+fma(w,w,z2)": f32(fma(y, y, sq(x)) + fma(w, w, sq(z))),
        "pair_xz (x2+z2)+(y2+w2)": f32(f32(sq(x) + sq(z)) + f32(sq(y) + sq(w))),
    }
    out = {}
    for name, n2 in cands.items():
        n = np.maximum(f32(np.sqrt(n2.astype(np.float64))), np.float32(1e-12))
        qn = f32(q.numpy().astype(np.float64) / n[:, None].astype(np.float64))
        out[name] = float(np.mean(np.all(qn == ref, axis=1)))
    v = torch.randn(400000, generator=g) * 3
    e = torch.exp(v.cuda()).cpu().numpy()
    s = torch.sigmoid(v.cuda()).cpu().numpy()
    vd = v.numpy().astype(np.float64)
    out["exp vs correctly rounded"] = float(np.mean(e == f32(np.exp(vd))))
    ef = f32(np.exp(-vd))
    out["sigmoid vs 1/(1+expf(-x)) (expf correctly rounded)"] = float(
        np.mean(s == f32(1.0 / f32(1.0 + ef.astype(np.float64)).astype(np.float64))))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
