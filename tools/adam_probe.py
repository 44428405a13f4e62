#!/usr/bin/env python3
"""Bit-level agreement of FusedAdam with torch.optim.Adam (foreach) on the
reference's parameter groups: fraction of identical fp32 words per state."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd.optim import FusedAdam  # noqa: E402
from tests.test_optim import _clone, make_opt, make_params, set_grads  # noqa: E402

ref = make_params()
ours = _clone(ref)
o_ref, o_ours = make_opt(torch.optim.Adam, ref), make_opt(FusedAdam, ours)
for step in range(6):
    set_grads(ref, step)
    set_grads(ours, step)
    o_ref.step()
    o_ours.step()
    out = {}
    for k in ref:
        sr, so = o_ref.state[ref[k]], o_ours.state[ours[k]]
        out[k] = [round((ours[k].detach() == ref[k].detach()).float().mean().item(), 6)] + \
                 [round((so[x] == sr[x]).float().mean().item(), 6) for x in ("exp_avg", "exp_avg_sq")]
    print(json.dumps({"step": step, "exact_frac[param, m, v]": out}))
