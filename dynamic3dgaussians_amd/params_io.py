"""The reference's parameter output format:
params2cpu / save_params (helpers.py:149-167) and the matching loader.

`output/<exp>/<seq>/params.npz`: for every key of the first timestep's
params, either a stack over timesteps ([T, ...], keys saved every timestep:
means3D, rgb_colors, unnorm_rotations) or the first timestep's array (keys
saved once).  Plain numpy, no pickles (load with allow_pickle=False).
"""
from __future__ import annotations

import os

import numpy as np


def params2cpu(params: dict, is_initial_timestep: bool) -> dict:
    """helpers.py:149-155."""
    keep = None if is_initial_timestep else ("means3D", "rgb_colors", "unnorm_rotations")
    return {k: v.detach().cpu().contiguous().numpy() for k, v in params.items() if keep is None or k in keep}


def save_params(output_params: list, seq: str, exp: str, root: str = "./output") -> str:
    """helpers.py:158-167; returns the written path."""
    to_save = {}
    for k in output_params[0].keys():
        if len(output_params) > 1 and k in output_params[1].keys():
            to_save[k] = np.stack([p[k] for p in output_params])
        else:
            to_save[k] = output_params[0][k]
    out_dir = os.path.join(root, exp, seq)
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "params")
    np.savez(path, **to_save)
    return path + ".npz"


def load_params(path: str) -> dict:
    """Read a params.npz back (no pickles)."""
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
