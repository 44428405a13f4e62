"""The training loop's helpers around the rasterizer against the reference's
own Python (tests/golden/train_helpers.npz, made by tests/golden/make_golden.py
from helpers.py and external.py): the camera every caller builds, the
activations GS_FLAG_ACTIVATE folds into the kernels, the losses, the PSNR
the bench reports, and the neighbour-loss oracle that checks the HIP
neighbour kernels (oracle/neighbor.py; Open3D's k-NN graph itself stays
unpinned -- the fixture's neighbour indices are given, not searched)."""
from __future__ import annotations

import os

import numpy as np
import torch

from dynamic3dgaussians_amd.camera import setup_camera
from dynamic3dgaussians_amd.timesteps import params2rendervar
from oracle import neighbor as onb

# torch's CPU elementwise kernels (exp, sqrt, division) dispatch on the host's
# vector ISA (AVX2 / AVX512), so results are bit-equal to the fixture only on
# a host of the fixture's ISA; across hosts they agree to a couple of ulp.
ULP2 = dict(rtol=2.5e-7, atol=0)

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "train_helpers.npz"))


def test_setup_camera_matches_helpers_setup_camera():
    """helpers.py:68-95, off-centre principal points included: the same
    view / full-projection matrices (column-major, as the rasterizer reads
    them), camera centre, tan(fov/2) and principal point."""
    for i in range(len(G["cam_w"])):
        c = setup_camera(int(G["cam_w"][i]), int(G["cam_h"][i]), G["cam_k"][i], G["cam_w2c"][i])
        np.testing.assert_allclose(c.viewmatrix, G["cam_viewmatrix"][i], rtol=0, atol=1e-6)
        np.testing.assert_allclose(c.projmatrix, G["cam_projmatrix"][i], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(c.campos, G["cam_campos"][i], rtol=1e-6, atol=1e-6)
        assert c.tanfovx == float(G["cam_tanfovx"][i]) and c.tanfovy == float(G["cam_tanfovy"][i])
        assert c.c_x == float(G["cam_c_x"][i]) and c.c_y == float(G["cam_c_y"][i])


def test_params2rendervar_matches_helpers():
    """helpers.py:98-107 on the CPU: normalise / sigmoid / exp (the same torch
    ops, so bit-equal on a host of the fixture's ISA; within 2 ulp on any)."""
    params = {k[2:]: torch.from_numpy(G[k]) for k in G.files if k.startswith("p_")}
    rv = params2rendervar(params)
    for k in ("rotations", "opacities", "scales"):
        torch.testing.assert_close(rv[k], torch.from_numpy(G[f"rv_{k}"]), **ULP2, msg=k)


def test_losses_and_psnr_match_reference():
    from bench import calc_psnr
    x, y, w = (torch.from_numpy(G[k]) for k in ("loss_x", "loss_y", "loss_w"))
    # reductions: bit-equal on the fixture's host ISA, 1e-6 relative on any
    def close(got, key):
        return abs(got - float(G[key])) <= 1e-6 * abs(float(G[key]))
    assert close(torch.abs(x - y).mean().item(), "l1_v1")          # helpers.py:110-111
    assert close(onb._wl2_v1(x, y, w).item(), "wl2_v1")            # helpers.py:117-118
    assert close(onb._wl2_v2(x, y, w[:, 0]).item(), "wl2_v2")      # helpers.py:121-122
    # bench.py's PSNR: external.py:85-87 per channel, averaged over the channels
    ref = np.asarray(G["psnr"], np.float64).reshape(-1)
    assert abs(calc_psnr(G["psnr_img1"], G["psnr_img2"]) - ref.mean()) < 1e-4


def test_neighbour_loss_oracle_matches_reference_composition():
    """oracle/neighbor.py's torch restatement (fp32, the checker of the HIP
    neighbour kernels) against train.py:256-270 composed from the
    reference's quat_mult / build_rotation / weighted_l2 losses; its float64
    numpy restatement within fp32 rounding."""
    fg_pts, fg_rot = torch.from_numpy(G["nb_fg_pts"]), torch.from_numpy(G["nb_fg_rot"])
    variables = {"neighbor_indices": torch.from_numpy(G["nb_indices"]),
                 "neighbor_weight": torch.from_numpy(G["nb_weight"]),
                 "prev_inv_rot_fg": torch.from_numpy(G["nb_prev_inv_rot"]),
                 "prev_offset": torch.from_numpy(G["nb_prev_offset"]),
                 "neighbor_dist": torch.from_numpy(G["nb_dist"])}
    torch.testing.assert_close(onb._quat_mult(fg_rot, variables["prev_inv_rot_fg"]),
                               torch.from_numpy(G["nb_rel_rot"]), **ULP2)
    # build_rotation divides by a sqrt: 2 ulp of the entries' magnitude (<= 1)
    torch.testing.assert_close(onb._build_rotation(torch.from_numpy(G["nb_rel_rot"])),
                               torch.from_numpy(G["nb_rot"]), rtol=0, atol=5e-7)
    rigid, rot, iso = onb.torch_reference(fg_pts, fg_rot, variables)
    for got, key in ((rigid, "nb_rigid"), (rot, "nb_rot_loss"), (iso, "nb_iso")):
        assert abs(got.item() - float(G[key])) <= 1e-6 * abs(float(G[key])), (key, got.item(), float(G[key]))
    r64 = onb.numpy_losses(G["nb_fg_pts"], G["nb_fg_rot"], G["nb_indices"], G["nb_weight"], G["nb_dist"],
                           G["nb_prev_offset"], G["nb_prev_inv_rot"])
    for got, key in zip(r64, ("nb_rigid", "nb_rot_loss", "nb_iso")):
        assert abs(got - float(G[key])) <= 2e-6 * abs(float(G[key])), key
