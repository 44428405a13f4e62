"""CPU tests of the drop-in boundary (no GPU needed):
  * the C ABI library loads and exports every symbol include/gsplat_hip.h declares;
  * the autograd wrapper reproduces the reference wrapper's conventions exactly
    (golden fixture recorded from DGR/diff_gaussian_rasterization/__init__.py);
  * the caller-generation arity dispatch (G1..G4) and the settings superset;
  * no CPU fallback: host tensors are rejected loudly.
"""
import ctypes
import json
import os
import re
import subprocess

import pytest
import torch

import dynamic3dgaussians_amd.rasterizer as R
from dynamic3dgaussians_amd import _C, _lib
from tests.golden.make_golden import Recorder, conventions_case, run_wrapper

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden", "boundary_conventions.json")


def _declared_symbols():
    names = set()
    for h in ("gsplat_hip.h", "gs_neighbor.h", "gs_optim.h", "gs_knn.h"):
        txt = open(os.path.join(REPO, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(gs_[a-z_0-9]+)\s*\(", txt))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    names = _declared_symbols()
    assert len(names) >= 14
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.PROTOTYPES, f"{n} has no ctypes prototype"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.lib_path()], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r" T (gs_[a-z_0-9]+)", out))
    assert set(names) <= exported


def test_abi_version_and_sizes():
    L = _lib.load()
    assert L.gs_version() == _lib.ABI_VERSION == 13
    assert L.gs_geom_buffer_bytes(1) >= 64  # one 64-B render record at least
    for a, b in [(1000, 2000), (10_000, 300_000)]:
        assert L.gs_geom_buffer_bytes(b) > L.gs_geom_buffer_bytes(a)
        assert L.gs_binning_buffer_bytes(b) > L.gs_binning_buffer_bytes(a)
    assert L.gs_image_buffer_bytes(800, 800) >= 800 * 800 * 4
    assert L.gs_backward_scratch_bytes(1000, 32) >= 1000 * 10 * 4  # feature grads go to the output


def test_invalid_arguments_report_errors_without_gpu():
    L = _lib.load()
    g = _lib.GsGaussians(P=-1)
    c = _lib.GsCamera(image_width=8, image_height=8)
    import ctypes
    n = ctypes.c_int64(0)
    code = L.gs_forward_plan(ctypes.byref(g), ctypes.byref(c), 0, 0, 0, None, None, None,
                             ctypes.byref(n), None, None)
    assert code < 0 and b"P must be" in L.gs_last_error()
    g = _lib.GsGaussians(P=10, F=7)
    code = L.gs_forward_plan(ctypes.byref(g), ctypes.byref(c), 0, 0, 0, None, None, None,
                             ctypes.byref(n), None, None)
    assert code < 0 and b"feature width" in L.gs_last_error()


def test_debug_checks_reject_corrupted_state_without_gpu():
    """debug=True validates the forward's state on the host before the blend
    kernels dereference it (gsplat_hip.h, gs_check_*): a corrupted plan
    header, non-contiguous or out-of-bound ranges and out-of-range Gaussian
    ids must be refused with a message, valid ones accepted.  Host
    functions: no GPU needed, no GPU fault provoked."""
    import numpy as np
    L = _lib.load()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    # {L, longest, num_rendered, status, p1, q1, p2, -}
    good = np.array([500, 120, 640, 0, 3, 2, 1, 0], np.uint32)
    assert L.gs_check_plan_header(p(good), 50) == 0
    for i, v, msg in [(0, 700, b"exceed"), (1, 501, b"longest tile"), (3, 8, b"status"),
                      (4, 51, b"sort-class"), (5, 4, b"sort-class"), (6, 4, b"sort-class")]:
        bad = good.copy()
        bad[i] = v
        assert L.gs_check_plan_header(p(bad), 50) < 0, (i, v)
        assert msg in L.gs_last_error(), (i, L.gs_last_error())
    # 4 tiles, 10 instances: [0,4) [4,4) [4,9) [9,10)
    rg = np.array([0, 4, 4, 4, 4, 9, 9, 10], np.uint32)
    assert L.gs_check_ranges(p(rg), 4, 10, 5) == 0
    assert L.gs_check_ranges(p(rg), 4, 10, -1) == 0
    assert L.gs_check_ranges(p(rg), 4, 10, 4) < 0 and b"planned longest" in L.gs_last_error()
    gap = rg.copy(); gap[4] = 5                     # [5,9): a hole at 4
    assert L.gs_check_ranges(p(gap), 4, 10, -1) < 0 and b"contiguous" in L.gs_last_error()
    over = rg.copy(); over[7] = 11                  # past L
    assert L.gs_check_ranges(p(over), 4, 10, -1) < 0 and b"outside" in L.gs_last_error()
    short = rg.copy(); short[7] = 9; short[6] = 9   # covers 9 of 10
    assert L.gs_check_ranges(p(short), 4, 10, -1) < 0 and b"cover" in L.gs_last_error()
    neg = rg.copy(); neg[2], neg[3] = 6, 5          # end < begin
    assert L.gs_check_ranges(p(neg), 4, 10, -1) < 0
    ids = np.array([0, 5, 99, 3], np.uint32)
    assert L.gs_check_point_list(p(ids), 4, 100) == 0
    ids[2] = 100
    assert L.gs_check_point_list(p(ids), 4, 100) < 0 and b"id 100" in L.gs_last_error()
    assert L.gs_check_point_list(p(ids), 2, 100) == 0  # only the first L entries count


def test_conventions_match_reference_wrapper(monkeypatch):
    """Golden: positional packing of _C.rasterize_gaussians / _backward
    (including Q2's swapped camera scalars), the returned 5-tuple and the
    label masking (Q12) are identical to the reference wrapper's."""
    gold = json.load(open(GOLD))
    rec = Recorder()
    monkeypatch.setattr(R, "_C", rec)
    tensors, settings = conventions_case()
    ours = run_wrapper(R, rec, tensors, settings)
    assert ours["n_outputs"] == gold["n_outputs"] == 5
    assert ours["radii"] == gold["radii"]
    assert len(ours["forward_args"]) == len(gold["forward_args"]) == 22
    assert ours["forward_args"] == gold["forward_args"]
    assert len(ours["backward_args"]) == len(gold["backward_args"]) == 28
    assert ours["backward_args"] == gold["backward_args"]
    assert ours["grads"].keys() == gold["grads"].keys()
    for k in gold["grads"]:
        assert ours["grads"][k] == pytest.approx(gold["grads"][k], rel=1e-12, abs=1e-12), k
    # the reference's settings fields are a prefix of ours (superset)
    assert list(R.GaussianRasterizationSettings._fields[:15]) == gold["settings_fields"]


def test_fixed_mode_passes_camera_scalars_in_binding_order(monkeypatch):
    rec = Recorder()
    monkeypatch.setattr(R, "_C", rec)
    tensors, settings = conventions_case()
    settings = dict(settings, compat="fixed")
    run_wrapper(R, rec, tensors, settings)
    assert rec.bwd_args[11:15] == [2.25, 1.75, 0.61, 0.47]


def _stub_call(monkeypatch, **kw):
    rec = Recorder()
    monkeypatch.setattr(R, "_C", rec)
    tensors, settings = conventions_case()
    s = R.GaussianRasterizationSettings(**settings)
    t = tensors
    return R.GaussianRasterizer(s)(means3D=t["means3D"], means2D=torch.zeros_like(t["means3D"]),
                                   opacities=t["opacities"], colors_precomp=t["colors_precomp"],
                                   scales=t["scales"], rotations=t["rotations"], **kw)


def test_arity_dispatch_g1_to_g4(monkeypatch):
    t, _ = conventions_case()
    g1 = _stub_call(monkeypatch)
    assert len(g1) == 3 and g1[1].dtype == torch.int32               # color, radii, depth
    g2 = _stub_call(monkeypatch, label=t["label"])
    assert len(g2) == 4 and g2[1].dtype == torch.int32               # + alpha
    g3 = _stub_call(monkeypatch, label=t["label"], semantic_feature=t["semantic_feature"])
    assert len(g3) == 5 and g3[2].shape[0] == 32                     # color, radii, feat, depth, alpha
    g4 = _stub_call(monkeypatch, semantic_feature=t["semantic_feature"])
    assert len(g4) == 4 and g4[2].dtype == torch.int32 and g4[1].shape[0] == 32


def test_settings_superset_defaults():
    s = R.GaussianRasterizationSettings(image_height=10, image_width=20, tanfovx=0.5, tanfovy=0.4,
                                        bg=torch.zeros(3), viewmatrix=torch.eye(4),
                                        projmatrix=torch.eye(4), sh_degree=0,
                                        campos=torch.zeros(3), prefiltered=False, debug=False)
    assert s.c_x is None and s.confidence is None and s.compat is None
    assert R._principal_point(s) == (10.0, 5.0)


def test_input_validation_messages(monkeypatch):
    rec = Recorder()
    monkeypatch.setattr(R, "_C", rec)
    t, settings = conventions_case()
    ras = R.GaussianRasterizer(R.GaussianRasterizationSettings(**settings))
    with pytest.raises(Exception, match="exactly one of either SHs or precomputed colors|excatly"):
        ras(means3D=t["means3D"], means2D=t["means3D"], opacities=t["opacities"],
            scales=t["scales"], rotations=t["rotations"])
    with pytest.raises(Exception, match="scale/rotation pair"):
        ras(means3D=t["means3D"], means2D=t["means3D"], opacities=t["opacities"],
            colors_precomp=t["colors_precomp"], scales=t["scales"])


def test_no_cpu_fallback():
    t, settings = conventions_case()
    with pytest.raises(_lib.GsplatError, match="device tensors"):
        _C.rasterize_gaussians(settings["bg"], t["means3D"], t["colors_precomp"], None,
                               t["opacities"], t["scales"], t["rotations"], 1.0, torch.Tensor([]),
                               settings["viewmatrix"], settings["projmatrix"], 1.0, 1.0, 0.5, 0.5,
                               4, 5, torch.Tensor([]), 0, settings["campos"], False, False)
    with pytest.raises(RuntimeError, match=r"means3D must have dimensions \(num_points, 3\)"):
        _C.rasterize_gaussians(settings["bg"], t["means3D"][:, :2], None, None, None, None, None,
                               1.0, None, None, None, 1, 1, 1, 1, 4, 5, None, 0, None, False, False)


def test_compat_validation():
    with pytest.raises(ValueError):
        _C.set_default_compat("nope")
    _C.set_default_compat("fixed")
    assert _C.get_default_compat() == "fixed"
    _C.set_default_compat("reference")


def test_drop_in_import_name():
    import diff_gaussian_rasterization as d
    from diff_gaussian_rasterization import _C as c2
    assert d.GaussianRasterizer is R.GaussianRasterizer and c2 is _C


@pytest.mark.parametrize("P,F,M", [(1000, 32, 0), (777, 8, 16), (5, 0, 1)])
def test_flat_backward_buffers_carving(P, F, M):
    """GradientSink's per-stream slot: one flat buffer whose per-gradient views
    have the binding's shapes, are contiguous, start on 256-byte boundaries
    and do not overlap, so a whole gradient set sums with one add."""
    plain = _C.backward_buffers(P, F, M, "cpu")
    views, buf, offs = _C.backward_buffers(P, F, M, "cpu", flat=True)
    assert set(views) == set(plain)
    spans = []
    for k, v in views.items():
        assert v.shape == plain[k].shape, k
        assert v.is_contiguous(), k
        assert v.untyped_storage().data_ptr() == buf.untyped_storage().data_ptr(), k
        o, n, _ = offs[k]
        assert o % 64 == 0, k  # 64 floats = 256 B
        assert v.numel() == n
        spans.append((o, o + n))
    spans.sort()
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    # a sum of two flat slots carves back to the per-gradient sums
    buf.normal_()
    other = torch.randn_like(buf)
    summed = _C.carve_buffers(buf + other, offs)
    ov = _C.carve_buffers(other, offs)
    for k in views:
        torch.testing.assert_close(summed[k], views[k] + ov[k], rtol=0, atol=0)


def _header_struct_fields(name):
    """Field names of `typedef struct <name> { ... } <name>;` in include/gsplat_hip.h, in order."""
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "gsplat_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, flags=re.S).group(1)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        # "float c_x, c_y, tan_fovx" / "const float *means3D" / "int32_t tile_x0, tile_y0"
        first, *rest = [p.strip() for p in decl.split(",")]
        names.append(re.findall(r"[A-Za-z_]\w*", first)[-1])
        names += [re.findall(r"[A-Za-z_]\w*", p)[-1] for p in rest]
    return names


@pytest.mark.parametrize("struct,mirror", [("gs_gaussians", "GsGaussians"), ("gs_camera", "GsCamera"),
                                           ("gs_batch_hint", "GsBatchHint")])
def test_ctypes_structs_mirror_the_header(struct, mirror):
    """The ctypes mirrors name the header's fields in order (ctypes would
    silently accept a stale keyword as a plain attribute)."""
    fields = [f for f, _ in getattr(_lib, mirror)._fields_]
    assert fields == _header_struct_fields(struct)


def test_integration_stub_uses_real_field_names():
    """INTEGRATION.md's ctypes stub passes only field names of the structs."""
    import re
    doc = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "INTEGRATION.md")).read()
    for mirror in ("GsGaussians", "GsCamera"):
        fields = {f for f, _ in getattr(_lib, mirror)._fields_}
        calls = []
        for m in re.finditer(r"%s\(" % mirror, doc):
            depth, i = 1, m.end()
            while depth:
                depth += {"(": 1, ")": -1}.get(doc[i], 0)
                i += 1
            calls.append(re.sub(r"#[^\n]*", "", doc[m.end():i - 1]))
        assert calls, mirror
        for call in calls:
            for kw in re.findall(r"(\w+)=", call):
                assert kw in fields, (mirror, kw)
