"""Timing-only build variants of libgsplat_hip.so, as source patches.

The product sources carry no experiment switches.  A variant listed here is
built by dynamic3dgaussians_amd/build.py (GSPLAT_VARIANT=<name>) from a copy
of csrc/ with these text substitutions applied; every anchor must occur
exactly once, so a patch that no longer matches the kernel fails the build
instead of silently timing the product.  Their results are wrong by
construction (DESIGN.md section 4 "Measured design experiments"): they bound
what removing a piece of work could buy.

    GSPLAT_VARIANT=exp_noatomic python -m dynamic3dgaussians_amd.build
"""
from __future__ import annotations

# render_bwd's per-Gaussian commit: a store that never happens (the value is
# never 12345) instead of the float atomic -- the atomic-free ceiling
_ACC_ATOMIC = ("gs_render.hip",
               "      if (slot < nb) atomicAdd(dst, s_out[i]);\n",
               "      if (slot < nb && s_out[i] == 12345.f) *dst = 0.f;  // timing only\n")
_FEAT_ATOMIC = ("gs_render.hip",
                "        if (slot < nb) atomicAdd(dsem + (size_t)gi * FS + 16 * cb + g, cf[cb][r]);\n",
                "        if (slot < nb && cf[cb][r] == 12345.f) dsem[(size_t)gi * FS + 16 * cb + g] = 0.f;"
                "  // timing only\n")
# render_fwd: the feature planes are not written (their store traffic)
_FWD_FEAT_STORE = ("gs_render.hip",
                   "          const uint32_t voff = (uint32_t)(pix + (size_t)(4 * (lane >> 5)) * HW) * 4u;\n",
                   "          continue;  // timing only: no feature planes\n"
                   "          const uint32_t voff = (uint32_t)(pix + (size_t)(4 * (lane >> 5)) * HW) * 4u;\n")
# tile_sort_kernel: each tile's segment copied unsorted (the launch's floor)
_SORT_COPY = ("gs_tiles.hip",
              "  if (n <= cap) {\n    // keys straight from global memory",
              "  for (int i = threadIdx.x; i < n; i += NT) plist[r.x + i] = (uint32_t)keys[r.x + i];  // timing only\n"
              "  return;\n"
              "  if (n <= cap) {\n    // keys straight from global memory")

# strip_of_block: the XCD rotation at every camera count (C >= 8 too)
_ROT_ALL = ("gs_render.hip",
            "    u = k * 8 + ((x + (C < CAM_GROUP ? k : 0)) & 7);\n",
            "    u = k * 8 + ((x + k) & 7);\n")

# render_fwd's flush: every feature row read from row (g & 7) -- always
# cached -- instead of the batch's Gaussians: the gather latency's share
_FWD_ROW0 = ("gs_render.hip",
             "          const uint32_t off = (g * (uint32_t)F + (uint32_t)(fb * 32 + (ln & 31))) * 4u;\n",
             "          const uint32_t off = ((g & 7u) * (uint32_t)F + (uint32_t)(fb * 32 + (ln & 31))) * 4u;"
             "  // timing only\n")

PATCHES = {
    "exp_nofeat": [_FEAT_ATOMIC],
    "exp_noacc": [_ACC_ATOMIC],
    "exp_noatomic": [_FEAT_ATOMIC, _ACC_ATOMIC],
    "exp_fwd_nofeatst": [_FWD_FEAT_STORE],
    "exp_sort_copy": [_SORT_COPY],
    "exp_rot_all": [_ROT_ALL],
    "exp_fwd_row0": [_FWD_ROW0],
}


def apply(name: str, file: str, text: str) -> str:
    """`text` (csrc/<file>) with variant `name`'s substitutions for that file."""
    for f, old, new in PATCHES.get(name, ()):
        if f != file:
            continue
        n = text.count(old)
        if n != 1:
            raise RuntimeError(f"variant {name}: anchor found {n} times in {file}: {old[:60]!r}")
        text = text.replace(old, new)
    return text
