"""Build libgsplat_hip.so (hand-written HIP kernels for gfx950) in-tree.

    python -m dynamic3dgaussians_amd.build          # build if stale
    python -m dynamic3dgaussians_amd.build --force  # rebuild

Each .hip translation unit is compiled to an object with hipcc and the objects
are linked into one shared library exposing the C ABI of include/gsplat_hip.h.
The library is written next to this file (lib/), so it travels with the repo
snapshot to the GPU box.  hipcc cross-compiles for gfx950 without a GPU.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
OUT_DIR = os.path.join(PKG, "lib")
BUILD_DIR = os.path.join(OUT_DIR, "obj")
LIB = os.path.join(OUT_DIR, "libgsplat_hip.so")
# Build variants ("" = the product library): see VARIANT_FLAGS.
VARIANT = os.environ.get("GSPLAT_VARIANT", "")
if VARIANT:
    LIB = os.path.join(OUT_DIR, f"libgsplat_hip_{VARIANT}.so")
    BUILD_DIR = os.path.join(OUT_DIR, f"obj_{VARIANT}")
# Build variants: "stats" (work counters of the blend and sort kernels,
# tools/render_stats.py), "stamps" / "stamps_fine" (per-wave lifetime stamps,
# tools/batch_steps.py --stamps) and timing-only removals whose results are
# wrong by construction (the backward's atomic-free ceiling, the tile sort's
# floor).  The timing-only removals are not in the
# product sources: they are text patches (tools/variants.py) applied to a
# copy of csrc/ for that variant's build.  A variant name not listed here is
# a frozen snapshot (e.g. a copy of a previous product library for A/B
# timing) and is never rebuilt.
VARIANT_FLAGS = {"": [], "stats": ["-DGS_STATS"], "stamps": ["-DGS_STAMPS"],
                 "stamps_fine": ["-DGS_STAMPS", "-DGS_STAMPS_FINE"],
                 "exp_nofeat": [], "exp_noacc": [], "exp_noatomic": [],  # the backward's atomics (tools/variants.py)
                 "exp_fwd_nofeatst": [],  # traffic of the feature planes
                 "exp_sort_copy": [],  # the tile sort's floor: copy, no sort
                 "exp_rot_all": [],  # strip_of_block's XCD rotation at C >= 8 too
                 "exp_fwd_row0": [],  # render_fwd's feature rows from 8 cached rows (gather latency)
                 "ctl": []}  # the product's flags under a variant's (ctypes) binding: the A/B control
PATCHED = ("exp_nofeat", "exp_noacc", "exp_noatomic", "exp_fwd_nofeatst", "exp_sort_copy", "exp_rot_all", "exp_fwd_row0")
ARCH = os.environ.get("GSPLAT_OFFLOAD_ARCH", "gfx950")

# Per-file flags.  The preprocess kernels are compiled without FMA
# contraction so that they follow the CPU oracle's operation order exactly.
SOURCES = {
    "gs_preprocess.hip": ["-ffp-contract=off"],
    "gs_binning.hip": [],
    "gs_tiles.hip": [],
    "gs_render.hip": [],
    "gs_neighbor.hip": [],
    "gs_optim.hip": ["-ffp-contract=off"],
    "gs_knn.hip": ["-ffp-contract=off"],
    "gs_api.hip": [],
    "gs_host.cpp": [],  # host-only C++ (also built by oracle/Makefile's sanitizer target)
}
COMMON = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
          "-Wno-unused-function", "-I", CSRC, "-I", INCLUDE]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (ROCm) is required to build libgsplat_hip.so")


def _headers() -> list[str]:
    """Every public header: the C ABI and the structs the ctypes mirrors
    follow (gs_optim.h, gs_neighbor.h, gs_knn.h)."""
    return [os.path.join(INCLUDE, f) for f in sorted(os.listdir(INCLUDE)) if f.endswith(".h")]


def _deps() -> list[str]:
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f != "gs_torch_binding.cpp"]
    files += _headers()
    files.append(os.path.abspath(__file__))
    if VARIANT in PATCHED:
        files.append(os.path.join(REPO, "tools", "variants.py"))
    return files


def is_stale() -> bool:
    if not os.path.exists(LIB):
        return True
    if VARIANT not in VARIANT_FLAGS:
        return False  # a frozen snapshot (e.g. "old" = a previous product build for A/B timing)
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in _deps())


def _patched_sources() -> str:
    """A copy of csrc/ with the variant's text patches (tools/variants.py)."""
    sys.path.insert(0, REPO)
    from tools import variants
    out = os.path.join(OUT_DIR, f"src_{VARIANT}")
    os.makedirs(out, exist_ok=True)
    for f in os.listdir(CSRC):
        if f.endswith((".hip", ".h", ".cpp")):
            with open(os.path.join(CSRC, f)) as fh:
                text = variants.apply(VARIANT, f, fh.read())
            with open(os.path.join(out, f), "w") as fh:
                fh.write(text)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not is_stale():
        return LIB
    os.makedirs(BUILD_DIR, exist_ok=True)
    cc = hipcc()
    src_dir = _patched_sources() if VARIANT in PATCHED else CSRC

    def compile_one(item):
        src, extra = item
        obj = os.path.join(BUILD_DIR, os.path.splitext(src)[0] + ".o")
        if src.endswith(".cpp"):  # host-only translation unit
            cmd = [cc, "-x", "c++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I", CSRC, "-I", INCLUDE, *extra,
                   "-c", os.path.join(CSRC, src), "-o", obj]
        else:
            cmd = [cc, *COMMON, *VARIANT_FLAGS[VARIANT], *extra, "-c", os.path.join(src_dir, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, SOURCES.items()))
    tmp = LIB + ".tmp"
    cmd = [cc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


NATIVE_SRC = os.path.join(CSRC, "gs_torch_binding.cpp")
NATIVE = os.path.join(OUT_DIR, "_gs_native.so")


def native_is_stale() -> bool:
    if not os.path.exists(NATIVE):
        return True
    t = os.path.getmtime(NATIVE)
    return any(os.path.getmtime(f) > t for f in (NATIVE_SRC, *_headers(), LIB))


def build_native(force: bool = False, verbose: bool = False) -> str:
    """The C++ fast path of the `_C` binding (csrc/gs_torch_binding.cpp): a
    torch extension (host code only) linked against libgsplat_hip.so, written
    to lib/_gs_native.so next to it (rpath $ORIGIN)."""
    if VARIANT:
        return ""
    if not force and not native_is_stale():
        return NATIVE
    from torch.utils import cpp_extension  # heavy import, only when building
    bdir = os.path.join(OUT_DIR, "native_obj")
    os.makedirs(bdir, exist_ok=True)
    os.environ.setdefault("MAX_JOBS", "4")
    cpp_extension.load(name="_gs_native", sources=[NATIVE_SRC], build_directory=bdir,
                       extra_include_paths=[INCLUDE], extra_cflags=["-O2"],
                       # rpath $ORIGIN (lib/) and $ORIGIN/.. (the build dir's parent, lib/),
                       # escaped for ninja ($$) and the shell ('')
                       extra_ldflags=[f"-L{OUT_DIR}", "-lgsplat_hip", "-Wl,-rpath,'$$ORIGIN:$$ORIGIN/..'"],
                       with_cuda=False, verbose=verbose, is_python_module=True)
    built = os.path.join(bdir, "_gs_native.so")
    tmp = NATIVE + ".tmp"
    shutil.copyfile(built, tmp)
    os.replace(tmp, NATIVE)
    return NATIVE


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    args = ap.parse_args()
    print(build(force=args.force, verbose=args.verbose))
    if not VARIANT:
        print(build_native(force=args.force, verbose=args.verbose))


if __name__ == "__main__":
    main()
