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
# Build variants: "" = the product library; "stats" adds the blend kernels'
# work counters (-DGS_STATS, tools/render_stats.py only).
VARIANT = os.environ.get("GSPLAT_VARIANT", "")
if VARIANT:
    LIB = os.path.join(OUT_DIR, f"libgsplat_hip_{VARIANT}.so")
    BUILD_DIR = os.path.join(OUT_DIR, f"obj_{VARIANT}")
VARIANT_FLAGS = {"": [], "stats": ["-DGS_STATS"], "stamps": ["-DGS_STAMPS"], "stamps_fine": ["-DGS_STAMPS", "-DGS_STAMPS_FINE"],
                 # timing experiments only (results are wrong by construction)
                 "exp_nofeat": ["-DGS_EXP_NO_FEAT_ATOMIC"], "exp_noacc": ["-DGS_EXP_NO_ACC_ATOMIC"],
                 "exp_noatomic": ["-DGS_EXP_NO_FEAT_ATOMIC", "-DGS_EXP_NO_ACC_ATOMIC"],
                 "exp_occ5": ["-DGS_EXP_FWD_LDS_PAD=18000"], "exp_occ3": ["-DGS_EXP_FWD_LDS_PAD=40000"],
                 "exp_wg1": ["-DGS_WPB_FWD=1"], "exp_tilegroup": ["-DGS_XCD_TILE_GROUP"], "exp_strip16x4": ["-DGS_STRIP_16X4"], "exp_tb512": ["-DGS_TB_THREADS=512"], "exp_fwd_nopair": ["-DGS_FWD_NO_PAIR"], "exp_acc10": ["-DGS_ACC_STRIDE=10"], "exp_wg4": ["-DGS_WPB_BWD=4"], "exp_bwd_wpe3": ["-DGS_BWD_WPE=3"],  "exp_fwd_wpe5": ["-DGS_FWD_WPE=5"], "exp_fwd_wpe6": ["-DGS_FWD_WPE=6"],
                 "exp_oldmath": ["-DGS_OLD_MATH"], "exp_oldepi": ["-DGS_OLD_EPILOGUE"], "exp_oldpro": ["-DGS_OLD_PROLOGUE"], "exp_radixsort": ["-DGS_NO_BUCKET_SORT"], "exp_bs8": ["-DGS_BS_BITS=8"], "exp_bs9": ["-DGS_BS_BITS=9"], "exp_bs11": ["-DGS_BS_BITS=11"], "exp_bs12": ["-DGS_BS_BITS=12"],
                 "exp_ssmall512": ["-DGS_SORT_SMALL=512"], "exp_ssmall768": ["-DGS_SORT_SMALL=768"],
                 "exp_ssmall1536": ["-DGS_SORT_SMALL=1536"], "exp_cammajor": ["-DGS_CAM_MAJOR"], "exp_camg4": ["-DGS_CAM_GROUP=4"], "exp_camg9": ["-DGS_CAM_GROUP=9"], "exp_camg2": ["-DGS_CAM_GROUP=2"],
                 "exp_kpt16": ["-DGS_BS_KPT=16"], "exp_bsl10": ["-DGS_BS_BITS_LONG=10"], "exp_bsl12": ["-DGS_BS_BITS_LONG=12"],
                 "exp_tbb64": ["-DGS_TB_BLOCKS=64"], "exp_tbb128": ["-DGS_TB_BLOCKS=128"], "exp_tbb256": ["-DGS_TB_BLOCKS=256"],
                 "exp_fulw": ["-DGS_FWD_ULW", "-DGS_FWD_SLAST"],
                 "exp_ulw": ["-DGS_FWD_ULW", "-DGS_FWD_SLAST", "-DGS_BWD_ULW"],
                 "exp_bkt_batch": ["-DGS_BUCKET_BATCH"],
                 "exp_fdummy": ["-DGS_FWD_DUMMY"], "exp_fdummy_ulw": ["-DGS_FWD_DUMMY", "-DGS_FWD_ULW", "-DGS_FWD_SLAST"],
                 "exp_pb1": ["-DGS_PBWD_GROUP=1"], "exp_pb3": ["-DGS_PBWD_GROUP=3"],
                 "exp_mid512": ["-DGS_SORT_MID512"], "exp_rs256": ["-DGS_RS_THREADS=256"],
                 "exp_split2": ["-DGS_SPLIT_PIECES=2"], "exp_bwd_wpe2": ["-DGS_BWD_WPE=2"], "exp_fwd_wpe3": ["-DGS_FWD_WPE=3"],
                 "exp_fwd_noflush": ["-DGS_EXP_FWD_NO_FLUSH"], "exp_bwd_nomfma": ["-DGS_EXP_BWD_NO_MFMA"],
                 "exp_noatomic_nomfma": ["-DGS_EXP_NO_FEAT_ATOMIC", "-DGS_EXP_NO_ACC_ATOMIC", "-DGS_EXP_BWD_NO_MFMA"],
                 "exp_fwd_dma": ["-DGS_FWD_DMA"], "exp_camgrp_all": ["-DGS_CAM_GROUP=64"], "exp_oldsplit": ["-DGS_OLD_SPLIT"], "exp_split_pk": ["-DGS_SPLIT_PK"], "exp_fwd_gather64": ["-DGS_FWD_GATHER64"], "exp_bwd_buffer_atomic": ["-DGS_BWD_BUFFER_ATOMIC"], "exp_bucket_store2": ["-DGS_EXP_BUCKET_STORE2"], "exp_bucket_direct": ["-DGS_BUCKET_DIRECT"]}
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
    return files


def is_stale() -> bool:
    if not os.path.exists(LIB):
        return True
    if VARIANT not in VARIANT_FLAGS:
        return False  # a frozen snapshot (e.g. "old" = a previous product build for A/B timing)
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(f) > t for f in _deps())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not is_stale():
        return LIB
    os.makedirs(BUILD_DIR, exist_ok=True)
    cc = hipcc()

    def compile_one(item):
        src, extra = item
        obj = os.path.join(BUILD_DIR, src.replace(".hip", ".o"))
        cmd = [cc, *COMMON, *VARIANT_FLAGS[VARIANT], *extra, "-c", os.path.join(CSRC, src), "-o", obj]
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
