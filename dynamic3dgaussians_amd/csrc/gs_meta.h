// gs_meta.h -- the binning plan's 8-word header (one per camera): shared by
// the kernels (gs_common.h), the C-ABI host code and the host-only validators
// (gs_host.cpp, also built under the CPU sanitizers: oracle/Makefile).
#pragma once

namespace gs {
// M_L = list instances (after the exact tile test), M_MAXN = longest tile,
// M_LREF = the reference's num_rendered (bounding-rect instances), M_STATUS,
// the tile-order prefixes of the sort launches (tile_offsets_kernel), and a
// last word the kernel writes 0 (the host's check that a header was written)
enum ImgMeta { M_L = 0, M_MAXN = 1, M_LREF = 2, M_STATUS = 3,
               M_SORT_P1 = 4, M_SORT_Q1 = 5, M_SORT_P2 = 6, M_WORDS = 8 };
}  // namespace gs

// Host-side error state of the C ABI (gs_last_error): sets the thread's
// message, returns `code`.
int gs_set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
