// gs_host.cpp -- host-only part of the C ABI: the thread's error message
// (gs_last_error) and the debug-mode validators of the forward's state
// (gs_check_plan_header / gs_check_ranges / gs_check_point_list,
// include/gsplat_hip.h).  Plain C++ with no HIP dependency, so the same file
// is linked into libgsplat_hip.so and into the CPU sanitizer build
// (oracle/Makefile `sanitize`: AddressSanitizer + UndefinedBehaviorSanitizer
// over these validators and the C oracle).
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include <string>
#include <vector>

#include "../../include/gsplat_hip.h"
#include "gs_meta.h"

using namespace gs;

namespace {
thread_local std::string g_err;
}  // namespace

int gs_set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

extern "C" {

const char* gs_last_error(void) { return g_err.c_str(); }

int gs_check_plan_header(const uint32_t* hdr, int64_t tiles) {
  if (!hdr) return gs_set_error(-1, "plan header: null");
  const uint64_t L = hdr[M_L], maxn = hdr[M_MAXN], lref = hdr[M_LREF], st = hdr[M_STATUS];
  const uint64_t p1 = hdr[M_SORT_P1], q1 = hdr[M_SORT_Q1], p2 = hdr[M_SORT_P2];
  if (st > 3u) return gs_set_error(-3, "plan header: status word %llu has unknown bits", (unsigned long long)st);
  if (L > lref)
    return gs_set_error(-3, "plan header: %llu list instances exceed the %llu bounding-rect instances",
                        (unsigned long long)L, (unsigned long long)lref);
  if (maxn > L)
    return gs_set_error(-3, "plan header: longest tile %llu > %llu instances", (unsigned long long)maxn,
                        (unsigned long long)L);
  if (tiles < 0 || p1 > (uint64_t)tiles || p2 > p1 || q1 > p1)
    return gs_set_error(-3, "plan header: sort-class prefixes p1=%llu q1=%llu p2=%llu inconsistent with %lld tiles",
                        (unsigned long long)p1, (unsigned long long)q1, (unsigned long long)p2, (long long)tiles);
  return 0;
}

int gs_check_ranges(const uint32_t* ranges, int64_t tiles, int64_t L, int64_t max_len) {
  if (!ranges && tiles > 0) return gs_set_error(-1, "ranges: null");
  int64_t next = 0;
  for (int64_t t = 0; t < tiles; ++t) {
    const int64_t a = ranges[2 * t], b = ranges[2 * t + 1];
    if (b < a || b > L)
      return gs_set_error(-3, "ranges: tile %lld has [%lld, %lld) outside [0, %lld]", (long long)t, (long long)a,
                          (long long)b, (long long)L);
    if (b > a) {
      if (a != next)
        return gs_set_error(-3, "ranges: tile %lld starts at %lld, expected %lld (lists not contiguous)",
                            (long long)t, (long long)a, (long long)next);
      if (max_len >= 0 && b - a > max_len)
        return gs_set_error(-3, "ranges: tile %lld holds %lld instances > the planned longest %lld", (long long)t,
                            (long long)(b - a), (long long)max_len);
      next = b;
    }
  }
  if (next != L) return gs_set_error(-3, "ranges: lists cover %lld of %lld instances", (long long)next, (long long)L);
  return 0;
}

int gs_check_point_list(const uint32_t* ids, int64_t L, int64_t P) {
  if (!ids && L > 0) return gs_set_error(-1, "point list: null");
  for (int64_t i = 0; i < L; ++i)
    if ((int64_t)ids[i] >= P)
      return gs_set_error(-3, "point list: entry %lld holds Gaussian id %u >= P = %lld", (long long)i, ids[i],
                          (long long)P);
  return 0;
}

int gs_check_walk_order(const int32_t* order, int64_t P) {
  if (!order && P > 0) return gs_set_error(-1, "walk order: null");
  std::vector<unsigned char> seen((size_t)(P > 0 ? P : 0), 0);
  for (int64_t i = 0; i < P; ++i) {
    const int64_t v = order[i];
    if (v < 0 || v >= P)
      return gs_set_error(-3, "walk order: entry %lld holds id %lld outside [0, %lld)", (long long)i, (long long)v,
                          (long long)P);
    if (seen[(size_t)v]++)
      return gs_set_error(-3, "walk order: id %lld appears twice (entry %lld): not a permutation", (long long)v,
                          (long long)i);
  }
  return 0;
}

}  // extern "C"
