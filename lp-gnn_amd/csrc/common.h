// Internal helpers shared by the liblpgnn_hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "lpgnn.h"

namespace lpg {

// Thread-local last-error buffer behind lpg_last_error().
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

#define LPG_REQUIRE(cond, ...)              \
  do {                                      \
    if (!(cond)) {                          \
      ::lpg::set_error(__VA_ARGS__);        \
      return LPG_ERR_INVALID;               \
    }                                       \
  } while (0)

#define LPG_HIP(call)                                                        \
  do {                                                                       \
    hipError_t _e = (call);                                                  \
    if (_e != hipSuccess) {                                                  \
      ::lpg::set_error("%s failed: %s", #call, hipGetErrorString(_e));       \
      return LPG_ERR_HIP;                                                    \
    }                                                                        \
  } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Compute units of the current device (cached per device id).
inline int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// Workgroups of `kernel` (block of `threads`) that stay resident on the whole device at once:
// the grid of a persistent (row-range) kernel, so that no tail round follows.  The occupancy query
// runs once per (kernel, block size, device) and host thread (a thread-local cache: no locks).
template <typename K>
inline int64_t resident_blocks(K kernel, int threads) {
  struct Entry {
    const void *k;
    int threads, dev;
    int64_t blocks;
  };
  thread_local Entry cache[32];
  thread_local int used = 0;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  const void *key = reinterpret_cast<const void *>(kernel);
  for (int i = 0; i < used; ++i)
    if (cache[i].k == key && cache[i].threads == threads && cache[i].dev == dev) return cache[i].blocks;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  const int64_t blocks = (int64_t)per_cu * device_cus();
  if (used < 32) cache[used++] = Entry{key, threads, dev, blocks};
  return blocks;
}

}  // namespace lpg
