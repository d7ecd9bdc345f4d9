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

}  // namespace lpg
