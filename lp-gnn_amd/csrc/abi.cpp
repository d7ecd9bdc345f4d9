// Error state and build info of the C ABI (include/lpgnn.h).
#include <cstring>

#include "common.h"

namespace lpg {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

}  // namespace lpg

extern "C" const char *lpg_last_error(void) { return lpg::g_err; }

extern "C" const char *lpg_build_info(void) {
  return "liblpgnn_hip: gfx950 (CDNA4), wave64, fp32/bf16/fp16 CSR SpMM + MFMA FC (fp32 as f16x2 or x3 on the "
         "16-bit matrix cores, exact fp32, bf16, fp16), deterministic (no float atomics), -ffp-contract=off";
}
