// Error state + library metadata for the C ABI (include/gpt2mi.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "common.h"
#include "gpt2mi.h"

namespace gpt2mi {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}
}  // namespace gpt2mi

GPT2MI_EXPORT const char* gpt2mi_last_error(void) { return gpt2mi::g_err; }

GPT2MI_EXPORT int gpt2mi_abi_version(void) { return GPT2MI_ABI_VERSION; }
