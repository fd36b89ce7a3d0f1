// Error text + version for the kinet_amd C-ABI (include/kinet_common.h).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/kinet_common.h"
#include "common.h"

namespace kinet {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace kinet

extern "C" const char* kinet_last_error(void) { return kinet::g_err; }

extern "C" const char* kinet_version(void) { return "kinet_amd 0.1 gfx950 built " __DATE__ " " __TIME__; }
