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

#ifndef KINET_SRC_HASH
#define KINET_SRC_HASH "unknown"
#endif

// "kinet_amd <ver> gfx950 src <hash>": <hash> = kinet_amd.build.source_hash() of the sources
// this library was compiled from (tests/test_native_cpu.py / test_build_gpu compare it).
extern "C" const char* kinet_version(void) { return "kinet_amd 0.2 gfx950 src " KINET_SRC_HASH; }
