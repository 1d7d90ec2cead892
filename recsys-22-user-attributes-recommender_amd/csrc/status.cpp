// C-ABI status plumbing: thread-local last-error message (include/asme_mi.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "common.h"

namespace asme {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int hip_status(hipError_t e, const char* where) {
    if (e == hipSuccess) return 0;
    char buf[512];
    std::snprintf(buf, sizeof(buf), "%s: HIP error %d (%s)", where, (int)e, hipGetErrorString(e));
    g_last_error = buf;
    return -2;
}
}  // namespace asme

ASME_API const char* asme_mi_last_error(void) { return asme::g_last_error.c_str(); }

ASME_API int asme_mi_abi_version(void) { return 1; }
