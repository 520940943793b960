// Error reporting and build info for libcsu_hip.so.
#include <string>

#include "common.hpp"

namespace csu {
namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& s) { g_last_error = s; }

int fail(int code, const std::string& s) {
    g_last_error = s;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_error = std::string(what) + ": " + hipGetErrorString(e);
        return (int)e;
    }
    return 0;
}

}  // namespace csu

extern "C" const char* csu_last_error_string(void) { return csu::g_last_error.c_str(); }

extern "C" const char* csu_build_info(void) { return "libcsu_hip 0.1 (gfx950, CDNA4; bf16/fp32 MFMA)"; }
