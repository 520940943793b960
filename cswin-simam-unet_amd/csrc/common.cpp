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

extern "C" int csu_event_create(void** event) {
    if (!event) return csu::fail(CSU_E_ARG, "event_create: null");
    hipEvent_t e = nullptr;
    // timing only (the ledger reads them after a full synchronize): no system-scope fence, so recording
    // one between two kernels of a replayed graph does not add an L2 write-back to the kernel before it
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess)
        return csu::fail(CSU_E_ARG, "event_create: hipEventCreateWithFlags failed");
    *event = e;
    return CSU_OK;
}
extern "C" int csu_event_destroy(void* event) {
    if (event && hipEventDestroy((hipEvent_t)event) != hipSuccess) return csu::fail(CSU_E_ARG, "event_destroy failed");
    return CSU_OK;
}
extern "C" int csu_event_record_ext(void* event, void* stream) {
    if (!event) return csu::fail(CSU_E_ARG, "event_record_ext: null event");
    hipStream_t st = csu::as_stream(stream);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    hipError_t e = hipStreamGetCaptureInfo_v2(st, &cs, nullptr, &g, &deps, &nd);
    if (e != hipSuccess) return csu::fail(CSU_E_ARG, std::string("event_record_ext: hipStreamGetCaptureInfo_v2: ") + hipGetErrorString(e));
    if (cs != hipStreamCaptureStatusActive) {
        e = hipEventRecord((hipEvent_t)event, st);
    } else {
        // capturing: append an event-record node after the stream's current dependencies and make it
        // the new dependency set (the runtime this library shares with torch refuses
        // hipEventRecordWithFlags(..., hipEventRecordExternal) inside a capture)
        hipGraphNode_t node = nullptr;
        e = hipGraphAddEventRecordNode(&node, g, deps, nd, (hipEvent_t)event);
        if (e == hipSuccess) e = hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies);
    }
    if (e != hipSuccess) return csu::fail(CSU_E_ARG, std::string("event_record_ext: ") + hipGetErrorString(e));
    return CSU_OK;
}
extern "C" int csu_event_elapsed_ms(void* start, void* end, float* ms) {
    if (!start || !end || !ms) return csu::fail(CSU_E_ARG, "event_elapsed_ms: null");
    if (hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end) != hipSuccess)
        return csu::fail(CSU_E_ARG, "event_elapsed_ms: hipEventElapsedTime failed (not yet complete?)");
    return CSU_OK;
}
