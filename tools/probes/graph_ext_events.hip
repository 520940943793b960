// Probe: hipEventRecordWithFlags(..., hipEventRecordExternal) inside a stream capture -> event record
// nodes whose hipEventElapsedTime gives per-kernel durations on every graph launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void spin(float* p, int iters) {
    float v = p[threadIdx.x + blockIdx.x * blockDim.x];
    for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 0.5f;
    p[threadIdx.x + blockIdx.x * blockDim.x] = v;
}
int main() {
    float* buf; CK(hipMalloc(&buf, 1 << 24));
    hipStream_t s; CK(hipStreamCreate(&s));
    const int n = 4, iters[n] = {20000, 5000, 80000, 1000};
    hipEvent_t ev[n + 1];
    for (int k = 0; k <= n; ++k) CK(hipEventCreate(&ev[k]));
    // eager reference
    for (int k = 0; k < n; ++k) {
        CK(hipEventRecord(ev[0], s)); spin<<<1024, 256, 0, s>>>(buf, iters[k]); CK(hipEventRecord(ev[1], s));
        CK(hipStreamSynchronize(s)); float ms; CK(hipEventElapsedTime(&ms, ev[0], ev[1])); printf("eager k%d %.1f us\n", k, ms * 1e3);
    }
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecordWithFlags(ev[0], s, hipEventRecordExternal));
    for (int k = 0; k < n; ++k) { spin<<<1024, 256, 0, s>>>(buf, iters[k]); CK(hipEventRecordWithFlags(ev[k + 1], s, hipEventRecordExternal)); }
    CK(hipStreamEndCapture(s, &g));
    size_t nn = 0; CK(hipGraphGetNodes(g, nullptr, &nn)); printf("graph nodes %zu\n", nn);
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 3; ++r) {
        CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
        printf("replay %d:", r);
        for (int k = 0; k < n; ++k) { float ms; CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1])); printf(" %.1f", ms * 1e3); }
        printf(" us\n");
    }
    return 0;
}
