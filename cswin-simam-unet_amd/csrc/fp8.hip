// fp8-e4m3 weight quantization for the 1024x1024 configuration (BASELINE config 5: "fp8-e4m3
// weights, bf16 activations, fp32 accumulate", SURVEY §8 d).  Each row (output feature) of a
// Linear weight gets a power-of-two scale s = 2^ceil(log2(amax / 448)) (448 = e4m3fn max), so
// every quantised value q * s is exactly representable in bf16 and the kernels that consume the
// dequantised bf16 shadow compute on exactly the e4m3 weights.  Round-to-nearest-even, OCP
// e4m3fn (v_cvt_pk_fp8_f32); |w / s| <= 448 by construction, so nothing saturates.
// One launch per step for every weight: block = one row of one item (items sorted by row0).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ float e4m3_round(float v) {
    const int p = __builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false);
    return __builtin_amdgcn_cvt_f32_fp8(p, 0);
}

__global__ __launch_bounds__(NT) void quant_e4m3_rows(const csu_fp8_item* __restrict__ items, int count) {
    __shared__ float red[NT / 64];
    // item of this row: last item with row0 <= blockIdx.x (binary search, uniform)
    int lo = 0, hi = count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].row0 <= (long)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    const csu_fp8_item it = items[lo];
    const long row = (long)blockIdx.x - it.row0;
    const float* src = it.src + row * it.cols;
    float amax = 0.f;
    for (int c = threadIdx.x; c < it.cols; c += NT) amax = fmaxf(amax, fabsf(src[c]));
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // power-of-two scale: the smallest 2^e with amax / 2^e <= 448
    const float s = amax > 0.f ? exp2f(ceilf(log2f(amax / 448.f))) : 1.f;
    const float inv = 1.f / s;   // exact (power of two)
    if (threadIdx.x == 0 && it.scales) it.scales[row] = s;
    for (int c = threadIdx.x; c < it.cols; c += NT) {
        const float v = src[c] * inv;
        const int p = __builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false);
        it.dst[row * it.cols + c] = __builtin_amdgcn_cvt_f32_fp8(p, 0) * s;
        if (it.dst_q) it.dst_q[row * it.cols + c] = (uint8_t)(p & 0xff);
    }
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_quant_e4m3_batch(const csu_fp8_item* items, int count, long total_rows, void* stream) {
    if (count < 1 || total_rows < 1 || !items) return fail(CSU_E_ARG, "quant_e4m3: bad args");
    quant_e4m3_rows<<<(unsigned)total_rows, NT, 0, as_stream(stream)>>>(items, count);
    return check_launch("quant_e4m3");
}
