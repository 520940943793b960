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


// e4m3 byte layouts (csu_e4m3_layout_batch): one thread per 4-byte dst word
__global__ __launch_bounds__(NT) void e4m3_layout_kernel(const csu_e4m3_layout_item* __restrict__ items, int count,
                                                         long total) {
    const long w = (long)blockIdx.x * NT + threadIdx.x;
    if (w >= total) return;
    int lo = 0, hi = count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].word0 <= w) lo = mid; else hi = mid - 1;
    }
    const csu_e4m3_layout_item it = items[lo];
    const bool tr = it.mode & 1, perm = it.mode & 2;
    const int dcols = tr ? it.rows : it.cols;
    const long p0 = (w - it.word0) * 4;                 // first dst byte of the word
    const long drow = p0 / dcols;
    int dcol = (int)(p0 % dcols);
    if (perm) {   // dst 32h + 16t + 4g (+ i) <- 32t + 8g + 4h (+ i)
        const int b = dcol & 63, h = b >> 5, t = (b >> 4) & 1, g = (b >> 2) & 3;
        dcol = (dcol & ~63) + 32 * t + 8 * g + 4 * h;
    }
    unsigned v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const long sidx = tr ? (long)(dcol + i) * it.cols + drow : drow * it.cols + dcol + i;
        v |= (unsigned)it.src[sidx] << (8 * i);
    }
    *reinterpret_cast<unsigned*>(it.dst + p0) = v;
}
}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_quant_e4m3_batch(const csu_fp8_item* items, int count, long total_rows, void* stream) {
    if (count < 1 || total_rows < 1 || !items) return fail(CSU_E_ARG, "quant_e4m3: bad args");
    quant_e4m3_rows<<<(unsigned)total_rows, NT, 0, as_stream(stream)>>>(items, count);
    return check_launch("quant_e4m3");
}

extern "C" int csu_e4m3_layout_batch(const csu_e4m3_layout_item* items, int count, long total_words, void* stream) {
    if (count < 1 || total_words < 1 || !items) return fail(CSU_E_ARG, "e4m3_layout: bad args");
    e4m3_layout_kernel<<<(unsigned)((total_words + NT - 1) / NT), NT, 0, as_stream(stream)>>>(items, count, total_words);
    return check_launch("e4m3_layout");
}
