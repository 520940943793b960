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



// Quantisation straight into the kernels' bf16 shadows (csu_quant_e4m3_shadow_batch): block = 64 rows of
// one item, thread = (row tr, 16 columns tc of each 64-column tile).  Phase 1: the row amax (two tiles
// of loads in flight per thread, the 4 threads of a row combined by lane shuffles) and its scale (the
// rule of quant_e4m3_rows, bit for bit).  Phase 2, per tile: e4m3 bytes, the exact bf16 of q * s (the
// shadow), and through LDS tiles the transposed shadow and the fp8 fused Mlp's operand layouts
// (q_perm: columns permuted within 64-groups; q_t: transposed; q_tp: transposed with permuted columns).
constexpr int T8S = 68;   // byte row stride of the e4m3 transposition tile (4 column groups on distinct banks)

__device__ __forceinline__ float row_scale_of(float amax) { return amax > 0.f ? exp2f(ceilf(log2f(amax / 448.f))) : 1.f; }

__global__ __launch_bounds__(NT) void quant_e4m3_shadow(const csu_fp8_shadow_item* __restrict__ items, int count) {
    __shared__ __attribute__((aligned(16))) bf16 T[64][64 + 8];
    __shared__ __attribute__((aligned(16))) uint8_t T8[64 * T8S];
    int lo = 0, hi = count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].blk0 <= (long)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    const csu_fp8_shadow_item it = items[lo];
    const int rows = it.rows, cols = it.cols;
    const int rb = (int)((long)blockIdx.x - it.blk0) * 64;
    const int tr = threadIdx.x >> 2, tc = (threadIdx.x & 3) * 16;
    const int row = rb + tr;
    const bool rok = row < rows;
    const float* src = it.src + (long)(rok ? row : 0) * cols;
    auto load16 = [&](int col, float* v) {   // cols % 16 == 0: whole 16-column runs
        if (rok && col < cols) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(src + col + 4 * k);
                v[4 * k] = x[0]; v[4 * k + 1] = x[1]; v[4 * k + 2] = x[2]; v[4 * k + 3] = x[3];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = 0.f;
        }
    };
    float amax = 0.f;
    for (int c0 = 0; c0 < cols; c0 += 128) {
        float a[16], b[16];
        load16(c0 + tc, a);
        load16(c0 + 64 + tc, b);
#pragma unroll
        for (int k = 0; k < 16; ++k) amax = fmaxf(amax, fmaxf(fabsf(a[k]), fabsf(b[k])));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    const float sc = row_scale_of(amax);
    if (rok && (threadIdx.x & 3) == 0 && it.scales) it.scales[row] = sc;
    const float inv = 1.f / sc;   // exact: a power of two
    bf16* const sh = (bf16*)it.shadow;
    bf16* const st = (bf16*)it.shadow_t;
    const bool tiles = st || it.q_t || it.q_tp;
    for (int c0 = 0; c0 < cols; c0 += 64) {
        const int col = c0 + tc;
        const bool ok = rok && col < cols;
        float v[16];
        load16(col, v);
        unsigned w[4];
        float dq[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int p = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * k] * inv, v[4 * k + 1] * inv, 0, false);
            p = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * k + 2] * inv, v[4 * k + 3] * inv, p, true);
            w[k] = (unsigned)p;
            const auto a = __builtin_amdgcn_cvt_pk_f32_fp8(p, false);
            const auto b = __builtin_amdgcn_cvt_pk_f32_fp8(p, true);
            dq[4 * k] = a[0] * sc; dq[4 * k + 1] = a[1] * sc; dq[4 * k + 2] = b[0] * sc; dq[4 * k + 3] = b[1] * sc;
        }
        if (ok) {
            const long o = (long)row * cols + col;
            if (it.q) *reinterpret_cast<u32x4*>(it.q + o) = u32x4{w[0], w[1], w[2], w[3]};
            if (it.q_perm) {   // dst 32h + 16t + 4g + i <- src 32t + 8g + 4h + i within the 64-group
                const int k = tc >> 4, t = k >> 1, d0 = 16 * t + 8 * (k & 1);
                *reinterpret_cast<u32x2*>(it.q_perm + (long)row * cols + c0 + d0) = u32x2{w[0], w[2]};
                *reinterpret_cast<u32x2*>(it.q_perm + (long)row * cols + c0 + 32 + d0) = u32x2{w[1], w[3]};
            }
            store8(sh + o, dq);
            store8(sh + o + 8, dq + 8);
        }
        if (tiles) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                T[tc + j][tr] = (bf16)dq[j];
                T8[(tc + j) * T8S + tr] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
            }
            __syncthreads();
            const int tcol = threadIdx.x >> 2, r16 = (threadIdx.x & 3) * 16;   // dst row = c0 + tcol
            if (c0 + tcol < cols) {
                const long drow = c0 + tcol;
                if (st) {
                    bf16* dst = st + drow * rows + rb + r16;
                    if (rb + r16 + 16 <= rows && (rows & 7) == 0) {
                        *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(&T[tcol][r16]);
                        *reinterpret_cast<u32x4*>(dst + 8) = *reinterpret_cast<const u32x4*>(&T[tcol][r16 + 8]);
                    } else {
                        for (int j = 0; j < 16 && rb + r16 + j < rows; ++j) dst[j] = T[tcol][r16 + j];
                    }
                }
                const unsigned* t8 = reinterpret_cast<const unsigned*>(T8 + tcol * T8S);
                if (it.q_t)   // rows % 64 == 0 (host-checked)
                    *reinterpret_cast<u32x4*>(it.q_t + drow * rows + rb + r16) =
                        u32x4{t8[r16 / 4], t8[r16 / 4 + 1], t8[r16 / 4 + 2], t8[r16 / 4 + 3]};
                if (it.q_tp) {   // dst col 32h + 16t + 4g + i <- src row 32t + 8g + 4h + i (k = r16 / 16 = 2h + t)
                    const int k = r16 >> 4, b = 32 * (k & 1) + 4 * (k >> 1);
                    *reinterpret_cast<u32x4*>(it.q_tp + drow * rows + rb + r16) =
                        u32x4{t8[b / 4], t8[(b + 8) / 4], t8[(b + 16) / 4], t8[(b + 24) / 4]};
                }
            }
            __syncthreads();
        }
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

extern "C" int csu_quant_e4m3_shadow_batch(const csu_fp8_shadow_item* items, int count, long total_blocks, void* stream) {
    if (count < 1 || total_blocks < 1 || !items) return fail(CSU_E_ARG, "quant_e4m3_shadow: bad args");
    quant_e4m3_shadow<<<(unsigned)total_blocks, NT, 0, as_stream(stream)>>>(items, count);
    return check_launch("quant_e4m3_shadow");
}
