// Batched fp32 -> bf16 weight cast (+ transposed copy) for gfx950: one launch refreshes every
// bf16 shadow of the fp32 master weights per step (the per-Linear weight casts autocast would do,
// cswin:185-195/314-368) and writes W^T (K, N) next to W (N, K), so the input-gradient GEMM
// dX = dY W is a plain b[n][k] GEMM (csu_gemm_ex, b_trans = 0).
// One workgroup = one 64 x 64 tile of one item; items are found by binary search on tile0.
// Conv-weight items (taps > 0) write the two channels-last layouts of the implicit-GEMM conv
// kernels instead (OHWI for the forward / transposed-conv input gradient, IHWO for the
// input gradient / transposed-conv forward), 4096 elements per workgroup.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int T = 64;

__global__ __launch_bounds__(NT) void cast_batch(const csu_cast_item* __restrict__ items, int count) {
    __shared__ bf16 tile[T][T + 2];
    const long b = blockIdx.x;
    int lo = 0, hi = count - 1;
    while (lo < hi) {   // last item with tile0 <= b
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].tile0 <= b) lo = mid; else hi = mid - 1;
    }
    const csu_cast_item it = items[lo];
    if (it.taps > 0) {   // conv weight (rows = N, cols = C, taps = KH*KW): OHWI and IHWO bf16 layouts
        const int n_el = it.rows * it.cols * it.taps;       // < 2^31 (conv weights)
        const unsigned CT = it.cols * it.taps, TP = it.taps;
        const unsigned CP = it.cols_pad > it.cols ? it.cols_pad : it.cols;
        bf16* o = (bf16*)it.dst;
        bf16* t = (bf16*)it.dst_t;
        const int e0 = (int)(b - it.tile0) * (T * T), e1 = min(n_el, e0 + T * T);
        for (int e = e0 + threadIdx.x; e < e1; e += NT) {
            const unsigned n = (unsigned)e / CT, rem = (unsigned)e - n * CT, c = rem / TP, k = rem - c * TP;
            const bf16 v = (bf16)it.src[e];                        // src [n][c][k]
            o[(n * TP + k) * CP + c] = v;                          // OHWI [n][k][c] (channel stride CP)
            if (t) t[(c * TP + k) * it.rows + n] = v;              // IHWO [c][k][n]
        }
        return;
    }
    const int tk = (it.cols + T - 1) / T;
    const long t = b - it.tile0;
    const int r0 = (int)(t / tk) * T, c0 = (int)(t % tk) * T;
    const float* src = it.src;
    bf16* dst = (bf16*)it.dst;
    bf16* dstT = (bf16*)it.dst_t;
    // rows r0.., 64 columns: thread -> (row = tid / 16 + 16 i, 4 columns)
    const int cq = (threadIdx.x & 15) * 4, rr = threadIdx.x >> 4;
#pragma unroll
    for (int i = 0; i < T / 16; ++i) {
        const int r = r0 + rr + 16 * i;
        if (r >= it.rows) continue;
        const int c = c0 + cq;
        float v[4];
        if (c + 4 <= it.cols && (it.cols & 3) == 0) {
            load4(src + (long)r * it.cols + c, v);
            store4(dst + (long)r * it.cols + c, v);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = c + j < it.cols ? src[(long)r * it.cols + c + j] : 0.f;
                if (c + j < it.cols) dst[(long)r * it.cols + c + j] = (bf16)v[j];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[rr + 16 * i][cq + j] = (bf16)v[j];
    }
    if (!dstT) return;
    __syncthreads();
    // transposed: rows c0.. of dstT (cols rows), thread -> (col = tid / 16 + 16 i, 4 rows)
#pragma unroll
    for (int i = 0; i < T / 16; ++i) {
        const int c = c0 + rr + 16 * i;
        if (c >= it.cols) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = r0 + cq + j;
            if (r < it.rows) dstT[(long)c * it.rows + r] = tile[cq + j][rr + 16 * i];
        }
    }
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_cast_bf16_batch(const csu_cast_item* items, int count, long total_tiles, void* stream) {
    if (count < 1 || total_tiles < 1 || !items) return fail(CSU_E_ARG, "cast_bf16_batch: bad args");
    cast_batch<<<(unsigned)total_tiles, NT, 0, as_stream(stream)>>>(items, count);
    return check_launch("cast_bf16_batch");
}
