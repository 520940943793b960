// Fused multi-tensor AdamW for gfx950 (fp32 params / grads / moments).
//
// The optimizer of the reference training step (torch.optim.AdamW(lr 1e-4, betas (0.9, 0.999),
// eps 1e-8, weight_decay 1e-4), cswin:937-941) over all 463 parameter tensors in ONE launch:
// a device table of (param, grad, exp_avg, exp_avg_sq, numel, first chunk) items, one workgroup per
// 4096-element chunk (items found by binary search), 16-B vector loads/stores; the update is
// torch's AdamW arithmetic operation for operation (decoupled decay, lerp first moment,
// sqrt(v)/sqrt(bc2) + eps denominator).  lr and step may live on the device (HIP-graph capture:
// the scheduler updates the lr tensor between replays, a graph node increments the step).
// Streaming kernel: 28 B per parameter (read p, g, m, v; write p, m, v), HBM-bound; + 2 B per bf16
// shadow layout written (the forward's weight copies, csu.h), which replaces a separate cast pass
// re-reading every fp32 weight (4 B + the same 2 B per layout).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int PER = 16;                  // elements per thread
constexpr long CH = (long)NT * PER;      // elements per chunk (workgroup)

struct AdamConst {
    float beta1, beta2, eps, wd, step_size, bc2s, decay;
};

template <bool L2> __device__ __forceinline__ void adam4(const AdamConst& k, float* pv, const float* gv0, float* mv, float* vv) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float g = gv0[j];
        if constexpr (L2) g = fmaf(k.wd, pv[j], g);
        else pv[j] *= k.decay;
        mv[j] = fmaf(1.f - k.beta1, g - mv[j], mv[j]);   // lerp(m, g, 1 - beta1)
        vv[j] = fmaf(1.f - k.beta2, g * g, vv[j] * k.beta2);
        const float denom = sqrtf(vv[j]) / k.bc2s + k.eps;
        pv[j] = fmaf(-k.step_size, mv[j] / denom, pv[j]);
    }
}

// n (<= 4) elements at index i: one 16-B vector when vec (n == 4, 16-B aligned), else scalars
__device__ __forceinline__ void ld4n(const float* p, long i, int n, bool vec, float* v) {
    if (vec) load4(p + i, v);
    else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = j < n ? p[i + j] : 0.f;
    }
}
template <typename T> __device__ __forceinline__ void st4n(T* p, long i, int n, bool vec, const float* v) {
    if (vec) store4(p + i, v);
    else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < n) p[i + j] = from_f<T>(v[j]);
    }
}

template <bool L2>
__device__ __forceinline__ void update(const AdamConst& k, float* p, const float* g, float* m, float* v, long i, int n,
                                       bool vec, float* pv) {
    float gv[4], mv[4], vv[4];
    ld4n(p, i, n, vec, pv);
    ld4n(g, i, n, vec, gv);
    ld4n(m, i, n, vec, mv);
    ld4n(v, i, n, vec, vv);
    adam4<L2>(k, pv, gv, mv, vv);
    st4n(p, i, n, vec, pv);
    st4n(m, i, n, vec, mv);
    st4n(v, i, n, vec, vv);
}

// L2 = false: AdamW (decoupled decay, cswin:937-941); L2 = true: Adam with L2 weight decay, the
// plain UNet's optim.Adam(weight_decay) (unet:486-490): g += wd * param before the moments.
// Shadow modes (csu.h): tile items update a 64 x 64 tile and write W and, through LDS, W^T in
// bf16; flat items write the bf16 copy at the same index, conv items scatter the OHWI / IHWO
// layouts (the csu_cast_bf16_batch layouts, now made from the updated fp32 value in registers).
template <bool L2>
__global__ __launch_bounds__(NT) void adamw_kernel(const csu_adamw_item* __restrict__ items, int count, const float* lr_dev,
                                                   float lr_host, float beta1, float beta2, float eps, float wd,
                                                   const float* step_dev, float step_host) {
    __shared__ bf16 tile[64][64 + 2];
    const long b = blockIdx.x;
    int lo = 0, hi = count - 1;
    while (lo < hi) {   // last item with chunk0 <= b
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].chunk0 <= b) lo = mid; else hi = mid - 1;
    }
    const csu_adamw_item it = items[lo];
    const float lr = lr_dev ? *lr_dev : lr_host;
    const float step = step_dev ? *step_dev : step_host;
    const float bc1 = 1.f - powf(beta1, step), bc2 = 1.f - powf(beta2, step);
    const AdamConst k{beta1, beta2, eps, wd, lr / bc1, sqrtf(bc2), L2 ? 1.f : 1.f - lr * wd};
    float* p = it.param;
    const float* g = it.grad;
    float* m = it.exp_avg;
    float* v = it.exp_avg_sq;
    bf16* sh = (bf16*)it.shadow;
    bf16* sht = (bf16*)it.shadow_t;
    if (sh && sht && it.taps == 0) {   // 64 x 64 tile of a rows x cols matrix: W and W^T shadows
        const int tk = (it.cols + 63) / 64;
        const long t = b - it.chunk0;
        const int r0 = (int)(t / tk) * 64, c0 = (int)(t % tk) * 64;
        const int cq = (threadIdx.x & 15) * 4, rr = threadIdx.x >> 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = r0 + rr + 16 * i, c = c0 + cq;
            float pv[4] = {0.f, 0.f, 0.f, 0.f};
            if (r < it.rows && c < it.cols) {
                const int n = min(4, it.cols - c);
                const bool vec = (it.cols & 3) == 0;   // then n == 4 and the row segment is 16-B aligned
                const long e = (long)r * it.cols + c;
                update<L2>(k, p, g, m, v, e, n, vec, pv);
                st4n(sh, e, n, vec, pv);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) tile[rr + 16 * i][cq + j] = (bf16)pv[j];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // W^T rows c0.. (cols rows): thread -> (column c, 4 rows)
            const int c = c0 + rr + 16 * i;
            if (c >= it.cols) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = r0 + cq + j;
                if (r < it.rows) sht[(long)c * it.rows + r] = tile[cq + j][rr + 16 * i];
            }
        }
        return;
    }
    const long base = (b - it.chunk0) * CH;
    const bool vec = (it.numel & 3) == 0;
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const long i = base + ((long)q * NT + threadIdx.x) * 4;   // 4 consecutive elements, coalesced per q
        if (i >= it.numel) break;
        const int n = vec ? 4 : (int)(it.numel - i < 4 ? it.numel - i : 4);
        float pv[4];
        update<L2>(k, p, g, m, v, i, n, vec, pv);
        if (!sh) continue;
        if (it.taps > 0) {   // conv weight [n][c][tap] -> OHWI [n][tap][c] (stride cols_pad), IHWO [c][tap][n]
            const unsigned TP = it.taps, CT = (unsigned)it.cols * TP;
            const unsigned CP = it.cols_pad > it.cols ? it.cols_pad : it.cols;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (j >= n) break;
                const unsigned e = (unsigned)(i + j), o = e / CT, rem = e - o * CT, c = rem / TP, t = rem - c * TP;
                const bf16 w = (bf16)pv[j];
                sh[(o * TP + t) * CP + c] = w;
                if (sht) sht[(c * TP + t) * (unsigned)it.rows + o] = w;
            }
        } else {
            st4n(sh, i, n, vec, pv);
        }
    }
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" long csu_adamw_chunk_elems(void) { return CH; }

extern "C" int csu_adamw_step(const csu_adamw_item* items, int count, long total_chunks, const float* lr_dev, float lr,
                              float beta1, float beta2, float eps, float weight_decay, const float* step_dev, float step,
                              void* stream) {
    if (!items || count < 1 || total_chunks < 1) return fail(CSU_E_ARG, "adamw: empty item table");
    adamw_kernel<false><<<(unsigned)total_chunks, NT, 0, as_stream(stream)>>>(items, count, lr_dev, lr, beta1, beta2, eps,
                                                                              weight_decay, step_dev, step);
    return check_launch("adamw");
}

extern "C" int csu_adam_l2_step(const csu_adamw_item* items, int count, long total_chunks, const float* lr_dev, float lr,
                                float beta1, float beta2, float eps, float weight_decay, const float* step_dev, float step,
                                void* stream) {
    if (!items || count < 1 || total_chunks < 1) return fail(CSU_E_ARG, "adam_l2: empty item table");
    adamw_kernel<true><<<(unsigned)total_chunks, NT, 0, as_stream(stream)>>>(items, count, lr_dev, lr, beta1, beta2, eps,
                                                                             weight_decay, step_dev, step);
    return check_launch("adam_l2");
}
