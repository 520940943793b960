// Fused multi-tensor AdamW for gfx950 (fp32 params / grads / moments).
//
// The optimizer of the reference training step (torch.optim.AdamW(lr 1e-4, betas (0.9, 0.999),
// eps 1e-8, weight_decay 1e-4), cswin:937-941) over all 463 parameter tensors in ONE launch:
// a device table of (param, grad, exp_avg, exp_avg_sq, numel, first chunk) items, one workgroup per
// 4096-element chunk (items found by binary search), 16-B vector loads/stores; the update is
// torch's AdamW arithmetic operation for operation (decoupled decay, lerp first moment,
// sqrt(v)/sqrt(bc2) + eps denominator).  lr and step may live on the device (HIP-graph capture:
// the scheduler updates the lr tensor between replays, a graph node increments the step).
// Streaming kernel: 28 B per parameter (read p, g, m, v; write p, m, v), HBM-bound.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int PER = 16;                  // elements per thread
constexpr long CH = (long)NT * PER;      // elements per chunk (workgroup)

// L2 = false: AdamW (decoupled decay, cswin:937-941); L2 = true: Adam with L2 weight decay, the
// plain UNet's optim.Adam(weight_decay) (unet:486-490): g += wd * param before the moments
template <bool L2>
__global__ __launch_bounds__(NT) void adamw_kernel(const csu_adamw_item* __restrict__ items, int count, const float* lr_dev,
                                                   float lr_host, float beta1, float beta2, float eps, float wd,
                                                   const float* step_dev, float step_host) {
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
    const float step_size = lr / bc1, bc2s = sqrtf(bc2), decay = L2 ? 1.f : 1.f - lr * wd;
    float* p = it.param;
    const float* g = it.grad;
    float* m = it.exp_avg;
    float* v = it.exp_avg_sq;
    const long base = (b - it.chunk0) * CH;
    const bool vec = (it.numel & 3) == 0;
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const long i = base + ((long)q * NT + threadIdx.x) * 4;   // 4 consecutive elements, coalesced per q
        if (i >= it.numel) break;
        float pv[4], gv[4], mv[4], vv[4];
        const int n = vec ? 4 : (int)(it.numel - i < 4 ? it.numel - i : 4);
        if (vec) {
            load4(p + i, pv); load4(g + i, gv); load4(m + i, mv); load4(v + i, vv);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = j < n;
                pv[j] = ok ? p[i + j] : 0.f; gv[j] = ok ? g[i + j] : 0.f;
                mv[j] = ok ? m[i + j] : 0.f; vv[j] = ok ? v[i + j] : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (L2) gv[j] = fmaf(wd, pv[j], gv[j]);
            else pv[j] *= decay;
            mv[j] = fmaf(1.f - beta1, gv[j] - mv[j], mv[j]);   // lerp(m, g, 1 - beta1)
            vv[j] = fmaf(1.f - beta2, gv[j] * gv[j], vv[j] * beta2);
            const float denom = sqrtf(vv[j]) / bc2s + eps;
            pv[j] = fmaf(-step_size, mv[j] / denom, pv[j]);
        }
        if (vec) {
            store4(p + i, pv); store4(m + i, mv); store4(v + i, vv);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (j < n) { p[i + j] = pv[j]; m[i + j] = mv[j]; v[i + j] = vv[j]; }
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
