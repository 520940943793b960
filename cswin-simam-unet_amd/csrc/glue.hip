// Small fused passes that replace the PyTorch elementwise kernels left between the csu kernels of a
// training step:
//   * grad_join: the gradient of an fp32 activation that was cast once to bf16 for two consumers
//     (encoder skip -> Merge conv + decoder concat_linear, cswin:530-545 / 568-592; decoder block
//     output -> CARAFE down conv + reassembly, cswin:408-432): out = a + b in fp32 plus the bf16
//     copy the upstream GEMM backward consumes -- one pass instead of cast, add, cast;
//   * BCE loss (nn.BCELoss, mean, cswin:935): forward as fixed-order per-block partial sums + one
//     final block (deterministic), backward elementwise with torch's clamps (log >= -100,
//     denominator >= 1e-12);
//   * image pack: the fp32 NCHW image -> bf16 NHWC with the channels zero-padded to a multiple of
//     8 (the patch-embed conv's 16-B gathers), one pass instead of zeros + strided copy.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ void load8_any(int dt, const void* p, long e, float* v) {
    if (dt == CSU_BF16) load8((const bf16*)p + e, v);
    else load8((const float*)p + e, v);
}

__global__ __launch_bounds__(NT) void grad_join_kernel(long n8, int adt, const void* __restrict__ a, int bdt,
                                                       const void* __restrict__ b, float* __restrict__ out,
                                                       bf16* __restrict__ outb) {
    for (long g = (long)blockIdx.x * NT + threadIdx.x; g < n8; g += (long)gridDim.x * NT) {
        const long e = g * 8;
        float va[8], vb[8];
        load8_any(adt, a, e, va);
        if (b) {
            load8_any(bdt, b, e, vb);
#pragma unroll
            for (int j = 0; j < 8; ++j) va[j] += vb[j];
        }
        if (out) store8(out + e, va);
        if (outb) store8(outb + e, va);
    }
}

// ATen's binary_cross_entropy: (t - 1) * max(log1p(-p), -100) - t * max(log p, -100) -- log1p, so
// p near 0 contributes ~p, not the 0 that logf(1 - p) rounds to for p < 6e-8
__device__ __forceinline__ float bce_term(float p, float t) {
    const float lp = fmaxf(logf(p), -100.f), lq = fmaxf(log1pf(-p), -100.f);
    return (t - 1.f) * lq - t * lp;
}

constexpr int BCE_BLOCKS = 1024;

// partial[block] = sum over the block's fixed element range (fixed order: per-thread strided sum,
// then a fixed shuffle + LDS tree)
__global__ __launch_bounds__(NT) void bce_partial(long n, const float* __restrict__ p, const float* __restrict__ t,
                                                  float* __restrict__ partial, int stats) {
    // stats: also the per-step segmentation sums of the reference loop (cswin:789-795, thresholded
    // predictions pred = p > 0.5): sum(pred * t), sum(pred), sum(t) -> partial[k * gridDim.x + block]
    __shared__ float red[4][NT / 64];
    const long per = (n + gridDim.x - 1) / gridDim.x;
    const long b0 = (long)blockIdx.x * per, b1 = min(n, b0 + per);
    float s = 0.f, si = 0.f, sp = 0.f, st = 0.f;
    auto acc = [&](float pv, float tv) {
        s += bce_term(pv, tv);
        const float pr = pv > 0.5f ? 1.f : 0.f;
        si += pr * tv;
        sp += pr;
        st += tv;
    };
    if ((per & 3) == 0 && (n & 3) == 0) {
        for (long e = b0 + 4 * threadIdx.x; e < b1; e += 4 * NT) {
            float pv[4], tv[4];
            load4(p + e, pv);
            load4(t + e, tv);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc(pv[j], tv[j]);
        }
    } else {
        for (long e = b0 + threadIdx.x; e < b1; e += NT) acc(p[e], t[e]);
    }
    const float v[4] = {s, si, sp, st};
    const int nk = stats ? 4 : 1;
    for (int k = 0; k < nk; ++k) {
        const float w = wave_sum(v[k]);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = w;
    }
    __syncthreads();
    if (threadIdx.x < nk) {
        const int k = threadIdx.x;
        partial[(long)k * gridDim.x + blockIdx.x] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    }
}

__global__ __launch_bounds__(NT) void bce_final(int nb, long n, const float* __restrict__ partial, float* __restrict__ loss,
                                                float* __restrict__ stats) {
    __shared__ float red[NT / 64];
    const int nk = stats ? 4 : 1;
    for (int k = 0; k < nk; ++k) {
        float s = 0.f;
        for (int i = threadIdx.x; i < nb; i += NT) s += partial[(long)k * nb + i];
        s = wave_sum(s);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            const float tot = (red[0] + red[1]) + (red[2] + red[3]);
            if (k == 0) loss[0] = tot / (float)n;
            else stats[k - 1] = tot;
        }
        __syncthreads();
    }
}

// dp = dloss * (p - t) / max((1 - p) p, 1e-12) * (1 / n)   (torch: bce backward, then div by numel
// as a multiplication by the fp32 reciprocal)
__global__ __launch_bounds__(NT) void bce_backward(long n, const float* __restrict__ p, const float* __restrict__ t,
                                                   const float* __restrict__ dloss, float* __restrict__ dp) {
    const float g = dloss[0], inv = 1.f / (float)n;
    for (long e = (long)blockIdx.x * NT + threadIdx.x; e < n; e += (long)gridDim.x * NT) {
        const float pv = p[e];
        dp[e] = (g * (pv - t[e]) / fmaxf((1.f - pv) * pv, 1e-12f)) * inv;
    }
}

// one thread per output pixel: C fp32 channel reads (plane stride H*W, coalesced across threads),
// one 16-B store per 8 output channels
__global__ __launch_bounds__(NT) void pack_nhwc(long pixels, int C, int Cp, long hw, const float* __restrict__ x,
                                                bf16* __restrict__ y) {
    for (long q = (long)blockIdx.x * NT + threadIdx.x; q < pixels; q += (long)gridDim.x * NT) {
        const long b = q / hw, s = q - b * hw;
        const float* src = x + b * C * hw + s;
        for (int c0 = 0; c0 < Cp; c0 += 8) {
            bf16x8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = (bf16)(c0 + j < C ? src[(long)(c0 + j) * hw] : 0.f);
            *reinterpret_cast<bf16x8*>(y + q * Cp + c0) = v;
        }
    }
}

unsigned grid_for(long work) {
    const long g = (work + NT - 1) / NT;
    return (unsigned)(g < 1 ? 1 : g > 8192 ? 8192 : g);
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_grad_join(long n, int adtype, const void* a, int bdtype, const void* b, float* out, void* out_bf16,
                             void* stream) {
    if (n < 0 || !a || (!out && !out_bf16) || (n % 8))
        return fail(CSU_E_ARG, "grad_join: bad args (n must be a multiple of 8, one output at least)");
    if ((adtype != CSU_BF16 && adtype != CSU_F32) || (b && bdtype != CSU_BF16 && bdtype != CSU_F32))
        return fail(CSU_E_ARG, "grad_join: bad dtype");
    if (n == 0) return 0;
    grad_join_kernel<<<grid_for(n / 8), NT, 0, as_stream(stream)>>>(n / 8, adtype, a, bdtype, b, out, (bf16*)out_bf16);
    return check_launch("grad_join");
}

extern "C" size_t csu_bce_loss_workspace(long n) { return (size_t)4 * BCE_BLOCKS * sizeof(float); }

static int bce_fwd(long n, const float* p, const float* t, float* loss, float* stats, void* workspace, size_t ws_bytes,
                   void* stream) {
    if (n < 1 || !p || !t || !loss) return fail(CSU_E_ARG, "bce_loss_fwd: bad args");
    if (!workspace || ws_bytes < csu_bce_loss_workspace(n)) return fail(CSU_E_WORKSPACE, "bce_loss_fwd: workspace");
    const long want = (n + 4 * NT - 1) / (4 * NT);
    const int nb = (int)(want < BCE_BLOCKS ? want : BCE_BLOCKS);
    hipStream_t st = as_stream(stream);
    bce_partial<<<nb, NT, 0, st>>>(n, p, t, (float*)workspace, stats != nullptr);
    if (int e = check_launch("bce_loss_fwd")) return e;
    bce_final<<<1, NT, 0, st>>>(nb, n, (const float*)workspace, loss, stats);
    return check_launch("bce_loss_fwd");
}

extern "C" int csu_bce_loss_fwd(long n, const float* p, const float* t, float* loss, void* workspace, size_t ws_bytes,
                                void* stream) {
    return bce_fwd(n, p, t, loss, nullptr, workspace, ws_bytes, stream);
}

extern "C" int csu_bce_loss_fwd_stats(long n, const float* p, const float* t, float* loss, float* stats, void* workspace,
                                      size_t ws_bytes, void* stream) {
    if (!stats) return fail(CSU_E_ARG, "bce_loss_fwd_stats: null stats");
    return bce_fwd(n, p, t, loss, stats, workspace, ws_bytes, stream);
}

extern "C" int csu_bce_loss_bwd(long n, const float* p, const float* t, const float* dloss, float* dp, void* stream) {
    if (n < 1 || !p || !t || !dloss || !dp) return fail(CSU_E_ARG, "bce_loss_bwd: bad args");
    bce_backward<<<grid_for(n), NT, 0, as_stream(stream)>>>(n, p, t, dloss, dp);
    return check_launch("bce_loss_bwd");
}

extern "C" int csu_pack_nhwc_bf16(int B, int C, int H, int W, int Cp, const float* x, void* y, void* stream) {
    if (B < 1 || C < 1 || H < 1 || W < 1 || Cp < C || Cp % 8 || !x || !y) return fail(CSU_E_ARG, "pack_nhwc_bf16: bad args");
    const long pixels = (long)B * H * W;
    pack_nhwc<<<grid_for(pixels), NT, 0, as_stream(stream)>>>(pixels, C, Cp, (long)H * W, x, (bf16*)y);
    return check_launch("pack_nhwc_bf16");
}
