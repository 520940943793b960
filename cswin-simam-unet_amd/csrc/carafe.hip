// Fused CARAFE content-aware reassembly (+ the 1-class output head) for gfx950.
//
// Replaces, of CARAFE/CARAFE4.forward (cswin:401-437 / 450-486), everything between the encoder
// conv and the `out` 1x1 conv: pixel_shuffle of the kernel logits (cswin:410), softmax over the
// k^2 = 9 taps (cswin:412), both unfolds/reshape/permute (cswin:413-427), the per-pixel
// (C x 9) @ (9 x s^2) matmul (cswin:429) and the final pixel_shuffle (cswin:432).  Token-major
// (NHWC) in and out; the 9x-expanded unfold tensor and every layout copy disappear.
//   out[b, Y, X, c] = sum_t w[b, y, x, t, i, j] * x[b, y + ky - 1, x + kx - 1, c]   (zero padded)
//   with Y = y*s + i, X = x*s + j, t = 3*ky + kx, w = softmax_t(enc[b, y, x, t*s*s + i*s + j]).
// HBM-bound: one thread = one output pixel x 8 channels (16-B vectors); neighbour rows of x are
// re-read from L1/L2.  The softmax weights are saved (fp32) for the backward pass.
//
// Head (up_x4 + sigmoid, cswin:674-688): prob[b, p] = sigmoid(sum_c x[b, p, c] * w[c]) for the
// 1-class 1x1 conv without bias; backward gives dx = dlogit * w and deterministic dW partials.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int KT = 9;   // 3x3 taps

// 8 consecutive elements at byte offset `off` of a raw buffer resource (kOOB: zeros).  The 9 tap
// gathers are issued together: a predicated `if (inside) load` made hipcc wait vmcnt(0) per tap.
__device__ __forceinline__ void ld8_rs(__amdgpu_buffer_rsrc_t rs, unsigned off, const bf16*, float* v) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    bf16x8 b;
    __builtin_memcpy(&b, &x, 16);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (float)b[k];
}
__device__ __forceinline__ void ld8_rs(__amdgpu_buffer_rsrc_t rs, unsigned off, const float*, float* v) {
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    const u32x4 c = __builtin_amdgcn_raw_buffer_load_b128(rs, off == kOOB ? kOOB : off + 16, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = __uint_as_float(a[k]);
        v[4 + k] = __uint_as_float(c[k]);
    }
}

// One thread = one INPUT pixel x 8 channels and all S^2 output sub-pixels of it: the 9 neighbour
// vectors are gathered once per input pixel (not once per output pixel: S^2 x fewer L2 reads), and
// the pixel's 9 S^2 logits are read as contiguous vectors.
template <typename T, int S>
__global__ __launch_bounds__(NT) void carafe_fwd(int B, int H, int W, int C, const T* __restrict__ x,
                                                 const T* __restrict__ enc, T* __restrict__ out,
                                                 float* __restrict__ wsave) {
    constexpr int S2 = S * S;
    const int G = C / 8;
    const long gid = xcd_tile(blockIdx.x, gridDim.x) * NT + threadIdx.x;   // neighbour blocks share one L2
    const long total = (long)B * H * W * G;
    if (gid >= total) return;
    const int g = gid % G;
    long p = gid / G;
    const int xx = p % W; p /= W;
    const int y = p % H;
    const int b = p / H;
    const size_t lpix = ((size_t)b * H + y) * W + xx;
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x, (long)B * H * W * C * (long)sizeof(T));
    float v[KT][8];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        const int yy = y + t / 3 - 1, xq = xx + t % 3 - 1;
        const bool in = yy >= 0 && yy < H && xq >= 0 && xq < W;
        ld8_rs(rx, in ? (unsigned)(((((b * H + yy) * W + xq) * C) + 8 * g) * (int)sizeof(T)) : kOOB, x, v[t]);
    }
    float lg[KT * S2];   // logit of tap t, sub-pixel q at t * S2 + q
    const T* e = enc + lpix * KT * S2;
#pragma unroll
    for (int k = 0; k < KT * S2; k += 4) load4(e + k, lg + k);   // 9 S^2 is a multiple of 4
    const int sW = S * W, sH = S * H;
#pragma unroll
    for (int q = 0; q < S2; ++q) {
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < KT; ++t) mx = fmaxf(mx, lg[t * S2 + q]);
        float w[KT], den = 0.f;
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            w[t] = __expf(lg[t * S2 + q] - mx);
            den += w[t];
        }
        const float inv = 1.f / den;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            w[t] *= inv;
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += w[t] * v[t][k];
        }
        const int Y = y * S + q / S, X = xx * S + q % S;
        store8(out + (((size_t)b * sH + Y) * sW + X) * C + 8 * g, acc);
        if (g == 0) {
            float* ws = wsave + lpix * KT * S2 + q;
#pragma unroll
            for (int t = 0; t < KT; ++t) ws[t * S2] = w[t];
        }
    }
}

// d enc: per output pixel, dw_t = sum_c dout[c] x[nbr_t][c]; dlogit_t = w_t (dw_t - sum_u w_u dw_u).
// One thread = one input pixel x 8 channels x its S^2 output sub-pixels (the neighbour gathers once
// per input pixel); G = C/8 lanes cooperate on the channel sum (G in {8, 16, 32, 64} divides the wave).
template <typename T, int S>
__global__ __launch_bounds__(NT) void carafe_bwd_enc(int B, int H, int W, int C, const T* __restrict__ x,
                                                     const float* __restrict__ wsave, const T* __restrict__ dout,
                                                     T* __restrict__ denc) {
    constexpr int S2 = S * S;
    const int G = C / 8;
    const long gid = xcd_tile(blockIdx.x, gridDim.x) * NT + threadIdx.x;   // neighbour blocks share one L2
    const long total = (long)B * H * W * G;
    const bool live = gid < total;
    const long gg = live ? gid : 0;
    const int g = gg % G;
    long p = gg / G;
    const int xx = p % W; p /= W;
    const int y = p % H;
    const int b = p / H;
    const size_t lpix = ((size_t)b * H + y) * W + xx;
    const int sW = S * W, sH = S * H;
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(x, (long)B * H * W * C * (long)sizeof(T));
    float v[KT][8];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        const int yy = y + t / 3 - 1, xq = xx + t % 3 - 1;
        const bool in = yy >= 0 && yy < H && xq >= 0 && xq < W;
        ld8_rs(rx, in ? (unsigned)(((((b * H + yy) * W + xq) * C) + 8 * g) * (int)sizeof(T)) : kOOB, x, v[t]);
    }
    float go[S2][8];
#pragma unroll
    for (int q = 0; q < S2; ++q)
        load8(dout + (((size_t)b * sH + y * S + q / S) * sW + xx * S + q % S) * C + 8 * g, go[q]);
    float dw[S2][KT];
#pragma unroll
    for (int q = 0; q < S2; ++q)
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            float d = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) d += go[q][k] * v[t][k];
            dw[q][t] = d;
        }
    if constexpr (S == 2) {
        if (G >= 4) {
            // reduce-scatter over the pixel's G lanes (aligned groups of G consecutive lanes): the
            // top lane bit keeps sub-pixels {0,1} / {2,3}, the next one sub-pixel q of those (18 + 9
            // exchanges), then the lanes of one q sum its 9 tap values -- 18 + 9 + 9 log2(G/4)
            // exchanges instead of 36 log2(G); each lane ends with its q's 9 sums
            const int h = G >> 1, qq = G >> 2;
            const bool hi = (g & h) != 0, lo = (g & qq) != 0;
            float d2[2][KT], d1[KT];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int t = 0; t < KT; ++t) {
                    const float keep = hi ? dw[2 + j][t] : dw[j][t], send = hi ? dw[j][t] : dw[2 + j][t];
                    d2[j][t] = keep + __shfl_xor(send, h, 64);
                }
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                const float keep = lo ? d2[1][t] : d2[0][t], send = lo ? d2[0][t] : d2[1][t];
                d1[t] = keep + __shfl_xor(send, qq, 64);
            }
            for (int o = qq >> 1; o > 0; o >>= 1)
#pragma unroll
                for (int t = 0; t < KT; ++t) d1[t] += __shfl_xor(d1[t], o, 64);
            if (!live) return;
            const int q = (hi ? 2 : 0) + (lo ? 1 : 0);
            const float* ws = wsave + lpix * KT * S2 + q;
            T* de = denc + lpix * KT * S2 + q;
            float wt[KT], sum = 0.f;
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                wt[t] = ws[t * S2];
                sum += wt[t] * d1[t];
            }
            // the q's 9 outputs over its G/4 lanes (a runtime tap index into registers -> select chain)
            for (int t = g & (qq - 1); t < KT; t += qq) {
                float d = 0.f, w = 0.f;
#pragma unroll
                for (int k = 0; k < KT; ++k)
                    if (k == t) { d = d1[k]; w = wt[k]; }
                de[t * S2] = from_f<T>(w * (d - sum));
            }
            return;
        }
    }
    // reduce over the G lanes of this pixel (aligned groups of G consecutive lanes)
    for (int o = G >> 1; o > 0; o >>= 1)
#pragma unroll
        for (int q = 0; q < S2; ++q)
#pragma unroll
            for (int t = 0; t < KT; ++t) dw[q][t] += __shfl_xor(dw[q][t], o, 64);
    if (!live) return;
    if constexpr (S != 2) {   // S = 4 (144 values per pixel): one lane writes them
        if (g != 0) return;
        const float* ws = wsave + lpix * KT * S2;
        T* de = denc + lpix * KT * S2;
#pragma unroll
        for (int q = 0; q < S2; ++q) {
            float wt[KT], sum = 0.f;
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                wt[t] = ws[t * S2 + q];
                sum += wt[t] * dw[q][t];
            }
#pragma unroll
            for (int t = 0; t < KT; ++t) de[t * S2 + q] = from_f<T>(wt[t] * (dw[q][t] - sum));
        }
        return;
    }
    // S = 2, G < 4: every lane of the pixel now holds all 9 S^2 sums: the lanes split the pixel's outputs
    // (index i = t S^2 + q, consecutive lanes -> consecutive elements: coalesced stores instead of
    // one lane writing all 9 S^2 values)
    const float* ws = wsave + lpix * KT * S2;
    T* de = denc + lpix * KT * S2;
    float sum[S2];
#pragma unroll
    for (int q = 0; q < S2; ++q) sum[q] = 0.f;
#pragma unroll
    for (int i = 0; i < KT * S2; i += 4) {   // the pixel's softmax weights (same 16-B vectors in every lane)
        const f32x4 wv = *reinterpret_cast<const f32x4*>(ws + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) sum[(i + e) % S2] += wv[e] * dw[(i + e) % S2][(i + e) / S2];
    }
    // outputs g, g + G, ... (G = C / 8 lanes: 1..64 -- every one of the 9 S^2 outputs is written)
    for (int i = g; i < KT * S2; i += G) {
        // the lane's own (q, t) = (i % S2, i / S2): a runtime index into registers -> select chain
        float d = 0.f, sq = 0.f;
#pragma unroll
        for (int k = 0; k < KT * S2; ++k)
            if (k == i) { d = dw[k % S2][k / S2]; sq = sum[k % S2]; }
        de[i] = from_f<T>(ws[i] * (d - sq));
    }
}

// dx[y', x', c] = sum_t sum_{i,j} w[(y,x), t, (i,j)] dout[(y s + i, x s + j), c],  (y, x) = (y'-ky+1, x'-kx+1).
// One thread = one input pixel x 8 channels; taps in groups whose loads (the S^2 weights as 16-B
// vectors, the S^2 dout vectors) are all issued before their FMAs -- branch-free raw buffer loads,
// out-of-image neighbours at an out-of-range offset (zeros): the per-tap `continue` loop with a runtime
// s waited for every load in turn
template <typename T, int S>
__global__ __launch_bounds__(NT, 4) void carafe_bwd_x(int B, int H, int W, int C, const float* __restrict__ wsave,
                                                   const T* __restrict__ dout, T* __restrict__ dx) {
    constexpr int S2 = S * S;
    constexpr int TG = S == 2 && sizeof(T) == 2 ? 3 : 1;   // taps per load group
    const int G = C / 8;
    const long gid = xcd_tile(blockIdx.x, gridDim.x) * NT + threadIdx.x;   // neighbour blocks share one L2
    const long total = (long)B * H * W * G;
    if (gid >= total) return;
    const int g = gid % G;
    long p = gid / G;
    const int xp = p % W; p /= W;
    const int yp = p % H;
    const int b = p / H;
    const int sW = S * W, sH = S * H;
    const __amdgpu_buffer_rsrc_t rd = buf_rsrc(dout, (long)B * sH * sW * C * (long)sizeof(T));
    const __amdgpu_buffer_rsrc_t rw = buf_rsrc(wsave, (long)B * H * W * KT * S2 * 4);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int t0 = 0; t0 < KT; t0 += TG) {
        // dout vectors kept raw (bf16: 4 VGPRs per 8 channels) until their FMAs
        u32x4 v[TG][S2][sizeof(T) / 2];
        float w[TG][S2];
#pragma unroll
        for (int u = 0; u < TG; ++u) {
            const int t = t0 + u;
            const int y = yp - (t / 3 - 1), xx = xp - (t % 3 - 1);
            const bool in = y >= 0 && y < H && xx >= 0 && xx < W;
            const unsigned wo = in ? (unsigned)(((((long)b * H + y) * W + xx) * KT * S2 + t * S2) * 4) : kOOB;
#pragma unroll
            for (int q = 0; q < S2; q += 4) {
                const u32x4 wv = __builtin_amdgcn_raw_buffer_load_b128(rw, wo == kOOB ? kOOB : wo + 4 * q, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; ++e) w[u][q + e] = __uint_as_float(wv[e]);
            }
#pragma unroll
            for (int q = 0; q < S2; ++q) {
                const unsigned o = in ? (unsigned)(((((long)b * sH + y * S + q / S) * sW + xx * S + q % S) * C + 8 * g) *
                                                   (long)sizeof(T))
                                      : kOOB;
#pragma unroll
                for (int h = 0; h < (int)(sizeof(T) / 2); ++h)
                    v[u][q][h] = __builtin_amdgcn_raw_buffer_load_b128(rd, o == kOOB ? kOOB : o + 16 * h, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < TG; ++u)
#pragma unroll
            for (int q = 0; q < S2; ++q) {
                float f[8];
                if constexpr (sizeof(T) == 2) {
                    bf16x8 bv;
                    __builtin_memcpy(&bv, &v[u][q][0], 16);
#pragma unroll
                    for (int k = 0; k < 8; ++k) f[k] = (float)bv[k];
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) f[k] = __uint_as_float(v[u][q][k / 4][k % 4]);
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[k] += w[u][q] * f[k];
            }
    }
    store8(dx + (((size_t)b * H + yp) * W + xp) * C + 8 * g, acc);
}

// ---- 1-class head: prob = sigmoid(x . w) ----------------------------------------------------
template <typename T>
__global__ __launch_bounds__(NT) void head_fwd(long P, int C, const T* __restrict__ x, const float* __restrict__ w,
                                               float* __restrict__ prob) {
    const int G = C / 8;   // lanes per pixel
    const long gid = (long)blockIdx.x * NT + threadIdx.x;
    const bool live = gid < P * G;
    const long p = live ? gid / G : 0;
    const int g = live ? gid % G : 0;
    float v[8];
    load8(x + p * C + 8 * g, v);
    float d = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) d += v[k] * w[8 * g + k];
    for (int o = G >> 1; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
    if (live && g == 0) prob[p] = 1.f / (1.f + __expf(-d));
}

// dlogit = dprob * p (1 - p); dx = dlogit * w; per-block partial of dW = sum_p dlogit x
template <typename T>
__global__ __launch_bounds__(NT) void head_bwd(long P, int C, long pix_per_block, const T* __restrict__ x,
                                               const float* __restrict__ w, const float* __restrict__ prob,
                                               const float* __restrict__ dprob, T* __restrict__ dx,
                                               float* __restrict__ part) {
    __shared__ float red[NT][8];
    const int G = C / 8;              // lanes per pixel (C <= 64)
    const int PPI = NT / G;           // pixels per iteration
    const int g = threadIdx.x % G, pl = threadIdx.x / G;
    const long p0 = (long)blockIdx.x * pix_per_block, p1 = min(P, p0 + pix_per_block);
    float wv[8], acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 8; ++k) wv[k] = w[8 * g + k];
    for (long p = p0 + pl; p < p1; p += PPI) {
        const float pr = prob[p];
        const float dl = dprob[p] * pr * (1.f - pr);
        float v[8], o[8];
        load8(x + p * C + 8 * g, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc[k] += dl * v[k];
            o[k] = dl * wv[k];
        }
        store8(dx + p * C + 8 * g, o);
    }
    // combine the PPI pixel lanes in a fixed order
#pragma unroll
    for (int k = 0; k < 8; ++k) red[threadIdx.x][k] = acc[k];
    __syncthreads();
    if (threadIdx.x < C) {
        const int gc = threadIdx.x / 8, kc = threadIdx.x % 8;
        float s = 0.f;
        for (int q = 0; q < PPI; ++q) s += red[q * G + gc][kc];
        part[(size_t)blockIdx.x * C + threadIdx.x] = s;
    }
}

__global__ void head_wreduce(int C, int nb, const float* __restrict__ part, float* __restrict__ dw) {
    __shared__ float red[4][64];
    const int c = threadIdx.x & 63, l = threadIdx.x >> 6;
    float s = 0.f;
    if (c < C)
        for (int b = l; b < nb; b += 4) s += part[(size_t)b * C + c];
    red[l][c] = s;
    __syncthreads();
    if (l == 0 && c < C) dw[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

unsigned blocks(long threads) { return (unsigned)((threads + NT - 1) / NT); }

int check_args(int B, int H, int W, int C, int s) {
    if (B < 1 || H < 1 || W < 1 || (s != 2 && s != 4) || C < 8 || C % 8 || C / 8 > 64 || ((C / 8) & (C / 8 - 1)))
        return fail(CSU_E_ARG, "carafe: need s in {2, 4} and C = 8 * 2^k <= 512");
    if ((long)B * H * W * C * 4 >= (1L << 31))   // 32-bit buffer offsets into the input (fp32 worst case)
        return fail(CSU_E_UNSUPPORTED, "carafe: input larger than 2 GiB");
    return 0;
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_carafe_fwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                              void* out, float* wsave, void* stream) {
    if (int e = check_args(B, H, W, C, s)) return e;
    if (!x || !enc || !out || !wsave) return fail(CSU_E_ARG, "carafe_fwd: null buffer");
    const long n = (long)B * H * W * (C / 8);   // one thread per input pixel x 8 channels
    hipStream_t st = as_stream(stream);
#define CSU_CF(T, S_) carafe_fwd<T, S_><<<blocks(n), NT, 0, st>>>(B, H, W, C, (const T*)x, (const T*)enc, (T*)out, wsave)
    if (dtype == CSU_BF16) { if (s == 4) CSU_CF(bf16, 4); else CSU_CF(bf16, 2); }
    else if (dtype == CSU_F32) { if (s == 4) CSU_CF(float, 4); else CSU_CF(float, 2); }
    else return fail(CSU_E_ARG, "carafe_fwd: bad dtype");
#undef CSU_CF
    return check_launch("carafe_fwd");
}

extern "C" int csu_carafe_bwd(int B, int H, int W, int C, int s, int dtype, const void* x, const float* wsave,
                              const void* dout, void* dx, void* denc, void* stream) {
    if (int e = check_args(B, H, W, C, s)) return e;
    if (!x || !wsave || !dout || !dx || !denc) return fail(CSU_E_ARG, "carafe_bwd: null buffer");
    const long n_in = (long)B * H * W * (C / 8);
    hipStream_t st = as_stream(stream);
#define CSU_CE(T, S_) carafe_bwd_enc<T, S_><<<blocks(n_in), NT, 0, st>>>(B, H, W, C, (const T*)x, wsave, (const T*)dout, (T*)denc)
#define CSU_CX(T, S_) carafe_bwd_x<T, S_><<<blocks(n_in), NT, 0, st>>>(B, H, W, C, wsave, (const T*)dout, (T*)dx)
    if (dtype == CSU_BF16) {
        if (s == 4) CSU_CE(bf16, 4); else CSU_CE(bf16, 2);
        if (s == 4) CSU_CX(bf16, 4); else CSU_CX(bf16, 2);
    } else if (dtype == CSU_F32) {
        if (s == 4) CSU_CE(float, 4); else CSU_CE(float, 2);
        if (s == 4) CSU_CX(float, 4); else CSU_CX(float, 2);
    } else {
        return fail(CSU_E_ARG, "carafe_bwd: bad dtype");
    }
#undef CSU_CE
#undef CSU_CX
    return check_launch("carafe_bwd");
}

static long head_ppb(long P) { long r = (P + 1023) / 1024; return r < 64 ? 64 : r; }

extern "C" size_t csu_head_bwd_workspace(long P, int C) {
    const long ppb = head_ppb(P);
    return (size_t)((P + ppb - 1) / ppb) * C * sizeof(float);
}

extern "C" int csu_head_fwd(long P, int C, int dtype, const void* x, const float* w, float* prob, void* stream) {
    if (P < 1 || C < 8 || C > 64 || C % 8 || ((C / 8) & (C / 8 - 1)) || !x || !w || !prob)
        return fail(CSU_E_ARG, "head_fwd: need C in {8,16,32,64}");
    hipStream_t st = as_stream(stream);
    if (dtype == CSU_BF16) head_fwd<bf16><<<blocks(P * (C / 8)), NT, 0, st>>>(P, C, (const bf16*)x, w, prob);
    else if (dtype == CSU_F32) head_fwd<float><<<blocks(P * (C / 8)), NT, 0, st>>>(P, C, (const float*)x, w, prob);
    else return fail(CSU_E_ARG, "head_fwd: bad dtype");
    return check_launch("head_fwd");
}

extern "C" int csu_head_bwd(long P, int C, int dtype, const void* x, const float* w, const float* prob,
                            const float* dprob, void* dx, float* dw, void* workspace, size_t ws_bytes, void* stream) {
    if (P < 1 || C < 8 || C > 64 || C % 8 || ((C / 8) & (C / 8 - 1)) || !x || !w || !prob || !dprob || !dx || !dw)
        return fail(CSU_E_ARG, "head_bwd: bad args");
    if (!workspace || ws_bytes < csu_head_bwd_workspace(P, C)) return fail(CSU_E_WORKSPACE, "head_bwd: workspace");
    hipStream_t st = as_stream(stream);
    const long ppb = head_ppb(P);
    const int nb = (int)((P + ppb - 1) / ppb);
    float* part = (float*)workspace;
    if (dtype == CSU_BF16)
        head_bwd<bf16><<<nb, NT, 0, st>>>(P, C, ppb, (const bf16*)x, w, prob, dprob, (bf16*)dx, part);
    else if (dtype == CSU_F32)
        head_bwd<float><<<nb, NT, 0, st>>>(P, C, ppb, (const float*)x, w, prob, dprob, (float*)dx, part);
    else
        return fail(CSU_E_ARG, "head_bwd: bad dtype");
    head_wreduce<<<1, 256, 0, st>>>(C, nb, part, dw);
    return check_launch("head_bwd");
}
