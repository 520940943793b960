// BatchNorm2d (+ ReLU) and MaxPool2d(2) of the plain UNet (train_unet_segmentation.py unet:177-204)
// on NHWC rows for gfx950 -- the ops between the implicit-GEMM convs of DoubleConv / Down.
//
// BatchNorm statistics are per channel over the M = B*H*W rows.  One row of C channels is
// contiguous, so a block owns 64 channels (8 lanes x 8 channels, 16-B bf16 / 2 x 16-B fp32 loads: a
// 128-B row segment per 8 lanes) and a chunk of rows; the 32 row groups of the block stride over the
// chunk.  Three launches per direction, each deterministic (fixed-order sums, no atomics):
//   1. partial:  per (chunk, channel) pivot-shifted sums  S1 = sum(x - p), S2 = sum((x - p)^2)
//                (p = x[row 0][c]: no cancellation for data far from 0);  backward: sum(g),
//                sum(g (x - mean)) with g = dy * [y > 0] (ReLU folded in);
//   2. finalize: one pass per 64 channels sums the chunk partials in chunk order -> mean / rstd
//                (biased variance, as F.batch_norm normalises) + the running-stat update (momentum,
//                unbiased variance, unet:183); backward: dgamma, dbeta;
//   3. apply:    y = relu((x - mean) rstd gamma + beta) in the input's dtype;  backward
//                dx = gamma rstd (g - dbeta / M - xhat dgamma / M)  (training) or gamma rstd g (eval).
// MaxPool2d(2): one thread per (output pixel, 8 channels); the backward recomputes the window's
// first maximum (torch's scan order, NaN wins) and writes all four input gradients of the window.
#include "common.hpp"

#include <numeric>

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int CW = 64;         // channels per block
constexpr int LPR = CW / 8;    // lanes per row (8 channels each)
constexpr int RG = NT / LPR;   // row groups per block (32)
constexpr int MAXCH = 256;     // row chunks per launch
constexpr int RIF = 8;         // rows in flight per thread

struct BnGeo {
    long M;
    int C, ncb, nch;
    long chunk;
};

BnGeo bn_geo(long M, int C) {
    BnGeo g{M, C, (C + CW - 1) / CW, 0, 0};
    long nch = (512 + g.ncb - 1) / g.ncb;                 // ~512 partial blocks per launch
    const long maxc = (M + RIF * RG - 1) / (RIF * RG);    // >= one full pass of rows in flight per block
    if (nch > maxc) nch = maxc;
    if (nch > MAXCH) nch = MAXCH;
    if (nch < 1) nch = 1;
    g.chunk = (M + nch - 1) / nch;
    g.nch = (int)((M + g.chunk - 1) / g.chunk);
    return g;
}

// pass 1, forward: S1, S2 of (x - pivot) per (chunk, channel) -> part[(chunk * C + c) * 2 + k]
template <typename T>
__global__ __launch_bounds__(NT) void bn_stats_partial(BnGeo g, const T* __restrict__ x, float* __restrict__ part) {
    __shared__ float red[RG][CW * 2 + 1];
    const int cb = blockIdx.x % g.ncb, ch = blockIdx.x / g.ncb;
    const int l8 = threadIdx.x % LPR, rg = threadIdx.x / LPR;
    const int c0 = cb * CW + 8 * l8;
    const bool cv = c0 < g.C;
    float p[8], s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = s1[j] = s2[j] = 0.f;
    if (cv) load8(x + c0, p);
    const long r0 = ch * g.chunk, r1 = min(g.M, r0 + g.chunk);
    if (cv) {
        // 8 rows in flight per thread (branch-free: rows past the chunk read a clamped row and add 0)
        for (long r = r0 + rg; r < r1; r += RIF * RG) {
            float v[RIF][8];
#pragma unroll
            for (int u = 0; u < RIF; ++u) load8(x + min(r + u * RG, r1 - 1) * g.C + c0, v[u]);
#pragma unroll
            for (int u = 0; u < RIF; ++u) {
                const float on = r + u * RG < r1 ? 1.f : 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float d = (v[u][j] - p[j]) * on;
                    s1[j] += d;
                    s2[j] = fmaf(d, d, s2[j]);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[rg][(8 * l8 + j) * 2] = s1[j];
        red[rg][(8 * l8 + j) * 2 + 1] = s2[j];
    }
    __syncthreads();
    if (threadIdx.x < CW * 2) {
        const int c = cb * CW + threadIdx.x / 2;
        float s = 0.f;
        for (int k = 0; k < RG; ++k) s += red[k][threadIdx.x];
        if (c < g.C) part[((long)ch * g.C + c) * 2 + (threadIdx.x & 1)] = s;
    }
}

// pass 1, backward: sum(g), sum(g (x - mean)) with g = dy [relu: y > 0], y recomputed from x
template <typename T, typename G>
__global__ __launch_bounds__(NT) void bn_grad_partial(BnGeo g, const T* __restrict__ x, const G* __restrict__ dy,
                                                      const float* __restrict__ save, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int relu,
                                                      float* __restrict__ part) {
    __shared__ float red[RG][CW * 2 + 1];
    const int cb = blockIdx.x % g.ncb, ch = blockIdx.x / g.ncb;
    const int l8 = threadIdx.x % LPR, rg = threadIdx.x / LPR;
    const int c0 = cb * CW + 8 * l8;
    const bool cv = c0 < g.C;
    float mu[8], a[8], b[8], sg[8], sgx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) mu[j] = a[j] = b[j] = sg[j] = sgx[j] = 0.f;
    if (cv)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            mu[j] = save[c0 + j];
            a[j] = save[g.C + c0 + j] * gamma[c0 + j];   // y = (x - mu) a + b
            b[j] = beta[c0 + j];
        }
    const long r0 = ch * g.chunk, r1 = min(g.M, r0 + g.chunk);
    if (cv) {
        for (long r = r0 + rg; r < r1; r += RIF * RG) {   // 8 rows of x and dy in flight
            float xv[RIF][8], gv[RIF][8];
#pragma unroll
            for (int u = 0; u < RIF; ++u) {
                const long rr = min(r + u * RG, r1 - 1);
                load8(x + rr * g.C + c0, xv[u]);
                load8(dy + rr * g.C + c0, gv[u]);
            }
#pragma unroll
            for (int u = 0; u < RIF; ++u) {
                const bool on = r + u * RG < r1;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float d = xv[u][j] - mu[j];
                    const float gg = (on && (!relu || fmaf(d, a[j], b[j]) > 0.f)) ? gv[u][j] : 0.f;
                    sg[j] += gg;
                    sgx[j] = fmaf(gg, d, sgx[j]);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        red[rg][(8 * l8 + j) * 2] = sg[j];
        red[rg][(8 * l8 + j) * 2 + 1] = sgx[j];
    }
    __syncthreads();
    if (threadIdx.x < CW * 2) {
        const int c = cb * CW + threadIdx.x / 2;
        float s = 0.f;
        for (int k = 0; k < RG; ++k) s += red[k][threadIdx.x];
        if (c < g.C) part[((long)ch * g.C + c) * 2 + (threadIdx.x & 1)] = s;
    }
}

// pass 2, forward: mean / rstd (save[0:C], save[C:2C]) and the running-stat update
__global__ __launch_bounds__(NT) void bn_stats_final(BnGeo g, const void* x, int xdt, const float* __restrict__ part,
                                                     float eps, float momentum, float* __restrict__ rmean,
                                                     float* __restrict__ rvar, float* __restrict__ save) {
    __shared__ float red[CW * 2][4];
    // 256 threads = 128 (channel, value) slots x 2 halves; half q sums the chunks i = 4j + q and
    // 4j + q + 2 into two registers, combined in a fixed order
    const int slot = threadIdx.x & (CW * 2 - 1), q = threadIdx.x / (CW * 2);
    const int c = blockIdx.x * CW + slot / 2, k = slot & 1;
    float s = 0.f, s2 = 0.f;
    if (c < g.C) {
        for (int i = q; i < g.nch; i += 4) s += part[((long)i * g.C + c) * 2 + k];
        for (int i = q + 2; i < g.nch; i += 4) s2 += part[((long)i * g.C + c) * 2 + k];
    }
    red[slot][q] = s;
    red[slot][q + 2] = s2;
    __syncthreads();
    if (threadIdx.x < CW && blockIdx.x * CW + threadIdx.x < g.C) {
        const int cc = blockIdx.x * CW + threadIdx.x;
        const float S1 = (red[2 * threadIdx.x][0] + red[2 * threadIdx.x][1]) + (red[2 * threadIdx.x][2] + red[2 * threadIdx.x][3]);
        const float S2 = (red[2 * threadIdx.x + 1][0] + red[2 * threadIdx.x + 1][1]) +
                         (red[2 * threadIdx.x + 1][2] + red[2 * threadIdx.x + 1][3]);
        const float pv = xdt == CSU_BF16 ? (float)((const bf16*)x)[cc] : ((const float*)x)[cc];
        const float n = (float)g.M;
        const float dm = S1 / n;
        const float var = fmaxf(S2 / n - dm * dm, 0.f);
        const float mean = pv + dm;
        save[cc] = mean;
        save[g.C + cc] = 1.f / sqrtf(var + eps);
        if (rmean) {
            const float uv = g.M > 1 ? var * (n / (n - 1.f)) : var;
            rmean[cc] = (1.f - momentum) * rmean[cc] + momentum * mean;
            rvar[cc] = (1.f - momentum) * rvar[cc] + momentum * uv;
        }
    }
}

// pass 2, backward: dbeta = sum(g), dgamma = rstd sum(g (x - mean)); coef[c] = dbeta / M,
// coef[C + c] = dgamma / M (the training-mode dx terms)
__global__ __launch_bounds__(NT) void bn_grad_final(BnGeo g, const float* __restrict__ part, const float* __restrict__ save,
                                                    float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                    float* __restrict__ coef) {
    __shared__ float red[CW * 2][4];
    const int slot = threadIdx.x & (CW * 2 - 1), q = threadIdx.x / (CW * 2);
    const int c = blockIdx.x * CW + slot / 2, k = slot & 1;
    float s = 0.f, s2 = 0.f;
    if (c < g.C) {
        for (int i = q; i < g.nch; i += 4) s += part[((long)i * g.C + c) * 2 + k];
        for (int i = q + 2; i < g.nch; i += 4) s2 += part[((long)i * g.C + c) * 2 + k];
    }
    red[slot][q] = s;
    red[slot][q + 2] = s2;
    __syncthreads();
    if (threadIdx.x < CW && blockIdx.x * CW + threadIdx.x < g.C) {
        const int cc = blockIdx.x * CW + threadIdx.x;
        const float sg = (red[2 * threadIdx.x][0] + red[2 * threadIdx.x][1]) + (red[2 * threadIdx.x][2] + red[2 * threadIdx.x][3]);
        const float sgx = (red[2 * threadIdx.x + 1][0] + red[2 * threadIdx.x + 1][1]) +
                          (red[2 * threadIdx.x + 1][2] + red[2 * threadIdx.x + 1][3]);
        const float dg = sgx * save[g.C + cc];
        if (dgamma) dgamma[cc] = dg;
        if (dbeta) dbeta[cc] = sg;
        coef[cc] = sg / (float)g.M;
        coef[g.C + cc] = dg / (float)g.M;
    }
}

// pass 3, forward: y = [relu]((x - mean) rstd gamma + beta); 8 channels per thread, grid-stride.
// The grid stride is a multiple of C/8 (grid_apply), so a thread's 8 channels never change: their
// per-channel terms are loaded once, and the loop is a pure 16-B stream (per-element loads of the
// small per-channel arrays made the backward VMEM-issue-bound at ~0.8 TB/s).
template <typename T>
__global__ __launch_bounds__(NT) void bn_apply(long n8, int C, const T* __restrict__ x, const float* __restrict__ save,
                                               const float* __restrict__ gamma, const float* __restrict__ beta,
                                               int relu, T* __restrict__ y) {
    const int c8 = C / 8;
    const long i0 = (long)blockIdx.x * NT + threadIdx.x;
    const int c0 = (int)(i0 % c8) * 8;
    float mu[8], a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        mu[j] = save[c0 + j];
        a[j] = save[C + c0 + j] * gamma[c0 + j];
        b[j] = beta[c0 + j];
    }
    for (long i = i0; i < n8; i += (long)gridDim.x * NT) {
        float v[8];
        load8(x + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float o = fmaf(v[j] - mu[j], a[j], b[j]);
            v[j] = relu ? fmaxf(o, 0.f) : o;
        }
        store8(y + i * 8, v);
    }
}

// pass 3, backward: dx = gamma rstd (g - coef0 - (x - mean) rstd coef1)   (coef == nullptr: eval);
// per-channel terms hoisted as in bn_apply
template <typename T, typename G>
__global__ __launch_bounds__(NT) void bn_grad_apply(long n8, int C, const T* __restrict__ x, const G* __restrict__ dy,
                                                    const float* __restrict__ save, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, const float* __restrict__ coef,
                                                    int relu, T* __restrict__ dx) {
    const int c8 = C / 8;
    const long i0 = (long)blockIdx.x * NT + threadIdx.x;
    const int c0 = (int)(i0 % c8) * 8;
    float mu[8], rs[8], a[8], b[8], k0[8], k1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        rs[j] = save[C + c];
        mu[j] = save[c];
        a[j] = rs[j] * gamma[c];
        b[j] = beta[c];
        k0[j] = coef ? coef[c] : 0.f;
        k1[j] = coef ? coef[C + c] : 0.f;
    }
    for (long i = i0; i < n8; i += (long)gridDim.x * NT) {
        float xv[8], gv[8], o[8];
        load8(x + i * 8, xv);
        load8(dy + i * 8, gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float d = xv[j] - mu[j];
            const float gg = (!relu || fmaf(d, a[j], b[j]) > 0.f) ? gv[j] : 0.f;
            o[j] = coef ? a[j] * (gg - k0[j] - d * rs[j] * k1[j]) : a[j] * gg;
        }
        store8(dx + i * 8, o);
    }
}

// eval-mode statistics: save = (running_mean, 1 / sqrt(running_var + eps))
__global__ void bn_eval_save(int C, const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
                             float* __restrict__ save) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C) {
        save[c] = rmean[c];
        save[C + c] = 1.f / sqrtf(rvar[c] + eps);
    }
}

// ---- MaxPool2d(2) -----------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(NT) void maxpool2_fwd(int B, int H, int W, int C, const T* __restrict__ x, T* __restrict__ y) {
    const int Ho = H / 2, Wo = W / 2, c8 = C / 8;
    const long n = (long)B * Ho * Wo * c8;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
        const int c0 = (int)(i % c8) * 8;
        const long p = i / c8;
        const int ox = (int)(p % Wo), oy = (int)((p / Wo) % Ho);
        const long b = p / ((long)Wo * Ho);
        const T* src = x + (((b * H + 2 * oy) * W) + 2 * ox) * C + c0;
        float v[4][8], m[8];
        load8(src, v[0]);
        load8(src + C, v[1]);
        load8(src + (long)W * C, v[2]);
        load8(src + (long)W * C + C, v[3]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            m[j] = v[0][j];
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (v[k][j] > m[j] || v[k][j] != v[k][j]) m[j] = v[k][j];
        }
        store8(y + p * C + c0, m);
    }
}

template <typename T, typename G>
__global__ __launch_bounds__(NT) void maxpool2_bwd(int B, int H, int W, int C, const T* __restrict__ x,
                                                   const G* __restrict__ dy, T* __restrict__ dx) {
    const int Ho = H / 2, Wo = W / 2, c8 = C / 8;
    const long n = (long)B * Ho * Wo * c8;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
        const int c0 = (int)(i % c8) * 8;
        const long p = i / c8;
        const int ox = (int)(p % Wo), oy = (int)((p / Wo) % Ho);
        const long b = p / ((long)Wo * Ho);
        const long base = (((b * H + 2 * oy) * W) + 2 * ox) * C + c0;
        const long off[4] = {0, C, (long)W * C, (long)W * C + C};
        float v[4][8], g[8], o[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k) load8(x + base + off[k], v[k]);
        load8(dy + p * C + c0, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float m = v[0][j];
            int arg = 0;
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (v[k][j] > m || v[k][j] != v[k][j]) { m = v[k][j]; arg = k; }
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k][j] = k == arg ? g[j] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) store8(dx + base + off[k], o[k]);
    }
}

unsigned grid_of(long n) {
    const long g = (n + NT - 1) / NT;
    return (unsigned)(g < 8192 ? (g < 1 ? 1 : g) : 8192);
}

// apply grid: the stride grid * NT must be a multiple of C/8 (a thread keeps its channels)
unsigned grid_apply(long n8, int C) {
    const int c8 = C / 8;
    unsigned g = grid_of(n8);
    if (NT % c8 == 0) return g;
    const long per = c8 / std::gcd(c8, NT);          // grid must be a multiple of per
    return (unsigned)(((g + per - 1) / per) * per);
}

size_t bn_ws(long M, int C) {
    const BnGeo g = bn_geo(M, C);
    return ((size_t)g.nch * C * 2 + 2 * (size_t)C) * sizeof(float);
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" size_t csu_bn_workspace(long M, int C) { return bn_ws(M, C); }

extern "C" int csu_bn_relu_fwd(long M, int C, int dtype, const void* x, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, float momentum, float eps, int training,
                               int relu, float* save, void* y, void* workspace, size_t ws_bytes, void* stream) {
    if (M < 1 || C < 8 || C % 8 || !x || !gamma || !beta || !save || !y) return fail(CSU_E_ARG, "bn_relu_fwd: bad args");
    if (dtype != CSU_BF16 && dtype != CSU_F32) return fail(CSU_E_ARG, "bn_relu_fwd: dtype must be bf16 or f32");
    hipStream_t st = as_stream(stream);
    const BnGeo g = bn_geo(M, C);
    if (training) {
        if (!workspace || ws_bytes < bn_ws(M, C)) return fail(CSU_E_ARG, "bn_relu_fwd: workspace too small");
        if ((running_mean == nullptr) != (running_var == nullptr)) return fail(CSU_E_ARG, "bn_relu_fwd: running stats");
        float* part = static_cast<float*>(workspace);
        if (dtype == CSU_BF16) bn_stats_partial<bf16><<<g.ncb * g.nch, NT, 0, st>>>(g, (const bf16*)x, part);
        else bn_stats_partial<float><<<g.ncb * g.nch, NT, 0, st>>>(g, (const float*)x, part);
        bn_stats_final<<<g.ncb, NT, 0, st>>>(g, x, dtype, part, eps, momentum, running_mean, running_var, save);
    } else {
        if (!running_mean || !running_var) return fail(CSU_E_ARG, "bn_relu_fwd: eval needs running stats");
        bn_eval_save<<<(C + 255) / 256, 256, 0, st>>>(C, running_mean, running_var, eps, save);
    }
    const long n8 = M * C / 8;
    if (dtype == CSU_BF16) bn_apply<bf16><<<grid_apply(n8, C), NT, 0, st>>>(n8, C, (const bf16*)x, save, gamma, beta, relu, (bf16*)y);
    else bn_apply<float><<<grid_apply(n8, C), NT, 0, st>>>(n8, C, (const float*)x, save, gamma, beta, relu, (float*)y);
    return check_launch("bn_relu_fwd");
}

extern "C" int csu_bn_relu_bwd(long M, int C, int dtype, const void* x, const float* gamma, const float* beta,
                               const float* save, int training, int relu, int gdtype, const void* dy, void* dx,
                               float* dgamma, float* dbeta, void* workspace, size_t ws_bytes, void* stream) {
    if (M < 1 || C < 8 || C % 8 || !x || !gamma || !beta || !save || !dy || !dx) return fail(CSU_E_ARG, "bn_relu_bwd: bad args");
    if ((dtype != CSU_BF16 && dtype != CSU_F32) || (gdtype != CSU_BF16 && gdtype != CSU_F32))
        return fail(CSU_E_ARG, "bn_relu_bwd: dtypes must be bf16 or f32");
    if (!workspace || ws_bytes < bn_ws(M, C)) return fail(CSU_E_ARG, "bn_relu_bwd: workspace too small");
    hipStream_t st = as_stream(stream);
    const BnGeo g = bn_geo(M, C);
    float* part = static_cast<float*>(workspace);
    float* coef = part + (size_t)g.nch * C * 2;
    const unsigned nb = g.ncb * g.nch;
#define BN_PART(T, G) bn_grad_partial<T, G><<<nb, NT, 0, st>>>(g, (const T*)x, (const G*)dy, save, gamma, beta, relu, part)
    if (dtype == CSU_BF16) { if (gdtype == CSU_BF16) BN_PART(bf16, bf16); else BN_PART(bf16, float); }
    else { if (gdtype == CSU_BF16) BN_PART(float, bf16); else BN_PART(float, float); }
#undef BN_PART
    bn_grad_final<<<g.ncb, NT, 0, st>>>(g, part, save, dgamma, dbeta, coef);
    const long n8 = M * C / 8;
    const float* cf = training ? coef : nullptr;
#define BN_APPLY(T, G) bn_grad_apply<T, G><<<grid_apply(n8, C), NT, 0, st>>>(n8, C, (const T*)x, (const G*)dy, save, gamma, beta, cf, relu, (T*)dx)
    if (dtype == CSU_BF16) { if (gdtype == CSU_BF16) BN_APPLY(bf16, bf16); else BN_APPLY(bf16, float); }
    else { if (gdtype == CSU_BF16) BN_APPLY(float, bf16); else BN_APPLY(float, float); }
#undef BN_APPLY
    return check_launch("bn_relu_bwd");
}

extern "C" int csu_maxpool2_fwd(int B, int H, int W, int C, int dtype, const void* x, void* y, void* stream) {
    if (B < 1 || H < 2 || W < 2 || C < 8 || C % 8 || !x || !y) return fail(CSU_E_ARG, "maxpool2_fwd: bad args");
    const long n = (long)B * (H / 2) * (W / 2) * (C / 8);
    hipStream_t st = as_stream(stream);
    if (dtype == CSU_BF16) maxpool2_fwd<bf16><<<grid_of(n), NT, 0, st>>>(B, H, W, C, (const bf16*)x, (bf16*)y);
    else if (dtype == CSU_F32) maxpool2_fwd<float><<<grid_of(n), NT, 0, st>>>(B, H, W, C, (const float*)x, (float*)y);
    else return fail(CSU_E_ARG, "maxpool2_fwd: dtype must be bf16 or f32");
    return check_launch("maxpool2_fwd");
}

extern "C" int csu_maxpool2_bwd(int B, int H, int W, int C, int dtype, const void* x, int gdtype, const void* dy,
                                void* dx, void* stream) {
    if (B < 1 || H < 2 || W < 2 || C < 8 || C % 8 || !x || !dy || !dx) return fail(CSU_E_ARG, "maxpool2_bwd: bad args");
    if ((dtype != CSU_BF16 && dtype != CSU_F32) || (gdtype != CSU_BF16 && gdtype != CSU_F32))
        return fail(CSU_E_ARG, "maxpool2_bwd: dtypes must be bf16 or f32");
    const long n = (long)B * (H / 2) * (W / 2) * (C / 8);
    hipStream_t st = as_stream(stream);
#define MP(T, G) maxpool2_bwd<T, G><<<grid_of(n), NT, 0, st>>>(B, H, W, C, (const T*)x, (const G*)dy, (T*)dx)
    if (dtype == CSU_BF16) { if (gdtype == CSU_BF16) MP(bf16, bf16); else MP(bf16, float); }
    else { if (gdtype == CSU_BF16) MP(float, bf16); else MP(float, float); }
#undef MP
    return check_launch("maxpool2_bwd");
}
