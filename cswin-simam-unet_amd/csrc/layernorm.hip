// LayerNorm over the channel dim of token rows (B*L, C) for gfx950.
//
// Replaces nn.LayerNorm at norm1/norm2 (cswin:315, 347, applied cswin:357/368), Merge_Block.norm
// (cswin:377/386), the patch-embed LN (cswin:507) and norm/norm_up (cswin:554/602).
// One wave64 per row, the row held in registers (C/64 elements per lane, vectorised loads),
// fp32 statistics; the output may be bf16 so it feeds the following GEMM directly (the same
// rounding autocast would apply at the GEMM input).  Backward writes dx and deterministic
// per-block partial sums of dgamma/dbeta, reduced in a second pass in a fixed order.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int WAVES = NT / 64;

template <typename T, int V> __device__ __forceinline__ void ldv(const T* p, float* v) {
    if constexpr (V == 8) load8(p, v);
    else if constexpr (V == 4) load4(p, v);
    else {
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = to_f(p[j]);
    }
}
template <typename T, int V> __device__ __forceinline__ void stv(T* p, const float* v) {
    if constexpr (V == 8) store8(p, v);
    else if constexpr (V == 4) store4(p, v);
    else {
#pragma unroll
        for (int j = 0; j < V; ++j) p[j] = from_f<T>(v[j]);
    }
}

template <typename TX, typename TY, int V>
__global__ __launch_bounds__(NT) void ln_fwd(int rows, int C, float eps, const TX* __restrict__ x,
                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                             TY* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int c0 = lane * V;
    float v[V];
    ldv<TX, V>(x + (size_t)row * C + c0, v);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) s += v[j];
    const float mu = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        v[j] -= mu;
        q += v[j] * v[j];
    }
    const float rs = rsqrtf(wave_sum(q) / C + eps);
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = v[j] * rs * gamma[c0 + j] + beta[c0 + j];
    stv<TY, V>(y + (size_t)row * C + c0, o);
    if (lane == 0) {
        mean[row] = mu;
        rstd[row] = rs;
    }
}

// dx = rstd * (g*gamma - mean(g*gamma) - xhat * mean(g*gamma*xhat)); partial dgamma/dbeta per block
template <typename TX, typename TG, int V>
__global__ __launch_bounds__(NT) void ln_bwd(int rows, int C, int rows_per_block, const TX* __restrict__ x,
                                             const float* __restrict__ gamma, const float* __restrict__ mean,
                                             const float* __restrict__ rstd, const TG* __restrict__ dy,
                                             TX* __restrict__ dx, float* __restrict__ part) {
    __shared__ float red[WAVES][2][512];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = lane * V;
    float gw[V], dg[V], db[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
        gw[j] = gamma[c0 + j];
        dg[j] = 0.f;
        db[j] = 0.f;
    }
    const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
    for (int row = r0 + wave; row < r1; row += WAVES) {
        float xv[V], g[V];
        ldv<TX, V>(x + (size_t)row * C + c0, xv);
        ldv<TG, V>(dy + (size_t)row * C + c0, g);
        const float mu = mean[row], rs = rstd[row];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            xv[j] = (xv[j] - mu) * rs;   // xhat
            const float gg = g[j] * gw[j];
            s1 += gg;
            s2 += gg * xv[j];
            dg[j] += g[j] * xv[j];
            db[j] += g[j];
        }
        s1 = wave_sum(s1) / C;
        s2 = wave_sum(s2) / C;
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = rs * (g[j] * gw[j] - s1 - xv[j] * s2);
        stv<TX, V>(dx + (size_t)row * C + c0, o);
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
        red[wave][0][c0 + j] = dg[j];
        red[wave][1][c0 + j] = db[j];
    }
    __syncthreads();
    // partials laid out [nblocks][2C] (dgamma | dbeta) for the column-sum pass
    for (int i = threadIdx.x; i < 2 * C; i += NT) {
        const int k = i / C, c = i % C;
        float s = 0.f;
#pragma unroll
        for (int wv = 0; wv < WAVES; ++wv) s += red[wv][k][c];
        part[(size_t)blockIdx.x * 2 * C + i] = s;
    }
}

int ln_blocks(int rows, int* rpb) {
    int r = (rows + 511) / 512;
    r = ((r + WAVES - 1) / WAVES) * WAVES;
    if (r < WAVES) r = WAVES;
    *rpb = r;
    return (rows + r - 1) / r;
}

int check_c(int C) {
    if (C % 64 || C < 64 || C > 512) return fail(CSU_E_UNSUPPORTED, "layernorm: C must be 64..512, multiple of 64");
    return 0;
}

template <typename TX, typename TY>
int launch_fwd(int rows, int C, float eps, const void* x, const float* g, const float* b, void* y, float* m,
               float* r, hipStream_t st) {
    const dim3 grid((rows + WAVES - 1) / WAVES);
    switch (C / 64) {
        case 1: ln_fwd<TX, TY, 1><<<grid, NT, 0, st>>>(rows, C, eps, (const TX*)x, g, b, (TY*)y, m, r); break;
        case 2: ln_fwd<TX, TY, 2><<<grid, NT, 0, st>>>(rows, C, eps, (const TX*)x, g, b, (TY*)y, m, r); break;
        case 4: ln_fwd<TX, TY, 4><<<grid, NT, 0, st>>>(rows, C, eps, (const TX*)x, g, b, (TY*)y, m, r); break;
        case 8: ln_fwd<TX, TY, 8><<<grid, NT, 0, st>>>(rows, C, eps, (const TX*)x, g, b, (TY*)y, m, r); break;
        default: return fail(CSU_E_UNSUPPORTED, "layernorm: C/64 must be 1, 2, 4 or 8");
    }
    return check_launch("layernorm_fwd");
}

template <typename TX, typename TG>
int launch_bwd(int rows, int C, const void* x, const float* g, const float* m, const float* r, const void* dy,
               void* dx, float* dgamma, float* dbeta, float* part, hipStream_t st) {
    int rpb;
    const int nb = ln_blocks(rows, &rpb);
    switch (C / 64) {
        case 1: ln_bwd<TX, TG, 1><<<nb, NT, 0, st>>>(rows, C, rpb, (const TX*)x, g, m, r, (const TG*)dy, (TX*)dx, part); break;
        case 2: ln_bwd<TX, TG, 2><<<nb, NT, 0, st>>>(rows, C, rpb, (const TX*)x, g, m, r, (const TG*)dy, (TX*)dx, part); break;
        case 4: ln_bwd<TX, TG, 4><<<nb, NT, 0, st>>>(rows, C, rpb, (const TX*)x, g, m, r, (const TG*)dy, (TX*)dx, part); break;
        case 8: ln_bwd<TX, TG, 8><<<nb, NT, 0, st>>>(rows, C, rpb, (const TX*)x, g, m, r, (const TG*)dy, (TX*)dx, part); break;
        default: return fail(CSU_E_UNSUPPORTED, "layernorm: C/64 must be 1, 2, 4 or 8");
    }
    if (int e = check_launch("layernorm_bwd")) return e;
    float* cws = part + (size_t)2 * nb * C;
    if (dbeta == dgamma + C) return colsum_launch(nb, 2 * C, CSU_F32, part, dgamma, cws, st);
    float* tmp = cws + colsum_workspace(nb, 2 * C, CSU_F32) / sizeof(float);
    if (int e = colsum_launch(nb, 2 * C, CSU_F32, part, tmp, cws, st)) return e;
    if (hipMemcpyAsync(dgamma, tmp, C * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dbeta, tmp + C, C * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return check_launch("layernorm_bwd copy");
    return 0;
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_layernorm_fwd(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                                 const float* beta, int ydtype, void* y, float* mean, float* rstd, void* stream) {
    if (int e = check_c(C)) return e;
    if (rows < 1 || !x || !gamma || !beta || !y || !mean || !rstd) return fail(CSU_E_ARG, "layernorm_fwd: bad args");
    hipStream_t st = as_stream(stream);
    if (xdtype == CSU_F32 && ydtype == CSU_F32) return launch_fwd<float, float>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    if (xdtype == CSU_F32 && ydtype == CSU_BF16) return launch_fwd<float, bf16>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    if (xdtype == CSU_BF16 && ydtype == CSU_F32) return launch_fwd<bf16, float>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    if (xdtype == CSU_BF16 && ydtype == CSU_BF16) return launch_fwd<bf16, bf16>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    return fail(CSU_E_ARG, "layernorm_fwd: bad dtype");
}

extern "C" size_t csu_layernorm_bwd_workspace(int rows, int C) {
    int rpb;
    const int nb = ln_blocks(rows, &rpb);
    return (size_t)nb * 2 * C * sizeof(float) + colsum_workspace(nb, 2 * C, CSU_F32) + 2 * C * sizeof(float);
}

extern "C" int csu_layernorm_bwd(int rows, int C, int xdtype, const void* x, const float* gamma, const float* mean,
                                 const float* rstd, int dydtype, const void* dy, void* dx, float* dgamma,
                                 float* dbeta, void* workspace, size_t ws_bytes, void* stream) {
    if (int e = check_c(C)) return e;
    if (rows < 1 || !x || !gamma || !mean || !rstd || !dy || !dx || !dgamma || !dbeta)
        return fail(CSU_E_ARG, "layernorm_bwd: bad args");
    if (!workspace || ws_bytes < csu_layernorm_bwd_workspace(rows, C))
        return fail(CSU_E_WORKSPACE, "layernorm_bwd: workspace too small");
    hipStream_t st = as_stream(stream);
    float* part = (float*)workspace;
    if (xdtype == CSU_F32 && dydtype == CSU_F32) return launch_bwd<float, float>(rows, C, x, gamma, mean, rstd, dy, dx, dgamma, dbeta, part, st);
    if (xdtype == CSU_F32 && dydtype == CSU_BF16) return launch_bwd<float, bf16>(rows, C, x, gamma, mean, rstd, dy, dx, dgamma, dbeta, part, st);
    if (xdtype == CSU_BF16 && dydtype == CSU_F32) return launch_bwd<bf16, float>(rows, C, x, gamma, mean, rstd, dy, dx, dgamma, dbeta, part, st);
    if (xdtype == CSU_BF16 && dydtype == CSU_BF16) return launch_bwd<bf16, bf16>(rows, C, x, gamma, mean, rstd, dy, dx, dgamma, dbeta, part, st);
    return fail(CSU_E_ARG, "layernorm_bwd: bad dtype");
}
