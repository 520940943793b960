// SimAM parameter-free attention gate on token rows (B, L, C) for gfx950.
//
// NOT in the reference: the public SimAM formula, per (b, c) over the
// n = L positions:  mu = mean(x),  d = x - mu,  v = sum(d^2) / (n - 1),  s = 4 (v + lambda),
// e = d^2 / s + 1/2,  y = x * sigmoid(e).
// Statistics: per (image, 64-channel tile, token chunk) Welford partials combined in a fixed
// order (Chan's formula) -> deterministic and cancellation-free.  Backward, with
// a = g * x * sigma'(e), A1 = sum(a d), A2 = sum(a d^2):
//   dx = g sigma(e) + (2/s)(a d - A1/n) - 8 d A2 / ((n-1) s^2).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int CT = 64;         // channels per block (one per lane of a wave)
constexpr int TL = NT / CT;    // token lanes per block

int simam_chunks(int L, int* chunk) {
    int nch = (L + 1023) / 1024;
    if (nch > 64) nch = 64;
    if (nch < 1) nch = 1;
    *chunk = (L + nch - 1) / nch;
    return nch;
}

// partial (count, mean, M2) per (b, c, chunk)
template <typename T>
__global__ __launch_bounds__(NT) void simam_stats_partial(int L, int C, int chunk, int nch, const T* __restrict__ x,
                                                          float* __restrict__ part) {
    __shared__ float sm[3][TL][CT];
    const int b = blockIdx.z, ch = blockIdx.y;
    const int cl = threadIdx.x % CT, tl = threadIdx.x / CT;
    const int c = blockIdx.x * CT + cl;
    const int t0 = ch * chunk, t1 = min(L, t0 + chunk);
    float n = 0.f, mu = 0.f, m2 = 0.f;
    if (c < C) {
        for (int t = t0 + tl; t < t1; t += TL) {
            const float v = to_f(x[((size_t)b * L + t) * C + c]);
            n += 1.f;
            const float dlt = v - mu;
            mu += dlt / n;
            m2 += dlt * (v - mu);
        }
    }
    sm[0][tl][cl] = n; sm[1][tl][cl] = mu; sm[2][tl][cl] = m2;
    __syncthreads();
    if (tl == 0 && c < C) {
        float N = 0.f, M = 0.f, Q = 0.f;
        for (int j = 0; j < TL; ++j) {
            const float nb = sm[0][j][cl];
            if (nb == 0.f) continue;
            const float dlt = sm[1][j][cl] - M, tot = N + nb;
            M += dlt * nb / tot;
            Q += sm[2][j][cl] + dlt * dlt * N * nb / tot;
            N = tot;
        }
        float* p = part + (((size_t)b * C + c) * nch + ch) * 3;
        p[0] = N; p[1] = M; p[2] = Q;
    }
}

// combine chunk partials -> stats[b][c] = (mu, s)
__global__ void simam_stats_final(int B, int L, int C, int nch, float lam, const float* __restrict__ part,
                                  float* __restrict__ stats) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * C) return;
    float N = 0.f, M = 0.f, Q = 0.f;
    for (int j = 0; j < nch; ++j) {
        const float* p = part + ((size_t)i * nch + j) * 3;
        if (p[0] == 0.f) continue;
        const float dlt = p[1] - M, tot = N + p[0];
        M += dlt * p[0] / tot;
        Q += p[2] + dlt * dlt * N * p[0] / tot;
        N = tot;
    }
    stats[2 * i] = M;
    stats[2 * i + 1] = 4.f * (Q / (float)(L - 1) + lam);
}

__device__ __forceinline__ float sigm(float e) { return 1.f / (1.f + __expf(-e)); }

template <typename T>
__global__ __launch_bounds__(NT) void simam_apply(int L, int C, const T* __restrict__ x,
                                                  const float* __restrict__ stats, T* __restrict__ y) {
    const int b = blockIdx.z;
    const int c = blockIdx.x * CT + threadIdx.x % CT;
    if (c >= C) return;
    const float mu = stats[2 * ((size_t)b * C + c)], rs = 1.f / stats[2 * ((size_t)b * C + c) + 1];
    for (int t = blockIdx.y * TL + threadIdx.x / CT; t < L; t += gridDim.y * TL) {
        const size_t i = ((size_t)b * L + t) * C + c;
        const float v = to_f(x[i]), d = v - mu;
        y[i] = from_f<T>(v * sigm(d * d * rs + 0.5f));
    }
}

// partial (A1, A2) per (b, c, chunk)
template <typename T>
__global__ __launch_bounds__(NT) void simam_bwd_partial(int L, int C, int chunk, int nch, const T* __restrict__ x,
                                                        const T* __restrict__ dy, const float* __restrict__ stats,
                                                        float* __restrict__ part) {
    __shared__ float sm[2][TL][CT];
    const int b = blockIdx.z, ch = blockIdx.y;
    const int cl = threadIdx.x % CT, tl = threadIdx.x / CT;
    const int c = blockIdx.x * CT + cl;
    const int t0 = ch * chunk, t1 = min(L, t0 + chunk);
    float a1 = 0.f, a2 = 0.f;
    if (c < C) {
        const float mu = stats[2 * ((size_t)b * C + c)], rs = 1.f / stats[2 * ((size_t)b * C + c) + 1];
        for (int t = t0 + tl; t < t1; t += TL) {
            const size_t i = ((size_t)b * L + t) * C + c;
            const float v = to_f(x[i]), g = to_f(dy[i]), d = v - mu;
            const float sg = sigm(d * d * rs + 0.5f);
            const float a = g * v * sg * (1.f - sg);
            a1 += a * d;
            a2 += a * d * d;
        }
    }
    sm[0][tl][cl] = a1; sm[1][tl][cl] = a2;
    __syncthreads();
    if (tl == 0 && c < C) {
        float s1 = 0.f, s2 = 0.f;
        for (int j = 0; j < TL; ++j) { s1 += sm[0][j][cl]; s2 += sm[1][j][cl]; }
        float* p = part + (((size_t)b * C + c) * nch + ch) * 2;
        p[0] = s1; p[1] = s2;
    }
}

template <typename T>
__global__ __launch_bounds__(NT) void simam_bwd_apply(int L, int C, int nch, const T* __restrict__ x,
                                                      const T* __restrict__ dy, const float* __restrict__ stats,
                                                      const float* __restrict__ part, T* __restrict__ dx) {
    const int b = blockIdx.z;
    const int c = blockIdx.x * CT + threadIdx.x % CT;
    if (c >= C) return;
    const size_t bc = (size_t)b * C + c;
    float A1 = 0.f, A2 = 0.f;
    for (int j = 0; j < nch; ++j) {
        A1 += part[(bc * nch + j) * 2];
        A2 += part[(bc * nch + j) * 2 + 1];
    }
    const float mu = stats[2 * bc], s = stats[2 * bc + 1], rs = 1.f / s;
    const float n = (float)L;
    const float k1 = 2.f * rs, k1n = 2.f * rs * A1 / n, k2 = 8.f * A2 * rs * rs / (n - 1.f);
    for (int t = blockIdx.y * TL + threadIdx.x / CT; t < L; t += gridDim.y * TL) {
        const size_t i = ((size_t)b * L + t) * C + c;
        const float v = to_f(x[i]), g = to_f(dy[i]), d = v - mu;
        const float sg = sigm(d * d * rs + 0.5f);
        const float a = g * v * sg * (1.f - sg);
        dx[i] = from_f<T>(g * sg + k1 * a * d - k1n - k2 * d);
    }
}

dim3 apply_grid(int B, int L, int C) {
    int ty = (L + TL * 16 - 1) / (TL * 16);   // ~16 tokens per thread
    if (ty < 1) ty = 1;
    return dim3((C + CT - 1) / CT, ty, B);
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" size_t csu_simam_workspace(int B, int L, int C) {
    int chunk;
    const int nch = simam_chunks(L, &chunk);
    return (size_t)B * C * nch * 3 * sizeof(float);
}

extern "C" int csu_simam_fwd(int B, int L, int C, float lam, int dtype, const void* x, void* y, float* stats,
                             void* workspace, size_t ws_bytes, void* stream) {
    if (B < 1 || L < 2 || C < 1 || !x || !y || !stats) return fail(CSU_E_ARG, "simam_fwd: bad args (need L >= 2)");
    if (!workspace || ws_bytes < csu_simam_workspace(B, L, C)) return fail(CSU_E_WORKSPACE, "simam_fwd: workspace");
    hipStream_t st = as_stream(stream);
    int chunk;
    const int nch = simam_chunks(L, &chunk);
    float* part = (float*)workspace;
    const dim3 pg((C + CT - 1) / CT, nch, B);
    if (dtype == CSU_BF16) {
        simam_stats_partial<bf16><<<pg, NT, 0, st>>>(L, C, chunk, nch, (const bf16*)x, part);
        simam_stats_final<<<(B * C + 255) / 256, 256, 0, st>>>(B, L, C, nch, lam, part, stats);
        simam_apply<bf16><<<apply_grid(B, L, C), NT, 0, st>>>(L, C, (const bf16*)x, stats, (bf16*)y);
    } else if (dtype == CSU_F32) {
        simam_stats_partial<float><<<pg, NT, 0, st>>>(L, C, chunk, nch, (const float*)x, part);
        simam_stats_final<<<(B * C + 255) / 256, 256, 0, st>>>(B, L, C, nch, lam, part, stats);
        simam_apply<float><<<apply_grid(B, L, C), NT, 0, st>>>(L, C, (const float*)x, stats, (float*)y);
    } else {
        return fail(CSU_E_ARG, "simam_fwd: bad dtype");
    }
    return check_launch("simam_fwd");
}

extern "C" int csu_simam_bwd(int B, int L, int C, int dtype, const void* x, const float* stats, const void* dy,
                             void* dx, void* workspace, size_t ws_bytes, void* stream) {
    if (B < 1 || L < 2 || C < 1 || !x || !stats || !dy || !dx) return fail(CSU_E_ARG, "simam_bwd: bad args");
    if (!workspace || ws_bytes < csu_simam_workspace(B, L, C)) return fail(CSU_E_WORKSPACE, "simam_bwd: workspace");
    hipStream_t st = as_stream(stream);
    int chunk;
    const int nch = simam_chunks(L, &chunk);
    float* part = (float*)workspace;
    const dim3 pg((C + CT - 1) / CT, nch, B);
    if (dtype == CSU_BF16) {
        simam_bwd_partial<bf16><<<pg, NT, 0, st>>>(L, C, chunk, nch, (const bf16*)x, (const bf16*)dy, stats, part);
        simam_bwd_apply<bf16><<<apply_grid(B, L, C), NT, 0, st>>>(L, C, nch, (const bf16*)x, (const bf16*)dy, stats, part, (bf16*)dx);
    } else if (dtype == CSU_F32) {
        simam_bwd_partial<float><<<pg, NT, 0, st>>>(L, C, chunk, nch, (const float*)x, (const float*)dy, stats, part);
        simam_bwd_apply<float><<<apply_grid(B, L, C), NT, 0, st>>>(L, C, nch, (const float*)x, (const float*)dy, stats, part, (float*)dx);
    } else {
        return fail(CSU_E_ARG, "simam_bwd: bad dtype");
    }
    return check_launch("simam_bwd");
}
