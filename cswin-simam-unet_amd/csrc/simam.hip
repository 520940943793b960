// SimAM parameter-free attention gate on token rows (B, L, C) for gfx950.
//
// NOT in the reference: the public SimAM formula, per (b, c) over the
// n = L positions:  mu = mean(x),  d = x - mu,  v = sum(d^2) / (n - 1),  s = 4 (v + lambda),
// e = d^2 / s + 1/2,  y = x * sigmoid(e).
// Backward, with a = g * x * sigma'(e), A1 = sum(a d), A2 = sum(a d^2):
//   dx = g sigma(e) + (2/s)(a d - A1/n) - 8 d A2 / ((n-1) s^2).
//
// Layout: one block = 64 channels x one token chunk of one image; lane quad q of a 16-lane row
// group owns channels 4q..4q+3 (16-B fp32 / 8-B bf16 vector loads, a 64-channel row segment per
// 16 lanes), the 16 row groups of the block stride over the chunk's tokens.  Statistics are
// pivot-shifted sums (pivot = the (b, c) value at token 0: cancellation-free to O(1) std of pivot
// offset) reduced in a fixed order -- per block through LDS, then over the chunks in chunk order
// by every consumer -- so results are deterministic.  Two launches per direction: partial sums,
// then the elementwise pass (which folds the chunk combine in and writes y in the consumer's
// dtype, e.g. bf16 for the concat_linear GEMM that reads the gated skip).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int CW = 64;           // channels per block
constexpr int QPR = CW / 4;      // channel quads per row group (16 lanes)
constexpr int TPP = NT / QPR;    // tokens per pass (16 row groups)

struct Geo {
    int L, C, chunk, nch, ns;   // ns: partial stride per (b, c) = nch rounded up to even (16-B rows)
};

Geo geo(int B, int L, int C) {
    Geo g{L, C, 0, 0, 0};
    const long blocks = (long)B * ((C + CW - 1) / CW);
    long nch = (1024 + blocks - 1) / blocks;               // ~1024 blocks per launch
    const long maxc = (L + 4 * TPP - 1) / (4 * TPP);       // >= 4 passes per block
    if (nch > maxc) nch = maxc;
    if (nch < 1) nch = 1;
    g.chunk = (int)((L + nch - 1) / nch);
    g.nch = (int)((L + g.chunk - 1) / g.chunk);
    g.ns = (g.nch + 1) & ~1;
    return g;
}

__device__ __forceinline__ float sigm(float e) { return __builtin_amdgcn_rcpf(1.f + __expf(-e)); }

// fixed-order sum over the 16 row groups of a block -> row group 0's lanes: the 4 row groups of a
// wave (lane bits 4, 5) by a wavefront xor-butterfly (every lane ends with the same bits), then
// the 4 waves through LDS in wave order.  sm: [NT / 64][QPR * K]
template <int K>
__device__ __forceinline__ void rowgroup_sum(float (*sm)[QPR * K], const float* v, float* out, int tl, int q) {
    float w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const float a = v[k] + __shfl_xor(v[k], 16, 64);
        w[k] = a + __shfl_xor(a, 32, 64);
    }
    if ((tl & 3) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sm[tl >> 2][q * K + k] = w[k];
    __syncthreads();
    if (tl == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) out[k] = ((sm[0][q * K + k] + sm[1][q * K + k]) + sm[2][q * K + k]) + sm[3][q * K + k];
    }
}

// Sums (over the g.nch chunk partials) of the 8 values (pairs of 4 channels) of channel quad q, computed
// by the whole block ONCE: row group tl sums chunks tl, tl + 16, ... (fixed order), row group 0 adds
// the 16 row groups in order and publishes the totals in LDS (sm2[q][8]); every thread then reads its
// quad's 8 totals.  (Each of the 16 row groups re-reading all partials of its quad cost 16x the
// partial bytes per block -- most of the apply passes' time at ~1024 blocks per launch.)
__device__ __forceinline__ void coop_chunk_sums(const Geo& g, const float* part, size_t bc0, int tl, int q, bool ok,
                                                float (*sm)[QPR * 8], float (*sm2)[8], float* tot) {
    float a[8] = {};
    if (ok)
        for (int j = tl; j < g.nch; j += 16) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float2 v = *reinterpret_cast<const float2*>(part + ((bc0 + k) * g.ns + j) * 2);
                a[2 * k] += v.x;
                a[2 * k + 1] += v.y;
            }
        }
#pragma unroll
    for (int i = 0; i < 8; ++i) sm[tl][q * 8 + i] = a[i];
    __syncthreads();
    if (tl == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float t = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) t += sm[r][q * 8 + i];
            sm2[q][i] = t;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) tot[i] = sm2[q][i];
}

// partial pivot-shifted (sum d, sum d^2) per (b, c, chunk); part[b][c][chunk][2]
template <typename T>
__global__ __launch_bounds__(NT) void simam_stats(Geo g, const T* __restrict__ x, float* __restrict__ part) {
    __shared__ float sm[NT / 64][QPR * 8];
    const int b = blockIdx.z, ch = blockIdx.x;
    const int q = threadIdx.x % QPR, tl = threadIdx.x / QPR;
    const int c0 = blockIdx.y * CW + 4 * q;
    const bool ok = c0 < g.C;
    const int t0 = ch * g.chunk, t1 = min(g.L, t0 + g.chunk);
    const T* xb = x + (size_t)b * g.L * g.C + c0;
    float piv[4] = {}, acc[8] = {};
    if (ok) {
        load4(xb, piv);
        auto body = [&](const float* v) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = v[k] - piv[k];
                acc[2 * k] += d;
                acc[2 * k + 1] += d * d;
            }
        };
        int t = t0 + tl;
        for (; t + 3 * TPP < t1; t += 4 * TPP) {   // 4 tokens' loads in flight
            float v[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) load4(xb + (size_t)(t + u * TPP) * g.C, v[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u) body(v[u]);
        }
        for (; t < t1; t += TPP) {
            float v[4];
            load4(xb + (size_t)t * g.C, v);
            body(v);
        }
    }
    float tot[8];
    rowgroup_sum<8>(sm, acc, tot, tl, q);
    if (tl == 0 && ok) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float* p = part + (((size_t)b * g.C + c0 + k) * g.ns + ch) * 2;
            p[0] = tot[2 * k];
            p[1] = tot[2 * k + 1];
        }
    }
}

// y = x * sigmoid(d^2 / s + 1/2); chunk-0 blocks also write stats[b][c] = (mu, s)
// CAST: also write xc = bf16(x) (the fork's second consumer, the Merge_Block conv) from the same pass
template <typename T, typename TO, bool CAST = false>
__global__ __launch_bounds__(NT) void simam_apply(Geo g, float lam, const T* __restrict__ x, const float* __restrict__ part,
                                                  TO* __restrict__ y, float* __restrict__ stats, bf16* __restrict__ xc = nullptr) {
    __shared__ float sm[16][QPR * 8];
    __shared__ float sm2[QPR][8];
    const int b = blockIdx.z, ch = blockIdx.x;
    const int q = threadIdx.x % QPR, tl = threadIdx.x / QPR;
    const int c0 = blockIdx.y * CW + 4 * q;
    const bool ok = c0 < g.C;
    const size_t off = (size_t)b * g.L * g.C + (ok ? c0 : 0);
    float piv[4], mu[4], s[4], rs[4], tot[8];
    coop_chunk_sums(g, part, (size_t)b * g.C + c0, tl, q, ok, sm, sm2, tot);
    if (!ok) return;
    load4(x + off, piv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float n = (float)g.L, md = tot[2 * k] / n;
        mu[k] = piv[k] + md;
        s[k] = 4.f * (fmaxf(tot[2 * k + 1] - tot[2 * k] * md, 0.f) / (n - 1.f) + lam);
        rs[k] = 1.f / s[k];
    }
    if (ch == 0 && tl == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            stats[2 * ((size_t)b * g.C + c0 + k)] = mu[k];
            stats[2 * ((size_t)b * g.C + c0 + k) + 1] = s[k];
        }
    }
    const int t0 = ch * g.chunk, t1 = min(g.L, t0 + g.chunk);
    auto body = [&](int t, const float* v) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float d = v[k] - mu[k];
            o[k] = v[k] * sigm(d * d * rs[k] + 0.5f);
        }
        store4(y + off + (size_t)t * g.C, o);
        if constexpr (CAST) store4(xc + off + (size_t)t * g.C, v);
    };
    int t = t0 + tl;
    for (; t + 3 * TPP < t1; t += 4 * TPP) {
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) load4(x + off + (size_t)(t + u * TPP) * g.C, v[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u) body(t + u * TPP, v[u]);
    }
    for (; t < t1; t += TPP) {
        float v[4];
        load4(x + off + (size_t)t * g.C, v);
        body(t, v);
    }
}

// partial (A1, A2) per (b, c, chunk)
template <typename T, typename TG>
__global__ __launch_bounds__(NT) void simam_bwd_partial(Geo g, const T* __restrict__ x, const TG* __restrict__ dy,
                                                        const float* __restrict__ stats, float* __restrict__ part) {
    __shared__ float sm[NT / 64][QPR * 8];
    const int b = blockIdx.z, ch = blockIdx.x;
    const int q = threadIdx.x % QPR, tl = threadIdx.x / QPR;
    const int c0 = blockIdx.y * CW + 4 * q;
    const bool ok = c0 < g.C;
    const int t0 = ch * g.chunk, t1 = min(g.L, t0 + g.chunk);
    const size_t off = (size_t)b * g.L * g.C + c0;
    float acc[8] = {};
    if (ok) {
        float mu[4], rs[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            mu[k] = stats[2 * ((size_t)b * g.C + c0 + k)];
            rs[k] = 1.f / stats[2 * ((size_t)b * g.C + c0 + k) + 1];
        }
        auto body = [&](const float* v, const float* gv) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = v[k] - mu[k];
                const float sg = sigm(d * d * rs[k] + 0.5f);
                const float a = gv[k] * v[k] * sg * (1.f - sg);
                acc[2 * k] += a * d;
                acc[2 * k + 1] += a * d * d;
            }
        };
        int t = t0 + tl;
        for (; t + 3 * TPP < t1; t += 4 * TPP) {
            float v[4][4], gv[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                load4(x + off + (size_t)(t + u * TPP) * g.C, v[u]);
                load4(dy + off + (size_t)(t + u * TPP) * g.C, gv[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) body(v[u], gv[u]);
        }
        for (; t < t1; t += TPP) {
            float v[4], gv[4];
            load4(x + off + (size_t)t * g.C, v);
            load4(dy + off + (size_t)t * g.C, gv);
            body(v, gv);
        }
    }
    float tot[8];
    rowgroup_sum<8>(sm, acc, tot, tl, q);
    if (tl == 0 && ok) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float* p = part + (((size_t)b * g.C + c0 + k) * g.ns + ch) * 2;
            p[0] = tot[2 * k];
            p[1] = tot[2 * k + 1];
        }
    }
}

// JOIN: dx = g2 + (the SimAM input gradient) with g2 (bf16) the fork's other gradient, and dxb =
// bf16(dx) for the upstream GEMM backward -- grad_join's outputs, in the same pass
template <typename T, typename TG, bool JOIN = false>
__global__ __launch_bounds__(NT) void simam_bwd_apply(Geo g, const T* __restrict__ x, const TG* __restrict__ dy,
                                                      const float* __restrict__ stats, const float* __restrict__ part,
                                                      T* __restrict__ dx, const bf16* __restrict__ g2 = nullptr,
                                                      bf16* __restrict__ dxb = nullptr) {
    __shared__ float sm[16][QPR * 8];
    __shared__ float sm2[QPR][8];
    const int b = blockIdx.z, ch = blockIdx.x;
    const int q = threadIdx.x % QPR, tl = threadIdx.x / QPR;
    const int c0 = blockIdx.y * CW + 4 * q;
    const bool ok = c0 < g.C;
    float tot[8];
    coop_chunk_sums(g, part, (size_t)b * g.C + c0, tl, q, ok, sm, sm2, tot);
    if (!ok) return;
    const size_t off = (size_t)b * g.L * g.C + c0;
    const float n = (float)g.L;
    float mu[4], rs[4], k1[4], k1n[4], k2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t bc = (size_t)b * g.C + c0 + k;
        const float A1 = tot[2 * k], A2 = tot[2 * k + 1];
        mu[k] = stats[2 * bc];
        rs[k] = 1.f / stats[2 * bc + 1];
        k1[k] = 2.f * rs[k];
        k1n[k] = 2.f * rs[k] * A1 / n;
        k2[k] = 8.f * A2 * rs[k] * rs[k] / (n - 1.f);
    }
    const int t0 = ch * g.chunk, t1 = min(g.L, t0 + g.chunk);
    auto body = [&](int t, const float* v, const float* gv) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float d = v[k] - mu[k];
            const float sg = sigm(d * d * rs[k] + 0.5f);
            const float a = gv[k] * v[k] * sg * (1.f - sg);
            o[k] = gv[k] * sg + k1[k] * a * d - k1n[k] - k2[k] * d;
        }
        if constexpr (JOIN) {
            float v2[4];
            load4(g2 + off + (size_t)t * g.C, v2);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] += v2[k];
            store4(dxb + off + (size_t)t * g.C, o);
        }
        store4(dx + off + (size_t)t * g.C, o);
    };
    int t = t0 + tl;
    for (; t + 3 * TPP < t1; t += 4 * TPP) {
        float v[4][4], gv[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            load4(x + off + (size_t)(t + u * TPP) * g.C, v[u]);
            load4(dy + off + (size_t)(t + u * TPP) * g.C, gv[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) body(t + u * TPP, v[u], gv[u]);
    }
    for (; t < t1; t += TPP) {
        float v[4], gv[4];
        load4(x + off + (size_t)t * g.C, v);
        load4(dy + off + (size_t)t * g.C, gv);
        body(t, v, gv);
    }
}

dim3 grid_of(int B, const Geo& g) { return dim3(g.nch, (g.C + CW - 1) / CW, B); }

template <typename T>
int fwd_typed(int B, const Geo& g, float lam, const T* x, int ydtype, void* y, float* stats, float* part, hipStream_t st) {
    simam_stats<T><<<grid_of(B, g), NT, 0, st>>>(g, x, part);
    if (ydtype == CSU_BF16) simam_apply<T, bf16><<<grid_of(B, g), NT, 0, st>>>(g, lam, x, part, (bf16*)y, stats);
    else simam_apply<T, float><<<grid_of(B, g), NT, 0, st>>>(g, lam, x, part, (float*)y, stats);
    return check_launch("simam_fwd");
}

template <typename T>
int bwd_typed(int B, const Geo& g, const T* x, const float* stats, int gdtype, const void* dy, T* dx, float* part,
              hipStream_t st) {
    if (gdtype == CSU_BF16) {
        simam_bwd_partial<T, bf16><<<grid_of(B, g), NT, 0, st>>>(g, x, (const bf16*)dy, stats, part);
        simam_bwd_apply<T, bf16><<<grid_of(B, g), NT, 0, st>>>(g, x, (const bf16*)dy, stats, part, dx);
    } else {
        simam_bwd_partial<T, float><<<grid_of(B, g), NT, 0, st>>>(g, x, (const float*)dy, stats, part);
        simam_bwd_apply<T, float><<<grid_of(B, g), NT, 0, st>>>(g, x, (const float*)dy, stats, part, dx);
    }
    return check_launch("simam_bwd");
}

bool dt_ok(int d) { return d == CSU_BF16 || d == CSU_F32; }

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" size_t csu_simam_workspace(int B, int L, int C) {
    if (B < 1 || L < 1 || C < 1) return 0;
    const Geo g = geo(B, L, C);
    return (size_t)B * C * g.ns * 2 * sizeof(float);
}

extern "C" int csu_simam_fwd(int B, int L, int C, float lam, int xdtype, const void* x, int ydtype, void* y,
                             float* stats, void* workspace, size_t ws_bytes, void* stream) {
    if (B < 1 || L < 2 || C < 4 || C % 4 || !x || !y || !stats)
        return fail(CSU_E_ARG, "simam_fwd: bad args (need L >= 2, C a multiple of 4)");
    if (!dt_ok(xdtype) || !dt_ok(ydtype)) return fail(CSU_E_ARG, "simam_fwd: bad dtype");
    if (!workspace || ws_bytes < csu_simam_workspace(B, L, C)) return fail(CSU_E_WORKSPACE, "simam_fwd: workspace");
    const Geo g = geo(B, L, C);
    hipStream_t st = as_stream(stream);
    if (xdtype == CSU_BF16) return fwd_typed<bf16>(B, g, lam, (const bf16*)x, ydtype, y, stats, (float*)workspace, st);
    return fwd_typed<float>(B, g, lam, (const float*)x, ydtype, y, stats, (float*)workspace, st);
}

extern "C" int csu_simam_fwd_fork(int B, int L, int C, float lam, const float* x, void* y_, void* xc_, float* stats,
                                  void* workspace, size_t ws_bytes, void* stream) {
    bf16* y = (bf16*)y_;
    bf16* xc = (bf16*)xc_;
    if (B < 1 || L < 2 || C < 4 || C % 4 || !x || !y || !xc || !stats)
        return fail(CSU_E_ARG, "simam_fwd_fork: bad args (need L >= 2, C a multiple of 4)");
    if (!workspace || ws_bytes < csu_simam_workspace(B, L, C)) return fail(CSU_E_WORKSPACE, "simam_fwd_fork: workspace");
    const Geo g = geo(B, L, C);
    hipStream_t st = as_stream(stream);
    float* part = (float*)workspace;
    simam_stats<float><<<grid_of(B, g), NT, 0, st>>>(g, x, part);
    simam_apply<float, bf16, true><<<grid_of(B, g), NT, 0, st>>>(g, lam, x, part, y, stats, xc);
    return check_launch("simam_fwd_fork");
}

extern "C" int csu_simam_bwd_join(int B, int L, int C, const float* x, const float* stats, int gdtype, const void* dy,
                                  const void* g2_, float* dx, void* dxb_, void* workspace, size_t ws_bytes, void* stream) {
    const bf16* g2 = (const bf16*)g2_;
    bf16* dxb = (bf16*)dxb_;
    if (B < 1 || L < 2 || C < 4 || C % 4 || !x || !stats || !dy || !g2 || !dx || !dxb)
        return fail(CSU_E_ARG, "simam_bwd_join: bad args");
    if (!dt_ok(gdtype)) return fail(CSU_E_ARG, "simam_bwd_join: bad dtype");
    if (!workspace || ws_bytes < csu_simam_workspace(B, L, C)) return fail(CSU_E_WORKSPACE, "simam_bwd_join: workspace");
    const Geo g = geo(B, L, C);
    hipStream_t st = as_stream(stream);
    float* part = (float*)workspace;
    if (gdtype == CSU_BF16) {
        simam_bwd_partial<float, bf16><<<grid_of(B, g), NT, 0, st>>>(g, x, (const bf16*)dy, stats, part);
        simam_bwd_apply<float, bf16, true><<<grid_of(B, g), NT, 0, st>>>(g, x, (const bf16*)dy, stats, part, dx, g2, dxb);
    } else {
        simam_bwd_partial<float, float><<<grid_of(B, g), NT, 0, st>>>(g, x, (const float*)dy, stats, part);
        simam_bwd_apply<float, float, true><<<grid_of(B, g), NT, 0, st>>>(g, x, (const float*)dy, stats, part, dx, g2, dxb);
    }
    return check_launch("simam_bwd_join");
}

extern "C" int csu_simam_bwd(int B, int L, int C, int xdtype, const void* x, const float* stats, int gdtype,
                             const void* dy, void* dx, void* workspace, size_t ws_bytes, void* stream) {
    if (B < 1 || L < 2 || C < 4 || C % 4 || !x || !stats || !dy || !dx) return fail(CSU_E_ARG, "simam_bwd: bad args");
    if (!dt_ok(xdtype) || !dt_ok(gdtype)) return fail(CSU_E_ARG, "simam_bwd: bad dtype");
    if (!workspace || ws_bytes < csu_simam_workspace(B, L, C)) return fail(CSU_E_WORKSPACE, "simam_bwd: workspace");
    const Geo g = geo(B, L, C);
    hipStream_t st = as_stream(stream);
    if (xdtype == CSU_BF16) return bwd_typed<bf16>(B, g, (const bf16*)x, stats, gdtype, dy, (bf16*)dx, (float*)workspace, st);
    return bwd_typed<float>(B, g, (const float*)x, stats, gdtype, dy, (float*)dx, (float*)workspace, st);
}
