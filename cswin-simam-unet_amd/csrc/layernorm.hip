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
// ln_bwd: row groups per wave iteration -- 8 (4 at V = 8, C = 512: the registers of 8 would not fit).
// 8 vs 4: layernorm_bwd 1086-1093 vs 1103-1105 us/step at 512x512 B16 (profiles/r08z_ln_lu_ab.txt)
template <int V> constexpr int lu_of() { return V == 8 ? 4 : 8; }
constexpr int FU = 4;       // ln_fwd: row groups per wave

struct e4m3 { uint8_t v; };  // ln_fwd output type: OCP e4m3fn bytes + one power-of-two scale per row

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

// branch-free V-element row segments through raw buffer ops (kOOB offsets: loads read 0, stores
// dropped) -- a predicated load / store makes hipcc wait vmcnt(0) at every branch join
template <typename T, int V> __device__ __forceinline__ void bld(__amdgpu_buffer_rsrc_t rs, unsigned off, float* v) {
    if constexpr (sizeof(T) == 4) {
        buf_ld4(rs, off, v);
        if constexpr (V == 8) buf_ld4(rs, off == kOOB ? kOOB : off + 16, v + 4);
    } else {
        if constexpr (V == 8) buf_ld8bf(rs, off, v);
        else buf_ld4bf(rs, off, v);
    }
}
template <typename T, int V> __device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t rs, unsigned off, const float* v) {
    if constexpr (sizeof(T) == 4) {
        buf_st4(rs, off, v);
        if constexpr (V == 8) buf_st4(rs, off == kOOB ? kOOB : off + 16, v + 4);
    } else {
        if constexpr (V == 8) buf_st8bf(rs, off, v);
        else buf_st4bf(rs, off, v);
    }
}

// LPR lanes per row (C = LPR * V, 16-B or 8-B vectors), 64 / LPR rows per wave: C = 64 rows take a
// quarter wave each instead of a whole wave of 2-4-byte accesses.
template <int LPR> __device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// FU row groups per wave, every load issued before any math (one memory round trip per FU rows:
// the one-row-per-wave form was latency-bound at ~0.5 of the HBM roofline), branch-free raw
// buffer loads / stores (rows past the end: out-of-range offsets).  Same arithmetic per row.
template <typename TX, typename TY, int V, int LPR>
__global__ __launch_bounds__(NT) void ln_fwd(int rows, int C, float eps, const TX* __restrict__ x,
                                             const float* __restrict__ gamma, const float* __restrict__ beta,
                                             TY* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd,
                                             float* __restrict__ ysc, bf16* __restrict__ ydq) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int rb = (blockIdx.x * WAVES + (threadIdx.x >> 6)) * RPW * FU + lane / LPR;
    const int c0 = (lane % LPR) * V;
    const long n = (long)rows * C;
    const auto rs_x = buf_rsrc(x, n * sizeof(TX)), rs_y = buf_rsrc(y, n * sizeof(TY));
    const auto rs_m = buf_rsrc(mean, (long)rows * 4), rs_s = buf_rsrc(rstd, (long)rows * 4);
    float v[FU][V];
    unsigned e0[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
        const int row = rb + u * RPW;
        e0[u] = row < rows ? (unsigned)((long)row * C + c0) : kOOB;   // element offset of the lane's segment
        bld<TX, V>(rs_x, e0[u] == kOOB ? kOOB : e0[u] * (unsigned)sizeof(TX), v[u]);
    }
    float gw[V], bw[V];
    ldv<float, V>(gamma + c0, gw);
    ldv<float, V>(beta + c0, bw);
#pragma unroll
    for (int u = 0; u < FU; ++u) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) s += v[u][j];
        const float mu = group_sum<LPR>(s) / C;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            v[u][j] -= mu;
            q += v[u][j] * v[u][j];
        }
        const float rs = rsqrtf(group_sum<LPR>(q) / C + eps);
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) o[j] = v[u][j] * rs * gw[j] + bw[j];
        const unsigned e = e0[u];
        const int row = rb + u * RPW;
        const unsigned ro = (lane % LPR == 0 && row < rows) ? (unsigned)row * 4u : kOOB;
        if constexpr (sizeof(TY) == 1) {
            // fp8 output (the e4m3 GEMM's activation operand, csrc/fp8gemm.hip): the row's amax over
            // its LPR lanes, power-of-two scale s = 2^ceil(log2(amax / 448)) as the weights'
            // (csrc/fp8.hip), y / s rounded to e4m3 (RNE; |y / s| <= 448, nothing saturates)
            float am = 0.f;
#pragma unroll
            for (int j = 0; j < V; ++j) am = fmaxf(am, fabsf(o[j]));
#pragma unroll
            for (int m = LPR / 2; m > 0; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
            const float s = am > 0.f ? exp2f(ceilf(log2f(am / 448.f))) : 1.f;
            const float inv = 1.f / s;
            unsigned w[V / 4];
#pragma unroll
            for (int k = 0; k < V / 4; ++k) {
                int p = __builtin_amdgcn_cvt_pk_fp8_f32(o[4 * k] * inv, o[4 * k + 1] * inv, 0, false);
                w[k] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(o[4 * k + 2] * inv, o[4 * k + 3] * inv, p, true);
            }
            if constexpr (V == 8) __builtin_amdgcn_raw_buffer_store_b64(u32x2{w[0], w[1]}, rs_y, e, 0, 0);
            else __builtin_amdgcn_raw_buffer_store_b32(w[0], rs_y, e, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s), buf_rsrc(ysc, (long)rows * 4), ro, 0, 0);
            if (ydq) {   // the dequantised value in bf16 (exact): the weight gradient's operand
                float dq[V];
#pragma unroll
                for (int k = 0; k < V / 4; ++k) {
                    const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[k], false);
                    const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w[k], true);
                    dq[4 * k] = lo[0] * s;
                    dq[4 * k + 1] = lo[1] * s;
                    dq[4 * k + 2] = hi[0] * s;
                    dq[4 * k + 3] = hi[1] * s;
                }
                bst<bf16, V>(buf_rsrc(ydq, n * 2), e == kOOB ? kOOB : e * 2u, dq);
            }
        } else {
            bst<TY, V>(rs_y, e == kOOB ? kOOB : e * (unsigned)sizeof(TY), o);
        }
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mu), rs_m, ro, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(rs), rs_s, ro, 0, 0);
    }
}

// dx = dres + rstd * (g*gamma - mean(g*gamma) - xhat * mean(g*gamma*xhat)); optionally also a bf16
// copy of dx (the next GEMM's operand).  dres = the gradient reaching x through the residual branch
// (x + f(LN(x)) of CSWinBlock, cswin:367-368): the autograd add of the two branches is fused here.
// dgamma/dbeta: per-block partials, written [nblocks][2C] (one coalesced row per block: the
// [2C][nblocks] column layout's scattered 4-B stores cost 3-4 us per launch) for ln_cols_sum.
template <typename TX, typename TG, int V, int LPR>
__global__ __launch_bounds__(NT) void ln_bwd(int rows, int C, int rows_per_block, const TX* __restrict__ x,
                                             const float* __restrict__ gamma, const float* __restrict__ mean,
                                             const float* __restrict__ rstd, const TG* __restrict__ dy,
                                             const float* __restrict__ dres, TX* __restrict__ dx,
                                             bf16* __restrict__ dxb, float* __restrict__ part) {
    constexpr int RPW = 64 / LPR;
    constexpr int LU = lu_of<V>();
    __shared__ float red[WAVES][2][512];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = (lane % LPR) * V;
    float gw[V], dg[V], db[V];
    ldv<float, V>(gamma + c0, gw);
#pragma unroll
    for (int j = 0; j < V; ++j) dg[j] = db[j] = 0.f;
    const int r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
    // LU row groups per wave iteration, all loads issued before any math: one memory round trip
    // per LU rows instead of per row (the loop is latency-bound, not bandwidth-bound).  Raw buffer
    // loads / stores (rows past the end: out-of-range offsets) keep them in flight together.
    const long n = (long)rows * C;
    const auto rs_x = buf_rsrc(x, n * sizeof(TX)), rs_g = buf_rsrc(dy, n * sizeof(TG));
    const auto rs_r = buf_rsrc(dres, dres ? n * 4 : 0), rs_dx = buf_rsrc(dx, n * sizeof(TX));
    const auto rs_db = buf_rsrc(dxb, dxb ? n * 2 : 0);
    const auto rs_m = buf_rsrc(mean, (long)rows * 4), rs_s = buf_rsrc(rstd, (long)rows * 4);
    for (int rb = r0 + wave * RPW * LU; rb < r1; rb += WAVES * RPW * LU) {
        float xv[LU][V], g[LU][V], rv[LU][V], mu[LU], rs[LU];
        unsigned e0[LU];
#pragma unroll
        for (int u = 0; u < LU; ++u) {
            const int row = rb + u * RPW + lane / LPR;
            const bool ok = row < r1;
            e0[u] = ok ? (unsigned)((long)row * C + c0) : kOOB;   // element offset of the lane's segment
            bld<TX, V>(rs_x, ok ? e0[u] * (unsigned)sizeof(TX) : kOOB, xv[u]);
            bld<TG, V>(rs_g, ok ? e0[u] * (unsigned)sizeof(TG) : kOOB, g[u]);
            bld<float, V>(rs_r, ok ? e0[u] * 4u : kOOB, rv[u]);
            mu[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_m, ok ? (unsigned)row * 4u : kOOB, 0, 0));
            rs[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_s, ok ? (unsigned)row * 4u : kOOB, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < LU; ++u) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int j = 0; j < V; ++j) {
                xv[u][j] = (xv[u][j] - mu[u]) * rs[u];   // xhat (0 on rows past the end: g = 0 there)
                const float gg = g[u][j] * gw[j];
                s1 += gg;
                s2 += gg * xv[u][j];
                dg[j] += g[u][j] * xv[u][j];
                db[j] += g[u][j];
            }
            s1 = group_sum<LPR>(s1) / C;
            s2 = group_sum<LPR>(s2) / C;
            float o[V];
#pragma unroll
            for (int j = 0; j < V; ++j) o[j] = rs[u] * (g[u][j] * gw[j] - s1 - xv[u][j] * s2) + rv[u][j];
            const unsigned e = e0[u];
            bst<TX, V>(rs_dx, e == kOOB ? kOOB : e * (unsigned)sizeof(TX), o);
            if (dxb) bst<bf16, V>(rs_db, e == kOOB ? kOOB : e * 2u, o);
        }
    }
    // column partials: lanes of one column inside the wave (fixed xor tree), then the waves
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < V; ++j) {
            dg[j] += __shfl_xor(dg[j], o, 64);
            db[j] += __shfl_xor(db[j], o, 64);
        }
    if (lane < LPR)
#pragma unroll
        for (int j = 0; j < V; ++j) {
            red[wave][0][c0 + j] = dg[j];
            red[wave][1][c0 + j] = db[j];
        }
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * C; i += NT) {
        const int k = i / C, c = i % C;
        float s = 0.f;
#pragma unroll
        for (int wv = 0; wv < WAVES; ++wv) s += red[wv][k][c];
        part[(size_t)blockIdx.x * 2 * C + i] = s;
    }
}

// out[v] = sum_b part[b][v] (v < 2C: dgamma | dbeta) for the 64 values v0 + lane of one workgroup
// of RT threads: wave w sums blocks w, w + RW, ... (8 loads in flight, coalesced 256-B rows), then
// the RW wave sums in order -- fixed association, deterministic
constexpr int RT = 1024, RW = RT / 64;
__device__ __forceinline__ void ln_cols_sum(const float* __restrict__ part, int C, int nb, int v0,
                                            float* __restrict__ dgamma, float* __restrict__ dbeta) {
    __shared__ float red[RW][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long ld = 2L * C;
    const float* p = part + v0 + lane;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int b = wave;
    for (; b + 7 * RW < nb; b += 8 * RW)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += p[(b + k * RW) * ld];
    for (; b < nb; b += RW) a[0] += p[b * ld];
    red[wave][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (wave == 0) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < RW; ++w) s += red[w][lane];
        const int v = v0 + lane;
        (v < C ? dgamma[v] : dbeta[v - C]) = s;
    }
}

__global__ __launch_bounds__(RT) void ln_param_reduce(int C, int nb, const float* __restrict__ part,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta) {
    ln_cols_sum(part, C, nb, blockIdx.x * 64, dgamma, dbeta);
}

int ln_blocks(int rows, int rpw, int lu, int* rpb) {   // <= 512 blocks, rows per block a multiple of a block's row step
    const int step = WAVES * rpw * lu;
    int r = (rows + 511) / 512;   // (1024 / 2048 blocks measured no faster: tools/ln_probe.py)
    r = ((r + step - 1) / step) * step;
    *rpb = r;
    return (rows + r - 1) / r;
}

// the backward's block count for rows x C (rows per wave 64 / LPR = C >= 256 ? 1 : 256 / C; V = 8 at C = 512)
int ln_bwd_blocks(int rows, int C, int* rpb) { return ln_blocks(rows, C >= 256 ? 1 : 256 / C, C == 512 ? 4 : 8, rpb); }

int check_c(int C) {
    if (C % 64 || C < 64 || C > 512) return fail(CSU_E_UNSUPPORTED, "layernorm: C must be 64..512, multiple of 64");
    return 0;
}

int check_rows(int rows, int C) {   // 32-bit byte offsets of the raw buffer ops (fp32 rows)
    if ((long)rows * C * 4 >= 0x7fffffffL) return fail(CSU_E_UNSUPPORTED, "layernorm: rows * C * 4 must be < 2^31");
    return 0;
}

template <typename TX, typename TY>
int launch_fwd(int rows, int C, float eps, const void* x, const float* g, const float* b, void* y, float* m,
               float* r, hipStream_t st, float* ysc = nullptr, bf16* ydq = nullptr) {
#define CSU_LNF(V, LPR)                                                                                           \
    ln_fwd<TX, TY, V, LPR><<<(rows + WAVES * (64 / LPR) * FU - 1) / (WAVES * (64 / LPR) * FU), NT, 0, st>>>(rows, C, eps, \
                                                                                                  (const TX*)x, g, b, \
                                                                                                  (TY*)y, m, r, ysc, ydq)
    switch (C / 64) {
        case 1: CSU_LNF(4, 16); break;
        case 2: CSU_LNF(4, 32); break;
        case 4: CSU_LNF(4, 64); break;
        case 8: CSU_LNF(8, 64); break;
        default: return fail(CSU_E_UNSUPPORTED, "layernorm: C/64 must be 1, 2, 4 or 8");
    }
#undef CSU_LNF
    return check_launch("layernorm_fwd");
}

template <typename TX, typename TG>
int launch_bwd(int rows, int C, const void* x, const float* g, const float* m, const float* r, const void* dy,
               const float* dres, void* dx, bf16* dxb, float* dgamma, float* dbeta, float* part, hipStream_t st) {
    int rpb, nb;
#define CSU_LNB(V, LPR)                                                                                              \
    nb = ln_bwd_blocks(rows, C, &rpb);                                                                               \
    ln_bwd<TX, TG, V, LPR><<<nb, NT, 0, st>>>(rows, C, rpb, (const TX*)x, g, m, r, (const TG*)dy, dres, (TX*)dx, dxb, \
                                             part)
    switch (C / 64) {
        case 1: CSU_LNB(4, 16); break;
        case 2: CSU_LNB(4, 32); break;
        case 4: CSU_LNB(4, 64); break;
        case 8: CSU_LNB(8, 64); break;
        default: return fail(CSU_E_UNSUPPORTED, "layernorm: C/64 must be 1, 2, 4 or 8");
    }
#undef CSU_LNB
    if (int e = check_launch("layernorm_bwd")) return e;
    if (!dgamma) return 0;   // partials stay in the workspace: csu_layernorm_param_reduce
    ln_param_reduce<<<2 * C / 64, RT, 0, st>>>(C, nb, part, dgamma, dbeta);
    return check_launch("layernorm_bwd reduce");
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_layernorm_fwd(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                                 const float* beta, int ydtype, void* y, float* mean, float* rstd, void* stream) {
    if (int e = check_c(C)) return e;
    if (int e = check_rows(rows, C)) return e;
    if (rows < 1 || !x || !gamma || !beta || !y || !mean || !rstd) return fail(CSU_E_ARG, "layernorm_fwd: bad args");
    hipStream_t st = as_stream(stream);
    if (xdtype == CSU_F32 && ydtype == CSU_F32) return launch_fwd<float, float>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    if (xdtype == CSU_F32 && ydtype == CSU_BF16) return launch_fwd<float, bf16>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    if (xdtype == CSU_BF16 && ydtype == CSU_F32) return launch_fwd<bf16, float>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    if (xdtype == CSU_BF16 && ydtype == CSU_BF16) return launch_fwd<bf16, bf16>(rows, C, eps, x, gamma, beta, y, mean, rstd, st);
    return fail(CSU_E_ARG, "layernorm_fwd: bad dtype");
}

extern "C" int csu_layernorm_fwd_fp8_dq(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                                        const float* beta, void* yq, float* yscale, void* ydq, float* mean, float* rstd,
                                        void* stream) {
    if (int e = check_c(C)) return e;
    if (int e = check_rows(rows, C)) return e;
    if (rows < 1 || !x || !gamma || !beta || !yq || !yscale || !mean || !rstd)
        return fail(CSU_E_ARG, "layernorm_fwd_fp8: bad args");
    hipStream_t st = as_stream(stream);
    bf16* dq = (bf16*)ydq;
    if (xdtype == CSU_F32) return launch_fwd<float, e4m3>(rows, C, eps, x, gamma, beta, yq, mean, rstd, st, yscale, dq);
    if (xdtype == CSU_BF16) return launch_fwd<bf16, e4m3>(rows, C, eps, x, gamma, beta, yq, mean, rstd, st, yscale, dq);
    return fail(CSU_E_ARG, "layernorm_fwd_fp8: bad dtype");
}

extern "C" int csu_layernorm_fwd_fp8(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                                     const float* beta, void* yq, float* yscale, float* mean, float* rstd, void* stream) {
    return csu_layernorm_fwd_fp8_dq(rows, C, eps, xdtype, x, gamma, beta, yq, yscale, nullptr, mean, rstd, stream);
}

extern "C" size_t csu_layernorm_bwd_workspace(int rows, int C) {
    int rpb;
    const int nb = ln_bwd_blocks(rows, C, &rpb);
    return (size_t)nb * 2 * C * sizeof(float);
}

extern "C" int csu_layernorm_bwd_ex(int rows, int C, int xdtype, const void* x, const float* gamma, const float* mean,
                                    const float* rstd, int dydtype, const void* dy, const float* dres, void* dx,
                                    void* dx_bf16, float* dgamma, float* dbeta, void* workspace, size_t ws_bytes,
                                    void* stream) {
    if (int e = check_c(C)) return e;
    if (int e = check_rows(rows, C)) return e;
    if (rows < 1 || !x || !gamma || !mean || !rstd || !dy || !dx || (!dgamma) != (!dbeta))
        return fail(CSU_E_ARG, "layernorm_bwd: bad args");
    if (!workspace || ws_bytes < csu_layernorm_bwd_workspace(rows, C))
        return fail(CSU_E_WORKSPACE, "layernorm_bwd: workspace too small");
    if (dres && xdtype != CSU_F32) return fail(CSU_E_ARG, "layernorm_bwd: a residual gradient needs fp32 x/dx");
    hipStream_t st = as_stream(stream);
    float* part = (float*)workspace;
    bf16* dxb = (bf16*)dx_bf16;
#define CSU_LNB_CALL(TX, TG) return launch_bwd<TX, TG>(rows, C, x, gamma, mean, rstd, dy, dres, dx, dxb, dgamma, dbeta, part, st)
    if (xdtype == CSU_F32 && dydtype == CSU_F32) CSU_LNB_CALL(float, float);
    if (xdtype == CSU_F32 && dydtype == CSU_BF16) CSU_LNB_CALL(float, bf16);
    if (xdtype == CSU_BF16 && dydtype == CSU_F32) CSU_LNB_CALL(bf16, float);
    if (xdtype == CSU_BF16 && dydtype == CSU_BF16) CSU_LNB_CALL(bf16, bf16);
#undef CSU_LNB_CALL
    return fail(CSU_E_ARG, "layernorm_bwd: bad dtype");
}

extern "C" int csu_layernorm_bwd(int rows, int C, int xdtype, const void* x, const float* gamma, const float* mean,
                                 const float* rstd, int dydtype, const void* dy, void* dx, float* dgamma,
                                 float* dbeta, void* workspace, size_t ws_bytes, void* stream) {
    return csu_layernorm_bwd_ex(rows, C, xdtype, x, gamma, mean, rstd, dydtype, dy, nullptr, dx, nullptr, dgamma, dbeta,
                                workspace, ws_bytes, stream);
}

// Batched parameter reduction: the item table travels as a kernel argument (no device table, so
// a captured launch needs no host buffer); workgroup w of the launch handles the 64-value chunk
// w - v0 of the item whose chunk range [v0, v0 + 2C / 64) contains it.
constexpr int LNB_MAX = 48;
struct LnBatch {
    const float* part[LNB_MAX];
    float* dg[LNB_MAX];
    float* db[LNB_MAX];
    int nb[LNB_MAX], C[LNB_MAX], v0[LNB_MAX + 1];
    int count;
};

__global__ __launch_bounds__(RT) void ln_param_reduce_batch(LnBatch t) {
    const int w = blockIdx.x;
    int i = 0;
    while (i + 1 < t.count && t.v0[i + 1] <= w) ++i;
    ln_cols_sum(t.part[i], t.C[i], t.nb[i], (w - t.v0[i]) * 64, t.dg[i], t.db[i]);
}

// dgamma / dbeta from the per-block partials a csu_layernorm_bwd_ex call with NULL dgamma/dbeta
// left in `workspace` (the same rows / C): lets the reduction run on another stream
extern "C" int csu_layernorm_param_reduce(int rows, int C, const void* workspace, float* dgamma, float* dbeta,
                                          void* stream) {
    if (int e = check_c(C)) return e;
    if (rows < 1 || !workspace || !dgamma || !dbeta) return fail(CSU_E_ARG, "layernorm_param_reduce: bad args");
    int rpb;
    const int nb = ln_bwd_blocks(rows, C, &rpb);
    ln_param_reduce<<<2 * C / 64, RT, 0, as_stream(stream)>>>(C, nb, (const float*)workspace, dgamma, dbeta);
    return check_launch("layernorm_param_reduce");
}

extern "C" int csu_layernorm_param_reduce_batch(const csu_ln_param_item* items, int count, void* stream) {
    if (count < 0 || (count && !items)) return fail(CSU_E_ARG, "layernorm_param_reduce_batch: bad args");
    for (int base = 0; base < count; base += LNB_MAX) {
        LnBatch t;
        t.count = count - base < LNB_MAX ? count - base : LNB_MAX;
        t.v0[0] = 0;
        for (int i = 0; i < t.count; ++i) {
            const csu_ln_param_item& it = items[base + i];
            if (int e = check_c(it.C)) return e;
            if (it.rows < 1 || !it.workspace || !it.dgamma || !it.dbeta)
                return fail(CSU_E_ARG, "layernorm_param_reduce_batch: bad item");
            int rpb;
            t.nb[i] = it.nblocks > 0 ? it.nblocks : ln_bwd_blocks(it.rows, it.C, &rpb);
            t.C[i] = it.C;
            t.part[i] = (const float*)it.workspace;
            t.dg[i] = it.dgamma;
            t.db[i] = it.dbeta;
            t.v0[i + 1] = t.v0[i] + 2 * it.C / 64;
        }
        ln_param_reduce_batch<<<t.v0[t.count], RT, 0, as_stream(stream)>>>(t);
        if (int e = check_launch("layernorm_param_reduce_batch")) return e;
    }
    return 0;
}
