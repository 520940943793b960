// gemm_ws: weight-streaming token GEMM for gfx950 -- the CSWinBlock qkv / proj Linears and their
// input gradients at the 16384- and 65536-token stages (cswin:314-366), where every tiled GEMM
// re-stages the weight panel through LDS once per 64-128-token tile and is bound by one CU's
// L2 -> LDS fill rate (gemm4 and hipBLASLt both at 18-20 us for 16384 x 768 x 256,
// tools/probes/gemm_vs_blas.py).
//
//   out[m][n] = epi( sum_k X[m][k] * W[n][k] )     X (M, K) bf16 tokens, W (N, K) bf16 weight
//
// Design (MI355X):
//  * one workgroup (4 waves) per 64-token panel; the panel is read ONCE (coalesced 16-B loads into
//    LDS) and, for K <= 256, held in registers as the MFMA B fragments (K > 256: B fragments are
//    read from LDS per k-step);
//  * the waves split N in 32-feature tiles (wave w: tiles w, w + 4, ...); each wave streams its
//    tiles' weight fragments straight global -> VGPR, with NO LDS and NO barrier in the main loop:
//    the weight is stored FRAGMENT-ORDERED (csu_frag_layout_batch: [N/32][K/16][64 lanes][8 bf16],
//    lane (r, h) = row r, k 8h..8h+7 of a 16-deep k-step), so every wave load is one contiguous
//    1 KB (fragment-shaped loads of the natural layout ran 2.5x slower, tools/probes/wstream_probe.hip);
//  * "units" of up to 16 k-steps: the next unit's 16 loads are interleaved 1 : 2 with this unit's
//    MFMAs (sched_group_barrier), so the texture path sees a steady stream;
//  * epilogue per tile through a per-wave LDS region (fp32 [64][36]): bias, residual, output
//    dtype, row-contiguous 16-B stores.
// Measured (probe, 16384 x 768 x 256): 8.6 us vs 18.0 (gemm4) / 19.6 (hipBLASLt).
//
// e4m3 weights (BASELINE config 5, F8 != 0): the same kernel streams the fp8 format's e4m3 bytes in
// the same fragment order ([N/32][K/16][64 lanes][8 bytes]: half the bytes of the weight stream that
// bounds these GEMMs at the 16384-token stage) and widens each fragment to bf16 in registers
// (v_cvt_scalef32_pk_bf16_fp8, scale 1) right before its MFMA; activations stay bf16.  The per-row
// power-of-two scales s[n] of W = q s are applied exactly: F8 = 1 (x W^T) multiplies the accumulator
// of output column n by s[n] in the epilogue, F8 = 2 (dy W: the weight operand is W^T, whose k index
// is n) multiplies the token panel's column n by s[n] once when it is loaded.  Both are exact for
// power-of-two scales, so the outputs are bitwise those of the bf16 kernel on the dequantised weight.
#include "common.hpp"

#include <type_traits>

namespace csu {
namespace {

enum { WS_PLAIN = 0, WS_RESID = 1, WS_LNBWD = 2, WS_RESID_LN = 3 };

// WS_RESID_LN epilogue: y = res + x W^T + b (fp32, written as WS_RESID) is the residual stream that
// CSWinBlock's norm2 normalises next (cswin:366-368): the workgroup holds all N = C features of its
// tokens, so it also writes LayerNorm(y) (bf16) and the per-token mean / rstd for norm2's backward.
struct WsLnF {
    const float* gamma;   // (C)
    const float* beta;    // (C)
    float eps;
    bf16* out;            // (M, C)
    float* mean;          // (M)
    float* rstd;          // (M)
};

// WS_LNBWD epilogue: the GEMM is the input gradient dh of a LayerNorm's output (the qkv Linear's
// input, CSWinBlock norm1, cswin:357 / 337): instead of writing dh, the workgroup (64 tokens x all
// C = N features) runs the LayerNorm backward on it -- dx = dres + rstd (g - mean(g) - xhat
// mean(g xhat)), g = dh * gamma -- and writes dx (fp32) + its bf16 copy and the block's dgamma / dbeta
// column partials (row blockIdx.x of part [M / 64][2C], csu_layernorm_param_reduce_batch's layout).
struct WsLn {
    const float* x;      // LayerNorm input (M, C) fp32
    const float* gamma;  // (C)
    const float* mean;   // (M)
    const float* rstd;   // (M)
    const float* dres;   // (M, C) fp32 gradient of the residual branch, or NULL
    float* dx;           // (M, C)
    bf16* dxb;           // (M, C) bf16 copy of dx
    float* part;         // [M / 64][2C]
};

constexpr int WS_BM = 64;   // tokens per wave group (the 64-token panel a wave's B fragments hold)
constexpr bool WS_ROT = true;

// k-steps per unit: the largest divisor of ks <= 16 that still gives the wave >= 2 units (so the
// next unit's weight loads overlap this unit's MFMAs), else the largest divisor <= 16
constexpr int ws_unit(int ks, int nt, int umax = 16) {
    for (int u = umax; u > 1; --u)
        if (ks % u == 0 && nt * (ks / u) >= 2) return u;
    for (int u = umax; u > 1; --u)
        if (ks % u == 0) return u;
    return 1;
}
// waves along N: 4 when the 32-feature tiles split evenly over 4 waves, else 2 (N = 64, 192: two token
// groups of 64 per workgroup, each split over 2 waves) or 1
constexpr int ws_wn(int n) { return (n / 32) % 4 == 0 ? 4 : (n / 32) % 2 == 0 ? 2 : 1; }
constexpr int ws_tokens(int n) { return WS_BM * (4 / ws_wn(n)); }   // tokens per workgroup
// N split over NS workgroups per token panel (grid.y): each streams 1/NS of the weight and writes 1/NS
// of the features, two workgroups per CU.  Only for the plain epilogue (bias; RESID spills), K <= 256 (the token
// panel in registers, two workgroups' LDS fit) and an even tile count per wave.  WS_NSPLIT = 1: off.
#ifndef WS_NSPLIT
#define WS_NSPLIT 1
#endif
constexpr int ws_ns(int k, int n, int epi) {
    return WS_NSPLIT > 1 && epi == 0 && k <= 256 && ws_wn(n) == 4 && (n / 128) % WS_NSPLIT == 0 ? WS_NSPLIT : 1;
}

// 8 e4m3 bytes (one 32x32x16 A-fragment half-lane) -> 8 bf16, exactly
__device__ __forceinline__ bf16x8 e4m3x8_bf16(u32x2 w) {
    typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
    const bf16x2v p0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[0], 1.f, false);
    const bf16x2v p1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[0], 1.f, true);
    const bf16x2v p2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[1], 1.f, false);
    const bf16x2v p3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[1], 1.f, true);
    return bf16x8{p0[0], p0[1], p1[0], p1[1], p2[0], p2[1], p3[0], p3[1]};
}

template <int K, int N, int EPI, typename TOUT, int NS = 1, int F8 = 0>
__global__ __launch_bounds__(256, ws_wn(N) < 4 || NS > 1 ? 2 : 1) void gemm_ws_kernel(long M, const bf16* __restrict__ X, int ldx,
                                                      const bf16* __restrict__ Wf, const float* __restrict__ bias,
                                                      const float* __restrict__ resid, TOUT* __restrict__ out,
                                                      WsLn ln = WsLn{}, WsLnF lnf = WsLnF{},
                                                      const float* __restrict__ wsc = nullptr) {
    static_assert(F8 == 0 || EPI != WS_LNBWD, "gemm_ws: e4m3 weights not with the LayerNorm-backward epilogue");
    constexpr int WN = ws_wn(N);                   // waves along N
    constexpr int NT = N / (32 * WN * NS);         // 32-feature tiles per wave (of this workgroup's N / NS)
    static_assert(NT * 32 * WN * NS == N, "gemm_ws: N = 32 WN NT NS");
    static_assert(NS == 1 || EPI == WS_PLAIN || EPI == WS_RESID, "gemm_ws: the LayerNorm epilogues need all N features");
    static_assert(EPI != WS_LNBWD || WN == 4, "gemm_ws: the LayerNorm epilogue needs all C features in one token group");
    constexpr int KS = K / 16;                     // k-steps
    constexpr int UK = ws_unit(KS, NT, NS > 1 ? 8 : 16);   // k-steps per unit (a divisor of KS; <= 8 at two WGs/CU)
    constexpr int CH = KS / UK;                    // units per tile
    static_assert(CH * UK == KS, "unit size");
    constexpr int U = NT * CH;                     // units per wave
    constexpr bool XREG = K <= 256;                // B fragments held in registers
    constexpr bool XLDS = !XREG || WN == 4;        // token panel staged through LDS (else direct fragment loads)
    constexpr int XS = K + 8;                      // LDS row stride of the token panel (bf16)
    constexpr int ES = 36;                         // fp32 row stride of the epilogue region
    __shared__ __attribute__((aligned(16))) bf16 xs[XLDS ? WS_BM * XS : 8];
    __shared__ __attribute__((aligned(16))) float ep_all[4 * WS_BM * ES];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wn = wave % WN;                      // this wave's N slot
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * ws_tokens(N) + WS_BM * (wave / WN);   // the wave's 64-token panel
    float* ep = ep_all + wave * WS_BM * ES;

    // tile order rotated per workgroup (its index within the XCD: ids x, x + 8, ... run on XCD x), so
    // the CUs of an XCD do not all read the same weight lines at the same moment
    const int rot = WS_ROT ? (int)((blockIdx.x >> 3) % NT) : 0;
    const int tb = NS > 1 ? (int)blockIdx.y * NT : 0;   // this workgroup's first tile of each wave
    auto tile_of = [&](int i) { return tb + (i + rot < NT ? i + rot : i + rot - NT); };
    using WFR = std::conditional_t<F8 != 0, u32x2, bf16x8>;   // a lane's weight fragment as loaded
    WFR wf[2][UK];
    auto wload1 = [&](int u, int s) {   // k-step s of unit u of this wave into buffer u & 1
        const int nt = wn + WN * tile_of(u / CH), ks = (u % CH) * UK + s;
        if constexpr (F8 != 0)
            wf[u & 1][s] = *reinterpret_cast<const u32x2*>(reinterpret_cast<const uint8_t*>(Wf) +
                                                           ((long)(nt * KS + ks) * 64 + lane) * 8);
        else
            wf[u & 1][s] = *reinterpret_cast<const bf16x8*>(Wf + ((long)(nt * KS + ks) * 64 + lane) * 8);
    };
    auto wfrag = [&](const WFR& w) {
        if constexpr (F8 != 0) return e4m3x8_bf16(w);
        else return w;
    };
#pragma unroll
    for (int s = 0; s < UK; ++s) wload1(0, s);
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 xf[XREG ? 2 : 1][XREG ? KS : 1];
    if constexpr (XLDS) {
        // token panel -> LDS (16-B pieces, row-contiguous; one token group: WN = 4)
        constexpr int PR = K / 8;   // pieces per row
#pragma unroll
        for (int i = 0; i < WS_BM * PR / 256; ++i) {
            const int p = threadIdx.x + 256 * i, row = p / PR, c = 8 * (p % PR);
            bf16x8 v = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * ldx + c);
            if constexpr (F8 == 2) {   // column c + e of the panel is k = n of W: times s[n] (exact)
                const f32x4 s0 = *reinterpret_cast<const f32x4*>(wsc + c), s1 = *reinterpret_cast<const f32x4*>(wsc + c + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = (bf16)((float)v[e] * s0[e]);
                    v[4 + e] = (bf16)((float)v[4 + e] * s1[e]);
                }
            }
            *reinterpret_cast<bf16x8*>(xs + row * XS + c) = v;
        }
        __syncthreads();
        if constexpr (XREG) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < KS; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(xs + (32 * t + r) * XS + 16 * s + 8 * h);
        }
    } else {
        // B fragments straight from the token rows (lane (r, h): row r, k 16 s + 8 h .. + 7; a row's
        // 16-B pieces over the KS loads cover its lines once)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                xf[t][s] = *reinterpret_cast<const bf16x8*>(X + (m0 + 32 * t + r) * ldx + 16 * s + 8 * h);
                if constexpr (F8 == 2) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) xf[t][s][e] = (bf16)((float)xf[t][s][e] * wsc[16 * s + 8 * h + e]);
                }
            }
    }
    __builtin_amdgcn_sched_barrier(0);

    f32x16 a0 = f32x16{}, a1 = f32x16{};
    const auto rs_b = buf_rsrc(bias, bias ? (long)N * 4 : 0);   // null bias: loads read 0
    constexpr bool BF = sizeof(TOUT) == 2;
    // epilogue loads of a tile are issued at the start of its last unit, BEFORE the next unit's
    // weight loads: vmcnt counts in issue order, so waiting for them then does not wait for the prefetch
    constexpr bool RES = EPI == WS_RESID || EPI == WS_RESID_LN;
    static_assert(EPI != WS_RESID_LN || !BF, "gemm_ws: the LayerNorm epilogue writes the fp32 residual stream");
    float bv[8], rv[8][4], sv[8];
    const auto rs_s = buf_rsrc(wsc, F8 == 1 ? (long)N * 4 : 0);
    f32x16 keep[EPI == WS_LNBWD ? NT : 1][2];
    float yk[EPI == WS_RESID_LN ? NT : 1][8][4];   // y of the wave's tiles in the store layout (LayerNorm)
    float lg[EPI == WS_RESID_LN ? NT : 1][4], lb[EPI == WS_RESID_LN ? NT : 1][4];
    if constexpr (EPI == WS_RESID_LN) {   // gamma / beta of the lane's 4 features of each tile
        const int cc = 4 * (lane & 7);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            load4(lnf.gamma + 32 * (wn + WN * tile_of(i)) + cc, lg[i]);
            load4(lnf.beta + 32 * (wn + WN * tile_of(i)) + cc, lb[i]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u % CH;
        if (EPI != WS_LNBWD && c == CH - 1) {
            const int n0 = 32 * (wn + WN * tile_of(u / CH));
            if constexpr (BF) {
                const int cc = 8 * (lane & 3);
                buf_ld4(rs_b, (unsigned)(n0 + cc) * 4, bv);
                buf_ld4(rs_b, (unsigned)(n0 + cc + 4) * 4, bv + 4);
                if constexpr (F8 == 1) {
                    buf_ld4(rs_s, (unsigned)(n0 + cc) * 4, sv);
                    buf_ld4(rs_s, (unsigned)(n0 + cc + 4) * 4, sv + 4);
                }
            } else {
                const int cc = 4 * (lane & 7);
                buf_ld4(rs_b, (unsigned)(n0 + cc) * 4, bv);
                if constexpr (F8 == 1) buf_ld4(rs_s, (unsigned)(n0 + cc) * 4, sv);
                if constexpr (RES) {
                    const auto rs_res = buf_rsrc(resid + m0 * N, (M - m0) * N * 4);
#pragma unroll
                    for (int q = 0; q < 8; ++q) buf_ld4(rs_res, (unsigned)((8 * q + (lane >> 3)) * N + n0 + cc) * 4, rv[q]);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < UK; ++s) {
            if (u + 1 < U) wload1(u + 1, s);
            const int ks = c * UK + s;
            bf16x8 b0, b1;
            if constexpr (XREG) {
                b0 = xf[0][ks];
                b1 = xf[XREG ? 1 : 0][ks];
            } else {
                b0 = *reinterpret_cast<const bf16x8*>(xs + r * XS + 16 * ks + 8 * h);
                b1 = *reinterpret_cast<const bf16x8*>(xs + (32 + r) * XS + 16 * ks + 8 * h);
            }
            const bf16x8 wa = wfrag(wf[u & 1][s]);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, b0, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa, b1, a1, 0, 0, 0);
            if (u + 1 < U) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // one weight load
            if constexpr (!XREG) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // two fragment reads
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                 // two MFMAs
        }
        __builtin_amdgcn_sched_barrier(0);
        if (c != CH - 1) continue;
        if constexpr (EPI == WS_LNBWD) {
            keep[u / CH][0] = a0;
            keep[u / CH][1] = a1;
            a0 = f32x16{};
            a1 = f32x16{};
            continue;
        }
        // ---- epilogue of tile nt: acc element (token 32 t + r, feature 32 nt + 8 g + 4 h + e)
        const int nt = wn + WN * tile_of(u / CH);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x16& a = t ? a1 : a0;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<f32x4*>(ep + (32 * t + r) * ES + 8 * g + 4 * h) =
                    f32x4{a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]};
        }
        asm volatile("" ::: "memory");   // the wave's own LDS writes, then its reads (in order per wave)
        const int n0 = 32 * nt;
        const auto rs_out = buf_rsrc(out + m0 * N, (M - m0) * N * (long)sizeof(TOUT));
        if constexpr (BF) {
            // 4 lanes x 8 features per token row, 16 rows per instruction
            const int cc = 8 * (lane & 3);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 16 * q + (lane >> 2);
                float v[8];
                load4(ep + row * ES + cc, v);
                load4(ep + row * ES + cc + 4, v + 4);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if constexpr (F8 == 1) v[e] *= sv[e];   // s[n] x (x q^T): exact (power of two)
                    v[e] += bv[e];
                }
                buf_st8bf(rs_out, (unsigned)(row * N + n0 + cc) * 2, v);
            }
        } else {
            // fp32: 8 lanes x 4 features per token row, 8 rows per instruction
            const int cc = 4 * (lane & 7);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int row = 8 * q + (lane >> 3);
                float v[4];
                load4(ep + row * ES + cc, v);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (F8 == 1) v[e] *= sv[e];
                    v[e] += bv[e];
                    if constexpr (RES) v[e] += rv[q][e];
                    if constexpr (EPI == WS_RESID_LN) yk[u / CH][q][e] = v[e];
                }
                buf_st4(rs_out, (unsigned)(row * N + n0 + cc) * 4, v);
            }
        }
        a0 = f32x16{};
        a1 = f32x16{};
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (EPI == WS_RESID_LN) {
        // lane: rows 8 q + (lane >> 3) of its 64-token panel, features cc..cc+3 of each of its tiles.
        // Two passes over the registers (mean, then the centred sum of squares), each: the lane's
        // sum, the 8 lanes of the row (DPP), the WN waves of the token group through LDS.
        __shared__ float lnx[2][4][WS_BM];
        const int rq = lane >> 3, g0 = (wave / WN) * WN;
        float mu[8], rsd[8];
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                float a = 0.f;
#pragma unroll
                for (int i = 0; i < NT; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float d = pass ? yk[i][q][e] - mu[q] : yk[i][q][e];
                        a = pass ? fmaf(d, d, a) : a + d;
                    }
                a = sum8_dpp(a);
                if ((lane & 7) == 0) lnx[pass][wave][8 * q + rq] = a;
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                float t = 0.f;
#pragma unroll
                for (int j = 0; j < WN; ++j) t += lnx[pass][g0 + j][8 * q + rq];
                if (pass) rsd[q] = rsqrtf(t * (1.f / N) + lnf.eps);
                else mu[q] = t * (1.f / N);
            }
        }
        const auto rs_ln = buf_rsrc(lnf.out + m0 * N, (M - m0) * N * 2);
        const int cc = 4 * (lane & 7);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int n0 = 32 * (wn + WN * tile_of(i));
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (yk[i][q][e] - mu[q]) * rsd[q] * lg[i][e] + lb[i][e];
                buf_st4bf(rs_ln, (unsigned)((8 * q + rq) * N + n0 + cc) * 2, o);
            }
        }
        if (wn == 0 && (lane & 7) == 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                lnf.mean[m0 + 8 * q + rq] = mu[q];
                lnf.rstd[m0 + 8 * q + rq] = rsd[q];
            }
        }
    }
    if constexpr (EPI == WS_LNBWD) {
        // lane (r, h) holds dh of tokens r (t = 0) and 32 + r (t = 1), features
        // 32 nt(i) + 8 g + 4 h + e of its tiles i.  Pass 1: xhat, g = dh gamma, the token sums of g and
        // g xhat (lane -> half pair by a shuffle -> the 4 waves through LDS in wave order) and the
        // column partials of dh xhat / dh over the 64 tokens.  Pass 2: dx.
        constexpr int C = N;
        const auto rs_x = buf_rsrc(ln.x + m0 * C, (M - m0) * C * 4);
        const auto rs_r = buf_rsrc(ln.dres ? ln.dres + m0 * C : nullptr, ln.dres ? (M - m0) * C * 4 : 0);
        float mu[2], rs[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            mu[t] = ln.mean[m0 + 32 * t + r];
            rs[t] = ln.rstd[m0 + 32 * t + r];
        }
        float xh[NT][2][16], gam[NT][16];
        float rv2[NT][2][16];
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int n0 = 32 * (wn + WN * tile_of(i));
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                load4(ln.gamma + n0 + 8 * g + 4 * h, gam[i] + 4 * g);
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const unsigned off = (unsigned)((32 * t + r) * C + n0 + 8 * g + 4 * h) * 4;
                    buf_ld4(rs_x, off, xh[i][t] + 4 * g);
                    buf_ld4(rs_r, off, rv2[i][t] + 4 * g);
                }
            }
        }
        float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
        float dgc[NT][16], dbc[NT][16];
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                dgc[i][j] = 0.f;
                dbc[i][j] = 0.f;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const float dh = keep[i][t][j];
                    const float x_h = (xh[i][t][j] - mu[t]) * rs[t];
                    xh[i][t][j] = x_h;
                    const float gg = dh * gam[i][j];
                    s1[t] += gg;
                    s2[t] += gg * x_h;
                    dgc[i][j] += dh * x_h;
                    dbc[i][j] += dh;
                }
            }
        float* lnx = ep_all;   // [4 waves][2 sums][64 tokens]
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            s1[t] += __shfl_xor(s1[t], 32, 64);
            s2[t] += __shfl_xor(s2[t], 32, 64);
            if (h == 0) {
                lnx[(wave * 2 + 0) * 64 + 32 * t + r] = s1[t];
                lnx[(wave * 2 + 1) * 64 + 32 * t + r] = s2[t];
            }
        }
        __syncthreads();
        float S1[2], S2[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            S1[t] = S2[t] = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                S1[t] += lnx[(w * 2 + 0) * 64 + 32 * t + r];
                S2[t] += lnx[(w * 2 + 1) * 64 + 32 * t + r];
            }
            S1[t] *= 1.f / C;
            S2[t] *= 1.f / C;
        }
        const auto rs_dx = buf_rsrc(ln.dx + m0 * C, (M - m0) * C * 4);
        const auto rs_dxb = buf_rsrc(ln.dxb + m0 * C, (M - m0) * C * 2);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int n0 = 32 * (wn + WN * tile_of(i));
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = 4 * g + e;
                        o[e] = rs[t] * (keep[i][t][j] * gam[i][j] - S1[t] - xh[i][t][j] * S2[t]) + rv2[i][t][j];
                    }
                    const unsigned off = (unsigned)((32 * t + r) * C + n0 + 8 * g + 4 * h);
                    buf_st4(rs_dx, off * 4, o);
                    buf_st4bf(rs_dxb, off * 2, o);
                }
        }
        // column partials: the 32 token lanes of each half (xor tree), then lanes r = 0 write the row
#pragma unroll
        for (int o = 1; o < 32; o <<= 1)
#pragma unroll
            for (int i = 0; i < NT; ++i)
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    dgc[i][j] += __shfl_xor(dgc[i][j], o, 64);
                    dbc[i][j] += __shfl_xor(dbc[i][j], o, 64);
                }
        if (r == 0) {
            float* prow = ln.part + (size_t)blockIdx.x * 2 * C;
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const int n0 = 32 * (wn + WN * tile_of(i));
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    store4(prow + n0 + 8 * g + 4 * h, dgc[i] + 4 * g);
                    store4(prow + C + n0 + 8 * g + 4 * h, dbc[i] + 4 * g);
                }
            }
        }
    }
}

template <int K, int N, int EPI, typename TOUT, int F8 = 0>
int ws_launch(long M, const bf16* X, int ldx, const bf16* Wf, const float* bias, const float* resid, void* out,
              hipStream_t st, const WsLn& ln = WsLn{}, const WsLnF& lnf = WsLnF{}, const float* wsc = nullptr) {
    constexpr int NS = F8 ? 1 : ws_ns(K, N, EPI);
    gemm_ws_kernel<K, N, EPI, TOUT, NS, F8><<<dim3((unsigned)(M / ws_tokens(N)), NS), 256, 0, st>>>(
        M, X, ldx, Wf, bias, resid, (TOUT*)out, ln, lnf, wsc);
    return check_launch("gemm_ws");
}

// the shapes instantiated: (K, N) of the CSWinBlock qkv / proj Linears at C = 64 / 128 / 256 and their
// input gradients (qkv^T: K = 3C, N = C).  Not (192, 64), the C = 64 qkv input gradient: 82.4 vs 67.7
// us/step on gemm4 in the step (profiles/r07q_ws_s1.txt); the C = 64 forward 60.7 vs 73.0.
#define WS_SHAPES(X_) X_(128, 384) X_(256, 768) X_(384, 128) X_(768, 256) X_(128, 128) X_(256, 256) \
    X_(64, 192) X_(64, 64)

}  // namespace

int gemm_ws_supported(long M, int N, int K, int resid, int out_dtype) {
    if (M < ws_tokens(N) || M % ws_tokens(N) || M > (1L << 30)) return 0;
    if (resid && out_dtype != CSU_F32) return 0;
    if (out_dtype != CSU_F32 && out_dtype != CSU_BF16) return 0;
#define WS_HAS(KK, NN) if (K == KK && N == NN) return 1;
    WS_SHAPES(WS_HAS)
#undef WS_HAS
    return 0;
}

int gemm_ws_run(long M, int N, int K, const bf16* X, int ldx, const bf16* Wf, const float* bias, const float* resid,
                int out_dtype, void* out, hipStream_t st) {
#define WS_GO(KK, NN)                                                                                             \
    if (K == KK && N == NN) {                                                                                     \
        if (resid) return ws_launch<KK, NN, WS_RESID, float>(M, X, ldx, Wf, bias, resid, out, st);          \
        if (out_dtype == CSU_F32) return ws_launch<KK, NN, WS_PLAIN, float>(M, X, ldx, Wf, bias, nullptr, out, st); \
        return ws_launch<KK, NN, WS_PLAIN, bf16>(M, X, ldx, Wf, bias, nullptr, out, st);                    \
    }
    WS_SHAPES(WS_GO)
#undef WS_GO
    return fail(CSU_E_ARG, "gemm_ws: shape not instantiated");
}

// e4m3 weights: mode 1 (x W^T, per-column scales in the epilogue) or 2 (dy W through the W^T fragments,
// per-k scales on the token panel); any epilogue of gemm_ws_run
int gemm_ws_e4m3_run(long M, int N, int K, const bf16* X, int ldx, const uint8_t* Wq, const float* wsc, int mode,
                     const float* bias, const float* resid, int out_dtype, void* out, hipStream_t st) {
    const bf16* W = reinterpret_cast<const bf16*>(Wq);
#define WS_GO8(KK, NN, MODE)                                                                                      \
    if (K == KK && N == NN && mode == MODE) {                                                                     \
        if (resid) return ws_launch<KK, NN, WS_RESID, float, MODE>(M, X, ldx, W, bias, resid, out, st, {}, {}, wsc); \
        if (out_dtype == CSU_F32)                                                                                 \
            return ws_launch<KK, NN, WS_PLAIN, float, MODE>(M, X, ldx, W, bias, nullptr, out, st, {}, {}, wsc);   \
        return ws_launch<KK, NN, WS_PLAIN, bf16, MODE>(M, X, ldx, W, bias, nullptr, out, st, {}, {}, wsc);        \
    }
#define WS_GO8B(KK, NN) WS_GO8(KK, NN, 1) WS_GO8(KK, NN, 2)
    WS_SHAPES(WS_GO8B)
#undef WS_GO8B
#undef WS_GO8
    return fail(CSU_E_ARG, "gemm_ws_e4m3: shape not instantiated");
}

// the LayerNorm (norm2) epilogue: proj + residual, K = N = C
int gemm_ws_ln_supported(long M, int N, int K) {
    if (M < ws_tokens(N) || M % ws_tokens(N) || M > (1L << 30)) return 0;
    return K == N && (N == 64 || N == 128 || N == 256);
}

int gemm_ws_ln_run(long M, int N, const bf16* X, int ldx, const bf16* Wf, const float* bias, const float* resid, float* out,
                   const WsLnF& lnf, hipStream_t st, const float* wsc = nullptr) {
    if (wsc) {   // e4m3 weight fragments, per-column scales
        if (N == 64) return ws_launch<64, 64, WS_RESID_LN, float, 1>(M, X, ldx, Wf, bias, resid, out, st, WsLn{}, lnf, wsc);
        if (N == 128) return ws_launch<128, 128, WS_RESID_LN, float, 1>(M, X, ldx, Wf, bias, resid, out, st, WsLn{}, lnf, wsc);
        if (N == 256) return ws_launch<256, 256, WS_RESID_LN, float, 1>(M, X, ldx, Wf, bias, resid, out, st, WsLn{}, lnf, wsc);
        return fail(CSU_E_ARG, "gemm_ws_ln_e4m3: shape not instantiated");
    }
    if (N == 64) return ws_launch<64, 64, WS_RESID_LN, float>(M, X, ldx, Wf, bias, resid, out, st, WsLn{}, lnf);
    if (N == 128) return ws_launch<128, 128, WS_RESID_LN, float>(M, X, ldx, Wf, bias, resid, out, st, WsLn{}, lnf);
    if (N == 256) return ws_launch<256, 256, WS_RESID_LN, float>(M, X, ldx, Wf, bias, resid, out, st, WsLn{}, lnf);
    return fail(CSU_E_ARG, "gemm_ws_ln: shape not instantiated");
}

// the LayerNorm-backward epilogue: the qkv input gradients at C = 128 / 256
int gemm_ws_lnbwd_supported(long M, int N, int K) {
    if (M < WS_BM || M % WS_BM || M > (1L << 30)) return 0;
    return (K == 384 && N == 128) || (K == 768 && N == 256);
}

int gemm_ws_lnbwd_run(long M, int N, int K, const bf16* dy, const bf16* Wtf, const WsLn& ln, hipStream_t st) {
    if (K == 384 && N == 128) return ws_launch<384, 128, WS_LNBWD, float>(M, dy, K, Wtf, nullptr, nullptr, nullptr, st, ln);
    if (K == 768 && N == 256) return ws_launch<768, 256, WS_LNBWD, float>(M, dy, K, Wtf, nullptr, nullptr, nullptr, st, ln);
    return fail(CSU_E_ARG, "gemm_ws_lnbwd: shape not instantiated");
}

// ---- fragment-ordered weight layout: 16-B chunk q (k 8q..8q+7) of row n of a bf16 (rows x cols)
// matrix -> chunk ((n / 32) * (cols / 16) + q / 2) * 64 + n % 32 + 32 (q % 2) of the output
__global__ __launch_bounds__(256) void frag_layout_kernel(const csu_frag_item* __restrict__ items, int count) {
    const long g = (long)blockIdx.x * 256 + threadIdx.x;   // global 16-B chunk index
    int lo = 0, hi = count - 1;
    while (lo < hi) {   // last item with chunk0 <= g
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].chunk0 <= g) lo = mid; else hi = mid - 1;
    }
    const csu_frag_item it = items[lo];
    const long q = g - it.chunk0;
    const int qc = it.cols / 8;
    if (q < 0 || q >= (long)it.rows * qc) return;
    const int n = (int)(q / qc), k8 = (int)(q % qc);
    const long dst = (((long)(n >> 5) * (it.cols >> 4) + (k8 >> 1)) * 64 + (n & 31) + 32 * (k8 & 1)) * 8;
    *reinterpret_cast<u32x4*>((bf16*)it.dst + dst) = *reinterpret_cast<const u32x4*>((const bf16*)it.src + q * 8);
}

// ---- e4m3 fragment order (csu_frag8_layout_batch): output matrix O (rows x cols) = src (transpose 0)
// or src^T (transpose 1) of an e4m3 (N x K) matrix; 8-byte chunk (row, c8 = col / 8) of O goes to chunk
// ((row / 32) * (cols / 16) + c8 / 2) * 64 + row % 32 + 32 (c8 % 2).  One thread per 8 x 8 byte block of
// the source: 8 rows x 8 bytes loaded, written as 8 chunks (transposed in registers for mode 1).
__device__ __forceinline__ long frag8_chunk(int row, int c8, int cols) {
    return ((long)(row >> 5) * (cols >> 4) + (c8 >> 1)) * 64 + (row & 31) + 32 * (c8 & 1);
}
__global__ __launch_bounds__(256) void frag8_layout_kernel(const csu_frag8_item* __restrict__ items, int count) {
    const long g = (long)blockIdx.x * 256 + threadIdx.x;   // global 8x8 block index
    int lo = 0, hi = count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (items[mid].block0 <= g) lo = mid; else hi = mid - 1;
    }
    const csu_frag8_item it = items[lo];
    const long b = g - it.block0;
    const int kb = it.K / 8;   // source column blocks
    if (b < 0 || b >= (long)(it.N / 8) * kb) return;
    const int n0 = 8 * (int)(b / kb), k0 = 8 * (int)(b % kb);
    const uint8_t* src = reinterpret_cast<const uint8_t*>(it.src);
    u32x2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const u32x2*>(src + (long)(n0 + i) * it.K + k0);
    u32x2* dst = reinterpret_cast<u32x2*>(it.dst);
    if (!it.transpose) {   // O = src (N x K): chunk (n0 + i, k0 / 8)
#pragma unroll
        for (int i = 0; i < 8; ++i) dst[frag8_chunk(n0 + i, k0 >> 3, it.K)] = v[i];
    } else {               // O = src^T (K x N): chunk (k0 + j, n0 / 8) = bytes src[n0 + i][k0 + j], i = 0..7
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            unsigned lo4 = 0, hi4 = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                lo4 |= ((v[i][j >> 2] >> (8 * (j & 3))) & 0xffu) << (8 * i);
                hi4 |= ((v[4 + i][j >> 2] >> (8 * (j & 3))) & 0xffu) << (8 * i);
            }
            dst[frag8_chunk(k0 + j, n0 >> 3, it.N)] = u32x2{lo4, hi4};
        }
    }
}

}  // namespace csu

using namespace csu;

extern "C" int csu_gemm_ws_supported(long M, int N, int K, int resid, int out_dtype) {
    return gemm_ws_supported(M, N, K, resid, out_dtype);
}

extern "C" int csu_gemm_ws(long M, int N, int K, const void* x, int ldx, const void* w_frag, const float* bias,
                           const float* resid, int out_dtype, void* out, void* stream) {
    if (!x || !w_frag || !out) return fail(CSU_E_ARG, "gemm_ws: null pointer");
    if (!gemm_ws_supported(M, N, K, resid != nullptr, out_dtype)) return fail(CSU_E_ARG, "gemm_ws: unsupported shape");
    if (ldx < K || ldx % 8) return fail(CSU_E_ARG, "gemm_ws: ldx must be >= K and a multiple of 8");
    return gemm_ws_run(M, N, K, (const bf16*)x, ldx, (const bf16*)w_frag, bias, resid, out_dtype, out, as_stream(stream));
}

extern "C" int csu_gemm_ws_e4m3(long M, int N, int K, const void* x, int ldx, const void* w_frag8, const float* w_scale,
                                int scale_mode, const float* bias, const float* resid, int out_dtype, void* out,
                                void* stream) {
    if (!x || !w_frag8 || !w_scale || !out) return fail(CSU_E_ARG, "gemm_ws_e4m3: null pointer");
    if (scale_mode != 1 && scale_mode != 2) return fail(CSU_E_ARG, "gemm_ws_e4m3: scale_mode 1 (x W^T) or 2 (dy W)");
    if (!gemm_ws_supported(M, N, K, resid != nullptr, out_dtype)) return fail(CSU_E_ARG, "gemm_ws_e4m3: unsupported shape");
    if (ldx < K || ldx % 8) return fail(CSU_E_ARG, "gemm_ws_e4m3: ldx must be >= K and a multiple of 8");
    return gemm_ws_e4m3_run(M, N, K, (const bf16*)x, ldx, (const uint8_t*)w_frag8, w_scale, scale_mode, bias, resid,
                            out_dtype, out, as_stream(stream));
}

extern "C" int csu_gemm_ws_ln_e4m3(long M, int C, const void* x, int ldx, const void* w_frag8, const float* w_scale,
                                   const float* bias, const float* resid, float* out, const float* gamma, const float* beta,
                                   float eps, void* ln_out, float* mean, float* rstd, void* stream) {
    if (!x || !w_frag8 || !w_scale || !resid || !out || !gamma || !beta || !ln_out || !mean || !rstd)
        return fail(CSU_E_ARG, "gemm_ws_ln_e4m3: null pointer");
    if (!gemm_ws_ln_supported(M, C, C)) return fail(CSU_E_ARG, "gemm_ws_ln_e4m3: unsupported shape");
    if (ldx < C || ldx % 8) return fail(CSU_E_ARG, "gemm_ws_ln_e4m3: ldx must be >= C and a multiple of 8");
    const WsLnF lnf{gamma, beta, eps, (bf16*)ln_out, mean, rstd};
    return gemm_ws_ln_run(M, C, (const bf16*)x, ldx, (const bf16*)w_frag8, bias, resid, out, lnf, as_stream(stream), w_scale);
}

extern "C" int csu_frag8_layout_batch(const csu_frag8_item* items, int count, long total_blocks, void* stream) {
    if (!items || count < 1 || total_blocks < 1) return fail(CSU_E_ARG, "frag8_layout: empty item table");
    frag8_layout_kernel<<<(unsigned)((total_blocks + 255) / 256), 256, 0, as_stream(stream)>>>(items, count);
    return check_launch("frag8_layout");
}

extern "C" int csu_gemm_ws_lnbwd_supported(long M, int C, int K) { return gemm_ws_lnbwd_supported(M, C, K); }

extern "C" int csu_gemm_ws_lnbwd(long M, int C, int K, const void* dy, const void* wt_frag, const float* x,
                                 const float* gamma, const float* mean, const float* rstd, const float* dres, float* dx,
                                 void* dx_bf16, float* part, void* stream) {
    if (!dy || !wt_frag || !x || !gamma || !mean || !rstd || !dx || !dx_bf16 || !part)
        return fail(CSU_E_ARG, "gemm_ws_lnbwd: null pointer");
    if (!gemm_ws_lnbwd_supported(M, C, K)) return fail(CSU_E_ARG, "gemm_ws_lnbwd: unsupported shape");
    const WsLn ln{x, gamma, mean, rstd, dres, dx, (bf16*)dx_bf16, part};
    return gemm_ws_lnbwd_run(M, C, K, (const bf16*)dy, (const bf16*)wt_frag, ln, as_stream(stream));
}

extern "C" int csu_gemm_ws_ln_supported(long M, int C, int K) { return gemm_ws_ln_supported(M, C, K); }

extern "C" int csu_gemm_ws_ln(long M, int C, const void* x, int ldx, const void* w_frag, const float* bias,
                              const float* resid, float* out, const float* gamma, const float* beta, float eps,
                              void* ln_out, float* mean, float* rstd, void* stream) {
    if (!x || !w_frag || !resid || !out || !gamma || !beta || !ln_out || !mean || !rstd)
        return fail(CSU_E_ARG, "gemm_ws_ln: null pointer");
    if (!gemm_ws_ln_supported(M, C, C)) return fail(CSU_E_ARG, "gemm_ws_ln: unsupported shape");
    if (ldx < C || ldx % 8) return fail(CSU_E_ARG, "gemm_ws_ln: ldx must be >= C and a multiple of 8");
    const WsLnF lnf{gamma, beta, eps, (bf16*)ln_out, mean, rstd};
    return gemm_ws_ln_run(M, C, (const bf16*)x, ldx, (const bf16*)w_frag, bias, resid, out, lnf, as_stream(stream));
}

extern "C" int csu_frag_layout_batch(const csu_frag_item* items, int count, long total_chunks, void* stream) {
    if (!items || count < 1 || total_chunks < 1) return fail(CSU_E_ARG, "frag_layout: empty item table");
    frag_layout_kernel<<<(unsigned)((total_chunks + 255) / 256), 256, 0, as_stream(stream)>>>(items, count);
    return check_launch("frag_layout");
}
