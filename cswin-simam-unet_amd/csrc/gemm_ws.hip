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
#include "common.hpp"

namespace csu {
namespace {

enum { WS_PLAIN = 0, WS_RESID = 1 };

constexpr int WS_BM = 64;   // tokens per workgroup
constexpr bool WS_ROT = true;

constexpr int ws_unit(int ks) {
    for (int u = 16; u > 1; --u)
        if (ks % u == 0) return u;
    return 1;
}

template <int K, int NT, int EPI, typename TOUT>
__global__ __launch_bounds__(256) void gemm_ws_kernel(long M, const bf16* __restrict__ X, int ldx,
                                                      const bf16* __restrict__ Wf, const float* __restrict__ bias,
                                                      const float* __restrict__ resid, TOUT* __restrict__ out) {
    constexpr int N = 128 * NT;
    constexpr int KS = K / 16;                     // k-steps
    constexpr int UK = ws_unit(KS);                // k-steps per unit (a divisor of KS, <= 16)
    constexpr int CH = KS / UK;                    // units per tile
    static_assert(CH * UK == KS, "unit size");
    constexpr int U = NT * CH;                     // units per wave
    constexpr bool XREG = K <= 256;                // B fragments held in registers
    constexpr int XS = K + 8;                      // LDS row stride of the token panel (bf16)
    constexpr int ES = 36;                         // fp32 row stride of the epilogue region
    __shared__ __attribute__((aligned(16))) bf16 xs[WS_BM * XS];
    __shared__ __attribute__((aligned(16))) float ep_all[4 * WS_BM * ES];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * WS_BM;
    float* ep = ep_all + wave * WS_BM * ES;

    // tile order rotated per workgroup (its index within the XCD: ids x, x + 8, ... run on XCD x), so
    // the CUs of an XCD do not all read the same weight lines at the same moment
    const int rot = WS_ROT ? (int)((blockIdx.x >> 3) % NT) : 0;
    auto tile_of = [&](int i) { return i + rot < NT ? i + rot : i + rot - NT; };
    bf16x8 wf[2][UK];
    auto wload1 = [&](int u, int s) {   // k-step s of unit u of this wave into buffer u & 1
        const int nt = wave + 4 * tile_of(u / CH), ks = (u % CH) * UK + s;
        wf[u & 1][s] = *reinterpret_cast<const bf16x8*>(Wf + ((long)(nt * KS + ks) * 64 + lane) * 8);
    };
#pragma unroll
    for (int s = 0; s < UK; ++s) wload1(0, s);
    __builtin_amdgcn_sched_barrier(0);
    // token panel -> LDS (16-B pieces, row-contiguous)
    constexpr int PR = K / 8;   // pieces per row
#pragma unroll
    for (int i = 0; i < WS_BM * PR / 256; ++i) {
        const int p = threadIdx.x + 256 * i, row = p / PR, c = 8 * (p % PR);
        *reinterpret_cast<bf16x8*>(xs + row * XS + c) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * ldx + c);
    }
    __syncthreads();
    bf16x8 xf[XREG ? 2 : 1][XREG ? KS : 1];
    if constexpr (XREG) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < KS; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(xs + (32 * t + r) * XS + 16 * s + 8 * h);
    }
    __builtin_amdgcn_sched_barrier(0);

    f32x16 a0 = f32x16{}, a1 = f32x16{};
    const auto rs_b = buf_rsrc(bias, bias ? (long)N * 4 : 0);   // null bias: loads read 0
    constexpr bool BF = sizeof(TOUT) == 2;
    // epilogue loads of a tile are issued at the start of its last unit, BEFORE the next unit's
    // weight loads: vmcnt counts in issue order, so waiting for them then does not wait for the prefetch
    float bv[8], rv[8][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int c = u % CH;
        if (c == CH - 1) {
            const int n0 = 32 * (wave + 4 * tile_of(u / CH));
            if constexpr (BF) {
                const int cc = 8 * (lane & 3);
                buf_ld4(rs_b, (unsigned)(n0 + cc) * 4, bv);
                buf_ld4(rs_b, (unsigned)(n0 + cc + 4) * 4, bv + 4);
            } else {
                const int cc = 4 * (lane & 7);
                buf_ld4(rs_b, (unsigned)(n0 + cc) * 4, bv);
                if constexpr (EPI == WS_RESID) {
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
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[u & 1][s], b0, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[u & 1][s], b1, a1, 0, 0, 0);
            if (u + 1 < U) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // one weight load
            if constexpr (!XREG) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // two fragment reads
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                 // two MFMAs
        }
        __builtin_amdgcn_sched_barrier(0);
        if (c != CH - 1) continue;
        // ---- epilogue of tile nt: acc element (token 32 t + r, feature 32 nt + 8 g + 4 h + e)
        const int nt = wave + 4 * tile_of(u / CH);
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
                for (int e = 0; e < 8; ++e) v[e] += bv[e];
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
                    v[e] += bv[e];
                    if constexpr (EPI == WS_RESID) v[e] += rv[q][e];
                }
                buf_st4(rs_out, (unsigned)(row * N + n0 + cc) * 4, v);
            }
        }
        a0 = f32x16{};
        a1 = f32x16{};
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int K, int NT, int EPI, typename TOUT>
int ws_launch(long M, const bf16* X, int ldx, const bf16* Wf, const float* bias, const float* resid, void* out,
              hipStream_t st) {
    gemm_ws_kernel<K, NT, EPI, TOUT><<<dim3((unsigned)(M / WS_BM)), 256, 0, st>>>(M, X, ldx, Wf, bias, resid, (TOUT*)out);
    return check_launch("gemm_ws");
}

// the shapes instantiated: (K, N) of the CSWinBlock qkv / proj Linears at C = 128 / 256 and their
// input gradients (qkv^T: K = 3C, N = C)
#define WS_SHAPES(X_) X_(128, 384) X_(256, 768) X_(384, 128) X_(768, 256) X_(128, 128) X_(256, 256)

}  // namespace

int gemm_ws_supported(long M, int N, int K, int resid, int out_dtype) {
    if (M < WS_BM || M % WS_BM || M > (1L << 30)) return 0;
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
        if (resid) return ws_launch<KK, NN / 128, WS_RESID, float>(M, X, ldx, Wf, bias, resid, out, st);          \
        if (out_dtype == CSU_F32) return ws_launch<KK, NN / 128, WS_PLAIN, float>(M, X, ldx, Wf, bias, nullptr, out, st); \
        return ws_launch<KK, NN / 128, WS_PLAIN, bf16>(M, X, ldx, Wf, bias, nullptr, out, st);                    \
    }
    WS_SHAPES(WS_GO)
#undef WS_GO
    return fail(CSU_E_ARG, "gemm_ws: shape not instantiated");
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

extern "C" int csu_frag_layout_batch(const csu_frag_item* items, int count, long total_chunks, void* stream) {
    if (!items || count < 1 || total_chunks < 1) return fail(CSU_E_ARG, "frag_layout: empty item table");
    frag_layout_kernel<<<(unsigned)((total_chunks + 255) / 256), 256, 0, as_stream(stream)>>>(items, count);
    return check_launch("frag_layout");
}
