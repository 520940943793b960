// fp8-e4m3 token GEMM for gfx950 (BASELINE config 5: "fp8 MFMA weights", 1024x1024 B4).
//
//   out[m][n] = bf16( sa[m] * sw[n] * sum_k A[m][k] W[n][k] + bias[n] )
//
// A = e4m3 activations with one fp32 scale per token (written by the LayerNorm that produces them,
// csu_layernorm_fwd_fp8: the producer holds the whole token row, so the per-token amax is free),
// W = e4m3 weights with one scale per output row (csu_quant_e4m3_batch).  The products run on
// v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3, unit block scales: the per-token / per-row scales
// are applied once, in the fp32 epilogue), fp32 accumulation.  Operand bytes are half the bf16
// GEMM's: A and W read once as 1 B / element.
//
// Tile 128 tokens x 64 features per 256-thread workgroup; wave (wm, wn) = 64 tokens x 32 features =
// two 32x32 MFMA tiles.  Weights are the MFMA A operand (rows = features), tokens the B operand
// (lane = token), so each lane ends with 16 features of one token: 8-B bf16 stores of 4 consecutive
// features.  K in steps of 64 (one MFMA k-step): the next step's tiles are loaded into registers
// while the current one is multiplied from LDS (two LDS buffers, one barrier per step).  LDS rows
// are 64 B + 16 B pad: the 16-lane groups of a ds_read_b128 hit 16 distinct 4-bank ranges.
// Operand lane map of the 32x32x64 f8 form: lane half h holds k = 16 h + 0..15 in bytes 0..15 and
// k = 32 + 16 h + 0..15 in bytes 16..31 (tools/probes/mx_layout_probe.hip).  Here both operands take
// the same 32 contiguous bytes per lane and the block scales are unit, so the contraction is exact
// whatever the hardware's k order.
#include "common.hpp"

namespace csu {
namespace {

constexpr int BM = 128, BN = 64, KS = 64, NT = 256;
constexpr int RS = KS + 16;                 // LDS row stride (bytes)
typedef int i32x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(NT) void fp8_gemm_kernel(long M, int N, int K, const uint8_t* __restrict__ A,
                                                      const float* __restrict__ sa, const uint8_t* __restrict__ W,
                                                      const float* __restrict__ sw, const float* __restrict__ bias,
                                                      bf16* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t As[2][BM * RS];
    __shared__ __attribute__((aligned(16))) uint8_t Ws[2][BN * RS];
    const int ntn = N / BN;
    const long id = xcd_tile(blockIdx.x, gridDim.x);      // n-tiles of one token panel on one XCD
    const long m0 = (id / ntn) * BM;
    const int n0 = (int)(id % ntn) * BN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = wave >> 1, wn = wave & 1;
    const long rows = M - m0;
    const auto rsA = buf_rsrc(A + m0 * K, rows * K);
    const auto rsW = buf_rsrc(W + (long)n0 * K, (long)BN * K);
    // global -> LDS: A tile 128 x 64 B (2 x 16 B per thread), W tile 64 x 64 B (1 x 16 B per thread)
    const int ar0 = threadIdx.x >> 2, ac = (threadIdx.x & 3) * 16;   // rows ar0, ar0 + 64
    const int wr = threadIdx.x >> 2;
    u32x4 ra[2], rw;
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = ar0 + 64 * i;
            ra[i] = __builtin_amdgcn_raw_buffer_load_b128(rsA, row < rows ? (unsigned)(row * K + k0 + ac) : kOOB, 0, 0);
        }
        rw = __builtin_amdgcn_raw_buffer_load_b128(rsW, (unsigned)(wr * K + k0 + ac), 0, 0);
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) *reinterpret_cast<u32x4*>(&As[buf][(ar0 + 64 * i) * RS + ac]) = ra[i];
        *reinterpret_cast<u32x4*>(&Ws[buf][wr * RS + ac]) = rw;
    };
    f32x16 acc[2] = {f32x16{}, f32x16{}};
    const int nk = K / KS;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load((kt + 1) * KS);
        i32x8 wf, tf[2];
        {
            const uint8_t* p = &Ws[buf][(wn * 32 + r) * RS + 32 * h];
            const u32x4 lo = *reinterpret_cast<const u32x4*>(p), hi = *reinterpret_cast<const u32x4*>(p + 16);
            wf = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint8_t* p = &As[buf][(wm * 64 + t * 32 + r) * RS + 32 * h];
            const u32x4 lo = *reinterpret_cast<const u32x4*>(p), hi = *reinterpret_cast<const u32x4*>(p + 16);
            tf[t] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)   // D[feature][token] += W A^T (e4m3 x e4m3, unit block scales)
            acc[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf, tf[t], acc[t], 0, 0, 0, 0, 0, 0);
        if (kt + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    // epilogue: lane = token m0 + wm*64 + t*32 + r, features n0 + wn*32 + crow(i, h)
    const auto rsO = buf_rsrc(out + m0 * N, rows * N * 2);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int tok = wm * 64 + t * 32 + r;
        const bool ok = tok < rows;
        const float s_tok = ok ? sa[m0 + tok] : 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = n0 + wn * 32 + 8 * g + 4 * h;
            const f32x4 swv = *reinterpret_cast<const f32x4*>(sw + n);
            const f32x4 bv = bias ? *reinterpret_cast<const f32x4*>(bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[t][4 * g + e] * (swv[e] * s_tok) + bv[e];
            buf_st4bf(rsO, ok ? (unsigned)(tok * N + n) * 2 : kOOB, v);
        }
    }
}

// e4m3 (per-row fp32 scale) -> bf16 rows: the backward's copy of a quantised activation (the weight
// gradient dW = dY^T X uses the X the forward multiplied)
__global__ __launch_bounds__(NT) void dequant_rows_kernel(long rows, int cols, const uint8_t* __restrict__ q,
                                                          const float* __restrict__ s, bf16* __restrict__ out) {
    const long i = ((long)blockIdx.x * NT + threadIdx.x) * 8;
    const long n = rows * cols;
    if (i >= n) return;
    const long row = i / cols;   // cols % 8 == 0: the 8 elements share a row
    const float sc = s[row];
    const u32x2 v = *reinterpret_cast<const u32x2*>(q + i);
    float f[8];
#pragma unroll
    for (int w = 0; w < 2; ++w) {
        const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[w], false);
        const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[w], true);
        f[4 * w] = lo[0] * sc;
        f[4 * w + 1] = lo[1] * sc;
        f[4 * w + 2] = hi[0] * sc;
        f[4 * w + 3] = hi[1] * sc;
    }
    store8(out + i, f);
}

}  // namespace
}  // namespace csu

using namespace csu;

namespace csu {
int gemm4_fp8_run(long M, int N, int K, const uint8_t* A, const float* sa, const uint8_t* W, const float* sw,
                  const float* bias, bf16* out, hipStream_t st);
}

extern "C" int csu_fp8_gemm(long M, int N, int K, const void* aq, const float* sa, const void* wq, const float* sw,
                            const float* bias, void* out, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !aq || !sa || !wq || !sw || !out) return fail(CSU_E_ARG, "fp8_gemm: bad arguments");
    if (N % BN || K % KS) return fail(CSU_E_UNSUPPORTED, "fp8_gemm: N % 64 == 0 and K % 64 == 0 required");
    if (M * (long)K > 0x7fffffffL || M * (long)N * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "fp8_gemm: tensor exceeds 2 GB");
    // K % 128 == 0: the persistent LDS-DMA design of the bf16 token GEMM (gemm4.hip, F8); K = 64 (the
    // stage-1 qkv at C = 64): the register-prefetch tile below
    if (K % 128 == 0) return gemm4_fp8_run(M, N, K, (const uint8_t*)aq, sa, (const uint8_t*)wq, sw, bias, (bf16*)out,
                                           as_stream(stream));
    const long tiles = ((M + BM - 1) / BM) * (N / BN);
    fp8_gemm_kernel<<<(unsigned)tiles, NT, 0, as_stream(stream)>>>(M, N, K, (const uint8_t*)aq, sa, (const uint8_t*)wq, sw,
                                                                   bias, (bf16*)out);
    return check_launch("fp8_gemm");
}

extern "C" int csu_dequant_e4m3_rows(long rows, int cols, const void* q, const float* scale, void* out, void* stream) {
    if (rows < 1 || cols < 8 || cols % 8 || !q || !scale || !out) return fail(CSU_E_ARG, "dequant_e4m3_rows: bad arguments");
    const long n = rows * cols / 8;
    dequant_rows_kernel<<<(unsigned)((n + NT - 1) / NT), NT, 0, as_stream(stream)>>>(rows, cols, (const uint8_t*)q, scale,
                                                                                    (bf16*)out);
    return check_launch("dequant_e4m3_rows");
}
