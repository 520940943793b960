// Fused Mlp + residual for gfx950: fc1 -> GELU -> fc2 with the 4C-wide hidden layer kept on chip.
//
//   forward   y  = res + fc2(gelu(fc1(x)))                     (Mlp cswin:180-196, residual cswin:368)
//   backward  h  = fc1(x) (recomputed), g = gelu(h)
//             dH = (dY W2) * gelu'(h),  dX = dH W1             (the two input-gradient GEMMs + GELU')
//             writes dH and g for the weight-gradient GEMMs dW1 = dH^T x, dW2 = dY^T g
//
// The unfused form moves the hidden layer (M x 4C bf16) through HBM three times in the forward
// (h and gelu(h) written, gelu(h) read) and three more in the backward; here the forward reads x
// and res and writes y only, and the backward reads x and dY and writes dH, g and dX.
//
// Design (MI355X):
//  * one workgroup (4 waves) per 64-token panel.  Wave (t, u) owns tokens 32t..32t+31 and, of
//    every 64-feature hidden chunk j, the 32 features 32u..32u+31: GEMM1 H = W1_sub x^T (K = C),
//    GELU on the accumulator, GEMM2 y_u += W2_sub g^T (K = 32) into a C x 32 partial output.
//    The two hidden halves' partials are added through LDS once, at the end.
//  * the token operands (x, dY) are loaded once into registers as MFMA B fragments; the weights
//    stream through a two-stage LDS ring (W1 chunk [64][C] + W2 chunk [C][64] per stage,
//    buffer_load ... lds DMA issued one chunk ahead, one barrier per chunk).
//  * the hidden activations never leave registers: the accumulator of lane (r, h) holds token r,
//    features 16s+4h+0..3 and 16s+8+4h+0..3 of k-step s, which is used directly as the B operand
//    of the next GEMM with the SAME permutation of k applied to the A operand (two 8-B reads, or
//    two transposed reads, of the weight image instead of one 16-B read): a contraction does not
//    care about the order of k.
//  * XOR swizzle of the 16-B chunks of every weight image (applied to the DMA source address),
//    key = bit-reversal of the row: ds_read_b128 row reads and ds_read_b64_tr_b16 transposed
//    reads are both bank-conflict free.
//  * v_mfma_f32_32x32x16_bf16 with weights as the A operand: lane (r, h) of an accumulator holds
//    token r and 4 consecutive features per register group; bias / GELU / GELU' / residual are
//    elementwise on registers.
#include "lds_dma.hpp"
#include "rng.hpp"

#include <cstdlib>
#include <type_traits>

namespace csu {
namespace {

constexpr int MT = 256;   // threads (4 waves)

// Mlp dropout (cswin:190/193) and DropPath (cswin:368) of one launch: hidden mask on g = gelu(h)
// (site_hidden, element m * 4C + f), output mask (site_out, element m * C + c) and the per-sample
// DropPath scale row_scale[m / rows_per_sample] on the Mlp output before the residual add.
struct MlpDrop {
    const uint64_t* rng;
    unsigned site_h, site_o;
    float p;
    const float* row_scale;
    long rps;
};

constexpr int BM = 64;    // tokens per workgroup
constexpr int HC = 64;    // hidden features per chunk

// the permuted-k form (see header): k = image rows k0 + 4h + 0..3 and k0 + 8 + 4h + 0..3
template <int RB>
__device__ __forceinline__ bf16x8 ptrfrag(const bf16* img, int c0, int k0, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = k0 + 4 * (grp >> 1) + q;
    return cat8(tr4(img + moff<RB>(row, col)), tr4(img + moff<RB>(row + 8, col)));
}
// permuted-k row fragment: row `row` of the image, k = columns k0 + 4h + 0..3, k0 + 8 + 4h + 0..3
template <int RB>
__device__ __forceinline__ bf16x8 pfrag(const bf16* img, int row, int k0, int h) {
    const bf16x4 lo = *reinterpret_cast<const bf16x4*>(img + moff<RB>(row, k0 + 4 * h));
    const bf16x4 hi = *reinterpret_cast<const bf16x4*>(img + moff<RB>(row, k0 + 8 + 4 * h));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// B operand of k-step s2 from accumulator-resident activations v (16 per lane, accumulator order)
__device__ __forceinline__ bf16x8 pack_b(const float* v, int s2) {
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (bf16)v[8 * s2 + i];
    return b;
}

// token-operand B fragments of 32 rows (lane: row r, k = 16 s + 8 h .. + 7); rows past the end
// read as 0
template <int C>
__device__ __forceinline__ void load_bfrags(__amdgpu_buffer_rsrc_t rs, int tok, bool ok, int h, bf16x8* f) {
#pragma unroll
    for (int s = 0; s < C / 16; ++s) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (unsigned)(tok * C + 16 * s + 8 * h) * 2 : kOOB, 0, 0);
        __builtin_memcpy(&f[s], &v, 16);
    }
}

// Add the partner wave's partial sums for this wave's half of the C x 32 output: acc[TF] holds the
// wave's partial over its hidden half for all C features; afterwards acc[U*HT .. U*HT+HT-1] hold
// the full sums of features [U*C/2, (U+1)*C/2).  xch: 4 x HT x 16 x 64 floats of LDS.
template <int C, int U>
__device__ __forceinline__ void exchange_half(f32x16* acc, float* xch, int wave, int lane) {
    constexpr int HT = C / 64;
#pragma unroll
    for (int q = 0; q < HT; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) xch[((wave * HT + q) * 16 + e) * 64 + lane] = acc[(1 - U) * HT + q][e];
    lds_sync();
    const int partner = wave ^ 1;
#pragma unroll
    for (int q = 0; q < HT; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[U * HT + q][e] += xch[((partner * HT + q) * 16 + e) * 64 + lane];
}

// A0: index of the first of the HT accumulator tiles holding features [U C/2, (U+1) C/2)
template <int C, int U, bool DROP, int A0 = U * (C / 64)>
__device__ __forceinline__ void fwd_epilogue(f32x16* acc, __amdgpu_buffer_rsrc_t rs_res, __amdgpu_buffer_rsrc_t rs_out,
                                             const float* b2, int tok, bool ok, int h, long mg, const MlpDrop& dd,
                                             bool keep = false) {
    constexpr int HT = C / 64;
    float sdp = 1.f;
    DropoutRng R;
    if constexpr (DROP) {
        R = load_rng(dd.rng, dd.site_o, dd.p);
        if (dd.row_scale) sdp = dd.row_scale[mg / dd.rps];
    }
#pragma unroll
    for (int q = 0; q < HT; ++q) {
        unsigned km = 0xffffu;
        if constexpr (DROP) if (dd.p > 0.f) km = keep16_crow(R, ((uint64_t)mg * C + (U * HT + q) * 32) >> 3, h);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = (U * HT + q) * 32 + 8 * g + 4 * h;
            const unsigned off = ok ? (unsigned)(tok * C + f) * 4 : kOOB;
            float rv[4], bv[4], v[4];
            buf_ld4(rs_res, off, rv);
            load4(b2 + f, bv);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float z = acc[A0 + q][4 * g + e] + bv[e];
                if constexpr (DROP) z *= ((km >> (4 * g + e)) & 1u) ? sdp * R.scale : 0.f;
                v[e] = z + rv[e];
                if (keep) acc[A0 + q][4 * g + e] = v[e];   // the block output, for ln_epilogue
            }
            buf_st4(rs_out, off, v);
        }
    }
}

// LayerNorm of the Mlp block's output (the NEXT CSWinBlock's norm1, cswin:357 -- the residual stream
// y = res + Mlp(x) is fully formed here): per token mean and rstd over its C values, two passes as
// ln_fwd (mean, then the centred sum of squares).  Lane (r, h) of wave (t, U) holds token 32 t + r,
// features (U HT + q) 32 + 8 g + 4 h + e in yv[q][4 g + e]; the two feature halves of a token meet by
// a shuffle (h) and the LDS exchange lnx with the partner wave (U ^ 1); both waves take part in the
// two barriers.  Writes the bf16 LN output and (wave U = 0) mean / rstd.
template <int C, int U, int NWV = 4, int A0 = U * (C / 64)>
__device__ __forceinline__ void ln_epilogue(const f32x16* yv, float* lnx, int wave, int r, int h, int tok, bool ok,
                                            const float* __restrict__ gam, const float* __restrict__ bet, float eps,
                                            __amdgpu_buffer_rsrc_t rs_ln, __amdgpu_buffer_rsrc_t rs_mean,
                                            __amdgpu_buffer_rsrc_t rs_rstd) {
    constexpr int HT = C / 64;
    // shifted one-pass moments (shift = the lane's first value, shared with the partner half and wave
    // through the exchange): one barrier instead of two, no cancellation for a large mean
    float sh = yv[A0][0];
    sh = __shfl(sh, r, 64);                         // token r's shift from lane (r, 0) of this wave
    constexpr int SEC = 32 * NWV;                   // lnx: [sums | squares | shifts] x NWV waves x 32 tokens
    if (h == 0) lnx[2 * SEC + wave * 32 + r] = sh;
    float s = 0.f, q2 = 0.f;
#pragma unroll
    for (int q = 0; q < HT; ++q)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float d = yv[A0 + q][i] - sh;
            s += d;
            q2 += d * d;
        }
    s += __shfl_xor(s, 32, 64);
    q2 += __shfl_xor(q2, 32, 64);
    if (h == 0) {
        lnx[wave * 32 + r] = s;
        lnx[SEC + wave * 32 + r] = q2;
    }
    lds_sync();
    const int pw = (wave ^ 1) * 32 + r;
    const float shp = lnx[2 * SEC + pw];             // the partner wave's shift for this token
    const float dsh = shp - sh;
    // partner moments re-centred on this wave's shift: sum(d + dsh), sum((d + dsh)^2)
    const float sp = lnx[pw], qp = lnx[SEC + pw];
    constexpr float HN = C / 2;
    const float S = s + sp + HN * dsh;
    const float Q = q2 + qp + 2.f * dsh * sp + HN * dsh * dsh;
    const float mu_s = S / C;                        // mean - sh
    const float mu = sh + mu_s;
    const float rs = rsqrtf(fmaxf(Q / C - mu_s * mu_s, 0.f) + eps);
#pragma unroll
    for (int q = 0; q < HT; ++q)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = (U * HT + q) * 32 + 8 * g + 4 * h;
            float gw[4], bw[4], o[4];
            load4(gam + f, gw);
            load4(bet + f, bw);
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (yv[A0 + q][4 * g + e] - mu) * rs * gw[e] + bw[e];
            buf_st4bf(rs_ln, ok ? (unsigned)(tok * C + f) * 2 : kOOB, o);
        }
    if (U == 0 && h == 0) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mu), rs_mean, ok ? (unsigned)tok * 4 : kOOB, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(rs), rs_rstd, ok ? (unsigned)tok * 4 : kOOB, 0, 0);
    }
}

// the next block's norm1 (ln_epilogue) for the fused forward, or all-null
struct MlpLn {
    const float* gamma;
    const float* beta;
    float eps;
    bf16* out;
    float* mean;
    float* rstd;
};

template <int C, int U>
__device__ __forceinline__ void bwd_epilogue(const f32x16* acc, __amdgpu_buffer_rsrc_t rs_dx, int tok, bool ok, int h) {
    constexpr int HT = C / 64;
#pragma unroll
    for (int q = 0; q < HT; ++q)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = (U * HT + q) * 32 + 8 * g + 4 * h;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[U * HT + q][4 * g + e];
            buf_st4bf(rs_dx, ok ? (unsigned)(tok * C + f) * 2 : kOOB, v);
        }
}

// b1 of the accumulator layout: hidden base + crow(e, h), from the LDS copy (4 x ds_read_b128)
__device__ __forceinline__ void bias16(const float* b1s, int base, int h, float* bv) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(b1s + base + 8 * g + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[4 * g + e] = v[e];
    }
}

template <bool V> using bconst = std::integral_constant<bool, V>;
template <int V> using iconst = std::integral_constant<int, V>;

// Forward.  Rings: W1 chunks in 2 stages, W2 chunks in 2 stages.  Step j (after one barrier):
// DMA W1(j+2), W2(j+1); GEMM1(j+1) on the MFMA pipe while GELU(j) runs on the VALU; GEMM2(j).
// DROP: hidden / output dropout and DropPath (MlpDrop)
template <int C, bool DROP, bool LN = false>
__global__ __launch_bounds__(MT) void mlp_fwd_kernel(long M, const bf16* __restrict__ X, const bf16* __restrict__ W1,
                                                     const float* __restrict__ b1, const bf16* __restrict__ W2,
                                                     const float* __restrict__ b2, const float* __restrict__ res,
                                                     float* __restrict__ out, MlpDrop dd, long rpi, MlpLn ln = MlpLn{}) {
    constexpr int NCH = 4 * C / HC;     // hidden chunks
    constexpr int KS = C / 16;          // k-steps of GEMM1
    constexpr int TF = C / 32;          // 32-feature output tiles (all C, partial over the hidden half)
    constexpr int IMG = HC * C;         // bf16 per weight-chunk image (W1 [HC][C] or W2 [C][HC])
    constexpr int NWV = 4, NTH = MT;
    using D1 = Dma<HC, 2 * C, NWV>;
    using D2 = Dma<C, 2 * HC, NWV>;
    __shared__ __attribute__((aligned(1024))) bf16 ring[4 * IMG];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    bf16* const w1r = ring;
    bf16* const w2r = ring + 2 * IMG;

    const long mw = (long)blockIdx.x * BM;           // the workgroup's first token
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long m0 = mw;
    const long rows = M - m0 > 0 ? M - m0 : 0;
    const int r = lane & 31, h = lane >> 5;
    const int t = (wave & 3) >> 1, u = wave & 1;
    const int tok = 32 * t + r;
    const bool ok = tok < rows;
    const int hs = 32 * u;              // this wave's hidden features within a chunk
    // hidden chunk of loop step j: rotated by the panel's position inside its image (rpi rows per
    // image, a multiple of the panel), so the workgroups running together stream different weight
    // chunks (every panel reads the same 2 x 4C x C weights: without the rotation all CUs of an XCD
    // hit the same L2 lines at once) while a token's sum order does not depend on the batch split
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((mw % rpi) / BM) & (NCH - 1)) : 0;
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += NTH) b1s[i] = b1[i];
    // LN epilogue: gamma / beta staged in LDS here -- read in the epilogue from LDS, a global load there
    // would wait (vmcnt, issue order) for the completion of every output store before it
    __shared__ __attribute__((aligned(16))) float lngb[LN ? 2 * C : 4];
    if constexpr (LN)
        for (int i = threadIdx.x; i < 2 * C; i += NTH) lngb[i] = i < C ? ln.gamma[i] : ln.beta[i - C];
    bf16x8 xf[KS];
    load_bfrags<C>(buf_rsrc(X + m0 * C, rows * C * 2), tok, ok, h, xf);

    D1 d1;
    D2 d2;
    d1.init(C, wave, lane);
    d2.init(4 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
    const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
    asm volatile("" ::: "memory");
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(0) * HC * C * 2, w1r, wave);
    dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(0) * HC * 2, w2r, wave);
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(1) * HC * C * 2, w1r + IMG, wave);

    auto gemm1 = [&](const bf16* img) {
        bf16x8 wf[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) wf[s] = frag(img, moff<2 * C>(hs + r, 16 * s + 8 * h));
        __builtin_amdgcn_sched_barrier(0);   // every fragment read in flight before the first MFMA
        f32x16 a = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s], xf[s], a, 0, 0, 0);
        return a;
    };
    f32x16 acc[TF];
#pragma unroll
    for (int i = 0; i < TF; ++i) acc[i] = f32x16{};
    const long mg = m0 + tok;   // global token of this lane (dropout element index)
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);
    vmwait<0>();
    lds_sync();
    f32x16 ha = gemm1(w1r), hb;

    // par = j & 1 as a compile-time constant: every LDS address is a per-lane base + immediate
    auto step = [&](auto more, auto par, int j, const f32x16& cur, f32x16& nxt) {
        constexpr int P = decltype(par)::value;
        vmwait<0>();                    // W1(j+1), W2(j): issued one step ago
        lds_sync();                     // every wave is past GEMM1(j) and GEMM2(j-1)
        if (j + 2 < NCH) dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(j + 2) * HC * C * 2, w1r + P * IMG, wave);
        if (j + 1 < NCH) dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(j + 1) * HC * 2, w2r + (1 - P) * IMG, wave);
        const int jc = chk(j);
        float bv[16], gv[16];
        bias16(b1s, jc * HC + hs, h, bv);
        if constexpr (decltype(more)::value) nxt = gemm1(w1r + (1 - P) * IMG);
#pragma unroll
        for (int e = 0; e < 16; ++e) gv[e] = gelu_fast(cur[e] + bv[e]);
        if constexpr (DROP) {   // hidden dropout on g (features j*HC + hs + crow(e, h) of token mg)
            if (dd.p > 0.f) {
                const unsigned km = keep16_crow(Rh, ((uint64_t)mg * 4 * C + jc * HC + hs) >> 3, h);
#pragma unroll
                for (int e = 0; e < 16; ++e) gv[e] = ((km >> e) & 1u) ? gv[e] * Rh.scale : 0.f;
            }
        }
        const bf16* w2c = w2r + P * IMG;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            bf16x8 wf2[TF];
#pragma unroll
            for (int ft = 0; ft < TF; ++ft) wf2[ft] = pfrag<2 * HC>(w2c, 32 * ft + r, hs + 16 * s2, h);
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8 gb = pack_b(gv, s2);
#pragma unroll
            for (int ft = 0; ft < TF; ++ft) acc[ft] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf2[ft], gb, acc[ft], 0, 0, 0);
        }
    };
    int j = 0;
    for (; j + 2 < NCH; j += 2) {
        step(bconst<true>{}, iconst<0>{}, j, ha, hb);
        step(bconst<true>{}, iconst<1>{}, j + 1, hb, ha);
    }
    step(bconst<true>{}, iconst<0>{}, j, ha, hb);
    step(bconst<false>{}, iconst<1>{}, j + 1, hb, ha);

    lds_sync();                         // ring free: partial-sum exchange
    float* xch = reinterpret_cast<float*>(ring);
    const auto rs_res = buf_rsrc(res + m0 * C, rows * C * 4);
    const auto rs_out = buf_rsrc(out + m0 * C, rows * C * 4);
    if constexpr (LN) {
        __shared__ float lnx[3 * 32 * NWV];
        const auto rs_ln = buf_rsrc(ln.out + m0 * C, rows * C * 2);
        const auto rs_mean = buf_rsrc(ln.mean + m0, rows * 4), rs_rstd = buf_rsrc(ln.rstd + m0, rows * 4);
        if (u == 0) {
            exchange_half<C, 0>(acc, xch, wave, lane);
            fwd_epilogue<C, 0, DROP>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd, true);
            ln_epilogue<C, 0, NWV>(acc, lnx, wave, r, h, tok, ok, lngb, lngb + C, ln.eps, rs_ln, rs_mean, rs_rstd);
        } else {
            exchange_half<C, 1>(acc, xch, wave, lane);
            fwd_epilogue<C, 1, DROP>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd, true);
            ln_epilogue<C, 1, NWV>(acc, lnx, wave, r, h, tok, ok, lngb, lngb + C, ln.eps, rs_ln, rs_mean, rs_rstd);
        }
        return;
    }
    if (u == 0) {
        exchange_half<C, 0>(acc, xch, wave, lane);
        fwd_epilogue<C, 0, DROP>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd);
    } else {
        exchange_half<C, 1>(acc, xch, wave, lane);
        fwd_epilogue<C, 1, DROP>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd);
    }
}

// Backward.  Rings: W1 chunks in 3 stages (GEMM1 of chunk j+1 and GEMM4 of chunk j overlap, plus
// the prefetch), W2 chunks in 2.  Step j (after one barrier): DMA W1(j+2), W2(j+2); GEMM1/GEMM3 of
// chunk j+1 on the MFMA pipe while chunk j's GELU / GELU' / g, dH stores run on the VALU; GEMM4(j).
// DROP: dY is the gradient of the dropped fc2 output (the output mask / DropPath were applied by
// the caller); the hidden mask is regenerated here: g stored = gelu(h) * mask, dH = (W2^T dY) * mask * gelu'(h).
template <int C, bool DROP>
__global__ __launch_bounds__(MT) void mlp_bwd_kernel(long M, const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                     const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                     const bf16* __restrict__ W2, bf16* __restrict__ dH,
                                                     bf16* __restrict__ G, bf16* __restrict__ dX, MlpDrop dd, long rpi) {
    constexpr int NCH = 4 * C / HC;
    constexpr int KS = C / 16;
    constexpr int TF = C / 32;
    constexpr int IMG = HC * C;
    using D1 = Dma<HC, 2 * C>;
    using D2 = Dma<C, 2 * HC>;
    // C = 256: two accumulator sets (overlap) would not fit in 512 registers -> plain order
    constexpr bool PIPE = C < 256;
    constexpr int W1S = PIPE ? 3 : 2;   // W1 ring stages
    __shared__ __attribute__((aligned(1024))) bf16 ring[(W1S + 2) * IMG];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    bf16* const w1r = ring;
    bf16* const w2r = ring + W1S * IMG;

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int t = wave >> 1, u = wave & 1;
    const int tok = 32 * t + r;
    const bool ok = tok < rows;
    const int hs = 32 * u;
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;   // see the forward
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += MT) b1s[i] = b1[i];
    bf16x8 xf[KS], dyf[KS];
    load_bfrags<C>(buf_rsrc(X + m0 * C, rows * C * 2), tok, ok, h, xf);
    load_bfrags<C>(buf_rsrc(dY + m0 * C, rows * C * 2), tok, ok, h, dyf);

    D1 d1;
    D2 d2;
    d1.init(C, wave, lane);
    d2.init(4 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
    const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
    const auto rs_dh = buf_rsrc(dH + m0 * 4 * C, rows * 4 * C * 2);
    const auto rs_g = buf_rsrc(G + m0 * 4 * C, rows * 4 * C * 2);
    asm volatile("" ::: "memory");
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(0) * HC * C * 2, w1r, wave);
    dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(0) * HC * 2, w2r, wave);
    if constexpr (PIPE) {
        dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(1) * HC * C * 2, w1r + IMG, wave);
        dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(1) * HC * 2, w2r + IMG, wave);
    }

    // GEMM1 (h = W1_sub x^T) and GEMM3 (dg = W2_sub^T dY^T) of one chunk
    auto gemm13 = [&](const bf16* w1c, const bf16* w2c, f32x16& ha, f32x16& ga) {
        ha = f32x16{};
        ga = f32x16{};
        // fragments of KS/2 k-steps in flight before their MFMAs (two halves: register budget)
        constexpr int KP = KS / 2;
#pragma unroll
        for (int s0 = 0; s0 < KS; s0 += KP) {
            bf16x8 fa[KP], fb[KP];
#pragma unroll
            for (int s = 0; s < KP; ++s) {
                fa[s] = frag(w1c, moff<2 * C>(hs + r, 16 * (s0 + s) + 8 * h));
                fb[s] = trfrag<2 * HC>(w2c, hs, s0 + s, lane);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < KP; ++s) {
                ha = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s], xf[s0 + s], ha, 0, 0, 0);
                ga = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[s], dyf[s0 + s], ga, 0, 0, 0);
            }
        }
    };
    f32x16 acc[TF];
#pragma unroll
    for (int i = 0; i < TF; ++i) acc[i] = f32x16{};
    // chunk j's epilogue (GELU, GELU', g / dH stores: 8 per wave) and GEMM4 (dx += W1_sub^T dH^T)
    const long mg = m0 + tok;
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);
    auto finish = [&](int jj, const f32x16& hc, const f32x16& gc, const float* bv, const bf16* w1c) {
        const int j = chk(jj);   // the chunk's hidden features
        float gv[16], dv[16];
        unsigned km = 0xffffu;
        if constexpr (DROP) if (dd.p > 0.f) km = keep16_crow(Rh, ((uint64_t)mg * 4 * C + j * HC + hs) >> 3, h);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            float dg;
            gelu_pair_fast(hc[e] + bv[e], gv[e], dg);
            if constexpr (DROP) {
                const float ms = ((km >> e) & 1u) ? Rh.scale : 0.f;
                gv[e] *= ms;                 // the dropped g feeds dW2
                dg *= ms;
            }
            dv[e] = gc[e] * dg;
        }
        const unsigned base = ok ? (unsigned)(tok * 4 * C + j * HC + hs + 4 * h) * 2 : kOOB;
#pragma unroll
        for (int g = 0; g < 4; ++g) {   // features 8g + 4h .. + 3 of the wave's 32
            const unsigned o = base == kOOB ? kOOB : base + 16 * g;
            buf_st4bf(rs_g, o, gv + 4 * g);
            buf_st4bf(rs_dh, o, dv + 4 * g);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const bf16x8 db = pack_b(dv, s2);
            bf16x8 fw[TF];
#pragma unroll
            for (int ft = 0; ft < TF; ++ft) fw[ft] = ptrfrag<2 * C>(w1c, 32 * ft, hs + 16 * s2, lane);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int ft = 0; ft < TF; ++ft) acc[ft] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[ft], db, acc[ft], 0, 0, 0);
        }
    };
    f32x16 ha, ga;
    if constexpr (PIPE) {
        vmwait<0>();
        lds_sync();
        f32x16 hb, gb;
        gemm13(w1r, w2r, ha, ga);
        auto step = [&](auto more, int j, const f32x16& hc, const f32x16& gc, f32x16& hn, f32x16& gn) {
            vmwait<8>();                // W1(j+1), W2(j+1) landed; only chunk j-1's 8 stores after them
            lds_sync();                 // every wave is past GEMM4(j-1) and GEMM3(j)
            if (j + 2 < NCH) {
                dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(j + 2) * HC * C * 2, w1r + ((j + 2) % 3) * IMG, wave);
                dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(j + 2) * HC * 2, w2r + (j & 1) * IMG, wave);
            }
            float bv[16];
            bias16(b1s, chk(j) * HC + hs, h, bv);
            if constexpr (decltype(more)::value) gemm13(w1r + ((j + 1) % 3) * IMG, w2r + ((j + 1) & 1) * IMG, hn, gn);
            finish(j, hc, gc, bv, w1r + (j % 3) * IMG);
        };
        int j = 0;
        for (; j + 2 < NCH; j += 2) {
            step(bconst<true>{}, j, ha, ga, hb, gb);
            step(bconst<true>{}, j + 1, hb, gb, ha, ga);
        }
        step(bconst<true>{}, j, ha, ga, hb, gb);
        step(bconst<false>{}, j + 1, hb, gb, ha, ga);
    } else {
        for (int j = 0; j < NCH; ++j) {
            // chunk j landed: after its DMA this wave issued only chunk j-1's 8 g / dH stores
            if (j == 0) vmwait<0>(); else vmwait<8>();
            lds_sync();                 // every wave is past chunk j-1: its stage is free
            if (j + 1 < NCH) {
                dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(j + 1) * HC * C * 2, w1r + ((j + 1) & 1) * IMG, wave);
                dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(j + 1) * HC * 2, w2r + ((j + 1) & 1) * IMG, wave);
            }
            float bv[16];
            bias16(b1s, chk(j) * HC + hs, h, bv);
            gemm13(w1r + (j & 1) * IMG, w2r + (j & 1) * IMG, ha, ga);
            finish(j, ha, ga, bv, w1r + (j & 1) * IMG);
        }
    }

    lds_sync();
    float* xch = reinterpret_cast<float*>(ring);
    const auto rs_dx = buf_rsrc(dX + m0 * C, rows * C * 2);
    if (u == 0) {
        exchange_half<C, 0>(acc, xch, wave, lane);
        bwd_epilogue<C, 0>(acc, rs_dx, tok, ok, h);
    } else {
        exchange_half<C, 1>(acc, xch, wave, lane);
        bwd_epilogue<C, 1>(acc, rs_dx, tok, ok, h);
    }
}


// Persistent backward for C = 64 (stage 1): W1 / W2 (2 x 256 x 64 bf16 = 64 KB) stay in LDS for the
// workgroup's lifetime -- the per-panel kernel above re-stages them for every 64-token panel (4096
// panels at 512x512 B16: 268 MB of L2 -> LDS traffic for 67 MB of token operands).  Two teams of 4
// waves (2 waves per SIMD) run their own panel streams through the same weight images; wave (t, u)
// of a team has the roles of the per-panel kernel; natural chunk order.  (The forward in this form
// measured slower than the per-panel kernel: its per-chunk work is too short to hide the token
// loads without the DMA ring's overlap.)
template <bool DROP>
__global__ __launch_bounds__(2 * MT) void mlp_bwd64_persist(long M, const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                            const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                            const bf16* __restrict__ W2, bf16* __restrict__ dH,
                                                            bf16* __restrict__ G, bf16* __restrict__ dX, MlpDrop dd) {
    constexpr int C = 64, NCH = 4 * C / HC, KS = C / 16, TF = C / 32, IMG = HC * C;
    using D1 = Dma<HC, 2 * C, 8>;
    using D2 = Dma<C, 2 * HC, 8>;
    __shared__ __attribute__((aligned(1024))) bf16 wimg[2 * NCH * IMG];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    __shared__ __attribute__((aligned(16))) float xch[2][4 * (C / 64) * 16 * 64];
    const int lane = threadIdx.x & 63;
    const int wave8 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int team = wave8 >> 2, wave = wave8 & 3;
    const int r = lane & 31, h = lane >> 5;
    const int t = wave >> 1, u = wave & 1;
    const int tok = 32 * t + r;
    const int hs = 32 * u;
    for (int i = threadIdx.x; i < 4 * C; i += 2 * MT) b1s[i] = b1[i];
    {
        D1 d1;
        D2 d2;
        d1.init(C, wave8, lane);
        d2.init(4 * C, wave8, lane);
        const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
        const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            dma<D1::NW>(rs_w1, d1.v, (unsigned)j * HC * C * 2, wimg + j * IMG, wave8);
            dma<D2::NW>(rs_w2, d2.v, (unsigned)j * HC * 2, wimg + (NCH + j) * IMG, wave8);
        }
        vmwait<0>();
        lds_sync();
    }
    const long npan = (M + BM - 1) / BM;
    const long mine = blockIdx.x < npan ? (npan - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    const long iters = (mine + 1) / 2;
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);
    float* xc = xch[team];
    for (long it = 0; it < iters; ++it) {
        const long k = 2 * it + team;
        const long m0 = (blockIdx.x + k * (long)gridDim.x) * BM;
        const long rows = k < mine ? M - m0 : 0;
        const long mb = rows > 0 ? m0 : 0;
        const bool ok = tok < rows;
        bf16x8 xf[KS], dyf[KS];
        load_bfrags<C>(buf_rsrc(X + mb * C, rows * C * 2), tok, ok, h, xf);
        load_bfrags<C>(buf_rsrc(dY + mb * C, rows * C * 2), tok, ok, h, dyf);
        const auto rs_dh = buf_rsrc(dH + mb * 4 * C, rows * 4 * C * 2);
        const auto rs_g = buf_rsrc(G + mb * 4 * C, rows * 4 * C * 2);
        const long mg = m0 + tok;
        f32x16 acc[TF];
#pragma unroll
        for (int i = 0; i < TF; ++i) acc[i] = f32x16{};
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const bf16* w1c = wimg + j * IMG;
            const bf16* w2c = wimg + (NCH + j) * IMG;
            f32x16 ha = f32x16{}, ga = f32x16{};
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                ha = __builtin_amdgcn_mfma_f32_32x32x16_bf16(frag(w1c, moff<2 * C>(hs + r, 16 * s2 + 8 * h)), xf[s2], ha, 0, 0, 0);
                ga = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<2 * HC>(w2c, hs, s2, lane), dyf[s2], ga, 0, 0, 0);
            }
            float bv[16], gv[16], dv[16];
            bias16(b1s, j * HC + hs, h, bv);
            unsigned km = 0xffffu;
            if constexpr (DROP) if (dd.p > 0.f) km = keep16_crow(Rh, ((uint64_t)mg * 4 * C + j * HC + hs) >> 3, h);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                float dg;
                gelu_pair_fast(ha[e] + bv[e], gv[e], dg);
                if constexpr (DROP) {
                    const float ms = ((km >> e) & 1u) ? Rh.scale : 0.f;
                    gv[e] *= ms;
                    dg *= ms;
                }
                dv[e] = ga[e] * dg;
            }
            const unsigned base = ok ? (unsigned)(tok * 4 * C + j * HC + hs + 4 * h) * 2 : kOOB;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const unsigned o = base == kOOB ? kOOB : base + 16 * g;
                buf_st4bf(rs_g, o, gv + 4 * g);
                buf_st4bf(rs_dh, o, dv + 4 * g);
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const bf16x8 db = pack_b(dv, s2);
#pragma unroll
                for (int ft = 0; ft < TF; ++ft)
                    acc[ft] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ptrfrag<2 * C>(w1c, 32 * ft, hs + 16 * s2, lane), db, acc[ft], 0, 0, 0);
            }
        }
        const auto rs_dx = buf_rsrc(dX + mb * C, rows * C * 2);
        if (u == 0) {
            exchange_half<C, 0>(acc, xc, wave, lane);
            bwd_epilogue<C, 0>(acc, rs_dx, tok, ok, h);
        } else {
            exchange_half<C, 1>(acc, xc, wave, lane);
            bwd_epilogue<C, 1>(acc, rs_dx, tok, ok, h);
        }
        lds_sync();
    }
}

int persist_grid(long M) {   // one workgroup (two panel streams) per CU, fewer for small M
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
    }
    const long pan = (M + BM - 1) / BM;
    return (int)(pan < 2L * cus ? (pan + 1) / 2 : cus);
}

// ================================================================================================
// Forward at C = 256 with two waves per SIMD (mlp_fwd8_kernel; no dropout: DROP launches keep the
// 4-wave kernel).  The 4-wave kernel keeps a C x 32 partial output per wave (128 accumulator
// registers) so that every wave needs every hidden feature of its token half, and one wave per SIMD
// runs the whole barrier -> GEMM1 -> GELU -> GEMM2 chain serially (profiles/r08b_mlp_ablate.txt:
// removing the DMA, the GELU or the MFMAs each saves 6-10 of 41 us, none dominates).  Here the
// hidden activations go through LDS, which splits the two GEMMs differently:
//  * GEMM1 + GELU: wave (tg, hq) = (wave >> 2, wave & 3) computes h = W1 x^T for the 16 hidden
//    features 16 hq .. of every 64-feature chunk and the 32 tokens 32 tg .. on 16x16x32 MFMAs (x as
//    B fragments in registers, W1 rows as A fragments from the ring), applies bias + GELU and writes
//    g (bf16) into a [64 tokens][64 hidden] LDS image (double-buffered by chunk parity);
//  * GEMM2: wave w owns the output features 32 w .. 32 w + 31 for all 64 tokens (two 32x32x16 tiles,
//    K = the chunk's 64 hidden): A = W2 rows from the ring, B = g from the LDS image -- no partial
//    outputs to exchange at the end, 32 accumulator registers per token tile.
// 154-158 VGPRs: two waves per SIMD.  Step j (one barrier): DMA W1(j+1), W2(j); GEMM1 + GELU of chunk j;
// GEMM2 of chunk j-1.  LDS per step and CU: 160 KB of fragment reads + 64 KB of DMA (256 B/clk: ~900
// cycles) against 1024 MFMA cycles per SIMD.
// HCK = 32: 32-hidden chunks through a 4-stage ring (the same 128 KB), the weight DMA up to three
// chunks ahead instead of one (GEMM1's wave tile 16 hidden x 16 tokens, GEMM2's K 32) -- measured, not
// used (kFwd8Hc): the DMA stream alone is 21-22 us of the 37-38 either way (w8_dmaonly,
// profiles/r08e_mlp_ablate.txt, r08f_mlp_ablate.txt), the rest is the compute chain.
template <int C, bool LN, int HCK>
__global__ __launch_bounds__(2 * MT) void mlp_fwd8_kernel(long M, const bf16* __restrict__ X, const bf16* __restrict__ W1,
                                                          const float* __restrict__ b1, const bf16* __restrict__ W2,
                                                          const float* __restrict__ b2, const float* __restrict__ res,
                                                          float* __restrict__ out, long rpi, MlpLn ln) {
    static_assert(C == 256, "mlp_fwd8: C = 256 (32 output features per wave)");
    static_assert(HCK == 64 || HCK == 32, "mlp_fwd8: 64- or 32-hidden chunks");
    constexpr int NCH = 4 * C / HCK;    // hidden chunks
    constexpr int IMG = HCK * C;        // bf16 per weight-chunk image
    constexpr int NST = 128 * 1024 / (4 * IMG);   // ring stages per matrix (2 at HCK 64, 4 at 32)
    constexpr int NWV = 8, NTH = 2 * MT;
    constexpr int KS = C / 32;          // GEMM1 k-steps (16x16x32)
    constexpr int HG = HCK / 16;        // GEMM1 hidden groups of 16 per chunk
    constexpr int TT = 4 / (NWV / HG);  // GEMM1 16-token tiles per wave (2 at HCK 64, 1 at 32)
    constexpr int K2 = HCK / 16;        // GEMM2 k-steps per chunk
    using D1 = Dma<HCK, 2 * C, NWV>;
    using D2 = Dma<C, 2 * HCK, NWV>;
    constexpr int DPS = D1::NW + D2::NW;   // DMA instructions per wave per step
    __shared__ __attribute__((aligned(1024))) bf16 ring[2 * NST * IMG];   // W1 x NST | W2 x NST stages
    __shared__ __attribute__((aligned(1024))) bf16 gimg[2][BM * HCK];    // g of a chunk: [token][hidden]
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    __shared__ __attribute__((aligned(16))) float lngb[LN ? 2 * C : 4];
    bf16* const w1r = ring;
    bf16* const w2r = ring + NST * IMG;

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0 > 0 ? M - m0 : 0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tg = wave / HG, hq = wave % HG;       // GEMM1 role: tokens 16 TT tg .., hidden 16 hq ..
    const int l16 = lane & 15, q4 = lane >> 4;      // 16x16x32 lane split
    const int r = lane & 31, h = lane >> 5;         // 32x32x16 lane split
    const int fo = 32 * wave;                       // GEMM2 role: output features fo .. fo + 31
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += NTH) b1s[i] = b1[i];
    if constexpr (LN)
        for (int i = threadIdx.x; i < 2 * C; i += NTH) lngb[i] = i < C ? ln.gamma[i] : ln.beta[i - C];

    // x as 16x16x32 B fragments: token 16 TT tg + 16 tt + l16, k = 32 s + 8 q4 .. + 7
    bf16x8 xf[TT][KS];
    {
        const auto rs_x = buf_rsrc(X + m0 * C, rows * C * 2);
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
            const int tok = 16 * TT * tg + 16 * tt + l16;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                    rs_x, tok < rows ? (unsigned)(tok * C + 32 * s + 8 * q4) * 2 : kOOB, 0, 0);
                __builtin_memcpy(&xf[tt][s], &v, 16);
            }
        }
    }
    D1 d1;
    D2 d2;
    d1.init(C, wave, lane);
    d2.init(4 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
    const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
    auto dma1 = [&](int c) { dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(c) * HCK * C * 2, w1r + (c % NST) * IMG, wave); };
    auto dma2 = [&](int c) { dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(c) * HCK * 2, w2r + (c % NST) * IMG, wave); };
    asm volatile("" ::: "memory");
    // prefetch: W1 runs NST - 1 chunks ahead of GEMM1, W2 NST - 2 ahead of GEMM2 (= GEMM1 - 1)
    dma1(0);
#pragma unroll
    for (int p = 1; p <= NST - 2; ++p) {
        dma1(p);
        dma2(p - 1);
    }

    f32x16 acc[2];
    acc[0] = f32x16{};
    acc[1] = f32x16{};

    // chunk j: h for (16 hidden of hq) x (16 TT tokens of tg), bias + GELU, g -> gimg[j & 1]
    auto gemm1 = [&](int j) {
        const bf16* w1c = w1r + (j % NST) * IMG;
        bf16x8 wf[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) wf[s] = frag(w1c, moff<2 * C>(16 * hq + l16, 32 * s + 8 * q4));
        f32x4 hv[TT];
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) hv[tt] = f32x4{};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) hv[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], xf[tt][s], hv[tt], 0, 0, 0);
        const f32x4 bv = *reinterpret_cast<const f32x4*>(b1s + chk(j) * HCK + 16 * hq + 4 * q4);
        bf16* gi = gimg[j & 1];
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
            bf16x4 gq;
#pragma unroll
            for (int e = 0; e < 4; ++e) gq[e] = (bf16)gelu_fast(hv[tt][e] + bv[e]);
            // token 16 TT tg + 16 tt + l16, hidden 16 hq + 4 q4 .. + 3
            *reinterpret_cast<bf16x4*>(gi + moff<2 * HCK>(16 * TT * tg + 16 * tt + l16, 16 * hq + 4 * q4)) = gq;
        }
    };
    // chunk j: acc[tt] += W2[fo .. fo + 31][chunk] g[chunk][32 tt ..]
    auto gemm2 = [&](int j) {
        const bf16* w2c = w2r + (j % NST) * IMG;
        const bf16* gi = gimg[j & 1];
        bf16x8 af[K2], bf[2][K2];
#pragma unroll
        for (int s = 0; s < K2; ++s) {
            af[s] = frag(w2c, moff<2 * HCK>(fo + r, 16 * s + 8 * h));
            bf[0][s] = frag(gi, moff<2 * HCK>(r, 16 * s + 8 * h));
            bf[1][s] = frag(gi, moff<2 * HCK>(32 + r, 16 * s + 8 * h));
        }
#pragma unroll
        for (int s = 0; s < K2; ++s) {
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf[0][s], acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf[1][s], acc[1], 0, 0, 0);
        }
    };

    // step j (one barrier): DMA W1(j + NST - 1), W2(j + NST - 2); GEMM1 + GELU of chunk j; GEMM2 of
    // chunk j - 1.  The wait leaves the last NST - 2 steps' DMAs in flight (all of them full groups
    // except near the end, where it waits for everything)
    for (int j = 0; j <= NCH; ++j) {
        if (NST > 2 && j + NST - 2 < NCH) vmwait<(NST > 2 ? (NST - 2) * DPS : 0)>();
        else vmwait<0>();
        lds_sync();                     // every wave is past step j-1 (its stages and g image are free)
        if (j + NST - 1 < NCH) dma1(j + NST - 1);
        if (j + NST - 2 < NCH) dma2(j + NST - 2);
        if (j < NCH) gemm1(j);
        if (j > 0) gemm2(j - 1);
    }

    // epilogue: lane holds token 32 tt + r, features fo + 8 g + 4 h + 0..3 in acc[tt][4 g + e]
    const auto rs_res = buf_rsrc(res + m0 * C, rows * C * 4);
    const auto rs_out = buf_rsrc(out + m0 * C, rows * C * 4);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const int tok = 32 * tt + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = fo + 8 * g + 4 * h;
            const unsigned off = tok < rows ? (unsigned)(tok * C + f) * 4 : kOOB;
            float rv[4], v[4];
            buf_ld4(rs_res, off, rv);
            const f32x4 bv = *reinterpret_cast<const f32x4*>(b2 + f);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = acc[tt][4 * g + e] + bv[e] + rv[e];
                acc[tt][4 * g + e] = v[e];
            }
            buf_st4(rs_out, off, v);
        }
    }
    if constexpr (LN) {
        // the next block's norm1 over the token's C values, spread over the 8 waves: two passes
        // (mean, centred squares) through an LDS [wave][token] table in the (now free) ring
        float* red = reinterpret_cast<float*>(ring);
        float mu[2], rs[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) s += acc[tt][i];
            s = xsum32(s);
            if (h == 0) red[wave * 64 + 32 * tt + r] = s;
        }
        lds_sync();
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < NWV; ++w) s += red[w * 64 + 32 * tt + r];
            mu[tt] = s * (1.f / C);
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float d = acc[tt][i] - mu[tt];
                q += d * d;
            }
            q = xsum32(q);
            if (h == 0) red[NWV * 64 + wave * 64 + 32 * tt + r] = q;
        }
        lds_sync();
        const auto rs_ln = buf_rsrc(ln.out + m0 * C, rows * C * 2);
        const auto rs_mean = buf_rsrc(ln.mean + m0, rows * 4), rs_rstd = buf_rsrc(ln.rstd + m0, rows * 4);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            float q = 0.f;
#pragma unroll
            for (int w = 0; w < NWV; ++w) q += red[NWV * 64 + w * 64 + 32 * tt + r];
            rs[tt] = rsqrtf(q * (1.f / C) + ln.eps);
            const int tok = 32 * tt + r;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f = fo + 8 * g + 4 * h;
                const f32x4 gw = *reinterpret_cast<const f32x4*>(lngb + f);
                const f32x4 bw = *reinterpret_cast<const f32x4*>(lngb + C + f);
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o[e] = (acc[tt][4 * g + e] - mu[tt]) * rs[tt] * gw[e] + bw[e];
                buf_st4bf(rs_ln, tok < rows ? (unsigned)(tok * C + f) * 2 : kOOB, o);
            }
            if (wave == 0 && h == 0) {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mu[tt]), rs_mean, tok < rows ? (unsigned)tok * 4 : kOOB, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(rs[tt]), rs_rstd, tok < rows ? (unsigned)tok * 4 : kOOB, 0, 0);
            }
        }
    }
}

// Backward at C = 256 with two waves per SIMD (mlp_bwd8_kernel; no dropout: DROP launches keep the
// 4-wave kernel).  The 4-wave kernel holds x, dY (64 + 64 registers) and a C x 32 partial dX (128) per
// wave, so at C = 256 it runs one wave per SIMD with no overlap between chunks (PIPE off); removing
// its DMA, MFMAs or g / dH stores each saved 11-17 of 60 us (profiles/r08b_mlp_ablate.txt).  Here
// per 64-hidden chunk, three phases separated by barriers, both waves of a SIMD busy in each:
//  A  waves 0-3: h = W1 x^T + b1 for (32 hidden of hh) x (32 tokens of tg) on 16x16x32 MFMAs (x in
//     registers); waves 4-7: dg = W2^T dY^T for the same tiles (dY in registers, W2 read transposed);
//     both written as bf16 (the reference's autocast rounds fc1's output and fc2's input gradient to
//     bf16 as well) into [token][hidden] LDS images;
//  B  all 512 threads: 8 consecutive hidden features of one token each -- g = gelu(h), dH = dg gelu'(h),
//     16-B stores of g and dH (the weight-gradient operands) and dH into an LDS image;
//  C  dX += W1^T dH: wave w owns the dX features 32 w .. for all 64 tokens (32x32x16, W1 read
//     transposed from the ring) -- no partial outputs to exchange.
// The next chunk's W1 / W2 land during the three phases (2-stage ring).
// 64-hidden chunks for mlp_fwd8_kernel: 32-hidden chunks with the weight DMA three chunks ahead (a
// 4-stage ring) measured no faster (38.6 vs 37.4 us isolated, mlp_fwd 1072-1079 vs 1038-1049 us/step
// in the step: profiles/r08f_mlp_ablate.txt, r08f bench pairs)
constexpr int kFwd8Hc = 64;
template <int C>
__global__ __launch_bounds__(2 * MT) void mlp_bwd8_kernel(long M, const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                          const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                          const bf16* __restrict__ W2, bf16* __restrict__ dH,
                                                          bf16* __restrict__ G, bf16* __restrict__ dX, long rpi) {
    static_assert(C == 256, "mlp_bwd8: C = 256 (32 dX features per wave)");
    constexpr int NCH = 4 * C / HC;
    constexpr int IMG = HC * C;
    constexpr int NWV = 8, NTH = 2 * MT;
    constexpr int KS = C / 32;          // k-steps of GEMM1 / GEMM3 (16x16x32)
    using D1 = Dma<HC, 2 * C, NWV>;
    using D2 = Dma<C, 2 * HC, NWV>;
    __shared__ __attribute__((aligned(1024))) bf16 ring[4 * IMG];      // W1 x 2 | W2 x 2 stages
    __shared__ __attribute__((aligned(1024))) bf16 himg[BM * HC];      // h + b1 (bf16), [token][hidden]
    __shared__ __attribute__((aligned(1024))) bf16 dgimg[BM * HC];     // dg
    __shared__ __attribute__((aligned(1024))) bf16 dhimg[BM * HC];     // dH
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    bf16* const w1r = ring;
    bf16* const w2r = ring + 2 * IMG;

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0 > 0 ? M - m0 : 0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool g1 = wave < 4;                       // GEMM1 (h) or GEMM3 (dg) role in phase A
    const int tg = (wave >> 1) & 1, hh = wave & 1;  // phase A tile: tokens 32 tg .., hidden 32 hh ..
    const int l16 = lane & 15, q4 = lane >> 4;
    const int r = lane & 31, h = lane >> 5;
    const int fo = 32 * wave;                       // phase C: dX features fo .. fo + 31
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += NTH) b1s[i] = b1[i];

    // phase-A token operand as 16x16x32 B fragments: x (GEMM1 waves) or dY (GEMM3 waves)
    bf16x8 tf[2][KS];
    {
        const auto rs_t = buf_rsrc((g1 ? X : dY) + m0 * C, rows * C * 2);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            const int tok = 32 * tg + 16 * tt + l16;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                    rs_t, tok < rows ? (unsigned)(tok * C + 32 * s + 8 * q4) * 2 : kOOB, 0, 0);
                __builtin_memcpy(&tf[tt][s], &v, 16);
            }
        }
    }
    D1 d1;
    D2 d2;
    d1.init(C, wave, lane);
    d2.init(4 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
    const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
    const auto rs_dh = buf_rsrc(dH + m0 * 4 * C, rows * 4 * C * 2);
    const auto rs_g = buf_rsrc(G + m0 * 4 * C, rows * 4 * C * 2);
    asm volatile("" ::: "memory");
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(0) * HC * C * 2, w1r, wave);
    dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(0) * HC * 2, w2r, wave);

    f32x16 acc[2];
    acc[0] = f32x16{};
    acc[1] = f32x16{};
    // phase B element of this thread: token tb, hidden 8 hb .. 8 hb + 7 of the chunk
    const int tb = threadIdx.x >> 3, hb = threadIdx.x & 7;

    for (int j = 0; j < NCH; ++j) {
        const int jc = chk(j);
        // chunk j landed; after its DMA this thread issued only chunk j-1's two phase-B stores
        if (j == 0) vmwait<0>(); else vmwait<2>();
        lds_sync();                     // every wave is past chunk j-1 (stages, images free)
        if (j + 1 < NCH) {
            dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(j + 1) * HC * C * 2, w1r + ((j + 1) & 1) * IMG, wave);
            dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(j + 1) * HC * 2, w2r + ((j + 1) & 1) * IMG, wave);
        }
        // ---- phase A
        {
            f32x4 a[2][2];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) a[mt][tt] = f32x4{};
            if (g1) {
                const bf16* w1c = w1r + (j & 1) * IMG;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    bf16x8 wf[KS];
#pragma unroll
                    for (int s = 0; s < KS; ++s) wf[s] = frag(w1c, moff<2 * C>(32 * hh + 16 * mt + l16, 32 * s + 8 * q4));
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        a[mt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], tf[0][s], a[mt][0], 0, 0, 0);
                        a[mt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], tf[1][s], a[mt][1], 0, 0, 0);
                    }
                }
            } else {
                const bf16* w2c = w2r + (j & 1) * IMG;
                const int grp = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    // A[m = hidden 32 hh + 16 mt + l16][k = 32 s + 8 q4 ..]: W2 image rows k, columns m
                    bf16x8 wf[KS];
                    const int col = 32 * hh + 16 * mt + 4 * p;
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        const int row = 32 * s + 8 * grp + q;
                        wf[s] = cat8(tr4(w2c + moff<2 * HC>(row, col)), tr4(w2c + moff<2 * HC>(row + 4, col)));
                    }
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        a[mt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], tf[0][s], a[mt][0], 0, 0, 0);
                        a[mt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s], tf[1][s], a[mt][1], 0, 0, 0);
                    }
                }
            }
            // D[m = 4 q4 + i][n = l16]: hidden 32 hh + 16 mt + 4 q4 + i, token 32 tg + 16 tt + l16
            bf16* img = g1 ? himg : dgimg;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const int hf = 32 * hh + 16 * mt + 4 * q4;
                f32x4 bv = f32x4{};
                if (g1) bv = *reinterpret_cast<const f32x4*>(b1s + jc * HC + hf);
#pragma unroll
                for (int tt = 0; tt < 2; ++tt) {
                    bf16x4 o;
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = (bf16)(a[mt][tt][e] + bv[e]);
                    *reinterpret_cast<bf16x4*>(img + moff<2 * HC>(32 * tg + 16 * tt + l16, hf)) = o;
                }
            }
        }
        lds_sync();
        // ---- phase B
        {
            const bf16x8 hv = frag(himg, moff<2 * HC>(tb, 8 * hb));
            const bf16x8 dv = frag(dgimg, moff<2 * HC>(tb, 8 * hb));
            float gv[8], dd[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float dg;
                gelu_pair_fast((float)hv[e], gv[e], dg);
                dd[e] = (float)dv[e] * dg;
            }
            const unsigned o = tb < rows ? (unsigned)(tb * 4 * C + jc * HC + 8 * hb) * 2 : kOOB;
            buf_st8bf(rs_g, o, gv);
            buf_st8bf(rs_dh, o, dd);
            bf16x8 db;
#pragma unroll
            for (int e = 0; e < 8; ++e) db[e] = (bf16)dd[e];
            *reinterpret_cast<bf16x8*>(dhimg + moff<2 * HC>(tb, 8 * hb)) = db;
        }
        lds_sync();
        // ---- phase C: acc[tt] += W1[chunk]^T[fo ..][hidden] dH[hidden][32 tt ..]
        {
            const bf16* w1c = w1r + (j & 1) * IMG;
            bf16x8 af[4], bf[2][4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                af[s] = trfrag<2 * C>(w1c, fo, s, lane);
                bf[0][s] = frag(dhimg, moff<2 * HC>(r, 16 * s + 8 * h));
                bf[1][s] = frag(dhimg, moff<2 * HC>(32 + r, 16 * s + 8 * h));
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf[0][s], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf[1][s], acc[1], 0, 0, 0);
            }
        }
    }
    // dX: lane holds token 32 tt + r, features fo + 8 g + 4 h + 0..3
    const auto rs_dx = buf_rsrc(dX + m0 * C, rows * C * 2);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
        const int tok = 32 * tt + r;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[tt][4 * g + e];
            buf_st4bf(rs_dx, tok < rows ? (unsigned)(tok * C + fo + 8 * g + 4 * h) * 2 : kOOB, v);
        }
    }
}

template <int C>
int fwd_launch(long M, const void* x, const void* w1, const float* b1, const void* w2, const float* b2, const float* res,
               float* out, const MlpDrop* d, long rpi, hipStream_t st, const MlpLn* ln = nullptr) {
    const dim3 grid((unsigned)((M + BM - 1) / BM));
    if constexpr (C == 256) {
        if (!d) {   // two waves per SIMD (dropout launches keep the 4-wave kernel)
            if (ln)
                mlp_fwd8_kernel<C, true, kFwd8Hc><<<grid, 2 * MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2,
                                                                   res, out, rpi, *ln);
            else
                mlp_fwd8_kernel<C, false, kFwd8Hc><<<grid, 2 * MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2,
                                                                    res, out, rpi, MlpLn{});
            return check_launch(ln ? "mlp_fwd_ln" : "mlp_fwd");
        }
    }
    if (ln) {
        if (d)
            mlp_fwd_kernel<C, true, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2,
                                                                      res, out, *d, rpi, *ln);
        else
            mlp_fwd_kernel<C, false, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2,
                                                                       b2, res, out, MlpDrop{}, rpi, *ln);
        return check_launch("mlp_fwd_ln");
    }
    if (d)
        mlp_fwd_kernel<C, true, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2, res,
                                                                   out, *d, rpi);
    else
        mlp_fwd_kernel<C, false, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2,
                                                                    res, out, MlpDrop{}, rpi);
    return check_launch("mlp_fwd");
}

template <int C>
int bwd_launch(long M, const void* x, const void* dy, const void* w1, const float* b1, const void* w2, void* dh, void* g,
               void* dx, const MlpDrop* d, long rpi, hipStream_t st) {
    const dim3 grid((unsigned)((M + BM - 1) / BM));
    if constexpr (C == 256) {
        if (!d) {   // two waves per SIMD (dropout launches keep the 4-wave kernel)
            mlp_bwd8_kernel<C><<<grid, 2 * MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                        (bf16*)dh, (bf16*)g, (bf16*)dx, rpi);
            return check_launch("mlp_bwd");
        }
    }
    if constexpr (C == 64) {   // persistent, weights resident (mlp_bwd64_persist)
        const dim3 pg((unsigned)persist_grid(M));
        if (d)
            mlp_bwd64_persist<true><<<pg, 2 * MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                           (bf16*)dh, (bf16*)g, (bf16*)dx, *d);
        else
            mlp_bwd64_persist<false><<<pg, 2 * MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                            (bf16*)dh, (bf16*)g, (bf16*)dx, MlpDrop{});
        return check_launch("mlp_bwd");
    }
    if (d)
        mlp_bwd_kernel<C, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                     (bf16*)dh, (bf16*)g, (bf16*)dx, *d, rpi);
    else
        mlp_bwd_kernel<C, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                      (bf16*)dh, (bf16*)g, (bf16*)dx, MlpDrop{}, rpi);
    return check_launch("mlp_bwd");
}


// ================================================================================================
// fp8-e4m3 fused Mlp (BASELINE config 5, "fp8 MFMA weights"): v_mfma_scale_f32_32x32x64_f8f6f4 with
// MX block scales -- every operand lane carries an E8M0 exponent for its 32 k-values (probe:
// tools/probes/mx_scale_probe.hip, 127 = 2^0, one scale per lane of A and of B).
//   GEMM1  h = W1 x   : A = e4m3 rows of W1 (the row's power-of-two scale sw1[f] = 2^e as the lane's
//                       E8M0), B = x quantised in registers per (token, 32 consecutive channels)
//   GEMM2  y += W2 g  : B = g = gelu(h + b1) quantised in registers per (token, 32 consecutive hidden
//                       features: the accumulator tile pair of a wave hands lane half h the features
//                       32 t + 8 g + 4 h + i in byte 16 t + 4 g + i, and the hardware's block b is bytes
//                       [16 b, 16 b + 16) of both halves = tile t = b), A = e4m3 rows of W2 (per-row scale
//                       sw2[c] as the lane's E8M0) with the columns permuted per 64-block so that a lane's
//                       32 k-bytes are contiguous: position 32h + 16t + 4g + i holds feature 32t + 8g +
//                       4h + i (csu_e4m3_layout_batch)
// Chunks of 128 hidden features (wave u: features 64u..64u+63 = two 32-row tiles, so one lane holds
// the 32 values of one f8 k-step of GEMM2); 64-token panel per workgroup as in the bf16 kernel.  A
// chunk's W1 + W2 bytes equal one 64-feature bf16 chunk's: half the weight stream per panel.  GEMM2
// is split by OUTPUT features: wave (t, u) accumulates y features [u C/2, (u+1) C/2) over the whole
// chunk, taking the partner wave's g_q through LDS (half the accumulators, no final exchange).
constexpr int HC8 = 128;
typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int e8m0_of(float s) { return (__float_as_int(s) >> 23) & 0xff; }

// MX quantisation of one f8 operand lane.  The hardware's k layout (tools/probes/mx_layout_probe.hip):
// bytes [0, 16) of lane half h are k = 16 h + 0..15 and bytes [16, 32) are k = 32 + 16 h + 0..15, and
// the E8M0 scale of lane half b applies to block b = k [32 b, 32 b + 32) = bytes [16 b, 16 b + 16) of
// BOTH lane halves.  So a block's amax combines this lane's half with the partner lane's (lane ^ 32):
// scale 2^e, e the smallest integer with amax <= 448 * 2^e (0 for an all-zero block, clamped to the
// E8M0 range), e4m3fn bytes round-to-nearest-even (no saturation).  v: the lane's 32 values in byte
// order; returns the lane's scale operand (E8M0 of block h); e0 / e1: both blocks' exponents.
__device__ __forceinline__ int mx_exp(float amax) {
    const int b = __float_as_int(amax);
    const int e = ((b >> 23) & 0xff) - 135 + ((b & 0x7fffff) > 0x600000 ? 1 : 0);
    return amax == 0.f ? 0 : (e < -127 ? -127 : (e > 127 ? 127 : e));
}
__device__ __forceinline__ int mx_quant32(const float* v, i32x8& q, int& e0, int& e1) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        a0 = fmaxf(a0, fabsf(v[i]));
        a1 = fmaxf(a1, fabsf(v[16 + i]));
    }
    a0 = fmaxf(a0, __shfl_xor(a0, 32, 64));
    a1 = fmaxf(a1, __shfl_xor(a1, 32, 64));
    e0 = mx_exp(a0);
    e1 = mx_exp(a1);
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const int e = d < 4 ? e0 : e1;
        int w = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * d], -e), ldexpf(v[4 * d + 1], -e), 0, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * d + 2], -e), ldexpf(v[4 * d + 3], -e), w, true);
        q[d] = w;
    }
    return ((threadIdx.x & 63) >> 5 ? e1 : e0) + 127;
}
__device__ __forceinline__ int mx_quant32(const float* v, i32x8& q) {
    int e0, e1;
    return mx_quant32(v, q, e0, e1);
}

// 16 + 16 k-bytes of row `row` of a swizzled byte image with RB-byte rows: bytes [kb, kb + 16) and
// [kb + 32, kb + 48) -- the k order of lane half h = (kb / 16) & 1 of an f8 k-step starting at kb - 16 h
// (two ds_read_b128, the bf16 images' 16-B slot swizzle)
template <int RB>
__device__ __forceinline__ i32x8 frag8s(const bf16* img, int row, int kb) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(img + moff<RB>(row, kb >> 1));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(img + moff<RB>(row, (kb + 32) >> 1));
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}
// 32 contiguous k-bytes [kb, kb + 32) of a row (operands whose k order is the accumulator tile
// pair's: byte j = 16 t + 4 g + i, see csu_e4m3_layout_batch)
template <int RB>
__device__ __forceinline__ i32x8 frag8(const bf16* img, int row, int kb) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(img + moff<RB>(row, kb >> 1));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(img + moff<RB>(row, (kb + 16) >> 1));
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}

// token operand of GEMM1 (or of the backward's dY GEMM): row `tok`, k-step s in the hardware's k
// order (channels 64 s + 16 h + 0..15 and 64 s + 32 + 16 h + 0..15), so MX blocks are 32 consecutive
// channels; optionally times a per-channel power-of-two factor colscale first
template <int C>
__device__ __forceinline__ void load_q8(__amdgpu_buffer_rsrc_t rs, int tok, bool ok, int h, i32x8* q, int* sc,
                                        const float* colscale = nullptr) {
#pragma unroll
    for (int s = 0; s < C / 64; ++s) {
        float v[32];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int ch = 64 * s + 32 * (p >> 1) + 16 * h + 8 * (p & 1);
            buf_ld8bf(rs, ok ? (unsigned)(tok * C + ch) * 2 : kOOB, v + 8 * p);
            if (colscale) {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[8 * p + i] *= colscale[ch + i];
            }
        }
        sc[s] = mx_quant32(v, q[s]);
    }
}

__device__ __forceinline__ f32x16 mfma8(const i32x8& a, const i32x8& b, const f32x16& c, int sa, int sb) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// Forward.  Rings as the bf16 forward: W1 chunk images [128][C B] in 2 stages, W2 chunk images [C][128 B]
// in 2 stages; step j: DMA W1(j+2), W2(j+1); GEMM1(j+1) on the MFMA pipe while GELU + quantisation of
// chunk j run on the VALU; GEMM2(j).
// LN: also the next block's norm1 on the output (ln_epilogue, as mlp_fwd_kernel's)
template <int C, bool DROP, bool LN = false>
__global__ __launch_bounds__(MT) void mlp_fp8_fwd_kernel(long M, const bf16* __restrict__ X, const uint8_t* __restrict__ W1,
                                                         const float* __restrict__ sw1, const float* __restrict__ b1,
                                                         const uint8_t* __restrict__ W2p, const float* __restrict__ sw2,
                                                         const float* __restrict__ b2, const float* __restrict__ res,
                                                         float* __restrict__ out, MlpDrop dd, long rpi, MlpLn ln = MlpLn{}) {
    constexpr int NCH = 4 * C / HC8;    // hidden chunks (even)
    constexpr int KS = C / 64;          // f8 k-steps of GEMM1
    constexpr int TF = C / 32;
    constexpr int IMG1 = HC8 * C / 2;   // bf16 units of a W1 chunk image
    constexpr int IMG2 = C * HC8 / 2;   // and of a W2 chunk image
    using D1 = Dma<HC8, C>;
    using D2 = Dma<C, HC8>;
    __shared__ __attribute__((aligned(1024))) bf16 ring[2 * IMG1 + 2 * IMG2];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    __shared__ int e1s[4 * C];
    __shared__ __attribute__((aligned(32))) i32x8 xg[4][64];   // quantised g of every wave's lanes
    __shared__ int xgs[4][64];
    bf16* const w1r = ring;
    bf16* const w2r = ring + 2 * IMG1;

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int t = wave >> 1, u = wave & 1;
    const int tok = 32 * t + r;
    const bool ok = tok < rows;
    const int hs = 64 * u;              // this wave's hidden features within a chunk
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;   // see mlp_fwd_kernel
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += MT) {
        b1s[i] = b1[i];
        e1s[i] = e8m0_of(sw1[i]);
    }
    __shared__ __attribute__((aligned(16))) float lngb[LN ? 2 * C : 4];   // gamma / beta (see mlp_fwd_kernel)
    if constexpr (LN)
        for (int i = threadIdx.x; i < 2 * C; i += MT) lngb[i] = i < C ? ln.gamma[i] : ln.beta[i - C];
    constexpr int TH = TF / 2;          // output tiles of one wave: features [u C/2, (u+1) C/2)
    int e2[TH];
#pragma unroll
    for (int q = 0; q < TH; ++q) e2[q] = e8m0_of(sw2[32 * (u * TH + q) + r]);
    i32x8 xq[KS];
    int xs[KS];
    load_q8<C>(buf_rsrc(X + m0 * C, rows * C * 2), tok, ok, h, xq, xs);

    D1 d1;
    D2 d2;
    d1.init(C / 2, wave, lane);         // ld in bf16 units: W1 rows are C bytes, W2p rows 4C bytes
    d2.init(2 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C);
    const i32x4 rs_w2 = rsrc4(W2p, 4L * C * C);
    asm volatile("" ::: "memory");
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(0) * HC8 * C, w1r, wave);
    dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(0) * HC8, w2r, wave);
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(1) * HC8 * C, w1r + IMG1, wave);

    auto gemm1 = [&](const bf16* img, int jc, f32x16* ha) {
        i32x8 wf[2][KS];
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int s = 0; s < KS; ++s) wf[t2][s] = frag8s<C>(img, hs + 32 * t2 + r, 64 * s + 16 * h);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
            const int sa = e1s[jc * HC8 + hs + 32 * t2 + r];
            f32x16 a = f32x16{};
#pragma unroll
            for (int s = 0; s < KS; ++s) a = mfma8(wf[t2][s], xq[s], a, sa, xs[s]);
            ha[t2] = a;
        }
    };
    f32x16 acc[TH];
#pragma unroll
    for (int i = 0; i < TH; ++i) acc[i] = f32x16{};
    const long mg = m0 + tok;
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);
    vmwait<0>();
    lds_sync();
    f32x16 ha[2], hb[2];
    gemm1(w1r, chk(0), ha);

    auto step = [&](auto more, auto par, int j, const f32x16* cur, f32x16* nxt) {
        constexpr int P = decltype(par)::value;
        vmwait<0>();                    // W1(j+1), W2(j): issued one step ago
        lds_sync();                     // every wave is past GEMM1(j) and GEMM2(j-1)
        if (j + 2 < NCH) dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(j + 2) * HC8 * C, w1r + P * IMG1, wave);
        if (j + 1 < NCH) dma<D2::NW>(rs_w2, d2.v, (unsigned)chk(j + 1) * HC8, w2r + (1 - P) * IMG2, wave);
        const int jc = chk(j);
        if constexpr (decltype(more)::value) gemm1(w1r + (1 - P) * IMG1, chk(j + 1), nxt);
        float gv[32];
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
            float bv[16];
            bias16(b1s, jc * HC8 + hs + 32 * t2, h, bv);
#pragma unroll
            for (int e = 0; e < 16; ++e) gv[16 * t2 + e] = gelu_fast(cur[t2][e] + bv[e]);
            if constexpr (DROP) {
                if (dd.p > 0.f) {
                    const unsigned km = keep16_crow(Rh, ((uint64_t)mg * 4 * C + jc * HC8 + hs + 32 * t2) >> 3, h);
#pragma unroll
                    for (int e = 0; e < 16; ++e) gv[16 * t2 + e] = ((km >> e) & 1u) ? gv[16 * t2 + e] * Rh.scale : 0.f;
                }
            }
        }
        i32x8 gq;
        const int gs = mx_quant32(gv, gq);
        xg[wave][lane] = gq;
        xgs[wave][lane] = gs;
        lds_sync();                     // the partner wave's g_q (same tokens, the other 64 features)
        const i32x8 gp = xg[wave ^ 1][lane];
        const int gsp = xgs[wave ^ 1][lane];
        const bf16* w2c = w2r + P * IMG2;
        const int hp = 64 * (1 - u);
        i32x8 wa[TH], wb[TH];
#pragma unroll
        for (int q = 0; q < TH; ++q) {
            wa[q] = frag8<HC8>(w2c, 32 * (u * TH + q) + r, hs + 32 * h);
            wb[q] = frag8<HC8>(w2c, 32 * (u * TH + q) + r, hp + 32 * h);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < TH; ++q) {
            acc[q] = mfma8(wa[q], gq, acc[q], e2[q], gs);
            acc[q] = mfma8(wb[q], gp, acc[q], e2[q], gsp);
        }
    };
    int j = 0;
    for (; j + 2 < NCH; j += 2) {
        step(bconst<true>{}, iconst<0>{}, j, ha, hb);
        step(bconst<true>{}, iconst<1>{}, j + 1, hb, ha);
    }
    step(bconst<true>{}, iconst<0>{}, j, ha, hb);
    step(bconst<false>{}, iconst<1>{}, j + 1, hb, ha);

    const auto rs_res = buf_rsrc(res + m0 * C, rows * C * 4);
    const auto rs_out = buf_rsrc(out + m0 * C, rows * C * 4);
    if constexpr (LN) {
        __shared__ float lnx[384];
        const auto rs_ln = buf_rsrc(ln.out + m0 * C, rows * C * 2);
        const auto rs_mean = buf_rsrc(ln.mean + m0, rows * 4), rs_rstd = buf_rsrc(ln.rstd + m0, rows * 4);
        if (u == 0) {
            fwd_epilogue<C, 0, DROP, 0>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd, true);
            ln_epilogue<C, 0, 4, 0>(acc, lnx, wave, r, h, tok, ok, lngb, lngb + C, ln.eps, rs_ln, rs_mean, rs_rstd);
        } else {
            fwd_epilogue<C, 1, DROP, 0>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd, true);
            ln_epilogue<C, 1, 4, 0>(acc, lnx, wave, r, h, tok, ok, lngb, lngb + C, ln.eps, rs_ln, rs_mean, rs_rstd);
        }
        return;
    }
    if (u == 0)
        fwd_epilogue<C, 0, DROP, 0>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd);
    else
        fwd_epilogue<C, 1, DROP, 0>(acc, rs_res, rs_out, b2, tok, ok, h, mg, dd);
}

template <int C>
int fp8_fwd_launch(long M, const void* x, const void* w1, const float* sw1, const float* b1, const void* w2p, const float* sw2,
                   const float* b2, const float* res, float* out, const MlpDrop* d, long rpi, hipStream_t st,
                   const MlpLn* ln = nullptr) {
    const dim3 grid((unsigned)((M + BM - 1) / BM));
    if (ln) {
        if (d)
            mlp_fp8_fwd_kernel<C, true, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const uint8_t*)w1, sw1, b1,
                                                                   (const uint8_t*)w2p, sw2, b2, res, out, *d, rpi, *ln);
        else
            mlp_fp8_fwd_kernel<C, false, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const uint8_t*)w1, sw1, b1,
                                                                    (const uint8_t*)w2p, sw2, b2, res, out, MlpDrop{}, rpi, *ln);
        return check_launch("mlp_fp8_fwd_ln");
    }
    if (d)
        mlp_fp8_fwd_kernel<C, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const uint8_t*)w1, sw1, b1, (const uint8_t*)w2p,
                                                         sw2, b2, res, out, *d, rpi);
    else
        mlp_fp8_fwd_kernel<C, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const uint8_t*)w1, sw1, b1, (const uint8_t*)w2p,
                                                          sw2, b2, res, out, MlpDrop{}, rpi);
    return check_launch("mlp_fp8_fwd");
}


// the 32 values of a packed e4m3 operand lane: bytes [0, 16) times 2^e0, [16, 32) times 2^e1
__device__ __forceinline__ void mx_dequant32(const i32x8& q, int e0, int e1, float* v) {
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const int e = d < 4 ? e0 : e1;
        const auto lo = __builtin_amdgcn_cvt_pk_f32_fp8(q[d], false);
        const auto hi = __builtin_amdgcn_cvt_pk_f32_fp8(q[d], true);
        v[4 * d] = ldexpf(lo[0], e);
        v[4 * d + 1] = ldexpf(lo[1], e);
        v[4 * d + 2] = ldexpf(hi[0], e);
        v[4 * d + 3] = ldexpf(hi[1], e);
    }
}

// Backward (straight-through for every quantisation):
//   h  = W1 x_q + b1 recomputed exactly as the forward (same operands, same instruction order),
//   dg = W2^T dY: A = W2^T e4m3 (csu_e4m3_layout_batch mode 1), B = dY * sw2 quantised per (token,
//        32 consecutive channels) -- the per-row scale of W2 lies along this contraction, so it is
//        folded into the token operand;
//   dh = dg * gelu'(h) (* hidden mask); dH (bf16) and G = the forward's g_q (bf16, exact) stored for
//        dW1 = dH^T x and dW2 = dY^T G;
//   dx = W1^T dh: A = W1^T e4m3 with permuted columns (mode 3), B = dh * sw1 quantised per lane as g.
// GEMM4 is split by OUTPUT features: wave (t, u) accumulates dx features [u C/2, (u+1) C/2) over the
// whole chunk, taking the partner wave's quantised dh (its 64 features) through LDS -- half the
// accumulator registers of a hidden-half split and no final exchange.
// LDS: W1 chunk images [128][C B] in 2 stages, one W2^T stage [128][C B], one W1^T stage [C][128 B]
// (C = 256: 128 KB).  Step j: DMA W1(j+1); GEMM1 + GEMM3(j); barrier, DMA W2^T(j+1); GELU', stores,
// quantisation, dh to LDS; wait for W1^T(j) by count; barrier; GEMM4(j); barrier, DMA W1^T(j+1).
template <int C, bool DROP>
__global__ __launch_bounds__(MT) void mlp_fp8_bwd_kernel(long M, const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                         const uint8_t* __restrict__ W1, const float* __restrict__ sw1,
                                                         const float* __restrict__ b1, const uint8_t* __restrict__ W2T,
                                                         const float* __restrict__ sw2, const uint8_t* __restrict__ W1Tp,
                                                         bf16* __restrict__ dH, bf16* __restrict__ G, bf16* __restrict__ dX,
                                                         MlpDrop dd, long rpi) {
    constexpr int NCH = 4 * C / HC8;
    constexpr int KS = C / 64;
    constexpr int TF = C / 32;
    constexpr int TH = TF / 2;          // dx tiles of one wave
    constexpr int IMG1 = HC8 * C / 2;   // W1 / W2^T chunk image (bf16 units)
    constexpr int IMG3 = C * HC8 / 2;   // W1^T chunk image
    using D1 = Dma<HC8, C>;
    using D3 = Dma<C, HC8>;
    constexpr int NST = 16;             // buffer stores per lane per chunk (8 G + 8 dH)
    __shared__ __attribute__((aligned(1024))) bf16 ring[3 * IMG1 + IMG3];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];
    __shared__ __attribute__((aligned(16))) uint8_t e1s[4 * C];
    __shared__ float s2s[C];
    __shared__ __attribute__((aligned(32))) i32x8 xdh[4][64];   // quantised dh of every wave's lanes
    __shared__ int xds[4][64];
    bf16* const w1r = ring;
    bf16* const w2r = ring + 2 * IMG1;
    bf16* const w3r = ring + 3 * IMG1;

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int t = wave >> 1, u = wave & 1;
    const int tok = 32 * t + r;
    const bool ok = tok < rows;
    const int hs = 64 * u;
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;   // see the forward
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += MT) {
        b1s[i] = b1[i];
        e1s[i] = (uint8_t)e8m0_of(sw1[i]);
    }
    for (int i = threadIdx.x; i < C; i += MT) s2s[i] = sw2[i];
    __syncthreads();
    i32x8 xq[KS], dq[KS];
    int xs[KS], ds[KS];
    load_q8<C>(buf_rsrc(X + m0 * C, rows * C * 2), tok, ok, h, xq, xs);
    load_q8<C>(buf_rsrc(dY + m0 * C, rows * C * 2), tok, ok, h, dq, ds, s2s);

    D1 d1, d2;
    D3 d3;
    d1.init(C / 2, wave, lane);
    d2.init(C / 2, wave, lane);
    d3.init(2 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C);
    const i32x4 rs_w2 = rsrc4(W2T, 4L * C * C);
    const i32x4 rs_w3 = rsrc4(W1Tp, 4L * C * C);
    const auto rs_dh = buf_rsrc(dH + m0 * 4 * C, rows * 4 * C * 2);
    const auto rs_g = buf_rsrc(G + m0 * 4 * C, rows * 4 * C * 2);
    asm volatile("" ::: "memory");
    dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(0) * HC8 * C, w1r, wave);
    dma<D1::NW>(rs_w2, d2.v, (unsigned)chk(0) * HC8 * C, w2r, wave);
    dma<D3::NW>(rs_w3, d3.v, (unsigned)chk(0) * HC8, w3r, wave);

    f32x16 acc[TH];
#pragma unroll
    for (int i = 0; i < TH; ++i) acc[i] = f32x16{};
    const long mg = m0 + tok;
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);

    auto step = [&](auto par, int j) {
        constexpr int P = decltype(par)::value;
        const bool more = j + 1 < NCH;
        vmwait<D3::NW>();               // W1(j), W2^T(j) landed (W1^T(j), the youngest, may still fly)
        lds_sync();
        if (more) dma<D1::NW>(rs_w1, d1.v, (unsigned)chk(j + 1) * HC8 * C, w1r + (1 - P) * IMG1, wave);
        const int jc = chk(j);
        const bf16* w1c = w1r + P * IMG1;
        float gv[32], dv[32];
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
            f32x16 ha, ga;
            {
                i32x8 fa[KS];
#pragma unroll
                for (int s = 0; s < KS; ++s) fa[s] = frag8s<C>(w1c, hs + 32 * t2 + r, 64 * s + 16 * h);
                __builtin_amdgcn_sched_barrier(0);
                const int sa = e1s[jc * HC8 + hs + 32 * t2 + r];
                ha = f32x16{};
#pragma unroll
                for (int s = 0; s < KS; ++s) ha = mfma8(fa[s], xq[s], ha, sa, xs[s]);   // as the forward
            }
            {
                i32x8 fb[KS];
#pragma unroll
                for (int s = 0; s < KS; ++s) fb[s] = frag8s<C>(w2r, hs + 32 * t2 + r, 64 * s + 16 * h);
                __builtin_amdgcn_sched_barrier(0);
                ga = f32x16{};
#pragma unroll
                for (int s = 0; s < KS; ++s) ga = mfma8(fb[s], dq[s], ga, 127, ds[s]);
            }
            float bv[16];
            bias16(b1s, jc * HC8 + hs + 32 * t2, h, bv);
            unsigned km = 0xffffu;
            if constexpr (DROP) if (dd.p > 0.f) km = keep16_crow(Rh, ((uint64_t)mg * 4 * C + jc * HC8 + hs + 32 * t2) >> 3, h);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                float gg, dg;
                gelu_pair_fast(ha[e] + bv[e], gg, dg);
                if constexpr (DROP) {
                    const float ms = ((km >> e) & 1u) ? Rh.scale : 0.f;
                    gg *= ms;
                    dg *= ms;
                }
                gv[16 * t2 + e] = gg;
                dv[16 * t2 + e] = ga[e] * dg;
            }
        }
        lds_sync();                     // every wave is past GEMM3(j): the W2^T stage is free
        if (more) dma<D1::NW>(rs_w2, d2.v, (unsigned)chk(j + 1) * HC8 * C, w2r, wave);
        {   // G = the forward's g_q, exactly
            i32x8 gq;
            int e0, e1;
            mx_quant32(gv, gq, e0, e1);
            mx_dequant32(gq, e0, e1, gv);
        }
        const int fb0 = jc * HC8 + hs;
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int f = fb0 + 32 * t2 + 8 * g + 4 * h;
                const unsigned o = ok ? (unsigned)(tok * 4 * C + f) * 2 : kOOB;
                buf_st4bf(rs_g, o, gv + 16 * t2 + 4 * g);
                buf_st4bf(rs_dh, o, dv + 16 * t2 + 4 * g);
            }
        // dh * sw1 (the per-row scale of W1 lies along GEMM4's contraction), quantised per lane
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const unsigned ew = *reinterpret_cast<const unsigned*>(e1s + fb0 + 32 * t2 + 8 * g + 4 * h);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    dv[16 * t2 + 4 * g + i] = ldexpf(dv[16 * t2 + 4 * g + i], (int)((ew >> (8 * i)) & 0xff) - 127);
            }
        i32x8 dhq;
        const int dhs = mx_quant32(dv, dhq);
        xdh[wave][lane] = dhq;
        xds[wave][lane] = dhs;
        // W1^T(j) landed: younger than it are W1(j+1), W2^T(j+1) (when issued) and this chunk's stores
        if (more) vmwait<2 * D1::NW + NST>(); else vmwait<NST>();
        lds_sync();                     // W1^T(j) and every wave's dh visible
        const i32x8 dhp = xdh[wave ^ 1][lane];
        const int dsp = xds[wave ^ 1][lane];
        const int hp = 64 * (1 - u);    // the partner's hidden features
#pragma unroll
        for (int q = 0; q < TH; ++q) {
            const int ft = u * TH + q;
            const i32x8 a0 = frag8<HC8>(w3r, 32 * ft + r, hs + 32 * h);
            const i32x8 a1 = frag8<HC8>(w3r, 32 * ft + r, hp + 32 * h);
            acc[q] = mfma8(a0, dhq, acc[q], 127, dhs);
            acc[q] = mfma8(a1, dhp, acc[q], 127, dsp);
        }
        lds_sync();                     // every wave is past GEMM4(j): the W1^T stage and xdh are free
        if (more) dma<D3::NW>(rs_w3, d3.v, (unsigned)chk(j + 1) * HC8, w3r, wave);
    };
    for (int j = 0; j < NCH; j += 2) {
        step(iconst<0>{}, j);
        step(iconst<1>{}, j + 1);
    }

    // dx features [u C/2, (u+1) C/2) of the wave's 32 tokens
    const auto rs_dx = buf_rsrc(dX + m0 * C, rows * C * 2);
#pragma unroll
    for (int q = 0; q < TH; ++q)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = (u * TH + q) * 32 + 8 * g + 4 * h;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[q][4 * g + e];
            buf_st4bf(rs_dx, ok ? (unsigned)(tok * C + f) * 2 : kOOB, v);
        }
}

template <int C>
int fp8_bwd_launch(long M, const void* x, const void* dy, const void* w1, const float* sw1, const float* b1, const void* w2t,
                   const float* sw2, const void* w1tp, void* dh, void* g, void* dx, const MlpDrop* d, long rpi, hipStream_t st) {
    const dim3 grid((unsigned)((M + BM - 1) / BM));
    if (d)
        mlp_fp8_bwd_kernel<C, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const uint8_t*)w1, sw1, b1,
                                                         (const uint8_t*)w2t, sw2, (const uint8_t*)w1tp, (bf16*)dh, (bf16*)g,
                                                         (bf16*)dx, *d, rpi);
    else
        mlp_fp8_bwd_kernel<C, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const uint8_t*)w1, sw1, b1,
                                                          (const uint8_t*)w2t, sw2, (const uint8_t*)w1tp, (bf16*)dh, (bf16*)g,
                                                          (bf16*)dx, MlpDrop{}, rpi);
    return check_launch("mlp_fp8_bwd");
}


// ================================================================================================
// Deep-ring forward (bf16): the per-panel kernel above keeps ONE 64-KB weight chunk in flight, and
// its step time is the DMA time of that chunk (~25 GB/s per CU: 2.5 us per chunk at C = 256, 16
// chunks); the LDS-DMA path delivers several times that with more bytes in flight
// (MI355X_MICROARCH.md, ring-gemm).  Here chunks are 32 hidden features (W1 [32][C] + W2 [C][32]
// = 128 C bytes) in an RS-stage ring with RS - 1 chunks in flight, and the waves split the panel by
// TOKENS: wave w owns tokens 16 w .. 16 w + 15 with every hidden feature of the chunk and every
// output feature (v_mfma_f32_16x16x32_bf16), so nothing is exchanged between waves.
//   GEMM1  h[32 hid][16 tok] = W1c x^T   (two 16-row tiles, k = C in steps of 32)
//   GELU   lane (tok, kg) holds hidden 4 kg + i of both tiles -> the 8 k-values of GEMM2's B
//          operand in the permuted order (4 kg + i, 16 + 4 kg + i); W2 is read in the same order
//   GEMM2  y[C][16 tok] += W2c g        (C / 16 tiles, one k-step of 32)
// Every step issues exactly one chunk's DMA (past the last chunk it re-fetches the last one into the
// free stage), so the wait for chunk j is a fixed count.
template <int C, int RS, bool DROP>
__global__ __launch_bounds__(MT) void mlp_fwd_deep(long M, const bf16* __restrict__ X, const bf16* __restrict__ W1,
                                                   const float* __restrict__ b1, const bf16* __restrict__ W2,
                                                   const float* __restrict__ b2, const float* __restrict__ res,
                                                   float* __restrict__ out, MlpDrop dd, long rpi) {
    constexpr int HD = 32;                 // hidden features per chunk
    constexpr int NCH = 4 * C / HD;
    constexpr int KS = C / 32;             // GEMM1 k-steps
    constexpr int OT = C / 16;             // output tiles
    constexpr int IMG1 = HD * C;           // bf16 of a W1 chunk image [32][C]
    constexpr int IMG2 = C * HD;           // and of a W2 chunk image [C][32]
    constexpr int STAGE = IMG1 + IMG2;
    using D1 = Dma<HD, 2 * C>;
    using D2 = Dma<C, 2 * HD>;
    constexpr int ND = D1::NW + D2::NW;    // DMA instructions per wave per chunk
    __shared__ __attribute__((aligned(1024))) bf16 ring[RS * STAGE];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int l16 = lane & 15, kg = lane >> 4;
    const int tok = 16 * wave + l16;
    const bool ok = tok < rows;
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;   // see mlp_fwd_kernel
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += MT) b1s[i] = b1[i];
    // x as GEMM1 B fragments: lane (tok, kg) of k-step s = x[tok][32 s + 8 kg .. + 7]
    bf16x8 xf[KS];
    {
        const auto rs = buf_rsrc(X + m0 * C, rows * C * 2);
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? (unsigned)(tok * C + 32 * s2 + 8 * kg) * 2 : kOOB, 0, 0);
            __builtin_memcpy(&xf[s2], &v, 16);
        }
    }
    D1 d1;
    D2 d2;
    d1.init(C, wave, lane);
    d2.init(4 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
    const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
    auto issue = [&](int j) {   // chunk min(j, NCH - 1) into stage j % RS
        const int jc = chk(j < NCH ? j : NCH - 1);
        bf16* st = ring + (j % RS) * STAGE;
        dma<D1::NW>(rs_w1, d1.v, (unsigned)jc * HD * C * 2, st, wave);
        dma<D2::NW>(rs_w2, d2.v, (unsigned)jc * HD * 2, st + IMG1, wave);
    };
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < RS - 1; ++j) issue(j);
    f32x4 acc[OT];
#pragma unroll
    for (int i = 0; i < OT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const long mg = m0 + tok;
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);
    __syncthreads();   // b1s
    for (int j = 0; j < NCH; ++j) {
        vmwait<(RS - 2) * ND>();          // chunk j landed (younger: chunks j + 1 .. j + RS - 2)
        lds_sync();                       // ... for every wave; stage (j - 1) % RS is free
        issue(j + RS - 1);
        const bf16* w1c = ring + (j % RS) * STAGE;
        const bf16* w2c = w1c + IMG1;
        const int jc = chk(j);
        f32x4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const bf16x8 a0 = frag(w1c, moff<2 * C>(l16, 32 * s2 + 8 * kg));
            const bf16x8 a1 = frag(w1c, moff<2 * C>(16 + l16, 32 * s2 + 8 * kg));
            h0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, xf[s2], h0, 0, 0, 0);
            h1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, xf[s2], h1, 0, 0, 0);
        }
        // GELU: hidden jc * 32 + 4 kg + i (tile 0) and + 16 (tile 1)
        const f32x4 bv0 = *reinterpret_cast<const f32x4*>(b1s + jc * HD + 4 * kg);
        const f32x4 bv1 = *reinterpret_cast<const f32x4*>(b1s + jc * HD + 16 + 4 * kg);
        float gv[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            gv[i] = gelu_fast(h0[i] + bv0[i]);
            gv[4 + i] = gelu_fast(h1[i] + bv1[i]);
        }
        if constexpr (DROP) {
            if (dd.p > 0.f) {
                const uint64_t e0 = (uint64_t)mg * 4 * C + jc * HD + 4 * kg;   // 4-aligned; its 8-group
                const unsigned m0b = keep8(Rh, e0 >> 3) >> (e0 & 7);
                const unsigned m1b = keep8(Rh, (e0 + 16) >> 3) >> ((e0 + 16) & 7);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    gv[i] = ((m0b >> i) & 1u) ? gv[i] * Rh.scale : 0.f;
                    gv[4 + i] = ((m1b >> i) & 1u) ? gv[4 + i] * Rh.scale : 0.f;
                }
            }
        }
        bf16x8 gb;
#pragma unroll
        for (int i = 0; i < 8; ++i) gb[i] = (bf16)gv[i];
#pragma unroll
        for (int ot = 0; ot < OT; ++ot) {   // A: W2[out][hidden 4 kg + i, 16 + 4 kg + i] (the same k order)
            const bf16x4 lo = *reinterpret_cast<const bf16x4*>(w2c + moff<2 * HD>(16 * ot + l16, 4 * kg));
            const bf16x4 hi = *reinterpret_cast<const bf16x4*>(w2c + moff<2 * HD>(16 * ot + l16, 16 + 4 * kg));
            const bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            acc[ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, gb, acc[ot], 0, 0, 0);
        }
    }
    // epilogue: acc[ot][i] = y[tok][16 ot + 4 kg + i]
    const auto rs_res = buf_rsrc(res + m0 * C, rows * C * 4);
    const auto rs_out = buf_rsrc(out + m0 * C, rows * C * 4);
    float sdp = 1.f;
    DropoutRng R;
    if constexpr (DROP) {
        R = load_rng(dd.rng, dd.site_o, dd.p);
        if (dd.row_scale) sdp = dd.row_scale[mg / dd.rps];
    }
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
        const int f = 16 * ot + 4 * kg;
        const unsigned off = ok ? (unsigned)(tok * C + f) * 4 : kOOB;
        float rv[4], bv[4], v[4];
        buf_ld4(rs_res, off, rv);
        load4(b2 + f, bv);
        unsigned km = 0xfu;
        if constexpr (DROP) if (dd.p > 0.f) {
            const uint64_t e = (uint64_t)mg * C + f;
            km = keep8(R, e >> 3) >> (e & 7);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float z = acc[ot][e] + bv[e];
            if constexpr (DROP) z *= ((km >> e) & 1u) ? sdp * R.scale : 0.f;
            v[e] = z + rv[e];
        }
        buf_st4(rs_out, off, v);
    }
    vmwait<0>();   // the re-fetch DMAs drained before the workgroup's LDS is released
}

template <int C, int RS>
int fwd_deep_launch(long M, const void* x, const void* w1, const float* b1, const void* w2, const float* b2, const float* res,
                    float* out, const MlpDrop* d, long rpi, hipStream_t st) {
    const dim3 grid((unsigned)((M + BM - 1) / BM));
    if (d)
        mlp_fwd_deep<C, RS, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2, res, out, *d, rpi);
    else
        mlp_fwd_deep<C, RS, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)w1, b1, (const bf16*)w2, b2, res, out,
                                                        MlpDrop{}, rpi);
    return check_launch("mlp_fwd (deep)");
}


// 16x16x32 operand fragments transposed out of a moff<RB> image whose ROWS are k and COLUMNS are i
// (ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3 and receives
// column l of the 4 rows):  A[i = c0 + (lane & 15)][k], k = k0 + 8 kg + 0..7 (natural order) ...
template <int RB>
__device__ __forceinline__ bf16x8 tr16n(const bf16* img, int c0, int k0, int lane) {
    const int kg = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    return cat8(tr4(img + moff<RB>(k0 + 8 * kg + q, c0 + 4 * p)), tr4(img + moff<RB>(k0 + 8 * kg + 4 + q, c0 + 4 * p)));
}
// ... or k = k0 + 4 kg + 0..3, k0 + 16 + 4 kg + 0..3 (the deep-ring kernels' permuted hidden order)
template <int RB>
__device__ __forceinline__ bf16x8 tr16p(const bf16* img, int c0, int k0, int lane) {
    const int kg = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    return cat8(tr4(img + moff<RB>(k0 + 4 * kg + q, c0 + 4 * p)), tr4(img + moff<RB>(k0 + 16 + 4 * kg + q, c0 + 4 * p)));
}

template <int N> __device__ __forceinline__ void vmwait_le(int c) {   // s_waitcnt vmcnt(c), c in [0, N] (c multiple of 4)
    if constexpr (N >= 4) {
        if (c >= N) { vmwait<N>(); return; }
        vmwait_le<N - 4>(c);
    } else {
        vmwait<0>();
    }
}

// Deep-ring backward (bf16): the forward's chunking and token split.  Per chunk j (32 hidden):
//   GEMM1  h  = W1c x^T                      (A: W1 image rows, as the forward)
//   GEMM3  dg = W2c^T dY^T                   (A: transposed reads of the W2 image [C][32], k = C natural)
//   dh = dg * gelu'(h) (* hidden mask), g = gelu(h) (* mask): stored (bf16) for the weight gradients
//   GEMM4  dx += W1c^T dh                    (A: transposed reads of the W1 image, k = the chunk's hidden
//                                             features in the permuted order the accumulators give)
// The wait for chunk j counts its younger DMAs and this wave's 4 stores per step since.
template <int C, int RS, bool DROP>
__global__ __launch_bounds__(MT) void mlp_bwd_deep(long M, const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                   const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                   const bf16* __restrict__ W2, bf16* __restrict__ dH, bf16* __restrict__ G,
                                                   bf16* __restrict__ dX, MlpDrop dd, long rpi) {
    constexpr int HD = 32;
    constexpr int NCH = 4 * C / HD;
    constexpr int KS = C / 32;
    constexpr int OT = C / 16;
    constexpr int IMG1 = HD * C;
    constexpr int IMG2 = C * HD;
    constexpr int STAGE = IMG1 + IMG2;
    using D1 = Dma<HD, 2 * C>;
    using D2 = Dma<C, 2 * HD>;
    constexpr int ND = D1::NW + D2::NW;
    constexpr int NS = 4;                  // buffer stores per lane per chunk (G, dH: 2 x 8 B each)
    __shared__ __attribute__((aligned(1024))) bf16 ring[RS * STAGE];
    __shared__ __attribute__((aligned(16))) float b1s[4 * C];

    const long m0 = (long)blockIdx.x * BM;
    const long rows = M - m0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int l16 = lane & 15, kg = lane >> 4;
    const int tok = 16 * wave + l16;
    const bool ok = tok < rows;
    const int j0 = kRot && rpi > 0 && rpi % BM == 0 ? (int)(((m0 % rpi) / BM) & (NCH - 1)) : 0;
    auto chk = [&](int j) { return (j + j0) & (NCH - 1); };
    for (int i = threadIdx.x; i < 4 * C; i += MT) b1s[i] = b1[i];
    bf16x8 xf[KS], yf[KS];
    {
        const auto rx = buf_rsrc(X + m0 * C, rows * C * 2);
        const auto ry = buf_rsrc(dY + m0 * C, rows * C * 2);
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const unsigned o = ok ? (unsigned)(tok * C + 32 * s2 + 8 * kg) * 2 : kOOB;
            const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0);
            const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(ry, o, 0, 0);
            __builtin_memcpy(&xf[s2], &a, 16);
            __builtin_memcpy(&yf[s2], &b, 16);
        }
    }
    D1 d1;
    D2 d2;
    d1.init(C, wave, lane);
    d2.init(4 * C, wave, lane);
    const i32x4 rs_w1 = rsrc4(W1, 4L * C * C * 2);
    const i32x4 rs_w2 = rsrc4(W2, 4L * C * C * 2);
    const auto rs_dh = buf_rsrc(dH + m0 * 4 * C, rows * 4 * C * 2);
    const auto rs_g = buf_rsrc(G + m0 * 4 * C, rows * 4 * C * 2);
    auto issue = [&](int j) {
        const int jc = chk(j < NCH ? j : NCH - 1);
        bf16* st = ring + (j % RS) * STAGE;
        dma<D1::NW>(rs_w1, d1.v, (unsigned)jc * HD * C * 2, st, wave);
        dma<D2::NW>(rs_w2, d2.v, (unsigned)jc * HD * 2, st + IMG1, wave);
    };
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < RS - 1; ++j) issue(j);
    f32x4 acc[OT];
#pragma unroll
    for (int i = 0; i < OT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const long mg = m0 + tok;
    DropoutRng Rh;
    if constexpr (DROP) Rh = load_rng(dd.rng, dd.site_h, dd.p);
    __syncthreads();
    for (int j = 0; j < NCH; ++j) {
        vmwait_le<(RS - 2) * ND + NS * (RS - 1)>((RS - 2) * ND + NS * (j < RS - 1 ? j : RS - 1));
        lds_sync();
        issue(j + RS - 1);
        const bf16* w1c = ring + (j % RS) * STAGE;
        const bf16* w2c = w1c + IMG1;
        const int jc = chk(j);
        f32x4 h[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}}, dg[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                h[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(w1c, moff<2 * C>(16 * t + l16, 32 * s2 + 8 * kg)), xf[s2], h[t],
                                                              0, 0, 0);
                dg[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr16n<2 * HD>(w2c, 16 * t, 32 * s2, lane), yf[s2], dg[t], 0, 0, 0);
            }
        // lane (tok, kg): hidden jc * 32 + 16 t + 4 kg + i
        float gv[8], dv[8];
        unsigned km[2] = {0xfu, 0xfu};
        if constexpr (DROP) if (dd.p > 0.f) {
            const uint64_t e0 = (uint64_t)mg * 4 * C + jc * HD + 4 * kg;
            km[0] = keep8(Rh, e0 >> 3) >> (e0 & 7);
            km[1] = keep8(Rh, (e0 + 16) >> 3) >> ((e0 + 16) & 7);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(b1s + jc * HD + 16 * t + 4 * kg);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float g, dgl;
                gelu_pair_fast(h[t][i] + bv[i], g, dgl);
                if constexpr (DROP) {
                    const float ms = ((km[t] >> i) & 1u) ? Rh.scale : 0.f;
                    g *= ms;
                    dgl *= ms;
                }
                gv[4 * t + i] = g;
                dv[4 * t + i] = dg[t][i] * dgl;
            }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const unsigned o = ok ? (unsigned)(tok * 4 * C + jc * HD + 16 * t + 4 * kg) * 2 : kOOB;
            buf_st4bf(rs_g, o, gv + 4 * t);
            buf_st4bf(rs_dh, o, dv + 4 * t);
        }
        bf16x8 db;
#pragma unroll
        for (int i = 0; i < 8; ++i) db[i] = (bf16)dv[i];
#pragma unroll
        for (int ot = 0; ot < OT; ++ot)
            acc[ot] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr16p<2 * C>(w1c, 16 * ot, 0, lane), db, acc[ot], 0, 0, 0);
    }
    const auto rs_dx = buf_rsrc(dX + m0 * C, rows * C * 2);
#pragma unroll
    for (int ot = 0; ot < OT; ++ot) {
        float v[4] = {acc[ot][0], acc[ot][1], acc[ot][2], acc[ot][3]};
        buf_st4bf(rs_dx, ok ? (unsigned)(tok * C + 16 * ot + 4 * kg) * 2 : kOOB, v);
    }
    vmwait<0>();
}

template <int C, int RS>
int bwd_deep_launch(long M, const void* x, const void* dy, const void* w1, const float* b1, const void* w2, void* dh, void* g,
                    void* dx, const MlpDrop* d, long rpi, hipStream_t st) {
    const dim3 grid((unsigned)((M + BM - 1) / BM));
    if (d)
        mlp_bwd_deep<C, RS, true><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                       (bf16*)dh, (bf16*)g, (bf16*)dx, *d, rpi);
    else
        mlp_bwd_deep<C, RS, false><<<grid, MT, 0, st>>>(M, (const bf16*)x, (const bf16*)dy, (const bf16*)w1, b1, (const bf16*)w2,
                                                        (bf16*)dh, (bf16*)g, (bf16*)dx, MlpDrop{}, rpi);
    return check_launch("mlp_bwd (deep)");
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_mlp_supported(int C) { return C == 64 || C == 128 || C == 256; }

static int mlp_drop_of(const csu_mlp_dropout* d, MlpDrop& md) {
    if (!d) return 0;
    if (d->p < 0.f || d->p >= 1.f || (d->p > 0.f && !d->rng) || (d->row_scale && d->rows_per_sample < 1))
        return fail(CSU_E_ARG, "mlp: bad dropout descriptor (0 <= p < 1, rng for p > 0, rows_per_sample >= 1)");
    md = MlpDrop{d->rng, d->site_hidden, d->site_out, d->p, d->row_scale, (long)d->rows_per_sample};
    return d->p > 0.f || d->row_scale ? 0 : 1;   // 1: nothing to apply -> the dropout-free kernel
}

extern "C" int csu_mlp_fwd_dp(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                              const float* res, float* out, const csu_mlp_dropout* d, void* stream) {
    if (M < 1 || !x || !w1 || !b1 || !w2 || !b2 || !res || !out) return fail(CSU_E_ARG, "mlp_fwd: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_fwd: tensor exceeds 2 GB buffer range");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;   // rows per image: the hidden-chunk rotation
    const hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return fwd_launch<64>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
        case 128: return fwd_launch<128>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
        case 256: return fwd_launch<256>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
        default: return fail(CSU_E_ARG, "mlp_fwd: C must be 64, 128 or 256");
    }
}

extern "C" int csu_mlp_fwd_ln(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                              const float* res, float* out, const csu_mlp_dropout* d, const float* ln_gamma,
                              const float* ln_beta, float ln_eps, void* ln_out, float* ln_mean, float* ln_rstd,
                              void* stream) {
    if (M < 1 || !x || !w1 || !b1 || !w2 || !b2 || !res || !out || !ln_gamma || !ln_beta || !ln_out || !ln_mean || !ln_rstd)
        return fail(CSU_E_ARG, "mlp_fwd_ln: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_fwd_ln: tensor exceeds 2 GB buffer range");
    if (res == out) return fail(CSU_E_ARG, "mlp_fwd_ln: out must not alias res");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const MlpLn ln{ln_gamma, ln_beta, ln_eps, (bf16*)ln_out, ln_mean, ln_rstd};
    const hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return fwd_launch<64>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st, &ln);
        case 128: return fwd_launch<128>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st, &ln);
        case 256: return fwd_launch<256>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st, &ln);
        default: return fail(CSU_E_ARG, "mlp_fwd_ln: C must be 64, 128 or 256");
    }
}

extern "C" int csu_mlp_fwd(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                           const float* res, float* out, void* stream) {
    return csu_mlp_fwd_dp(M, C, x, w1, b1, w2, b2, res, out, nullptr, stream);
}

extern "C" int csu_mlp_bwd_dp(long M, int C, const void* x, const void* dy, const void* w1, const float* b1, const void* w2,
                              void* dh, void* g, void* dx, const csu_mlp_dropout* d, void* stream) {
    if (M < 1 || !x || !dy || !w1 || !b1 || !w2 || !dh || !g || !dx) return fail(CSU_E_ARG, "mlp_bwd: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_bwd: tensor exceeds 2 GB buffer range");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return bwd_launch<64>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
        // C = 128: the deep ring (4 chunks of 32 hidden in flight) measured 61.0 vs 75.2 us at 65536
        // tokens (profiles/r06b_mlp8_probe.txt); C = 64 / 256: the per-panel kernels (equal or faster)
        case 128: return bwd_deep_launch<128, 4>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
        case 256: return bwd_launch<256>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
        default: return fail(CSU_E_ARG, "mlp_bwd: C must be 64, 128 or 256");
    }
}

extern "C" int csu_mlp_bwd(long M, int C, const void* x, const void* dy, const void* w1, const float* b1, const void* w2,
                           void* dh, void* g, void* dx, void* stream) {
    return csu_mlp_bwd_dp(M, C, x, dy, w1, b1, w2, dh, g, dx, nullptr, stream);
}

extern "C" int csu_mlp_fp8_supported(int C) { return C == 64 || C == 128 || C == 256; }

extern "C" int csu_mlp_fp8_fwd_ln(long M, int C, const void* x, const void* w1q, const float* sw1, const float* b1,
                                  const void* w2p, const float* sw2, const float* b2, const float* res, float* out,
                                  const csu_mlp_dropout* d, const float* ln_gamma, const float* ln_beta, float ln_eps,
                                  void* ln_out, float* ln_mean, float* ln_rstd, void* stream) {
    if (M < 1 || !x || !w1q || !sw1 || !b1 || !w2p || !sw2 || !b2 || !res || !out || !ln_gamma || !ln_beta || !ln_out ||
        !ln_mean || !ln_rstd)
        return fail(CSU_E_ARG, "mlp_fp8_fwd_ln: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_fp8_fwd_ln: tensor exceeds 2 GB buffer range");
    if (res == out) return fail(CSU_E_ARG, "mlp_fp8_fwd_ln: out must not alias res");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const MlpLn ln{ln_gamma, ln_beta, ln_eps, (bf16*)ln_out, ln_mean, ln_rstd};
    const hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return fp8_fwd_launch<64>(M, x, w1q, sw1, b1, w2p, sw2, b2, res, out, dp, rpi, st, &ln);
        case 128: return fp8_fwd_launch<128>(M, x, w1q, sw1, b1, w2p, sw2, b2, res, out, dp, rpi, st, &ln);
        case 256: return fp8_fwd_launch<256>(M, x, w1q, sw1, b1, w2p, sw2, b2, res, out, dp, rpi, st, &ln);
        default: return fail(CSU_E_UNSUPPORTED, "mlp_fp8_fwd_ln: C must be 64, 128 or 256");
    }
}

extern "C" int csu_mlp_fp8_fwd(long M, int C, const void* x, const void* w1q, const float* sw1, const float* b1,
                               const void* w2p, const float* sw2, const float* b2, const float* res, float* out,
                               const csu_mlp_dropout* d, void* stream) {
    if (M < 1 || !x || !w1q || !sw1 || !b1 || !w2p || !sw2 || !b2 || !res || !out)
        return fail(CSU_E_ARG, "mlp_fp8_fwd: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_fp8_fwd: tensor exceeds 2 GB buffer range");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return fp8_fwd_launch<64>(M, x, w1q, sw1, b1, w2p, sw2, b2, res, out, dp, rpi, st);
        case 128: return fp8_fwd_launch<128>(M, x, w1q, sw1, b1, w2p, sw2, b2, res, out, dp, rpi, st);
        case 256: return fp8_fwd_launch<256>(M, x, w1q, sw1, b1, w2p, sw2, b2, res, out, dp, rpi, st);
        default: return fail(CSU_E_UNSUPPORTED, "mlp_fp8_fwd: C must be 64, 128 or 256");
    }
}

extern "C" int csu_mlp_fp8_bwd(long M, int C, const void* x, const void* dy, const void* w1q, const float* sw1,
                               const float* b1, const void* w2t, const float* sw2, const void* w1tp, void* dh, void* g,
                               void* dx, const csu_mlp_dropout* d, void* stream) {
    if (M < 1 || !x || !dy || !w1q || !sw1 || !b1 || !w2t || !sw2 || !w1tp || !dh || !g || !dx)
        return fail(CSU_E_ARG, "mlp_fp8_bwd: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_fp8_bwd: tensor exceeds 2 GB buffer range");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const hipStream_t st = as_stream(stream);
    switch (C) {
        case 64: return fp8_bwd_launch<64>(M, x, dy, w1q, sw1, b1, w2t, sw2, w1tp, dh, g, dx, dp, rpi, st);
        case 128: return fp8_bwd_launch<128>(M, x, dy, w1q, sw1, b1, w2t, sw2, w1tp, dh, g, dx, dp, rpi, st);
        case 256: return fp8_bwd_launch<256>(M, x, dy, w1q, sw1, b1, w2t, sw2, w1tp, dh, g, dx, dp, rpi, st);
        default: return fail(CSU_E_UNSUPPORTED, "mlp_fp8_bwd: C must be 64, 128 or 256");
    }
}

// explicit forward variant (tests, tools/mlp8_probe.py): cfg 0 = the per-panel kernel, 1 = the deep ring
extern "C" int csu_mlp_fwd_ex(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                              const float* res, float* out, const csu_mlp_dropout* d, int cfg, void* stream) {
    if (cfg == 0) return csu_mlp_fwd_dp(M, C, x, w1, b1, w2, b2, res, out, d, stream);
    if (cfg != 1 && cfg != 2) return fail(CSU_E_ARG, "mlp_fwd_ex: cfg 0, 1 or 2");
    if (M < 1 || !x || !w1 || !b1 || !w2 || !b2 || !res || !out) return fail(CSU_E_ARG, "mlp_fwd: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_fwd: tensor exceeds 2 GB buffer range");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const hipStream_t st = as_stream(stream);
    if (cfg == 2) {   // deeper rings
        switch (C) {
            case 64: return fwd_deep_launch<64, 8>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
            case 128: return fwd_deep_launch<128, 6>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
            case 256: return fwd_deep_launch<256, 3>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
            default: return fail(CSU_E_ARG, "mlp_fwd: C must be 64, 128 or 256");
        }
    }
    switch (C) {
        case 64: return fwd_deep_launch<64, 6>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
        case 128: return fwd_deep_launch<128, 4>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
        case 256: return fwd_deep_launch<256, 4>(M, x, w1, b1, w2, b2, res, out, dp, rpi, st);
        default: return fail(CSU_E_ARG, "mlp_fwd: C must be 64, 128 or 256");
    }
}

// explicit backward variant: cfg 0 = the per-panel / persistent kernels, 1 / 2 = the deep ring (csu_mlp_bwd_dp:
// cfg 1 at C = 128, cfg 0 otherwise)
extern "C" int csu_mlp_bwd_ex(long M, int C, const void* x, const void* dy, const void* w1, const float* b1, const void* w2,
                              void* dh, void* g, void* dx, const csu_mlp_dropout* d, int cfg, void* stream) {
    if (cfg != 0 && cfg != 1 && cfg != 2) return fail(CSU_E_ARG, "mlp_bwd_ex: cfg 0, 1 or 2");
    if (M < 1 || !x || !dy || !w1 || !b1 || !w2 || !dh || !g || !dx) return fail(CSU_E_ARG, "mlp_bwd: bad arguments");
    if (M * 4L * C * 2 > 0x7fffffffL) return fail(CSU_E_ARG, "mlp_bwd: tensor exceeds 2 GB buffer range");
    MlpDrop md{};
    const int e = mlp_drop_of(d, md);
    if (e < 0) return e;
    const MlpDrop* dp = d && e == 0 ? &md : nullptr;
    const long rpi = d ? (long)d->rows_per_sample : 0;
    const hipStream_t st = as_stream(stream);
    if (cfg == 0) {   // the per-panel / persistent kernels
        switch (C) {
            case 64: return bwd_launch<64>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
            case 128: return bwd_launch<128>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
            case 256: return bwd_launch<256>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
            default: return fail(CSU_E_ARG, "mlp_bwd: C must be 64, 128 or 256");
        }
    }
    if (cfg == 2) {
        switch (C) {
            case 64: return bwd_deep_launch<64, 8>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
            case 128: return bwd_deep_launch<128, 6>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
            case 256: return bwd_deep_launch<256, 3>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
            default: return fail(CSU_E_ARG, "mlp_bwd: C must be 64, 128 or 256");
        }
    }
    switch (C) {
        case 64: return bwd_deep_launch<64, 6>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
        case 128: return bwd_deep_launch<128, 4>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
        case 256: return bwd_deep_launch<256, 4>(M, x, dy, w1, b1, w2, dh, g, dx, dp, rpi, st);
        default: return fail(CSU_E_ARG, "mlp_bwd: C must be 64, 128 or 256");
    }
}
