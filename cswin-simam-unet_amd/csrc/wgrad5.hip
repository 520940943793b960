// wgrad5: Linear weight + bias gradient over token rows with a deep LDS-DMA pipeline (gfx950).
//
//   dW[n][k] = sum_m dY[m][n] * X[m][k],   db[n] = sum_m dY[m][n]       (m = the B*L tokens)
//
// Same contract and split-K slab layout as wgrad_bf16_tr (wgrad.hip): workgroup (n-tile, k-tile,
// token chunk) writes its 128x128 partial tile (and, for k-tile 0, its db partial) to slab `chunk`
// of [chunk][N*K + N]; one fixed-order column-sum pass reduces the slabs (bitwise reproducible).
//
// Why another kernel: the register-staged kernel keeps one 64-token step in flight per workgroup,
// and PMC shows it waiting on memory (waitcnt ~35-60 % of wave cycles) while the operand re-reads
// already hit L2 (FETCH_SIZE = the algorithmic bytes).  Here the two operand panels of TMS tokens
// stream through an S-stage LDS ring by buffer_load ... lds DMA (inline asm: the compiler would
// otherwise wait vmcnt(0) before every LDS read), S-1 stages in flight, one barrier per stage.
//  * images are [TMS tokens][128 features] bf16 (256-B rows) with the row-bit-reversal XOR
//    swizzle of lds_dma.hpp: the ds_read_b64_tr_b16 gathers of both MFMA operands (k = tokens)
//    are bank-conflict free;
//  * 4 waves in 2 x 2, each 64 x 64 of the tile (2 x 2 v_mfma_f32_32x32x16_bf16 accumulators);
//  * the bias partial is an MFMA against a constant all-ones B fragment (k-tile-0 workgroups,
//    waves with wk = 0): db rides the matrix pipe instead of VALU column sums;
//  * the token chunk's rows are the buffer range, so rows past the chunk read as 0 and columns
//    past N or K only feed outputs that are not stored.
#include "lds_dma.hpp"

namespace csu {
namespace {

constexpr int W5_NT = 256;
constexpr int W5_T = 128;

template <int TMS, int S>
__global__ __launch_bounds__(W5_NT) void wgrad5_kernel(long M, int N, int K, long rpc, const bf16* __restrict__ dy,
                                                       const bf16* __restrict__ x, float* __restrict__ part) {
    constexpr int IMG = TMS * W5_T;             // bf16 per operand image
    constexpr int STG = 2 * IMG;
    using DA = Dma<TMS, 2 * W5_T>;
    constexpr int NW = DA::NW;                  // DMA instructions per wave per operand per stage
    __shared__ __attribute__((aligned(1024))) bf16 ring[S * STG];

    const int nt = (N + W5_T - 1) / W5_T, kt = (K + W5_T - 1) / W5_T;
    const long t = xcd_tile(blockIdx.x, gridDim.x);   // tiles of one chunk on one XCD
    const int chunk = (int)(t / (nt * kt)), tt = (int)(t % (nt * kt));
    const int n0 = (tt / kt) * W5_T, k0 = (tt % kt) * W5_T;
    const long m_begin = (long)chunk * rpc;
    const long m_end = min(M, m_begin + rpc);
    const int nsteps = (int)((m_end - m_begin + TMS - 1) / TMS);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave >> 1) * 64, wk = (wave & 1) * 64;
    const bool do_bias = k0 == 0 && wk == 0;

    DA da, db;
    da.init(N, wave, lane);
    db.init(K, wave, lane);
    const long rows = m_end - m_begin;
    const i32x4 rs_a = rsrc4(dy + m_begin * N + n0, rows * N * 2 - (long)n0 * 2);
    const i32x4 rs_b = rsrc4(x + m_begin * K + k0, rows * K * 2 - (long)k0 * 2);
    auto issue = [&](int s) {
        bf16* st = ring + (s % S) * STG;
        dma<NW>(rs_a, da.v, (unsigned)s * TMS * N * 2, st, wave);
        dma<NW>(rs_b, db.v, (unsigned)s * TMS * K * 2, st + IMG, wave);
    };
    // vmcnt(8 n) for n later stages in flight (immediate operand)
    auto wait_stage = [&](int later) {
        switch (later) {
            case 0: vmwait<0>(); break;
            case 1: vmwait<2 * NW>(); break;
            case 2: vmwait<4 * NW>(); break;
            default: vmwait<6 * NW>(); break;
        }
    };
    static_assert(S <= 4, "wait_stage covers at most 3 stages in flight");

    asm volatile("" ::: "memory");
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
        if (p < nsteps) issue(p);

    f32x16 acc[2][2], accb[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        accb[a] = f32x16{};
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
    }
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;

    for (int s = 0; s < nsteps; ++s) {
        const int later = min(S - 2, nsteps - 1 - s);   // stages issued after stage s
        wait_stage(later);
        lds_sync();                                     // stage s landed for all waves; stage s-1 free
        if (s + S - 1 < nsteps) issue(s + S - 1);
        const bf16* ia = ring + (s % S) * STG;
        const bf16* ib = ia + IMG;
#pragma unroll
        for (int kk = 0; kk < TMS / 16; ++kk) {
            bf16x8 fa[2], fb[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) fa[a] = trfrag<2 * W5_T>(ia, wn + 32 * a, kk, lane);
#pragma unroll
            for (int b = 0; b < 2; ++b) fb[b] = trfrag<2 * W5_T>(ib, wk + 32 * b, kk, lane);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
            if (do_bias)
#pragma unroll
                for (int a = 0; a < 2; ++a) accb[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], ones, accb[a], 0, 0, 0);
        }
    }

    // acc[a][b][reg] = dW[n0 + wn + 32a + crow(reg, h)][k0 + wk + 32b + r]
    const long slab = (long)N * K + N;
    float* out = part + (long)chunk * slab;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = n0 + wn + 32 * a + crow(reg, h), k = k0 + wk + 32 * b + r;
                if (n < N && k < K) out[(long)n * K + k] = acc[a][b][reg];
            }
    if (do_bias && r == 0) {   // every column of accb holds the token sum of row n
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = n0 + wn + 32 * a + crow(reg, h);
                if (n < N) out[(long)N * K + n] = accb[a][reg];
            }
    }
}

}  // namespace

// cfg: 0 -> TMS 64, S 4 (128 KB LDS, 1 workgroup / CU); 1 -> TMS 32, S 4 (64 KB, 2 / CU);
//      2 -> TMS 64, S 3 (96 KB)
int wgrad5_launch(int cfg, long M, int N, int K, long rpc, int chunks, const bf16* dy, const bf16* x, float* part,
                  hipStream_t st) {
    const int tiles = ((N + W5_T - 1) / W5_T) * ((K + W5_T - 1) / W5_T);
    const dim3 grid((unsigned)(tiles * chunks));
    switch (cfg) {
        case 1: wgrad5_kernel<32, 4><<<grid, W5_NT, 0, st>>>(M, N, K, rpc, dy, x, part); break;
        case 2: wgrad5_kernel<64, 3><<<grid, W5_NT, 0, st>>>(M, N, K, rpc, dy, x, part); break;
        default: wgrad5_kernel<64, 4><<<grid, W5_NT, 0, st>>>(M, N, K, rpc, dy, x, part); break;
    }
    return check_launch("wgrad5");
}

}  // namespace csu
