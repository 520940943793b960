// gemm4: token GEMM for gfx950 with LDS-DMA operand staging and a register epilogue.
//
//   out[m][n] = epi( sum_k A[m][k] * W[n][k] )      A (M, K) tokens, W (N, K) nn.Linear weight
//
// The nn.Linear forward / input-gradient GEMMs of CSWinBlock / Mlp (cswin:185-195, 314-368) and
// concat_linear (cswin:568-592) with bias / GELU / GELU' / residual fused into the epilogue.
//
// Design (MI355X):
//  * 256 threads = 4 waves in 2 x 2, tile BM x BN in {64,128}^2, BK = 64.
//  * Both operands go global -> LDS by global_load_lds_dwordx4 (no VGPR round trip): one wave
//    instruction fills 8 rows x 128 B of a [rows][64] bf16 image whose 16-B chunks are XOR-swizzled
//    by (row & 7) -- the swizzle is applied to the per-lane SOURCE address (the DMA destination is
//    lane-linear) and to the fragment reads, so ds_read_b128 fragment reads are conflict-free.
//  * Two LDS stages; the next K slice's DMA stays in flight across the barrier (counted vmcnt,
//    raw s_barrier), so a workgroup overlaps its own loads with its MFMAs.
//  * v_mfma_f32_32x32x16_bf16 with the WEIGHT fragment as the A operand: the accumulator of lane
//    (r, h) holds token r and features crow(reg, h) = 4 consecutive features per register group,
//    so the epilogue reads bias / GELU-aux / residual and writes outputs as 4-wide vectors
//    straight from registers (no LDS staging, no barriers).
//  * XCD-aware tile order (xcd_tile): the N tiles of one token panel run on one XCD's L2.
#include "lds_dma.hpp"

namespace csu {
namespace {


#ifdef G4_TIMING   // debug build only: per-workgroup phase timestamps (s_memtime), read by csu_debug_g4_ts
__device__ unsigned long long g4_ts[8][4096];
#define G4_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g4_ts[k][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define G4_STAMP(k) do {} while (0)
#endif
constexpr int G4_BK = 64;


enum { G4_PLAIN = 0, G4_GELU_OUT = 1, G4_GAUX = 2, G4_RESID = 3 };

// element offset of 16-B chunk `chunk` of row `row` in a swizzled [rows][64] bf16 image
__device__ __forceinline__ int g4_off(int row, int chunk) { return row * G4_BK + ((chunk ^ (row & 7)) << 3); }

// Per-lane byte offsets of the DMA of a ROWS x 64 bf16 slice (rows 0.., k 0..63 relative to the
// slice origin) of a row-major matrix with leading dimension ld into a swizzled [ROWS][64] image:
// wave instruction i of this wave fills image rows rb..rb+7 (rb = (wave * ROWS/32 + i) * 8), lane l
// row rb + l/8, 16-B chunk (l & 7) ^ (row & 7).  Constant for the whole kernel.
template <int ROWS, int NWV = 4>
__device__ __forceinline__ void g4_voff(int ld, int wave, int lane, unsigned* voff) {
    constexpr int NI = ROWS / (8 * NWV);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int row = (wave * NI + i) * 8 + (lane >> 3);
        voff[i] = (unsigned)row * ld * 2 + (((lane & 7) ^ (row & 7)) << 4);
    }
}

// DMA the slice: raw buffer loads to LDS from a resource whose base is the slice's first row and
// whose size ends at the matrix's last row, so rows past the end read as 0 (hardware range check);
// soff = the k offset in bytes (scalar).  Only scalar work per call: the lane offsets are fixed.
template <int ROWS, int NWV = 4>
__device__ __forceinline__ void g4_dma(i32x4 rs, const unsigned* voff, unsigned soff, bf16* img, int wave) {
    constexpr int NI = ROWS / (8 * NWV);
    // inline asm (lds_dma.hpp): the compiler would otherwise wait vmcnt(0) before LDS reads that may
    // alias an in-flight DMA stage, which makes every ring deeper than 2 stages useless
    dma<NI>(rs, voff, soff, img, wave);   // same lane-linear 1-KB blocks: (wave * NI + i) * 512
}

template <int N> __device__ __forceinline__ void g4_vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <typename T> struct V4;
template <> struct V4<float> {
    static __device__ __forceinline__ void ld(const float* p, float* v) { load4(p, v); }
    static __device__ __forceinline__ void st(float* p, const float* v) { store4(p, v); }
};
template <> struct V4<bf16> {
    static __device__ __forceinline__ void ld(const bf16* p, float* v) { load4(p, v); }
    static __device__ __forceinline__ void st(bf16* p, const float* v) { store4(p, v); }
};

// s_waitcnt vmcnt(k) for the largest multiple of 8 <= c (waiting for more than needed is safe)
__device__ __forceinline__ void g4_vmwait_floor(int c) {
    switch (c >= 63 ? 7 : c >> 3) {
        case 0: g4_vmwait<0>(); break;
        case 1: g4_vmwait<8>(); break;
        case 2: g4_vmwait<16>(); break;
        case 3: g4_vmwait<24>(); break;
        case 4: g4_vmwait<32>(); break;
        case 5: g4_vmwait<40>(); break;
        case 6: g4_vmwait<48>(); break;
        default: g4_vmwait<56>(); break;
    }
}

// Persistent workgroups, S-stage LDS ring.  A workgroup walks its tiles' K slices as one stream of
// "units" (tile, k-slice); the DMA of unit u + S - 1 is issued while unit u is multiplied, so the
// loads of the next tile overlap the last slices and the epilogue of the current one.
// vmcnt counts every vector-memory op of a wave in issue order (DMA, loads, stores), so the wait for
// unit u counts exactly the ops issued after its DMA.  Every step issues exactly D DMA ops (past
// the last unit it re-fetches the last unit into the free stage), and a tile's last step issues
// its L epilogue loads BEFORE its DMA (so waiting for them does not wait for the prefetch) and its
// ST stores after the MFMAs.
// F8: e4m3 operands (BASELINE config 5): A (M, K) / W (N, K) are e4m3 BYTE matrices with one fp32
// scale per row (sa per token, sw per output feature), K counted in bytes; a 128-byte K slice (the
// bf16 slice's bytes) is two k-steps of v_mfma_scale_f32_32x32x64_f8f6f4 at unit block scales, and
// the epilogue multiplies by sa[m] sw[n] before the bias.  lda / ldw are then given in bf16 units
// (bytes / 2) so that the DMA code is shared.
template <int BM, int BN, int S, int OCC, int EPI, typename TOUT, int WM = 2, int WN = 2, bool F8 = false>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm4_kernel(long M, int N, int K, const bf16* __restrict__ A, int lda,
                                                           const bf16* __restrict__ W, int ldw, const float* __restrict__ bias,
                                                           const bf16* __restrict__ gaux, const float* __restrict__ resid,
                                                           TOUT* __restrict__ out, bf16* __restrict__ gout, int ldc,
                                                           const float* __restrict__ sa = nullptr,
                                                           const float* __restrict__ sw = nullptr) {
    constexpr int NWV = WM * WN;                     // waves: WM along tokens x WN along features
    constexpr int TMW = BM / (32 * WM), TNW = BN / (32 * WN);   // 32x32 tiles per wave (tokens, features)
    static_assert(TMW >= 1 && TNW >= 1 && BM % (8 * NWV) == 0 && BN % (8 * NWV) == 0, "gemm4 wave layout");
    constexpr int STAGE = (BM + BN) * G4_BK;         // bf16 elements per stage
    constexpr int D = (BM + BN) / (8 * NWV);         // DMA instructions per wave per unit
    constexpr int P = S - 1;                         // units in flight ahead of the one multiplied
    constexpr bool PRE = EPI == G4_GAUX || EPI == G4_RESID;
    // epilogue: each wave transposes its (BM/2) x WC accumulator tile through its own fp32 LDS
    // region, 32 token rows per pass, and then reads/writes whole 8-feature row chunks (16/32-B
    // vectors, consecutive lanes along a row): row-contiguous loads and stores.
    constexpr int WC = BN / WN;                      // features per wave
    constexpr int CPR = WC / 8;                      // 8-feature chunks per row
    constexpr int RPS = 64 / CPR;                    // rows per wave instruction
    constexpr int Q = 32 / RPS;                      // instructions per 32-row pass
    constexpr int ERS = WC + 4;                      // fp32 row stride of the transposition region
    constexpr int OS = sizeof(TOUT);
    constexpr int L = 2 + (EPI == G4_RESID ? 2 : EPI == G4_GAUX ? 1 : 0) * TMW * Q   // epilogue loads per wave
                      + (F8 ? 2 + TMW * Q : 0);                                        // + sw (2), sa per row
    constexpr int ST = TMW * Q * ((OS == 4 ? 2 : 1) + (EPI == G4_GELU_OUT ? 1 : 0));   // epilogue stores per wave
    constexpr int EPB = 32 * ERS * 4;                // bytes per wave
    __shared__ __attribute__((aligned(1024))) bf16 smem[S * STAGE + NWV * EPB / 2];
    const unsigned nbn = (N + BN - 1) / BN;
    const unsigned T = (unsigned)((M + BM - 1) / BM) * nbn;
    // tiles of this workgroup: its XCD's contiguous tile range, strided by the XCD's workgroups
    const unsigned x = blockIdx.x % kXcds, kk = blockIdx.x / kXcds, nloc = gridDim.x / kXcds;
    const unsigned q = T / kXcds, rem = T % kXcds;
    const unsigned lo = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    const unsigned cnt = q + (x < rem ? 1 : 0);
    const int mytiles = kk < cnt ? (int)((cnt - kk + nloc - 1) / nloc) : 0;
    if (mytiles == 0) return;
    const int nk = F8 ? K / (2 * G4_BK) : K / G4_BK;   // K slices (F8: K in bytes, 128-byte slices)
    const int U = mytiles * nk;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int wm = (wave / WN) * (BM / WM), wn = (wave % WN) * (BN / WN);

    unsigned voffA[BM / (8 * NWV)], voffW[BN / (8 * NWV)];
    g4_voff<BM, NWV>(lda, wave, lane, voffA);
    g4_voff<BN, NWV>(ldw, wave, lane, voffW);
    auto issue = [&](int u) {   // DMA of unit min(u, U - 1) into stage u % S
        const int uu = u < U ? u : U - 1;
        const unsigned tile = lo + kk + (unsigned)(uu / nk) * nloc;
        const unsigned soff = (unsigned)(uu % nk) * G4_BK * 2;   // natural K order: rotating it by the N tile measured +3 % (profiles/r03y_*)
        bf16* st = smem + (u % S) * STAGE;
        const long ra = (long)(tile / nbn) * BM, rw = (long)(tile % nbn) * BN;
        g4_dma<BM, NWV>(rsrc4(A + ra * lda, (M - ra) * lda * 2), voffA, soff, st, wave);
        g4_dma<BN, NWV>(rsrc4(W + rw * ldw, (N - rw) * ldw * 2), voffW, soff, st + BM * G4_BK, wave);
    };
    auto wait_unit = [&](int u) {   // vector-memory ops issued after unit u's DMA (issued at step u - P)
        const int w = u - P;
        int c = (w >= 0 && w % nk == nk - 1) ? ST : 0;
        for (int v = w + 1; v < u; ++v) c += D + ((v >= 0 && v % nk == nk - 1) ? L + ST : 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        g4_vmwait_floor(c);
        __builtin_amdgcn_s_barrier();   // unit u landed for every wave; stage (u-1)%S is free
        __builtin_amdgcn_sched_barrier(0);
    };
    f32x16 acc[TMW][TNW];
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = f32x16{};
    auto mma = [&](int u) {
        const bf16* As = smem + (u % S) * STAGE;
        const bf16* Ws = As + BM * G4_BK;
        // fragments of k-step s + 1 are read while the MFMAs of step s run
        bf16x8 af[2][TMW], wf[2][TNW];
        auto frags = [&](int s, int b) {
#pragma unroll
            for (int i = 0; i < TMW; ++i) af[b][i] = *reinterpret_cast<const bf16x8*>(As + g4_off(wm + 32 * i + r, 2 * s + h));
#pragma unroll
            for (int j = 0; j < TNW; ++j) wf[b][j] = *reinterpret_cast<const bf16x8*>(Ws + g4_off(wn + 32 * j + r, 2 * s + h));
        };
        if constexpr (F8) {
            // 128-byte slice = k-steps s = 0, 1 of 64 bytes; lane (r, h) takes 32 contiguous bytes at 64 s + 32 h
            // of its row in both operands (16-B chunks 4 s + 2 h, + 1): the pairing is exact whatever the
            // hardware's k order, and the block scales are unit (the row scales come in the epilogue)
            typedef int i32x8 __attribute__((ext_vector_type(8)));
            auto f8 = [&](const bf16* img, int row, int s) {
                const u32x4 lo = *reinterpret_cast<const u32x4*>(img + g4_off(row, 4 * s + 2 * h));
                const u32x4 hi = *reinterpret_cast<const u32x4*>(img + g4_off(row, 4 * s + 2 * h + 1));
                return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            };
            i32x8 a8[2][TMW], w8[2][TNW];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
#pragma unroll
                for (int i = 0; i < TMW; ++i) a8[s][i] = f8(As, wm + 32 * i + r, s);
#pragma unroll
                for (int j = 0; j < TNW; ++j) w8[s][j] = f8(Ws, wn + 32 * j + r, s);
            }
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int i = 0; i < TMW; ++i)
#pragma unroll
                    for (int j = 0; j < TNW; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(w8[s][j], a8[s][i], acc[i][j], 0, 0, 0, 0,
                                                                                     0, 0);
        } else {
        frags(0, 0);
#pragma unroll
        for (int s = 0; s < G4_BK / 16; ++s) {
            if (s + 1 < G4_BK / 16) frags(s + 1, (s + 1) & 1);
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TNW; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s & 1][j], af[s & 1][i], acc[i][j], 0, 0, 0);
        }
        }
    };

    G4_STAMP(0);
#pragma unroll
    for (int p = 0; p < P; ++p) issue(p);
    int u = 0;
    for (int t = 0; t < mytiles; ++t) {
        for (int ks = 0; ks + 1 < nk; ++ks, ++u) {   // all but the tile's last K slice
            wait_unit(u);
            if (t == 0 && ks == 0) G4_STAMP(1);
            issue(u + P);
            mma(u);
        }
        // ---- last K slice + epilogue.  acc[i][j][4g + e] = C[wm + 32i + r][wn + 32j + 8g + 4h + e] of the
        // tile; after the transposition lane l holds row (l / CPR) + RPS q of pass i, features
        // 8 (l % CPR) .. + 7.  Raw buffer ops relative to the tile's first row; out-of-tile
        // elements get an out-of-range offset (no branches: see buf_rsrc).
        wait_unit(u);
        if (t == 0) G4_STAMP(2);
        const unsigned tile = lo + kk + (unsigned)t * nloc;
        const long m0 = (long)(tile / nbn) * BM;
        const int n0 = (int)(tile % nbn) * BN;
        const long rows = M - m0 < BM ? M - m0 : BM;
        const int c8 = lane % CPR, rr = lane / CPR;
        const int n = n0 + wn + 8 * c8;
        unsigned off[TMW][Q];   // element offsets, kOOB when outside
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int ml = wm + 32 * i + RPS * q + rr;
                off[i][q] = (ml < rows && n < N) ? (unsigned)(ml * ldc + n) : kOOB;
            }
        float bv[8];
        const auto rs_b = buf_rsrc(bias, bias ? (long)N * 4 : 0);   // null bias: every load reads 0
        buf_ld4(rs_b, n < N ? (unsigned)n * 4 : kOOB, bv);
        buf_ld4(rs_b, n < N ? (unsigned)n * 4 + 16 : kOOB, bv + 4);
        float swv[8], sav[TMW][Q];
        if constexpr (F8) {
            const auto rs_sw = buf_rsrc(sw, (long)N * 4);
            buf_ld4(rs_sw, n < N ? (unsigned)n * 4 : kOOB, swv);
            buf_ld4(rs_sw, n < N ? (unsigned)n * 4 + 16 : kOOB, swv + 4);
            const auto rs_sa = buf_rsrc(sa + m0, rows * 4);
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int q = 0; q < Q; ++q)
                    sav[i][q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        rs_sa, (unsigned)(wm + 32 * i + RPS * q + rr) * 4, 0, 0));
        }
        float pre[TMW][Q][8];
        if constexpr (PRE) {
            const auto rs_pre = EPI == G4_GAUX ? buf_rsrc(gaux + m0 * ldc, rows * ldc * 2) : buf_rsrc(resid + m0 * ldc, rows * ldc * 4);
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const unsigned o = off[i][q];
                    if constexpr (EPI == G4_GAUX) {
                        buf_ld8bf(rs_pre, o == kOOB ? kOOB : o * 2, pre[i][q]);
                    } else {
                        buf_ld4(rs_pre, o == kOOB ? kOOB : o * 4, pre[i][q]);
                        buf_ld4(rs_pre, o == kOOB ? kOOB : o * 4 + 16, pre[i][q] + 4);
                    }
                }
        }
        asm volatile("" ::: "memory");      // keep the epilogue loads ahead of the next DMA (vmcnt order)
        __builtin_amdgcn_sched_barrier(0);
        issue(u + P);
        mma(u);
        if (t == 0) G4_STAMP(3);
        const auto rs_out = buf_rsrc(out + m0 * ldc, rows * ldc * OS);
        const auto rs_g = buf_rsrc(gout ? gout + m0 * ldc : nullptr, gout ? rows * ldc * 2 : 0);
        float* ep = reinterpret_cast<float*>(smem + S * STAGE) + wave * (EPB / 4);
#pragma unroll
        for (int i = 0; i < TMW; ++i) {
#pragma unroll
            for (int j = 0; j < TNW; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                    *reinterpret_cast<f32x4*>(ep + r * ERS + 32 * j + 8 * g + 4 * h) = v;
                }
            asm volatile("" ::: "memory");  // the wave's own LDS writes, then its reads (in order per wave)
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const float* src = ep + (RPS * q + rr) * ERS + 8 * c8;
                const f32x4 lo4 = *reinterpret_cast<const f32x4*>(src);
                const f32x4 hi4 = *reinterpret_cast<const f32x4*>(src + 4);
                float v[8];
                if constexpr (F8) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v[e] = lo4[e] * (sav[i][q] * swv[e]) + bv[e];
                        v[e + 4] = hi4[e] * (sav[i][q] * swv[e + 4]) + bv[e + 4];
                    }
                } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = lo4[e] + bv[e];
                    v[e + 4] = hi4[e] + bv[e + 4];
                }
                }
                if constexpr (EPI == G4_GAUX) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] *= gelu_grad_as(pre[i][q][e]);
                } else if constexpr (EPI == G4_RESID) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += pre[i][q][e];
                }
                const unsigned o = off[i][q];
                if constexpr (OS == 4) {
                    buf_st4(rs_out, o == kOOB ? kOOB : o * 4, v);
                    buf_st4(rs_out, o == kOOB ? kOOB : o * 4 + 16, v + 4);
                } else {
                    buf_st8bf(rs_out, o == kOOB ? kOOB : o * 2, v);
                }
                if constexpr (EPI == G4_GELU_OUT) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = gelu_as(v[e]);
                    buf_st8bf(rs_g, o == kOOB ? kOOB : o * 2, v);
                }
            }
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
            for (int j = 0; j < TNW; ++j) acc[i][j] = f32x16{};
        ++u;
        if (t == 0) G4_STAMP(4);
    }
    g4_vmwait<0>();   // drain the re-fetch DMAs before the workgroup's LDS is released
    G4_STAMP(5);
}

// bm x bn tile, s-stage ring, occ workgroups per CU, wm x wn waves
struct G4Cfg { int bm, bn, s, occ, wm, wn; };
constexpr G4Cfg kG4Cfgs[] = {{64, 64, 3, 2, 2, 2}, {128, 64, 2, 2, 2, 2}, {128, 128, 2, 1, 2, 2}, {128, 128, 3, 1, 2, 2},
                             {64, 128, 2, 1, 2, 2}, {128, 64, 3, 1, 2, 2},
                             // 8-wave workgroups (as many DMA-issuing waves per CU as two 4-wave ones)
                             {128, 128, 2, 1, 2, 4}, {128, 128, 3, 1, 2, 4}, {256, 128, 2, 1, 2, 4}, {128, 256, 2, 1, 1, 8}};
constexpr int kG4NCfg = 10;

int g4_grid(int occ) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        cus = (cus + kXcds - 1) / kXcds * kXcds;
    }
    return cus * occ;
}

template <int BM, int BN, int S, int OCC, int EPI, typename TOUT, int WM, int WN>
int g4_launch(long M, int N, int K, const bf16* A, int lda, const bf16* W, int ldw, const float* bias, const bf16* gaux,
              const float* resid, void* out, bf16* gout, int ldc, hipStream_t st) {
    gemm4_kernel<BM, BN, S, OCC, EPI, TOUT, WM, WN><<<dim3(g4_grid(OCC)), 64 * WM * WN, 0, st>>>(M, N, K, A, lda, W, ldw, bias, gaux, resid,
                                                                                 (TOUT*)out, gout, ldc);
    return check_launch("gemm4");
}

template <int C>
int g4_epi(int epi, int odt, long M, int N, int K, const bf16* A, int lda, const bf16* W, int ldw, const float* bias,
           const bf16* gaux, const float* resid, void* out, bf16* gout, int ldc, hipStream_t st) {
    constexpr int BM = kG4Cfgs[C].bm, BN = kG4Cfgs[C].bn, S = kG4Cfgs[C].s, O = kG4Cfgs[C].occ, WM = kG4Cfgs[C].wm,
                  WN = kG4Cfgs[C].wn;
    switch (epi) {
        case G4_GELU_OUT: return g4_launch<BM, BN, S, O, G4_GELU_OUT, bf16, WM, WN>(M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case G4_GAUX:
            if (odt == CSU_F32) return g4_launch<BM, BN, S, O, G4_GAUX, float, WM, WN>(M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
            return g4_launch<BM, BN, S, O, G4_GAUX, bf16, WM, WN>(M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case G4_RESID: return g4_launch<BM, BN, S, O, G4_RESID, float, WM, WN>(M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        default:
            if (odt == CSU_F32) return g4_launch<BM, BN, S, O, G4_PLAIN, float, WM, WN>(M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
            return g4_launch<BM, BN, S, O, G4_PLAIN, bf16, WM, WN>(M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
    }
}

}  // namespace

// fp8 token GEMM (csu_fp8_gemm for K % 128 == 0): the 128 x 64 tile, 2-stage ring, 2 workgroups per
// CU of the bf16 path, bf16 output with bias
int gemm4_fp8_run(long M, int N, int K, const uint8_t* A, const float* sa, const uint8_t* W, const float* sw,
                  const float* bias, bf16* out, hipStream_t st) {
    gemm4_kernel<128, 64, 2, 2, G4_PLAIN, bf16, 2, 2, true><<<dim3(g4_grid(2)), 256, 0, st>>>(
        M, N, K, (const bf16*)A, K / 2, (const bf16*)W, K / 2, bias, nullptr, nullptr, out, nullptr, N, sa, sw);
    return check_launch("fp8_gemm");
}

// Tile choice (tools/linear_probe.py, tools/gemm_graph_probe.py: every token-GEMM shape of the 512x512
// step, graph-timed, profiles/r02al_gemm_probe.txt): 128 x 64 with a 2-stage ring at 2 workgroups per
// CU is fastest or within 5 % for N <= 256.  The 8-wave 256 x 128 tile wins the wide-output shapes
// with K >= 128 in isolation (qkv at C = 128: 21.2 -> 18.2 us, fc1 at C = 512: 17.7 -> 15.3), but the
// whole step with it there ran 0.7 % SLOWER (3 interleaved A/B pairs, profiles/r02am_ab.txt), so
// 128 x 64 stays everywhere; the 8-wave configurations stay selectable (cfg 16-19) and GPU-tested.
// The time per tile hardly follows its L2 -> LDS bytes (the 8-wave 128 x 128 tile moves 2/3 of the
// bytes of two 128 x 64 tiles in the same time).  cfg indexes kG4Cfgs.
// Exception (G4_SMALLM): when the 128 x 64 tiles cannot give every one of the 2 x CUs workgroups a
// tile (the 4096-token stage: 4096 x 512 outputs = 256 tiles), the 64 x 64 tile with a 3-stage ring
// doubles the tiles in flight -- those launches are latency-bound, one K loop per CU.
#ifndef G4_SMALLM
#define G4_SMALLM 1
#endif
int gemm4_pick(long M, int N, int) {
    if (G4_SMALLM && ((M + 127) / 128) * (long)((N + 63) / 64) < (long)g4_grid(2)) return 0;
    return 1;
}

int gemm4_run(int cfg, int epi, int odt, long M, int N, int K, const bf16* A, int lda, const bf16* W, int ldw,
              const float* bias, const bf16* gaux, const float* resid, void* out, bf16* gout, int ldc, hipStream_t st) {
    if (cfg < 0 || cfg >= kG4NCfg) cfg = gemm4_pick(M, N, K);
    switch (cfg) {
        case 9: return g4_epi<9>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 8: return g4_epi<8>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 7: return g4_epi<7>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 6: return g4_epi<6>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 5: return g4_epi<5>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 4: return g4_epi<4>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 3: return g4_epi<3>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 2: return g4_epi<2>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        case 1: return g4_epi<1>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
        default: return g4_epi<0>(epi, odt, M, N, K, A, lda, W, ldw, bias, gaux, resid, out, gout, ldc, st);
    }
}

}  // namespace csu

#ifdef G4_TIMING
extern "C" int csu_debug_g4_ts(unsigned long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(csu::g4_ts), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif
