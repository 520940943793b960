// Probe: token GEMM out[M][N] = x[M][K] W[N][K]^T (bf16, K = 256) with the 64-token x panel held in
// registers (MFMA B fragments) and the weights streamed global -> VGPR (no LDS), waves splitting N in
// 32-row tiles, double-buffered weight fragments.  Variants:
//   layout 0: natural [N][K] weights, fragment-shaped loads (lane (r, h): row r, 16 B at k 16 s + 8 h)
//   layout 1: fragment-ordered weights ([N/32][K/16][64 lanes][8]): one contiguous 1 KB per wave load
//   mode 0: loads + MFMA + epilogue; mode 1: loads only (sum kept live)
// Compared against the roofline bytes (x + W + out once) and reports per-CU weight stream rate.
//   hipcc --offload-arch=gfx950 -O3 -o wstream_probe wstream_probe.hip && ./wstream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int K = 256;
constexpr int KS = K / 16;
constexpr int BM = 64;

template <int LAYOUT, int MODE>
__global__ __launch_bounds__(256) void ws_gemm(int M, int N, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                               bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    bf16x8 xf[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            xf[t][s] = *reinterpret_cast<const bf16x8*>(X + (m0 + 32 * t + r) * K + 16 * s + 8 * h);
    const int ntiles = N / 32;
    auto wload = [&](int nt, bf16x8* wf) {
        if constexpr (LAYOUT == 0) {
#pragma unroll
            for (int s = 0; s < KS; ++s)
                wf[s] = *reinterpret_cast<const bf16x8*>(W + (long)(32 * nt + r) * K + 16 * s + 8 * h);
        } else {
#pragma unroll
            for (int s = 0; s < KS; ++s)
                wf[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
        }
    };
    bf16x8 wa[KS], wb[KS];
    int nt = wave;
    if (nt < ntiles) wload(nt, wa);
    float keep = 0.f;
    for (; nt < ntiles; nt += 8) {
        const int nt2 = nt + 4;
        if (nt2 < ntiles) wload(nt2, wb);
        auto body = [&](const bf16x8* wf, int n_t) {
            if constexpr (MODE == 0) {
                f32x16 a0 = f32x16{}, a1 = f32x16{};
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s], xf[0][s], a0, 0, 0, 0);
                    a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s], xf[1][s], a1, 0, 0, 0);
                }
                // out[token][n]: lane holds token r (+32), rows n = 32 n_t + 8 g + 4 h + e
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const f32x16& a = t ? a1 : a0;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
                        bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                        *reinterpret_cast<bf16x4*>(out + (m0 + 32 * t + r) * N + 32 * n_t + 8 * g + 4 * h) = v;
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < KS; ++s) keep += (float)wf[s][0] + (float)wf[s][7];
            }
        };
        body(wa, nt);
        if (nt2 >= ntiles) break;
        const int nt3 = nt + 8;
        if (nt3 < ntiles) wload(nt3, wa);
        body(wb, nt2);
    }
    if constexpr (MODE == 1)
        if (keep == 12345.f) out[0] = (bf16)keep;
}


// fully unrolled over the wave's n-tiles (compile-time N): the compiler can count vmcnt exactly
template <int N, int EPI>
__global__ __launch_bounds__(256) void ws_gemm_u(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                 bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    bf16x8 xf[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            xf[t][s] = *reinterpret_cast<const bf16x8*>(X + (m0 + 32 * t + r) * K + 16 * s + 8 * h);
    constexpr int NT = N / 32 / 4;     // n-tiles per wave
    __shared__ bf16 stage[4][64][40];  // per-wave epilogue transposition (32 n + 8 pad per token row)
    bf16x8 wf[2][KS];
    auto wload = [&](int nt, bf16x8* w) {
#pragma unroll
        for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
    wload(wave, wf[0]);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = wave + 4 * i;
        if (i + 1 < NT) wload(nt + 4, wf[(i + 1) & 1]);
        f32x16 a0 = f32x16{}, a1 = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i & 1][s], xf[0][s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i & 1][s], xf[1][s], a1, 0, 0, 0);
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        if constexpr (EPI == 0) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const f32x16& a = t ? a1 : a0;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                    *reinterpret_cast<bf16x4*>(out + (m0 + 32 * t + r) * N + 32 * nt + 8 * g + 4 * h) = v;
                }
            }
        } else {
            // through LDS: [64 tokens][32 n] then 16-B stores, 4 lanes per token row (64 B)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const f32x16& a = t ? a1 : a0;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                    *reinterpret_cast<bf16x4*>(&stage[wave][32 * t + r][8 * g + 4 * h]) = v;
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0) only (wave-private buffer)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 16 * q + (lane >> 2), c = 8 * (lane & 3);
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
                *reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * nt + c) = v;
            }
        }
    }
}

// v3: x panel staged once per workgroup through LDS (coalesced 16-B loads), B fragments read from it
// into registers; W prefetched D tiles ahead (ring of D+1 fragment sets), fully unrolled; LDS epilogue
template <int N, int D, int MF = 1, int ST = 1>
__global__ __launch_bounds__(256) void ws_gemm3(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    __shared__ __attribute__((aligned(16))) bf16 xs[BM][K + 8];
    __shared__ __attribute__((aligned(16))) bf16 stage[4][64][40];
    constexpr int NT = N / 32 / 4;
    bf16x8 wf[D + 1][KS];
    auto wload = [&](int nt, bf16x8* w) {
#pragma unroll
        for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
#pragma unroll
    for (int i = 0; i < D && i < NT; ++i) wload(wave + 4 * i, wf[i]);
    __builtin_amdgcn_sched_barrier(0);
    // x: 64 rows x 512 B = 2048 16-B pieces, 8 per thread, row-contiguous
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int p = threadIdx.x + 256 * i, row = p / (K / 8), c = 8 * (p % (K / 8));
        *reinterpret_cast<bf16x8*>(&xs[row][c]) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * K + c);
    }
    __syncthreads();
    bf16x8 xf[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(&xs[32 * t + r][16 * s + 8 * h]);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = wave + 4 * i;
        if (i + D < NT) wload(nt + 4 * D, wf[(i + D) % (D + 1)]);
        __builtin_amdgcn_sched_barrier(0);   // the prefetch stays here (hipcc sinks loads to their use)
        f32x16 a0 = f32x16{}, a1 = f32x16{};
        if constexpr (MF) {
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[0][s], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[1][s], a1, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int s = 0; s < KS; ++s) { a0[s] += (float)wf[i % (D + 1)][s][0]; a1[s] += (float)xf[1][s][1]; }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!ST) {
            if (a0[3] + a1[5] == 1234.5f) out[lane] = (bf16)a0[7];
            continue;
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x16& a = t ? a1 : a0;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                *reinterpret_cast<bf16x4*>(&stage[wave][32 * t + r][8 * g + 4 * h]) = v;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * q + (lane >> 2), c = 8 * (lane & 3);
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
            *reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * nt + c) = v;
        }
    }
}

// v4: as v3, but a wave's tiles come in adjacent pairs (64 output columns = one 128-B line per token
// row) and the pair is written with full-line stores after its second tile
template <int N, int D>
__global__ __launch_bounds__(256) void ws_gemm4(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    __shared__ __attribute__((aligned(16))) bf16 xs[BM][K + 8];
    __shared__ __attribute__((aligned(16))) bf16 stage[4][64][72];
    constexpr int NT = N / 32 / 4;                 // tiles per wave (even)
    auto tile_of = [&](int i) { return 8 * (i >> 1) + 2 * wave + (i & 1); };
    bf16x8 wf[D + 1][KS];
    auto wload = [&](int nt, bf16x8* w) {
#pragma unroll
        for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
#pragma unroll
    for (int i = 0; i < D && i < NT; ++i) wload(tile_of(i), wf[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int p = threadIdx.x + 256 * i, row = p / (K / 8), c = 8 * (p % (K / 8));
        *reinterpret_cast<bf16x8*>(&xs[row][c]) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * K + c);
    }
    __syncthreads();
    bf16x8 xf[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(&xs[32 * t + r][16 * s + 8 * h]);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = tile_of(i);
        if (i + D < NT) wload(tile_of(i + D), wf[(i + D) % (D + 1)]);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 a0 = f32x16{}, a1 = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[0][s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[1][s], a1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        const int c0 = 32 * (i & 1);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x16& a = t ? a1 : a0;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                *reinterpret_cast<bf16x4*>(&stage[wave][32 * t + r][c0 + 8 * g + 4 * h]) = v;
            }
        }
        if (i & 1) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int row = 8 * q + (lane >> 3), c = 8 * (lane & 7);
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
                *reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * (nt - 1) + c) = v;
            }
        }
    }
}

// v5: outputs collected in LDS ([64][N] bf16) and written at the end (NTS: nontemporal stores), or
// v3 with nontemporal stores (END = 0)
template <int N, int D, int END, int NTS>
__global__ __launch_bounds__(256) void ws_gemm5(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    __shared__ __attribute__((aligned(16))) bf16 xs[BM][K + 8];
    __shared__ __attribute__((aligned(16))) bf16 stage[END ? 1 : 4][64][END ? N + 8 : 40];
    constexpr int NT = N / 32 / 4;
    bf16x8 wf[D + 1][KS];
    auto wload = [&](int nt, bf16x8* w) {
#pragma unroll
        for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
#pragma unroll
    for (int i = 0; i < D && i < NT; ++i) wload(wave + 4 * i, wf[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int p = threadIdx.x + 256 * i, row = p / (K / 8), c = 8 * (p % (K / 8));
        *reinterpret_cast<bf16x8*>(&xs[row][c]) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * K + c);
    }
    __syncthreads();
    bf16x8 xf[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(&xs[32 * t + r][16 * s + 8 * h]);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = wave + 4 * i;
        if (i + D < NT) wload(nt + 4 * D, wf[(i + D) % (D + 1)]);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 a0 = f32x16{}, a1 = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[0][s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[1][s], a1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        const int sw = END ? 0 : wave, cb = END ? 32 * nt : 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x16& a = t ? a1 : a0;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                *reinterpret_cast<bf16x4*>(&stage[sw][32 * t + r][cb + 8 * g + 4 * h]) = v;
            }
        }
        if constexpr (!END) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 16 * q + (lane >> 2), c = 8 * (lane & 3);
                const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
                bf16x8* dst = reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * nt + c);
                if constexpr (NTS) __builtin_nontemporal_store(v, dst); else *dst = v;
            }
        }
    }
    if constexpr (END) {
        __syncthreads();
        constexpr int PR = N / 8;            // 16-B pieces per row
#pragma unroll
        for (int i = 0; i < 64 * PR / 256; ++i) {
            const int p = threadIdx.x + 256 * i, row = p / PR, c = 8 * (p % PR);
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[0][row][c]);
            bf16x8* dst = reinterpret_cast<bf16x8*>(out + (m0 + row) * N + c);
            if constexpr (NTS) __builtin_nontemporal_store(v, dst); else *dst = v;
        }
    }
}

// v6: 8 waves (2 per SIMD), x panel in LDS read per k-step (no register copy), W streamed D tiles
// ahead, per-wave LDS epilogue with (optionally nontemporal) 16-B stores
template <int N, int D, int NTS>
__global__ __launch_bounds__(512) void ws_gemm6(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    __shared__ __attribute__((aligned(16))) bf16 xs[BM][K + 8];
    __shared__ __attribute__((aligned(16))) bf16 stage[8][64][40];
    constexpr int NT = N / 32 / 8;
    bf16x8 wf[D + 1][KS];
    auto wload = [&](int nt, bf16x8* w) {
#pragma unroll
        for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
#pragma unroll
    for (int i = 0; i < D && i < NT; ++i) wload(wave + 8 * i, wf[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = threadIdx.x + 512 * i, row = p / (K / 8), c = 8 * (p % (K / 8));
        *reinterpret_cast<bf16x8*>(&xs[row][c]) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * K + c);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = wave + 8 * i;
        if (i + D < NT) wload(nt + 8 * D, wf[(i + D) % (D + 1)]);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 a0 = f32x16{}, a1 = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&xs[r][16 * s + 8 * h]);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&xs[32 + r][16 * s + 8 * h]);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], b0, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], b1, a1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x16& a = t ? a1 : a0;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                *reinterpret_cast<bf16x4*>(&stage[wave][32 * t + r][8 * g + 4 * h]) = v;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * q + (lane >> 2), c = 8 * (lane & 3);
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
            bf16x8* dst = reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * nt + c);
            if constexpr (NTS) __builtin_nontemporal_store(v, dst); else *dst = v;
        }
    }
}

// v7: TM token tiles of 32 per workgroup (BM7 = 32 TM tokens), N split over gridDim.y workgroups,
// 4 waves; x panel in LDS read per k-step; W D tiles ahead; nontemporal 16-B stores via LDS
template <int N, int D, int TM, int NSPLIT>
__global__ __launch_bounds__(256) void ws_gemm7(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                bf16* __restrict__ out) {
    constexpr int BM7 = 32 * TM;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM7;
    __shared__ __attribute__((aligned(16))) bf16 xs[BM7][K + 8];
    __shared__ __attribute__((aligned(16))) bf16 stage[4][BM7][40];
    constexpr int NT = N / NSPLIT / 32 / 4;
    const int ntb = blockIdx.y * (N / NSPLIT / 32);
    bf16x8 wf[D + 1][KS];
    auto wload = [&](int nt, bf16x8* w) {
#pragma unroll
        for (int s = 0; s < KS; ++s) w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
#pragma unroll
    for (int i = 0; i < D && i < NT; ++i) wload(ntb + wave + 4 * i, wf[i]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i) {
        const int p = threadIdx.x + 256 * i, row = p / (K / 8), c = 8 * (p % (K / 8));
        *reinterpret_cast<bf16x8*>(&xs[row][c]) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * K + c);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = ntb + wave + 4 * i;
        if (i + D < NT) wload(nt + 4 * D, wf[(i + D) % (D + 1)]);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 a[TM];
#pragma unroll
        for (int t = 0; t < TM; ++t) a[t] = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int t = 0; t < TM; ++t) {
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(&xs[32 * t + r][16 * s + 8 * h]);
                a[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], b, a[t], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int t = 0; t < TM; ++t) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 v = {(bf16)a[t][4 * g], (bf16)a[t][4 * g + 1], (bf16)a[t][4 * g + 2], (bf16)a[t][4 * g + 3]};
                *reinterpret_cast<bf16x4*>(&stage[wave][32 * t + r][8 * g + 4 * h]) = v;
            }
        }
#pragma unroll
        for (int q = 0; q < 2 * TM; ++q) {
            const int row = 16 * q + (lane >> 2), c = 8 * (lane & 3);
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
            __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * nt + c));
        }
    }
}

// v8: v5 (x in registers, W D tiles ahead, nontemporal LDS-staged stores) with the next tile's W loads
// interleaved with this tile's MFMAs by sched_group_barrier (1 load : 2 MFMA), so the TA sees a steady
// stream instead of a 16-load burst per tile
template <int N, int D>
__global__ __launch_bounds__(256) void ws_gemm8(int M, int, const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                bf16* __restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.x * BM;
    __shared__ __attribute__((aligned(16))) bf16 xs[BM][K + 8];
    __shared__ __attribute__((aligned(16))) bf16 stage[4][64][40];
    constexpr int NT = N / 32 / 4;
    bf16x8 wf[D + 1][KS];
    auto wload1 = [&](int nt, bf16x8* w, int s) {
        w[s] = *reinterpret_cast<const bf16x8*>(W + ((long)(nt * KS + s) * 64 + lane) * 8);
    };
#pragma unroll
    for (int i = 0; i < D && i < NT; ++i)
#pragma unroll
        for (int s = 0; s < KS; ++s) wload1(wave + 4 * i, wf[i], s);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int p = threadIdx.x + 256 * i, row = p / (K / 8), c = 8 * (p % (K / 8));
        *reinterpret_cast<bf16x8*>(&xs[row][c]) = *reinterpret_cast<const bf16x8*>(X + (m0 + row) * K + c);
    }
    __syncthreads();
    bf16x8 xf[2][KS];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < KS; ++s) xf[t][s] = *reinterpret_cast<const bf16x8*>(&xs[32 * t + r][16 * s + 8 * h]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int nt = wave + 4 * i;
        f32x16 a0 = f32x16{}, a1 = f32x16{};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (i + D < NT) wload1(nt + 4 * D, wf[(i + D) % (D + 1)], s);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[0][s], a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i % (D + 1)][s], xf[1][s], a1, 0, 0, 0);
            if (i + D < NT) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x16& a = t ? a1 : a0;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                bf16x4 v = {(bf16)a[4 * g], (bf16)a[4 * g + 1], (bf16)a[4 * g + 2], (bf16)a[4 * g + 3]};
                *reinterpret_cast<bf16x4*>(&stage[wave][32 * t + r][8 * g + 4 * h]) = v;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 16 * q + (lane >> 2), c = 8 * (lane & 3);
            const bf16x8 v = *reinterpret_cast<const bf16x8*>(&stage[wave][row][c]);
            __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(out + (m0 + row) * N + 32 * nt + c));
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

__global__ void fill_rand(bf16* p, long n, unsigned seed) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((float)(x & 0xffff) / 65536.f - 0.5f) * 0.1f);
}

int main(int argc, char** argv) {
    const int M = 16384;
    int Ns[] = {256, 768, 1024};
    bf16 *X, *W, *O;
    hipMalloc(&X, (size_t)M * K * 2);
    hipMalloc(&W, (size_t)2048 * K * 2);
    hipMalloc(&O, (size_t)M * 2048 * 2);
    hipMemset(X, 0, (size_t)M * K * 2);
    hipMemset(W, 0, (size_t)2048 * K * 2);
    if (argc > 1) {   // random operands instead of zeros
        fill_rand<<<(M * K + 255) / 256, 256>>>(X, (long)M * K, 1u);
        fill_rand<<<(2048 * K + 255) / 256, 256>>>(W, 2048L * K, 2u);
        hipDeviceSynchronize();
        printf("random operands\n");
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int N : Ns) {
        auto run = [&](auto kern, const char* name, int nthr = 256, int bm = 64, int ny = 1) {
            for (int i = 0; i < 3; ++i) kern<<<dim3(M / bm, ny), nthr>>>(M, N, X, W, O);
            hipEventRecord(e0);
            const int it = 20;
            for (int i = 0; i < it; ++i) kern<<<dim3(M / bm, ny), nthr>>>(M, N, X, W, O);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / it;
            const double bytes = (double)M * K * 2 + (double)N * K * 2 + (double)M * N * 2;
            const double wpcu = (double)N * K * 2 * (M / BM) / 256.0;   // weight bytes per CU
            printf("N=%5d %-22s %7.2f us  roof %5.2f us  frac %.3f  W per CU %.0f KB -> %.1f GB/s per CU\n", N, name, us,
                   bytes / 8e6, bytes / 8e6 / us, wpcu / 1024, wpcu / us / 1e3);
        };
        run(ws_gemm<0, 0>, "natural, mfma");
        run(ws_gemm<1, 0>, "fragment-ordered, mfma");
        if (N == 256) { run(ws_gemm_u<256, 0>, "unrolled, direct st"); run(ws_gemm_u<256, 1>, "unrolled, lds st"); }
        if (N == 768) { run(ws_gemm_u<768, 0>, "unrolled, direct st"); run(ws_gemm_u<768, 1>, "unrolled, lds st"); }
        if (N == 1024) { run(ws_gemm_u<1024, 0>, "unrolled, direct st"); run(ws_gemm_u<1024, 1>, "unrolled, lds st"); }
        if (N == 256) { run(ws_gemm8<256, 1>, "v8 D1 interleaved"); run(ws_gemm7<256, 1, 4, 2>, "v7 128tok N/2 D1", 256, 128, 2); run(ws_gemm7<256, 1, 4, 1>, "v7 128tok D1", 256, 128, 1);
            run(ws_gemm6<256, 1, 1>, "v6 8w D1 nt", 512); run(ws_gemm5<256, 2, 0, 1>, "v5 D2 nt stores"); run(ws_gemm3<256, 1>, "v3 D1"); run(ws_gemm3<256, 2>, "v3 D2"); run(ws_gemm4<256, 1>, "v4 D1 full lines"); }
        if (N == 768) { run(ws_gemm3<768, 1>, "v3 D1"); run(ws_gemm3<768, 2>, "v3 D2"); run(ws_gemm3<768, 3>, "v3 D3");
            run(ws_gemm4<768, 1>, "v4 D1 full lines"); run(ws_gemm4<768, 2>, "v4 D2 full lines");
            run(ws_gemm8<768, 1>, "v8 D1 interleaved"); run(ws_gemm8<768, 2>, "v8 D2 interleaved");
            run(ws_gemm7<768, 1, 4, 2>, "v7 128tok N/2 D1", 256, 128, 2); run(ws_gemm7<768, 1, 4, 3>, "v7 128tok N/3 D1", 256, 128, 3);
            run(ws_gemm7<768, 1, 2, 1>, "v7 64tok D1", 256, 64, 1); 
            run(ws_gemm7<768, 1, 4, 6>, "v7 128tok N/6 D1", 256, 128, 6);
            run(ws_gemm6<768, 1, 0>, "v6 8w D1", 512); run(ws_gemm6<768, 1, 1>, "v6 8w D1 nt", 512);
            run(ws_gemm6<768, 2, 1>, "v6 8w D2 nt", 512);
            run(ws_gemm5<768, 2, 0, 1>, "v5 D2 nt stores"); run(ws_gemm5<768, 2, 1, 0>, "v5 D2 stores at end");
            run(ws_gemm5<768, 2, 1, 1>, "v5 D2 nt stores at end");
            run(ws_gemm3<768, 2, 1, 0>, "v3 D2 no stores"); run(ws_gemm3<768, 2, 0, 1>, "v3 D2 no mfma"); run(ws_gemm3<768, 2, 0, 0>, "v3 D2 neither"); }
        if (N == 1024) { run(ws_gemm8<1024, 1>, "v8 D1 interleaved"); run(ws_gemm8<1024, 2>, "v8 D2 interleaved");
            run(ws_gemm7<1024, 1, 4, 2>, "v7 128tok N/2 D1", 256, 128, 2); run(ws_gemm7<1024, 1, 4, 4>, "v7 128tok N/4 D1", 256, 128, 4);
            run(ws_gemm6<1024, 1, 1>, "v6 8w D1 nt", 512); run(ws_gemm6<1024, 2, 1>, "v6 8w D2 nt", 512);
            run(ws_gemm5<1024, 2, 0, 1>, "v5 D2 nt stores"); run(ws_gemm4<1024, 1>, "v4 D1 full lines"); run(ws_gemm4<1024, 2>, "v4 D2 full lines"); run(ws_gemm3<1024, 1>, "v3 D1"); run(ws_gemm3<1024, 2>, "v3 D2"); run(ws_gemm3<1024, 3>, "v3 D3"); }
        run(ws_gemm<0, 1>, "natural, loads only");
        run(ws_gemm<1, 1>, "frag-ordered, loads");
    }
    return 0;
}
