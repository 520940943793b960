// Linear weight + bias gradient over token rows for gfx950 (bf16/fp32 in, fp32 out).
//
//   dW[n][k] = sum_m dY[m][n] * X[m][k],   db[n] = sum_m dY[m][n]       (m = the B*L tokens)
// This is the backward of every nn.Linear of the model (qkv/proj/fc1/fc2 cswin:185/187/314/323,
// concat_linear cswin:568/581/592, the CARAFE 1x1 convs cswin:396/399).  M is huge (up to 4M
// tokens) while N, K <= 2048: the output has few tiles, so the token (reduction) dimension is split
// into `chunks` and the chunk partials are summed in a fixed order (bitwise reproducible, no float
// atomics).
//
// bf16 path (wgrad_tile): one workgroup = one TN x TK output tile (TN, TK in {64, 128}) over one
// token chunk, 4 waves each owning a (TN/2) x (TK/2) block of 32x32x16 MFMA tiles.  Operands are
// staged row-major ([token][column], XOR-swizzled 16-B chunks) through TWO LDS buffers with a
// two-step register prefetch (branch-free buffer loads), fragments gathered with the transposing
// ds_read_b64_tr_b16.  Measured (tools/wgrad_timing.py, tools/wgrad_bench.py): a step is bound by
// the per-CU load rate (L2 hits ~70 GB/s/CU, the compulsory HBM part slower), not by latency
// (deeper prefetch, more workgroups per CU: no change) nor the MFMAs.  The chunk partials go to
// tile-local slabs reduced by ONE coalesced pass in chunk order (wslab_reduce): an in-launch
// combine (arrival counters, agent-scope release/acquire) measured 1.3-4x slower per launch.
// fp32 path: 64x64 tiles, v_mfma_f32_32x32x2f32, [chunk][N*K + N] slabs + csu_colsum.
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int TM = 64;    // tokens per LDS step

#ifdef WG_TIMING   // debug build only: per-workgroup phase timestamps (100 MHz), read by csu_debug_wgrad_ts
__device__ unsigned long long wg_ts[4][16384];
#define WG_STAMP(k) do { if (threadIdx.x < 1 && blockIdx.x < 16384) wg_ts[k][blockIdx.x + threadIdx.x] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ unsigned long long wg_steps[4][64];   // core-clock stamps of the phases of the first 64 steps of block 0
#define STEP_STAMP(k, i) do { if (blockIdx.x == 0 && threadIdx.x < 1 && (i) < 64) wg_steps[k][(i) + threadIdx.x] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define WG_STAMP(k) do {} while (0)
#define STEP_STAMP(k, i) do {} while (0)
#endif

// ------------------------------------------------------------------------------------------
// fp32 path
// ------------------------------------------------------------------------------------------
constexpr int TN32 = 64, TK32 = 64, S32 = TM + 4;

// stage a TM x 64 row-major fp32 tile (rows m0.., columns c0..) transposed into img[64][S32];
// rows >= M and columns >= ncols are zero.
__device__ __forceinline__ void stage_t32(const float* __restrict__ g, long M, int ld, int ncols, long m0, int c0,
                                          float* img) {
    for (int it = threadIdx.x; it < (TM / 2) * 16; it += NT) {
        const int pr = it / 16, q = it % 16;  // row pair, 4-column chunk
        const long m = m0 + 2 * pr;
        const int c = c0 + q * 4;
        float a[4], b[4];
        const bool cv = c < ncols;
        if (cv && m < M) load4(g + m * ld + c, a); else for (int j = 0; j < 4; ++j) a[j] = 0.f;
        if (cv && m + 1 < M) load4(g + (m + 1) * ld + c, b); else for (int j = 0; j < 4; ++j) b[j] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float* p = img + (q * 4 + j) * S32 + 2 * pr;
            p[0] = a[j];
            p[1] = b[j];
        }
    }
}

__global__ __launch_bounds__(NT) void wgrad_f32(long M, int N, int K, long rows_per_chunk, const float* __restrict__ dy,
                                                const float* __restrict__ x, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float At[TN32 * S32];   // dY^T tile [n][m]
    __shared__ __attribute__((aligned(16))) float Bt[TK32 * S32];   // X^T  tile [k][m]
    __shared__ float bred[NT];
    const int n0 = blockIdx.x * TN32, k0 = blockIdx.y * TK32;
    const long m_begin = (long)blockIdx.z * rows_per_chunk;
    const long m_end = min(M, m_begin + rows_per_chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave >> 1) * 32, wk = (wave & 1) * 32;
    const bool do_bias = blockIdx.y == 0;
    f32x16 acc = {};
    float bsum = 0.f;   // db partial of column n0 + (threadIdx.x & 63), rows threadIdx.x>>6 (mod 4)
    for (long m0 = m_begin; m0 < m_end; m0 += TM) {
        __syncthreads();
        stage_t32(dy, m_end, N, N, m0, n0, At);
        stage_t32(x, m_end, K, K, m0, k0, Bt);
        __syncthreads();
        if (do_bias) {
            const int n = threadIdx.x & 63, qq = threadIdx.x >> 6;
#pragma unroll
            for (int j = 0; j < TM / 4; ++j) bsum += At[n * S32 + qq * (TM / 4) + j];
        }
#pragma unroll
        for (int t = 0; t < TM / 2; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(At[(wn + r) * S32 + 2 * t + h], Bt[(wk + r) * S32 + 2 * t + h], acc,
                                                      0, 0, 0);
    }
    const long slab = (long)N * K + N;
    float* out = part + (long)blockIdx.z * slab;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int n = n0 + wn + crow(reg, h), k = k0 + wk + r;
        if (n < N && k < K) out[(long)n * K + k] = acc[reg];
    }
    if (do_bias) {
        bred[threadIdx.x] = bsum;
        __syncthreads();
        if (threadIdx.x < 64 && n0 + threadIdx.x < N)
            out[(long)N * K + n0 + threadIdx.x] =
                ((bred[threadIdx.x] + bred[threadIdx.x + 64]) + bred[threadIdx.x + 128]) + bred[threadIdx.x + 192];
    }
}

struct Plan32 {
    int nt, kt, chunks;
    long rpc;
};

Plan32 plan32(long M, int N, int K) {
    Plan32 p;
    p.nt = (N + TN32 - 1) / TN32;
    p.kt = (K + TK32 - 1) / TK32;
    long want = (1024 + p.nt * p.kt - 1) / (p.nt * p.kt);
    const long maxc = (M + 511) / 512;
    if (want > maxc) want = maxc;
    if (want > 256) want = 256;
    if (want < 1) want = 1;
    p.rpc = ((M + want - 1) / want + TM - 1) / TM * TM;
    p.chunks = (int)((M + p.rpc - 1) / p.rpc);
    return p;
}

// ------------------------------------------------------------------------------------------
// bf16 path
// ------------------------------------------------------------------------------------------
typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s tr_read(const bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

#ifndef WG_SB128
#define WG_SB128 1
#endif

// LDS operand images are [TM tokens][T columns] bf16 with no padding; the 16-B chunks of a row are
// XOR-swizzled so that a ds_read_b64_tr_b16 (each 32-lane half reads 4 consecutive rows x 64 B)
// and the ds_write_b128 staging are bank-conflict free: T = 128 (256-B rows, one bank row each):
// key = 4 (row & 3); T = 64 (two rows per bank row): key = 4 ((row >> 1) & 1).
template <int T>
__device__ __forceinline__ int swz(int row, int chunk) {
    const int key = T >= 128 ? 4 * (row & 3) : 4 * ((row >> 1) & 1);   // T = 256: 512-B rows, same key
    return row * T + ((chunk ^ key) << 3);
}

// 32x32x16 operand fragment of columns [c0, c0+32) at k-step rows [16s + 8h, +8) of a [TM][T]
// swizzled image: lane 4q+p of a 16-lane group reads row q, columns 4p..4p+3 and receives column
// (lane & 15) of the 4 rows; two reads (rows q and q+4) give the 8 tokens of the fragment.
template <int T>
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int c0, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = 16 * s + 8 * (grp >> 1) + q;
    const v4s lo = tr_read(img + swz<T>(row, col >> 3) + (col & 7));
    const v4s hi = tr_read(img + swz<T>(row + 4, col >> 3) + (col & 7));
    const v4s v[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

// f(i + J, set (J + 1) % D, LDS buffer (J + 1) % 2) for J = 0 .. U-1, all indices compile-time
template <int J, int U, int D, typename F>
__device__ __forceinline__ void unroll_steps(F& f, int i) {
    if constexpr (J < U) {
        f(i + J, std::integral_constant<int, (J + 1) % D>{}, std::integral_constant<int, (J + 1) % 2>{});
        unroll_steps<J + 1, U, D>(f, i);
    }
}

// NTH threads = NTH / 64 waves in a (NW / 2) x 2 grid over the tile (N x K): 4 waves for the 64 / 128
// tiles, 8 waves (64 x 64 per wave) for the 256 x 128 tile of the wide Linears (3/4 of the staged bytes
// per output of the 128 x 128 tile: the step is bound by operand staging; a 256 x 256 tile's 128
// accumulators per lane spilled)
template <int TN, int TK, int NTH = NT>
struct TileCfg {
    static constexpr int CPRA = TN / 8, RPPA = NTH / CPRA, NPA = TM / RPPA;   // 16-B chunks per row, rows per pass, passes
    static constexpr int CPRB = TK / 8, RPPB = NTH / CPRB, NPB = TM / RPPB;
    static constexpr int WNW = NTH / 128;                       // waves along N (2 along K)
    static constexpr int AN = TN / (32 * WNW), AK = TK / 64;    // 32x32 MFMA tiles per wave per dim
    static constexpr int BUF = TM * (TN + TK);                  // bf16 per LDS buffer (A image then B image)
};

// One TN x TK tile of dW (and db when k0 == 0) over tokens [m_begin, m_end).  chunks == 1: dW / db
// are written to dst (N*K + N fp32); else the partial tile goes to slab[tile][chunk][TN][TK] and the
// db partial to bslab[n_tile][chunk][TN]; wslab_reduce sums them.
// Pipeline per 64-token step i: stage step i+1 from registers into LDS buffer (i+1)&1, issue the
// global loads of step i+3 into the register set just freed, MFMAs of step i, one barrier -- two
// steps of MFMA work between a load's issue and its use, 64 KB LDS (T = 128) for 2 workgroups/CU.
// Body: logical workgroup t of one Linear (t = chunk * tiles + tile).
template <int TN, int TK, int D, int NTH = NT>
__device__ __forceinline__ void wgrad_tile_body(bf16* lds, int t, long M, int N, int K, long rpc, int chunks,
                                                const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                float* __restrict__ dst, float* __restrict__ slab) {
    using C = TileCfg<TN, TK, NTH>;
    const int nt = (N + TN - 1) / TN, kt = (K + TK - 1) / TK, tiles = nt * kt;
    const int chunk = __builtin_amdgcn_readfirstlane(t / tiles), tile = __builtin_amdgcn_readfirstlane(t % tiles);
    const int ntile = tile / kt;
    const int n0 = ntile * TN, k0 = (tile % kt) * TK;
    const long m_begin = (long)chunk * rpc;
    const long m_end = min(M, m_begin + rpc);
    const int nsteps = (int)((m_end - m_begin + TM - 1) / TM);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave >> 1) * (TN / C::WNW), wk = (wave & 1) * (TK / 2);
    const bool do_bias = k0 == 0;
    const int cga = threadIdx.x % C::CPRA, rra = threadIdx.x / C::CPRA;   // A: rows rra + RPPA i, chunk cga
    const int cgb = threadIdx.x % C::CPRB, rrb = threadIdx.x / C::CPRB;
    const bool nv = n0 + 8 * cga < N, kv = k0 + 8 * cgb < K;
    bf16x8 ra[D][C::NPA], rb[D][C::NPB];
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // buffer loads over this chunk's rows: rows past m_end fall outside the resource (read as 0) and
    // out-of-range columns get an offset past it -- no branches around the loads (a branch per load
    // makes hipcc wait for each one separately)
    const __amdgpu_buffer_rsrc_t rsa = buf_rsrc(dy + m_begin * N, (m_end - m_begin) * N * 2);
    const __amdgpu_buffer_rsrc_t rsb = buf_rsrc(x + m_begin * K, (m_end - m_begin) * K * 2);
    const unsigned offa = nv ? (unsigned)((rra * N + n0 + 8 * cga) * 2) : kOOB;
    const unsigned offb = kv ? (unsigned)((rrb * K + k0 + 8 * cgb) * 2) : kOOB;
    auto load = [&](bf16x8* A, bf16x8* B, int step) {   // rows m_begin + TM*step + ...
#pragma unroll
        for (int i = 0; i < C::NPA; ++i) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsa, offa + (unsigned)((TM * step + C::RPPA * i) * N * 2), 0, 0);
            __builtin_memcpy(&A[i], &v, 16);
        }
#pragma unroll
        for (int i = 0; i < C::NPB; ++i) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsb, offb + (unsigned)((TM * step + C::RPPB * i) * K * 2), 0, 0);
            __builtin_memcpy(&B[i], &v, 16);
        }
    };
    auto stage = [&](const bf16x8* A, const bf16x8* B, int buf) {
        bf16* la = lds + buf * C::BUF;
        bf16* lb = la + TM * TN;
#pragma unroll
        for (int i = 0; i < C::NPA; ++i) {
            *reinterpret_cast<bf16x8*>(la + swz<TN>(rra + C::RPPA * i, cga)) = A[i];
#pragma unroll
            for (int j = 0; j < 8; ++j) bsum[j] += (float)A[i][j];   // db partial (used when k0 == 0)
        }
#pragma unroll
        for (int i = 0; i < C::NPB; ++i) *reinterpret_cast<bf16x8*>(lb + swz<TK>(rrb + C::RPPB * i, cgb)) = B[i];
    };
    f32x16 acc[C::AN][C::AK];
#pragma unroll
    for (int a = 0; a < C::AN; ++a)
#pragma unroll
        for (int b = 0; b < C::AK; ++b) acc[a][b] = f32x16{};
    auto mfmas = [&](int buf) {
        const bf16* la = lds + buf * C::BUF;
        const bf16* lb = la + TM * TN;
#pragma unroll
        for (int s = 0; s < TM / 16; ++s) {
            bf16x8 fa[C::AN], fb[C::AK];
#pragma unroll
            for (int a = 0; a < C::AN; ++a) fa[a] = tr_frag<TN>(la, wn + 32 * a, s, lane);
#pragma unroll
            for (int b = 0; b < C::AK; ++b) fb[b] = tr_frag<TK>(lb, wk + 32 * b, s, lane);
#pragma unroll
            for (int a = 0; a < C::AN; ++a)
#pragma unroll
                for (int b = 0; b < C::AK; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
            // 256 x 256: one k-step's fragments live at a time (the 256 accumulators fill the AGPRs)
            // 128 x 128 (4 waves, 2 workgroups per CU): the same -- with every k-step's fragments hoisted
            // the kernel spilled an LDS address whose reload (vmcnt) waited for the whole load prefetch
            if constexpr (TN * TK > 256 * 128 || (WG_SB128 && TN * TK == 128 * 128 && NTH == NT))
                __builtin_amdgcn_sched_barrier(0);
        }
    };
    // Register set s % D holds step s, LDS buffer s & 1.  The loop runs a multiple of lcm(D, 2) steps
    // with no conditions inside (steps past the chunk load zeros from outside the buffer resource):
    // a conditional load or stage makes hipcc wait for every load in flight.
#pragma unroll
    for (int q = 0; q < D; ++q) load(ra[q], rb[q], q);
    stage(ra[0], rb[0], 0);
    load(ra[0], rb[0], D);
    __syncthreads();
    WG_STAMP(1);
    auto body = [&](int i, auto Q, auto B) {   // Q: register set of step i + 1, B: its LDS buffer
        constexpr int q = decltype(Q)::value, nb = decltype(B)::value;
        STEP_STAMP(0, i);
        stage(ra[q], rb[q], nb);                             // LDS buffer nb last read in step i - 1
        STEP_STAMP(1, i);
        load(ra[q], rb[q], i + 1 + D);
        mfmas(nb ^ 1);
        STEP_STAMP(2, i);
        __syncthreads();
        STEP_STAMP(3, i);
    };
    constexpr int U = D % 2 ? 2 * D : D;                     // unroll: lcm(D, 2)
    for (int i = 0; i < nsteps; i += U) unroll_steps<0, U, D>(body, i);
    WG_STAMP(2);
    // acc[a][b][reg] = dW[n0 + wn + 32a + crow(reg, h)][k0 + wk + 32b + r]
    if (chunks == 1) {   // buffer stores: out-of-range elements get an offset past the resource (dropped)
        const __amdgpu_buffer_rsrc_t rd = buf_rsrc(dst, (long)N * K * 4);
#pragma unroll
        for (int a = 0; a < C::AN; ++a)
#pragma unroll
            for (int b = 0; b < C::AK; ++b)
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int n = n0 + wn + 32 * a + crow(reg, h), k = k0 + wk + 32 * b + r;
                    const unsigned off = (n < N && k < K) ? (unsigned)(n * K + k) * 4u : kOOB;
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][reg]), rd, off, 0, 0);
                }
    } else {
        float* o = slab + ((long)tile * chunks + chunk) * (TN * TK);
#pragma unroll
        for (int a = 0; a < C::AN; ++a)
#pragma unroll
            for (int b = 0; b < C::AK; ++b)
#pragma unroll
                for (int reg = 0; reg < 16; ++reg)
                    o[(wn + 32 * a + crow(reg, h)) * TK + wk + 32 * b + r] = acc[a][b][reg];
    }
    if (do_bias) {   // column sums of dY: threads with the same cga hold the same 8 columns
        float* red = reinterpret_cast<float*>(lds);   // [NTH][9]: both LDS buffers are free now
#pragma unroll
        for (int j = 0; j < 8; ++j) red[threadIdx.x * 9 + j] = bsum[j];
        __syncthreads();
        if (threadIdx.x < TN) {
            const int g = threadIdx.x >> 3, j = threadIdx.x & 7;   // column n0 + 8g + j
            float sum = 0.f;
            for (int q = g; q < NTH; q += C::CPRA) sum += red[q * 9 + j];
            if (chunks == 1) {
                if (n0 + threadIdx.x < N) dst[(long)N * K + n0 + threadIdx.x] = sum;
            } else {
                float* bs = slab + (long)tiles * chunks * (TN * TK);
                bs[((long)ntile * chunks + chunk) * TN + threadIdx.x] = sum;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int TN, int TK, int D, int NTH = NT>
__global__ __launch_bounds__(NTH, D > 2 || NTH > NT ? 1 : 2) void wgrad_tile(long M, int N, int K, long rpc, int chunks,
                                                    const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                    float* __restrict__ dst, float* __restrict__ slab) {
    __shared__ __attribute__((aligned(16))) bf16 lds[2 * TileCfg<TN, TK, NTH>::BUF];
    WG_STAMP(0);
    // tiles of one token chunk are consecutive logical ids -> one XCD streams the chunk once
    // (readfirstlane: keep the tile decode in SGPRs -- a buffer resource built from a VGPR base
    // turns every buffer load into a waterfall loop)
    const int t = __builtin_amdgcn_readfirstlane((int)xcd_tile(blockIdx.x, gridDim.x));
    wgrad_tile_body<TN, TK, D, NTH>(lds, t, M, N, K, rpc, chunks, dy, x, dst, slab);
    WG_STAMP(3);
}

// Grouped form: the weight gradients of many Linears in ONE launch (the end-of-backward batch of
// every deferred token-Linear weight gradient).  Item table in the kernel arguments; logical
// workgroup -> item by a scan over the prefix sums (scalar), then the same tile body.  One launch
// has no per-Linear underfilled rounds or tails, so each Linear can use few token chunks (small
// partial slabs) and still keep every CU busy.
constexpr int WGG_MAX = 48;
struct WgGroup {
    const bf16* dy[WGG_MAX];
    const bf16* x[WGG_MAX];
    float* dst[WGG_MAX];
    float* slab[WGG_MAX];
    int M[WGG_MAX], N[WGG_MAX], K[WGG_MAX], chunks[WGG_MAX], rpc[WGG_MAX], b0[WGG_MAX + 1];
    int count;
};

template <int TN, int TK, int NTH = NT, int D = 2>
__global__ __launch_bounds__(NTH, NTH > NT || TN * TK > 256 * 128 ? 1 : 2) void wgrad_group(WgGroup g) {
    __shared__ __attribute__((aligned(16))) bf16 lds[2 * TileCfg<TN, TK, NTH>::BUF];
    const int lt = __builtin_amdgcn_readfirstlane((int)xcd_tile(blockIdx.x, gridDim.x));
    int i = 0;
    while (i + 1 < g.count && g.b0[i + 1] <= lt) ++i;
    i = __builtin_amdgcn_readfirstlane(i);
    wgrad_tile_body<TN, TK, D, NTH>(lds, lt - g.b0[i], g.M[i], g.N[i], g.K[i], g.rpc[i], g.chunks[i], g.dy[i], g.x[i],
                                    g.dst[i], g.slab[i]);
}

// dst[n][k] = sum_c slab[tile(n, k)][c][n % TN][k % TK], then dst[N*K + n] = sum_c bslab[n / TN][c][n % TN].
// A workgroup = NT / G output quads x G chunk groups: group g sums chunks g, g + G, ... (four 16-B
// loads in flight), then group 0 adds the G partials in order -- fixed association, deterministic.
// G grows with the chunk count: a Linear with ~170 chunks (stage 1, 262144 tokens) and few outputs
// otherwise serialises ~40 load round trips on a few thousand threads.
__host__ __device__ inline int wslab_groups(int chunks) {
    int g = 1;
    while (g < 16 && g * 8 < chunks) g <<= 1;
    return g;
}
inline long wslab_blocks(int N, int K, int chunks) {
    const long quads = ((long)N * K + N) / 4, qb = NT / wslab_groups(chunks);
    return (quads + qb - 1) / qb;
}

__device__ __forceinline__ void wslab_sum(long blk, int N, int K, int TN, int TK, int chunks,
                                          const float* __restrict__ slab, float* __restrict__ dst) {
    __shared__ f32x4 red[NT];
    const int G = wslab_groups(chunks), QB = NT / G;
    const int g = threadIdx.x / QB, qi = threadIdx.x % QB;
    const long e = (blk * QB + qi) * 4;   // first of the thread's 4 outputs
    const long NK = (long)N * K;
    const int kt = (K + TK - 1) / TK, nt = (N + TN - 1) / TN;
    const long step = (long)TN * TK;
    const float* p = slab;
    long stride = 0;
    const bool valid = e < NK + N;
    if (e < NK) {
        const int n = (int)(e / K), k = (int)(e % K);
        const long tile = (long)(n / TN) * kt + k / TK;
        p = slab + tile * chunks * step + (long)(n % TN) * TK + (k % TK);
        stride = step;
    } else if (valid) {
        const int n = (int)(e - NK);
        p = slab + (long)nt * kt * chunks * step + ((long)(n / TN) * chunks) * TN + (n % TN);
        stride = TN;
    }
    f32x4 a0 = {}, a1 = {}, a2 = {}, a3 = {};
    if (valid) {
        int c = g;
        for (; c + 3 * G < chunks; c += 4 * G) {
            a0 += *reinterpret_cast<const f32x4*>(p + c * stride);
            a1 += *reinterpret_cast<const f32x4*>(p + (c + G) * stride);
            a2 += *reinterpret_cast<const f32x4*>(p + (c + 2 * G) * stride);
            a3 += *reinterpret_cast<const f32x4*>(p + (c + 3 * G) * stride);
        }
        for (; c < chunks; c += G) a0 += *reinterpret_cast<const f32x4*>(p + c * stride);
    }
    const f32x4 s = (a0 + a1) + (a2 + a3);
    if (G == 1) {
        if (valid) *reinterpret_cast<f32x4*>(dst + e) = s;
        return;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (g == 0 && valid) {
        f32x4 t = red[qi];
        for (int j = 1; j < G; ++j) t += red[j * QB + qi];
        *reinterpret_cast<f32x4*>(dst + e) = t;
    }
}

__global__ __launch_bounds__(NT) void wslab_reduce(int N, int K, int TN, int TK, int chunks,
                                                   const float* __restrict__ slab, float* __restrict__ dst) {
    wslab_sum(blockIdx.x, N, K, TN, TK, chunks, slab, dst);
}

// many deferred slab reductions in one launch: item table in the kernel arguments (capturable),
// workgroup -> item by a scan over the block prefix sums (workgroup-uniform: scalar loads)
constexpr int WSB_MAX = 40;
struct WsBatch {
    const float* slab[WSB_MAX];
    float* dst[WSB_MAX];
    int N[WSB_MAX], K[WSB_MAX], tn[WSB_MAX], tk[WSB_MAX], chunks[WSB_MAX], b0[WSB_MAX + 1];
    int count;
};

__global__ __launch_bounds__(NT) void wslab_reduce_batch(WsBatch t) {
    const int b = blockIdx.x;
    int i = 0;
    while (i + 1 < t.count && t.b0[i + 1] <= b) ++i;
    wslab_sum(b - t.b0[i], t.N[i], t.K[i], t.tn[i], t.tk[i], t.chunks[i], t.slab[i], t.dst[i]);
}

int num_cus() {
    static int v = 0;
    if (!v) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess
            && n > 0)
            v = n;
        else
            v = 256;
    }
    return v;
}

struct Plan {
    int tn, tk, nt, kt, chunks, depth;
    long rpc;
};

// modelled launch time (us) of tile tn x tk with c chunks (tools/wgrad_bench.py): workgroup rounds x
// (tile bytes / c at ~70 GB/s per CU + ~3 us fixed per workgroup) + the slab reduction (~2 us + slab
// bytes at HBM rate).  One partial round doubles a launch (48 tiles: 6 chunks = 288 workgroups = 2
// rounds, 5 chunks = 240 = 1 round).
double model_us(long M, int N, int K, int tn, int tk, long c) {
    const long cus = num_cus();
    const long tiles = (long)((N + tn - 1) / tn) * ((K + tk - 1) / tk);
    const long rounds = (tiles * c + cus - 1) / cus;
    const double tile_us = (double)M * (tn + tk) * 2.0 / 70e3;   // 70 GB/s = 70e3 B/us
    double t = (double)rounds * (tile_us / (double)c + 3.0);
    if (c > 1) t += 2.0 + (double)c * ((double)N * K + N) * 8.0 / 8e6;
    return t;
}

// Plan: tile size and token chunks minimising model_us (each chunk >= 1024 tokens, >= 2048 with
// <= 2 tiles); 128-wide tiles need N, K multiples of 128.  tn / tk / chunks > 0 override
// (csu_linear_wgrad_tuned).
Plan make_plan(long M, int N, int K, int tn, int tk, int chunks) {
    Plan p;
    if (tn == 256) {   // explicit 256 x 128 tiles (the grouped path's choice for N % 256, K % 128 == 0)
        p.tn = 256;
        p.tk = 128;
        p.nt = (N + 255) / 256;
        p.kt = (K + 127) / 128;
        const long c = chunks > 0 ? chunks : 1;
        p.rpc = ((M + c - 1) / c + TM - 1) / TM * TM;
        p.chunks = (int)((M + p.rpc - 1) / p.rpc);
        p.depth = 2;
        return p;
    }
    double best = 1e30;
    p.tn = p.tk = 64;
    long want = 1;
    const int sizes[2] = {64, 128};
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            const int ctn = sizes[a], ctk = sizes[b];
            if ((tn > 0 && ctn != tn) || (tk > 0 && ctk != tk)) continue;
            if (tn <= 0 && tk <= 0 && ctn != ctk) continue;   // mixed tiles measured slower than the model says
            if ((ctn == 128 && N % 128) || (ctk == 128 && K % 128)) continue;
            const long tiles = (long)((N + ctn - 1) / ctn) * ((K + ctk - 1) / ctk);
            const long mintok = tiles <= 2 ? 2048 : 1024;
            const long maxc = chunks > 0 ? chunks : (M + mintok - 1) / mintok;
            for (long c = chunks > 0 ? chunks : 1; c <= maxc && c <= 4 * num_cus(); ++c) {
                const double t = model_us(M, N, K, ctn, ctk, c);
                if (t < best - 1e-9) {
                    best = t;
                    p.tn = ctn;
                    p.tk = ctk;
                    want = c;
                }
            }
        }
    p.nt = (N + p.tn - 1) / p.tn;
    p.kt = (K + p.tk - 1) / p.tk;
    if (want < 1) want = 1;
    p.rpc = ((M + want - 1) / want + TM - 1) / TM * TM;
    p.chunks = (int)((M + p.rpc - 1) / p.rpc);
    p.depth = 2;
    return p;
}

// workspace: [partial tiles [tile][chunk][TN][TK]][db partials [n_tile][chunk][TN]]
size_t plan_bytes(const Plan& p) {
    if (p.chunks == 1) return 0;
    return ((size_t)p.nt * p.kt * p.tn * p.tk + (size_t)p.nt * p.tn) * p.chunks * sizeof(float);
}

template <int TN, int TK>
void launch_tile(const Plan& p, unsigned grid, long M, int N, int K, const bf16* dy, const bf16* x, float* dst,
                 float* slab, hipStream_t st) {
    constexpr int NTH = TN == 256 ? 2 * NT : NT;
    wgrad_tile<TN, TK, 2, NTH><<<grid, NTH, 0, st>>>(M, N, K, p.rpc, p.chunks, dy, x, dst, slab);
}

int run_bf16(const Plan& p, long M, int N, int K, const bf16* dy, const bf16* x, float* dst, void* ws, hipStream_t st,
             bool defer = false) {
    const unsigned grid = (unsigned)((long)p.nt * p.kt * p.chunks);
    float* slab = p.chunks > 1 ? (float*)ws : nullptr;
    if (p.tn == 256 && p.tk == 128) launch_tile<256, 128>(p, grid, M, N, K, dy, x, dst, slab, st);
    else if (p.tn == 128 && p.tk == 128) launch_tile<128, 128>(p, grid, M, N, K, dy, x, dst, slab, st);
    else if (p.tn == 128 && p.tk == 64) launch_tile<128, 64>(p, grid, M, N, K, dy, x, dst, slab, st);
    else if (p.tn == 64 && p.tk == 128) launch_tile<64, 128>(p, grid, M, N, K, dy, x, dst, slab, st);
    else if (p.tn == 64 && p.tk == 64) launch_tile<64, 64>(p, grid, M, N, K, dy, x, dst, slab, st);
    else return fail(CSU_E_ARG, "linear_wgrad: tile must be 64 or 128 (or 256 x 128)");
    if (int e = check_launch("linear_wgrad")) return e;
    if (p.chunks > 1 && !defer) {
        wslab_reduce<<<(unsigned)wslab_blocks(N, K, p.chunks), NT, 0, st>>>(N, K, p.tn, p.tk, p.chunks, slab, dst);
        return check_launch("linear_wgrad reduce");
    }
    return 0;
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" size_t csu_linear_wgrad_tuned_workspace(long M, int N, int K, int tn, int tk, int chunks) {
    const Plan32 q = plan32(M, N, K);
    const size_t a = (size_t)q.chunks * ((size_t)N * K + N) * sizeof(float) +
                     colsum_workspace(q.chunks, (long)N * K + N, CSU_F32);
    const size_t b = plan_bytes(make_plan(M, N, K, tn, tk, chunks));
    return a > b ? a : b;
}

extern "C" size_t csu_linear_wgrad_workspace(long M, int N, int K) {
    return csu_linear_wgrad_tuned_workspace(M, N, K, 0, 0, 0);
}

extern "C" int csu_linear_wgrad_tuned(long M, int N, int K, int dtype, const void* dy, const void* x, float* dw_db,
                                      void* workspace, size_t ws_bytes, int tn, int tk, int chunks, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !dy || !x || !dw_db) return fail(CSU_E_ARG, "linear_wgrad: bad args");
    const int V = dtype == CSU_BF16 ? 8 : 4;
    if (N % V || K % V) return fail(CSU_E_ARG, "linear_wgrad: N and K must be multiples of 16 bytes");
    if (ws_bytes < csu_linear_wgrad_tuned_workspace(M, N, K, tn, tk, chunks) ||
        (!workspace && csu_linear_wgrad_tuned_workspace(M, N, K, tn, tk, chunks)))
        return fail(CSU_E_WORKSPACE, "linear_wgrad: workspace");
    hipStream_t st = as_stream(stream);
    if (dtype == CSU_BF16) {
        if ((tn && tn != 64 && tn != 128 && tn != 256) || (tk && tk != 64 && tk != 128) ||
            (tn == 256 && (tk != 128 || N % 256 || K % 128)))
            return fail(CSU_E_ARG, "linear_wgrad: tile");
        const Plan p = make_plan(M, N, K, tn, tk, chunks);
        return run_bf16(p, M, N, K, (const bf16*)dy, (const bf16*)x, dw_db, workspace, st);
    }
    if (dtype != CSU_F32) return fail(CSU_E_ARG, "linear_wgrad: bad dtype");
    const Plan32 q = plan32(M, N, K);
    const long slab = (long)N * K + N;
    float* part = (float*)workspace;
    wgrad_f32<<<dim3(q.nt, q.kt, q.chunks), NT, 0, st>>>(M, N, K, q.rpc, (const float*)dy, (const float*)x, part);
    if (int e = check_launch("linear_wgrad f32")) return e;
    return colsum_launch(q.chunks, slab, CSU_F32, part, dw_db, part + (size_t)q.chunks * slab, st);
}

extern "C" int csu_linear_wgrad(long M, int N, int K, int dtype, const void* dy, const void* x, float* dw_db,
                                void* workspace, size_t ws_bytes, void* stream) {
    return csu_linear_wgrad_tuned(M, N, K, dtype, dy, x, dw_db, workspace, ws_bytes, 0, 0, 0, stream);
}

extern "C" int csu_linear_wgrad_deferred(long M, int N, int K, const void* dy, const void* x, float* dw_db,
                                         void* workspace, size_t ws_bytes, csu_wslab_item* item, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !dy || !x || !dw_db || !item) return fail(CSU_E_ARG, "linear_wgrad_deferred: bad args");
    if (N % 8 || K % 8) return fail(CSU_E_ARG, "linear_wgrad_deferred: N and K must be multiples of 8");
    const Plan p = make_plan(M, N, K, 0, 0, 0);
    if (ws_bytes < plan_bytes(p) || (!workspace && plan_bytes(p))) return fail(CSU_E_WORKSPACE, "linear_wgrad_deferred: workspace");
    *item = csu_wslab_item{(const float*)workspace, dw_db, N, K, p.tn, p.tk, p.chunks, 0};
    return run_bf16(p, M, N, K, (const bf16*)dy, (const bf16*)x, dw_db, workspace, as_stream(stream), true);
}

// Plan of a Linear inside a grouped launch: 256 x 128 tiles (8 waves) when N % 256 == 0 and K % 128 == 0,
// 128 x 128 when both are multiples of 128, else 64 x 64; token chunks so
// that the fp32 partial slabs stay <= ~1/16 of the operand bytes (chunks <= M (N + K) / (32 N K)),
// >= 1024 tokens per chunk.  No occupancy target: the group fills the GPU.
// slab bytes <= operand bytes * 2 / kSlabDiv (A/B at 512 B16: 8 -> 1231 img/s, 16 -> 1249, 32 -> 1255, 64 -> 1227)
constexpr int kSlabDiv = 32;
// WG_RECT: 128 x 64 / 64 x 128 tiles for the C = 64 Linears whose other side is a multiple of 128
#ifndef WG_RECT
#define WG_RECT 1
#endif
static void group_plan(long M, int N, int K, int* tn, int* tk, int* chunks, long* rpc) {
    const int t = (N % 256 == 0 && K % 128 == 0) ? 256 : (N % 128 == 0 && K % 128 == 0) ? 128 : 64;
    long c = (long)((double)M * (N + K) / ((double)kSlabDiv * N * K) + 0.5);
    const long maxc = M / 1024 > 0 ? M / 1024 : 1;
    if (c > maxc) c = maxc;
    if (c < 1) c = 1;
    long r = ((M + c - 1) / c + TM - 1) / TM * TM;
    c = (M + r - 1) / r;
    *tn = t;
    *tk = t == 256 ? 128 : t;
    if (WG_RECT && t == 64) {   // one 128-wide side where it divides: 3/4 of the 64 x 64 tile's staged bytes per output
        if (N % 128 == 0) *tn = 128;
        else if (K % 128 == 0) *tk = 128;
    }
    *chunks = (int)c;
    *rpc = r;
}

extern "C" size_t csu_linear_wgrad_group_plan(long M, int N, int K, int* tn, int* tk, int* chunks) {
    int a, b, c;
    long r;
    group_plan(M, N, K, &a, &b, &c, &r);
    if (tn) *tn = a;
    if (tk) *tk = b;
    if (chunks) *chunks = c;
    if (c == 1) return 0;
    const long nt = (N + a - 1) / a, kt = (K + b - 1) / b;
    return ((size_t)nt * kt * a * b + (size_t)nt * a) * c * sizeof(float);
}

extern "C" int csu_linear_wgrad_group(const csu_wgrad_group_item* items, int count, void* stream) {
    if (count < 0 || (count && !items)) return fail(CSU_E_ARG, "linear_wgrad_group: bad args");
    hipStream_t st = as_stream(stream);
    constexpr int kPass[5][2] = {{256, 128}, {128, 128}, {128, 64}, {64, 128}, {64, 64}};
    for (int pass = 0; pass < 5; ++pass) {   // one launch per tile shape present
        const int T = kPass[pass][0], TK = kPass[pass][1];
        WgGroup g;
        g.count = 0;
        g.b0[0] = 0;
        auto flush = [&]() -> int {
            if (!g.count) return 0;
            if (T == 256) wgrad_group<256, 128, 2 * NT><<<(unsigned)g.b0[g.count], 2 * NT, 0, st>>>(g);
            else if (T == 128 && TK == 128) wgrad_group<128, 128><<<(unsigned)g.b0[g.count], NT, 0, st>>>(g);
            else if (T == 128) wgrad_group<128, 64><<<(unsigned)g.b0[g.count], NT, 0, st>>>(g);
            else if (TK == 128) wgrad_group<64, 128><<<(unsigned)g.b0[g.count], NT, 0, st>>>(g);
            else wgrad_group<64, 64><<<(unsigned)g.b0[g.count], NT, 0, st>>>(g);
            g.count = 0;
            return check_launch("linear_wgrad_group");
        };
        for (int i = 0; i < count; ++i) {
            const csu_wgrad_group_item& it = items[i];
            if (it.M < 1 || it.N % 8 || it.K % 8 || !it.dy || !it.x || !it.dw_db)
                return fail(CSU_E_ARG, "linear_wgrad_group: bad item");
            int tn, tk, c;
            long r;
            group_plan(it.M, it.N, it.K, &tn, &tk, &c, &r);
            if (tn != T || tk != TK) continue;
            if (c > 1 && !it.slab) return fail(CSU_E_WORKSPACE, "linear_wgrad_group: item needs a slab workspace");
            const long tiles = (long)((it.N + tn - 1) / tn) * ((it.K + tk - 1) / tk);
            if (g.count == WGG_MAX || (long)g.b0[g.count] + tiles * c > (1L << 30))
                if (int e = flush()) return e;
            const int k = g.count;
            g.dy[k] = (const bf16*)it.dy;
            g.x[k] = (const bf16*)it.x;
            g.dst[k] = it.dw_db;
            g.slab[k] = it.slab;
            g.M[k] = (int)it.M; g.N[k] = it.N; g.K[k] = it.K; g.chunks[k] = c; g.rpc[k] = (int)r;
            g.b0[k + 1] = g.b0[k] + (int)(tiles * c);
            g.count = k + 1;
        }
        if (int e = flush()) return e;
    }
    return 0;
}

extern "C" int csu_wslab_reduce_batch(const csu_wslab_item* items, int count, void* stream) {
    if (count < 0 || (count && !items)) return fail(CSU_E_ARG, "wslab_reduce_batch: bad args");
    WsBatch t;
    t.count = 0;
    t.b0[0] = 0;
    auto flush = [&]() -> int {
        if (!t.count) return 0;
        wslab_reduce_batch<<<(unsigned)t.b0[t.count], NT, 0, as_stream(stream)>>>(t);
        t.count = 0;
        return check_launch("wslab_reduce_batch");
    };
    for (int i = 0; i < count; ++i) {
        const csu_wslab_item& it = items[i];
        if (it.chunks <= 1) continue;   // written by the tile kernel itself
        if (!it.slab || !it.dst || it.N % 4 || it.K % 4) return fail(CSU_E_ARG, "wslab_reduce_batch: bad item");
        const long blocks = wslab_blocks(it.N, it.K, it.chunks);
        if (t.count == WSB_MAX || (long)t.b0[t.count] + blocks > (1L << 30))
            if (int e = flush()) return e;
        const int c = t.count;
        t.slab[c] = it.slab;
        t.dst[c] = it.dst;
        t.N[c] = it.N; t.K[c] = it.K; t.tn[c] = it.tn; t.tk[c] = it.tk; t.chunks[c] = it.chunks;
        t.b0[c + 1] = t.b0[c] + (int)blocks;
        t.count = c + 1;
    }
    return flush();
}

#ifdef WG_TIMING
extern "C" int csu_debug_wgrad_ts(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(csu::wg_ts), sizeof(csu::wg_ts), 0, hipMemcpyDeviceToHost);
}
extern "C" int csu_debug_wgrad_steps(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(csu::wg_steps), sizeof(csu::wg_steps), 0, hipMemcpyDeviceToHost);
}
#endif
