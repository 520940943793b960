// Linear weight + bias gradient over token rows for gfx950 (bf16/fp32 in, fp32 out).
//
//   dW[n][k] = sum_m dY[m][n] * X[m][k],   db[n] = sum_m dY[m][n]       (m = the B*L tokens)
// This is the backward of every nn.Linear of the model (qkv/proj/fc1/fc2 cswin:185/187/314/323,
// concat_linear cswin:568/581/592, the CARAFE 1x1 convs cswin:396/399).  M is huge (up to 4M
// tokens) while N, K <= 2048, so the reduction dim is split: workgroup (n-tile, k-tile, chunk)
// accumulates a 64x64 tile over its token chunk with v_mfma_f32_32x32x16_bf16 (f32: 32x32x2),
// both operands staged transposed in LDS ([n][m] / [k][m]) so MFMA fragments are 16-B reads.
// Partial tiles (and the db partials of the k-tile-0 workgroups) go to a [chunk][N*K + N] slab
// that one deterministic column-sum pass reduces in chunk order.
#include <cstdlib>

#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int TM = 64;    // tokens per LDS step
constexpr int TN = 64;    // output tile (n) per workgroup
constexpr int TK = 64;    // output tile (k) per workgroup

template <typename T> struct WCfg;
template <> struct WCfg<float> { static constexpr int S = TM + 4; };

// stage a TM x 64 row-major tile (rows m0.., columns c0..) of a (M, ld) matrix transposed into
// img[64][S]; rows >= M and columns >= ncols are zero.  Pairs of rows are packed per LDS write.
template <typename T>
__device__ __forceinline__ void stage_t(const T* __restrict__ g, long M, int ld, int ncols, long m0, int c0, T* img) {
    constexpr int V = 16 / sizeof(T);           // elements per 16-B load
    constexpr int CPR = 64 / V;                 // chunks per row
    constexpr int S = WCfg<T>::S;
    for (int it = threadIdx.x; it < (TM / 2) * CPR; it += NT) {
        const int pr = it / CPR, q = it % CPR;  // row pair, column chunk
        const long m = m0 + 2 * pr;
        const int c = c0 + q * V;
        float a[V], b[V];
        const bool cv = c < ncols;
        if (cv && m < M) { if constexpr (V == 8) load8(g + m * ld + c, a); else load4(g + m * ld + c, a); }
        else for (int j = 0; j < V; ++j) a[j] = 0.f;
        if (cv && m + 1 < M) { if constexpr (V == 8) load8(g + (m + 1) * ld + c, b); else load4(g + (m + 1) * ld + c, b); }
        else for (int j = 0; j < V; ++j) b[j] = 0.f;
#pragma unroll
        for (int j = 0; j < V; ++j) {
            T* p = img + (q * V + j) * S + 2 * pr;
            p[0] = from_f<T>(a[j]);
            p[1] = from_f<T>(b[j]);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(NT) void wgrad_kernel(long M, int N, int K, long rows_per_chunk, const T* __restrict__ dy,
                                                   const T* __restrict__ x, float* __restrict__ part) {
    constexpr int S = WCfg<T>::S;
    __shared__ __attribute__((aligned(16))) T At[TN * S];   // dY^T tile [n][m]
    __shared__ __attribute__((aligned(16))) T Bt[TK * S];   // X^T  tile [k][m]
    __shared__ float bred[NT];
    const int n0 = blockIdx.x * TN, k0 = blockIdx.y * TK;
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
        stage_t<T>(dy, m_end, N, N, m0, n0, At);
        stage_t<T>(x, m_end, K, K, m0, k0, Bt);
        __syncthreads();
        if (do_bias) {   // column sums of the staged dY^T image: thread -> (n, quarter of m)
            const int n = threadIdx.x & 63, qq = threadIdx.x >> 6;
#pragma unroll
            for (int j = 0; j < TM / 4; ++j) bsum += to_f(At[n * S + qq * (TM / 4) + j]);
        }
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int s = 0; s < TM / 16; ++s) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(At + (wn + r) * S + 16 * s + 8 * h);
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(Bt + (wk + r) * S + 16 * s + 8 * h);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int t = 0; t < TM / 2; ++t)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(At[(wn + r) * S + 2 * t + h], Bt[(wk + r) * S + 2 * t + h], acc, 0, 0, 0);
        }
    }
    // acc[reg] = dW[n0 + wn + crow(reg, h)][k0 + wk + r]
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

// bf16 fast path: row-major LDS tiles filled by coalesced 16-B loads (prefetched one step ahead
// in registers), MFMA fragments gathered with the gfx950 transposing read ds_read_b64_tr_b16
// (lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3; lane i receives column i of
// the 4 rows).  Rows padded by 64 B make the transposed reads of 4 rows bank-conflict free.
// Tile T x T (T = 64 or 128) per workgroup, each wave (T/2) x (T/2): at T = 128 every fragment
// feeds two MFMAs and the operand panels are re-read half as often (N/T + K/T passes).
typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4s tr_read(const bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// 32x32x16 operand fragment of columns [c0, c0+32) at k-step rows [16s + 8h, +8) of a [TM][RS] tile
template <int RS>
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int c0, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = 16 * s + 8 * (grp >> 1) + q;
    const v4s lo = tr_read(img + row * RS + col);
    const v4s hi = tr_read(img + (row + 4) * RS + col);
    const v4s v[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

__device__ __forceinline__ float gelu_w(float v) { return gelu_fast(v); }   // common.hpp (A-S 7.1.25)

template <int T, bool GELU_X>
__global__ __launch_bounds__(NT) void wgrad_bf16_tr(long M, int N, int K, long rows_per_chunk, const bf16* __restrict__ dy,
                                                   const bf16* __restrict__ x, float* __restrict__ part) {
    constexpr int RS = T + 32;          // bf16 elements per LDS row (T data + 64 B pad)
    constexpr int CPR = T / 8;          // 16-B chunks per row
    constexpr int RPP = NT / CPR;       // rows per pass of the workgroup
    constexpr int NP = TM / RPP;        // passes (chunks per thread per operand)
    constexpr int AT = T / 64;          // 32x32 tiles per wave per dim
    __shared__ __attribute__((aligned(16))) bf16 At[TM * RS];   // dY tile [m][n]
    __shared__ __attribute__((aligned(16))) bf16 Bt[TM * RS];   // X  tile [m][k]
    __shared__ float bred[NT][9];
    // tiles of one token chunk are consecutive logical ids -> one XCD reads the chunk once
    const int nt = (N + T - 1) / T, kt = (K + T - 1) / T;
    const long t = xcd_tile(blockIdx.x, gridDim.x);
    const int chunk = (int)(t / (nt * kt)), tt = (int)(t % (nt * kt));
    const int n0 = (tt / kt) * T, k0 = (tt % kt) * T;
    const long m_begin = (long)chunk * rows_per_chunk;
    const long m_end = min(M, m_begin + rows_per_chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave >> 1) * (T / 2), wk = (wave & 1) * (T / 2);
    const bool do_bias = k0 == 0;
    const int cg = threadIdx.x % CPR, rr = threadIdx.x / CPR;   // rows rr + RPP i
    const bool nv = n0 + 8 * cg < N, kv = k0 + 8 * cg < K;
    bf16x8 ra[NP], rb[NP];
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto load = [&](long m0) {
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const long m = m0 + rr + RPP * i;
            const bool mv = m < m_end;
            ra[i] = (mv && nv) ? *reinterpret_cast<const bf16x8*>(dy + m * N + n0 + 8 * cg) : bf16x8{};
            rb[i] = (mv && kv) ? *reinterpret_cast<const bf16x8*>(x + m * K + k0 + 8 * cg) : bf16x8{};
        }
    };
    f32x16 acc[AT][AT];
#pragma unroll
    for (int a = 0; a < AT; ++a)
#pragma unroll
        for (int b = 0; b < AT; ++b) acc[a][b] = f32x16{};
    load(m_begin);
    for (long m0 = m_begin; m0 < m_end; m0 += TM) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            *reinterpret_cast<bf16x8*>(At + (rr + RPP * i) * RS + 8 * cg) = ra[i];
            bf16x8 xv = rb[i];
            if constexpr (GELU_X) {   // X = gelu(h) on the fly (fc2's input, never materialised)
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[j] = (bf16)gelu_w((float)xv[j]);
            }
            *reinterpret_cast<bf16x8*>(Bt + (rr + RPP * i) * RS + 8 * cg) = xv;
            if (do_bias)
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[j] += (float)ra[i][j];
        }
        __syncthreads();
        if (m0 + TM < m_end) load(m0 + TM);      // next step's loads fly during the MFMAs
#pragma unroll
        for (int s = 0; s < TM / 16; ++s) {
            bf16x8 fa[AT], fb[AT];
#pragma unroll
            for (int a = 0; a < AT; ++a) fa[a] = tr_frag<RS>(At, wn + 32 * a, s, lane);
#pragma unroll
            for (int b = 0; b < AT; ++b) fb[b] = tr_frag<RS>(Bt, wk + 32 * b, s, lane);
#pragma unroll
            for (int a = 0; a < AT; ++a)
#pragma unroll
                for (int b = 0; b < AT; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
    }
    const long slab = (long)N * K + N;
    float* out = part + (long)chunk * slab;
#pragma unroll
    for (int a = 0; a < AT; ++a)
#pragma unroll
        for (int b = 0; b < AT; ++b)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = n0 + wn + 32 * a + crow(reg, h), k = k0 + wk + 32 * b + r;
                if (n < N && k < K) out[(long)n * K + k] = acc[a][b][reg];
            }
    if (do_bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bred[threadIdx.x][j] = bsum[j];
        __syncthreads();
        if (threadIdx.x < T) {
            const int g = threadIdx.x >> 3, j = threadIdx.x & 7;   // column n0 + 8g + j
            float sum = 0.f;
            for (int q = g; q < NT; q += CPR) sum += bred[q][j];
            if (n0 + 8 * g + j < N) out[(long)N * K + n0 + 8 * g + j] = sum;
        }
    }
}

struct WPlan {
    int t, nt, kt, chunks;
    long rpc;
};

// bf16 tiles: 128 x 128 when both N and K allow it (half the operand re-reads of 64 x 64), else
// 64 x 64; fp32 path 64 x 64.  ~1024 workgroups, >= 512 tokens per chunk.
int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
int wgrad_tile_env() {   // CSU_WGRAD_T=64|128 forces the tile (A/B comparisons)
    static int v = env_int("CSU_WGRAD_T", 0);
    return v;
}
int wgrad_target_env() {   // CSU_WGRAD_WGS: target workgroup count of the split-K plan
    static int v = env_int("CSU_WGRAD_WGS", 1024);
    return v;
}

int wgrad_mintok_env() {   // CSU_WGRAD_MINTOK: minimum tokens per split-K chunk
    static int v = env_int("CSU_WGRAD_MINTOK", 512);
    return v;
}

WPlan wplan(long M, int N, int K, bool bf16_path) {
    WPlan p;
    const int te = wgrad_tile_env();
    p.t = (bf16_path && N >= 128 && K >= 128 && te != 64) ? 128 : 64;
    p.nt = (N + p.t - 1) / p.t;
    p.kt = (K + p.t - 1) / p.t;
    const long target = wgrad_target_env();
    long want = (target + p.nt * p.kt - 1) / (p.nt * p.kt);
    const long mt = wgrad_mintok_env();
    const long maxc = (M + mt - 1) / mt;        // >= mt tokens per chunk
    if (want > maxc) want = maxc;
    if (want > 256) want = 256;
    if (want < 1) want = 1;
    p.chunks = (int)want;
    p.rpc = ((M + p.chunks - 1) / p.chunks + TM - 1) / TM * TM;
    p.chunks = (int)((M + p.rpc - 1) / p.rpc);
    return p;
}

}  // namespace

int wgrad5_launch(int cfg, long M, int N, int K, long rpc, int chunks, const bf16* dy, const bf16* x, float* part,
                  hipStream_t st);
bool wgrad4_ok(long M, int N, int K);
size_t wgrad4_workspace(long M, int N, int K);
int wgrad4_run(long M, int N, int K, const bf16* dy, const bf16* x, float* dw_db, void* ws, hipStream_t st);
}  // namespace csu

using namespace csu;

// CSU_WGRAD4=1 routes the bf16 path to wgrad4 (LDS-DMA + transposing reads).  Off by default: on
// the 512x512 step shapes it measured 0-40 % slower than the register-staged kernel below (both are
// bound by re-reading the operand panels once per output tile, tools/linear_probe.py).
static bool use_wgrad4() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("CSU_WGRAD4");
        v = e && e[0] == '1';
    }
    return v == 1;
}

// CSU_WGRAD5=<cfg> selects the deep LDS-DMA pipeline kernel (wgrad5.hip) for the bf16 128-tile
// plans; -1 = the register-staged kernel.
static int wgrad5_cfg() {
    static int v = -2;
    if (v == -2) {
        const char* e = getenv("CSU_WGRAD5");
        v = e ? atoi(e) : -1;
    }
    return v;
}

extern "C" size_t csu_linear_wgrad_workspace(long M, int N, int K) {
    const long slab = (long)N * K + N;
    size_t a = 0;
    for (int bf = 0; bf < 2; ++bf) {   // the dtype is not an argument: the larger of both plans
        const WPlan p = wplan(M, N, K, bf == 1);
        const size_t w = (size_t)p.chunks * slab * sizeof(float) + colsum_workspace(p.chunks, slab, CSU_F32);
        a = w > a ? w : a;
    }
    const size_t b = wgrad4_ok(M, N, K) ? wgrad4_workspace(M, N, K) : 0;
    return a > b ? a : b;
}

extern "C" int csu_linear_wgrad_ex(long M, int N, int K, int dtype, const void* dy, const void* x, int x_gelu,
                                   float* dw_db, void* workspace, size_t ws_bytes, void* stream);

extern "C" int csu_linear_wgrad(long M, int N, int K, int dtype, const void* dy, const void* x, float* dw_db,
                                void* workspace, size_t ws_bytes, void* stream) {
    return csu_linear_wgrad_ex(M, N, K, dtype, dy, x, 0, dw_db, workspace, ws_bytes, stream);
}

// split-K partial slabs only (the reduction is left to csu_colsum_batch)
static int wgrad_partials(const WPlan& p, long M, int N, int K, int dtype, const void* dy, const void* x, int x_gelu,
                          float* part, hipStream_t st) {
    const dim3 grid(p.nt, p.kt, p.chunks);
    const dim3 grid1((unsigned)(p.nt * p.kt * p.chunks));
    const bf16* dyb = (const bf16*)dy;
    const bf16* xb = (const bf16*)x;
    if (x_gelu && dtype != CSU_BF16) return fail(CSU_E_UNSUPPORTED, "linear_wgrad: GELU prologue is bf16-only");
    if (dtype == CSU_BF16 && p.t == 128 && !x_gelu && wgrad5_cfg() >= 0) {
        if (int e = wgrad5_launch(wgrad5_cfg(), M, N, K, p.rpc, p.chunks, dyb, xb, part, st)) return e;
    } else if (dtype == CSU_BF16 && p.t == 128 && x_gelu) wgrad_bf16_tr<128, true><<<grid1, NT, 0, st>>>(M, N, K, p.rpc, dyb, xb, part);
    else if (dtype == CSU_BF16 && p.t == 128) wgrad_bf16_tr<128, false><<<grid1, NT, 0, st>>>(M, N, K, p.rpc, dyb, xb, part);
    else if (dtype == CSU_BF16 && x_gelu) wgrad_bf16_tr<64, true><<<grid1, NT, 0, st>>>(M, N, K, p.rpc, dyb, xb, part);
    else if (dtype == CSU_BF16) wgrad_bf16_tr<64, false><<<grid1, NT, 0, st>>>(M, N, K, p.rpc, dyb, xb, part);
    else if (dtype == CSU_F32)
        wgrad_kernel<float><<<grid, NT, 0, st>>>(M, N, K, p.rpc, (const float*)dy, (const float*)x, part);
    else
        return fail(CSU_E_ARG, "linear_wgrad: bad dtype");
    return check_launch("linear_wgrad");
}

extern "C" size_t csu_linear_wgrad_partial_bytes(long M, int N, int K, int dtype) {
    const WPlan p = wplan(M, N, K, dtype == CSU_BF16);
    return (size_t)p.chunks * ((size_t)N * K + N) * sizeof(float);
}

extern "C" int csu_linear_wgrad_partial(long M, int N, int K, int dtype, const void* dy, const void* x, int x_gelu,
                                        float* slabs, size_t slab_bytes, int* chunks, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !dy || !x || !slabs || !chunks) return fail(CSU_E_ARG, "linear_wgrad_partial: bad args");
    const int V = dtype == CSU_BF16 ? 8 : 4;
    if (N % V || K % V) return fail(CSU_E_ARG, "linear_wgrad_partial: N and K must be multiples of 16 bytes");
    if (slab_bytes < csu_linear_wgrad_partial_bytes(M, N, K, dtype)) return fail(CSU_E_WORKSPACE, "linear_wgrad_partial: slabs");
    const WPlan p = wplan(M, N, K, dtype == CSU_BF16);
    *chunks = p.chunks;
    return wgrad_partials(p, M, N, K, dtype, dy, x, x_gelu, slabs, as_stream(stream));
}

extern "C" int csu_linear_wgrad_ex(long M, int N, int K, int dtype, const void* dy, const void* x, int x_gelu,
                                   float* dw_db, void* workspace, size_t ws_bytes, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !dy || !x || !dw_db) return fail(CSU_E_ARG, "linear_wgrad: bad args");
    const int V = dtype == CSU_BF16 ? 8 : 4;
    if (N % V || K % V) return fail(CSU_E_ARG, "linear_wgrad: N and K must be multiples of 16 bytes");
    if (!workspace || ws_bytes < csu_linear_wgrad_workspace(M, N, K)) return fail(CSU_E_WORKSPACE, "linear_wgrad: workspace");
    hipStream_t st = as_stream(stream);
    if (dtype == CSU_BF16 && !x_gelu && use_wgrad4() && wgrad4_ok(M, N, K))
        return wgrad4_run(M, N, K, (const bf16*)dy, (const bf16*)x, dw_db, workspace, st);
    const WPlan p = wplan(M, N, K, dtype == CSU_BF16);
    float* part = (float*)workspace;
    const long slab = (long)N * K + N;
    if (int e = wgrad_partials(p, M, N, K, dtype, dy, x, x_gelu, part, st)) return e;
    return colsum_launch(p.chunks, slab, CSU_F32, part, dw_db, part + (size_t)p.chunks * slab, st);
}
