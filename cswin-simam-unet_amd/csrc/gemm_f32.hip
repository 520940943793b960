// fp32 GEMMs for the fp32 (non-autocast) training path on gfx950 MFMA (v_mfma_f32_32x32x2_f32):
// the token Linear forward, its input gradient and its weight gradient (nn.Linear cswin:185/187/
// 314/323/568/581/592 in fp32, BASELINE config 2), replacing the platform BLAS on that path.
//
//   layout 0 (NT): C[m][n] = sum_k A[m][k] B[n][k]   (+ bias[n], + resid[m][n])   forward  y = x W^T + b
//   layout 1 (NN): C[m][n] = sum_k A[m][k] B[k][n]                                input gradient dx = dy W
//   layout 2 (TN): C[m][n] = sum_k A[k][m] B[k][n]                                weight gradient dW = dy^T x
//
// 128x128 output tiles, 4 waves of 64x64 (2x2 MFMA tiles of 32x32) -- or 64x64 tiles of 4 waves of
// 32x32 when 128-tiles would leave the GPU underfilled --, K staged 16 at a time through
// a double-buffered LDS image stored k-major ([k][m] and [k][n]): the MFMA operand of lane (r, h)
// is one float at [k0 + h][r], conflict-free ds_read_b32.  Global loads are 16-B vectors along
// whichever dimension is contiguous (k for A in layouts 0/1 and B in layout 0, m / n otherwise),
// one K tile ahead in registers.  The fp32 MFMA peak is 157 TFLOP/s; at AI = 2MNK / 4(MK+NK+MN)
// bytes every shape of the model is MFMA-bound.
//
// Products with few output tiles (layout 2 contracts over the 10^4..10^5 tokens; the stage-3/4
// input gradients have small outputs and long contractions) split K into fixed chunks, each writing
// its own fp32 slab, then one reduction sums the slabs in chunk order and applies bias / residual
// (deterministic, no atomics).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
#ifndef F32_T128
#define F32_T128 4   // 128-tiles when they give >= F32_T128 workgroups per CU
#endif
#ifndef F32_MINK2
#define F32_MINK2 256   // minimum split depth of the weight gradient (layout 2, tokens)
#endif
#ifndef F32_BK
#define F32_BK 32
#endif
constexpr int BK = F32_BK, PAD = 4;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// TM x BK tile of operand X into regs (TM BK / 1024 float4 per thread): element (i, k) of X at
// X[i * ld + k] (KC) or X[k * ld + i]
template <int TM, bool KC>
__device__ __forceinline__ void load_tile(const float* X, long ld, long i0, long ni, long k0, long k1, int tid, f32x4* v) {
    constexpr int QR = TM / 4;   // float4 per k row (!KC)
    constexpr int QK = BK / 4;   // float4 per i row (KC)
#pragma unroll
    for (int u = 0; u < TM * BK / 1024; ++u) {
        const int f = tid + u * NT;
        long i, k;
        if constexpr (KC) { i = i0 + f / QK; k = k0 + 4 * (f % QK); }
        else { k = k0 + f / QR; i = i0 + 4 * (f % QR); }
        const bool ok = i < ni && k < k1;   // the contiguous dimension is a multiple of 4
        v[u] = ok ? *reinterpret_cast<const f32x4*>(X + (KC ? i * ld + k : k * ld + i)) : f32x4{};
    }
}

template <int TM, bool KC, int W>
__device__ __forceinline__ void store_tile(float (*S)[W], int tid, const f32x4* v) {
    constexpr int QR = TM / 4, QK = BK / 4;
#pragma unroll
    for (int u = 0; u < TM * BK / 1024; ++u) {
        const int f = tid + u * NT;
        if constexpr (KC) {
            const int i = f / QK, k = 4 * (f % QK);
#pragma unroll
            for (int e = 0; e < 4; ++e) S[k + e][i] = v[u][e];
        } else {
            const int k = f / QR, i = 4 * (f % QR);
            *reinterpret_cast<f32x4*>(&S[k][i]) = v[u];
        }
    }
}

// AK: A(m, k) k-contiguous; BK: B(n, k) k-contiguous.  grid (n tiles, m tiles, k splits).
// TM x TM tile, waves 2 x 2 of (TM/2)^2, each F x F MFMA tiles of 32x32 (F = TM / 64).
template <int TM, bool AK, bool BKc>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(long M, long N, long K, long kchunk, const float* __restrict__ A,
                                                      long lda, const float* __restrict__ B, long ldb,
                                                      const float* __restrict__ bias, const float* __restrict__ resid,
                                                      float* __restrict__ C, long slab, float* __restrict__ asum) {
    constexpr int F = TM / 64, WT = TM / 2, NV = TM * BK / 1024;
    // asum (layout 2: the bias gradient): sum over this split's k of A(m, k), by the n-tile-0 blocks
    const bool do_sum = asum != nullptr && blockIdx.x == 0;
    float colacc = 0.f;
    __shared__ __attribute__((aligned(16))) float As[2][BK][TM + PAD];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK][TM + PAD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.y * TM, n0 = (long)blockIdx.x * TM;
    const long kb = (long)blockIdx.z * kchunk, ke = min(K, kb + kchunk);
    const int wm = (wave >> 1) * WT, wn = (wave & 1) * WT;
    f32x16 acc[F][F] = {};
    f32x4 va[NV], vb[NV];
    load_tile<TM, AK>(A, lda, m0, M, kb, ke, tid, va);
    load_tile<TM, BKc>(B, ldb, n0, N, kb, ke, tid, vb);
    store_tile<TM, AK>(As[0], tid, va);
    store_tile<TM, BKc>(Bs[0], tid, vb);
    __syncthreads();
    int cur = 0;
    for (long k0 = kb; k0 < ke; k0 += BK) {
        const bool more = k0 + BK < ke;
        if (more) {   // next K tile in flight during this tile's MFMAs
            load_tile<TM, AK>(A, lda, m0, M, k0 + BK, ke, tid, va);
            load_tile<TM, BKc>(B, ldb, n0, N, k0 + BK, ke, tid, vb);
        }
        if (do_sum && tid < TM) {
#pragma unroll
            for (int k = 0; k < BK; ++k) colacc += As[cur][k][tid];
        }
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            float a[F], b[F];
#pragma unroll
            for (int t = 0; t < F; ++t) {
                a[t] = As[cur][kk + h][wm + 32 * t + r];
                b[t] = Bs[cur][kk + h][wn + 32 * t + r];
            }
#pragma unroll
            for (int ti = 0; ti < F; ++ti)
#pragma unroll
                for (int tj = 0; tj < F; ++tj)
                    acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
        }
        if (more) {
            store_tile<TM, AK>(As[cur ^ 1], tid, va);
            store_tile<TM, BKc>(Bs[cur ^ 1], tid, vb);
        }
        __syncthreads();
        cur ^= 1;
    }
    if (do_sum && tid < TM && m0 + tid < M) asum[(long)blockIdx.z * M + m0 + tid] = colacc;
    // epilogue: lane holds column n = n0 + wn + 32 tj + r, rows 8 (v / 4) + 4 h + v % 4 of each tile
    float* Cz = C + (long)blockIdx.z * slab;
#pragma unroll
    for (int tj = 0; tj < F; ++tj) {
        const long n = n0 + wn + 32 * tj + r;
        if (n >= N) continue;
        const float bn = bias ? bias[n] : 0.f;
#pragma unroll
        for (int ti = 0; ti < F; ++ti)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const long m = m0 + wm + 32 * ti + 8 * (v >> 2) + 4 * h + (v & 3);
                if (m < M) {
                    float o = acc[ti][tj][v] + bn;
                    if (resid) o += resid[m * N + n];
                    Cz[m * N + n] = o;
                }
            }
    }
}

// out[e] = sum_z slab[z][e] in z order (+ bias[e % N], + resid[e]); the blocks past the slab's also
// sum the splits' A column sums (layout-2 bias gradient, asum[m] = sum_z apart[z][m], split order) --
// one launch instead of two (the fp32 path's per-Linear weight gradients: 105 launches of ~4 us each)
__global__ __launch_bounds__(NT) void slab_sum(long n4, int N, int splits, long slab, const float* __restrict__ part,
                                               const float* __restrict__ bias, const float* __restrict__ resid,
                                               float* __restrict__ out, long M, const float* __restrict__ apart,
                                               float* __restrict__ aout) {
    const long nb1 = (n4 + NT - 1) / NT;
    if ((long)blockIdx.x >= nb1) {
        const long m = ((long)blockIdx.x - nb1) * NT + threadIdx.x;
        if (m >= M) return;
        float s = apart[m];
        for (int z = 1; z < splits; ++z) s += apart[(long)z * M + m];
        aout[m] = s;
        return;
    }
    const long e = ((long)blockIdx.x * NT + threadIdx.x) * 4;
    if (e >= n4 * 4) return;
    f32x4 s = *reinterpret_cast<const f32x4*>(part + e);
    for (int z = 1; z < splits; ++z) s += *reinterpret_cast<const f32x4*>(part + (long)z * slab + e);
    if (bias) s += *reinterpret_cast<const f32x4*>(bias + e % N);
    if (resid) s += *reinterpret_cast<const f32x4*>(resid + e);
    *reinterpret_cast<f32x4*>(out + e) = s;
}

int num_cus_f32() {
    static int v = 0;
    if (!v) {
        int dev = 0, n = 0;
        v = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) ? n : 256;
    }
    return v;
}

struct PlanF32 {
    int tm;
    long splits, kchunk;
};

// 128-tiles when they give >= 2 workgroups per CU, else 64-tiles; K split so that a launch has
// about two workgroups per CU, each split >= 256 (layouts 0/1) or >= 512 (layout 2, tokens) deep
PlanF32 plan_f32(int layout, long M, long N, long K) {
    PlanF32 p;
    const long cus = num_cus_f32();
    const long t128 = ((M + 127) / 128) * ((N + 127) / 128);
    p.tm = t128 >= F32_T128 * cus ? 128 : 64;
    const long tiles = ((M + p.tm - 1) / p.tm) * ((N + p.tm - 1) / p.tm);
    long s = (2 * cus + tiles - 1) / tiles;
    const long mink = layout == 2 ? F32_MINK2 : 256;
    const long maxs = (K + mink - 1) / mink;
    if (s > maxs) s = maxs;
    if (s < 1) s = 1;
    p.kchunk = ((K + s - 1) / s + BK - 1) / BK * BK;
    p.splits = (K + p.kchunk - 1) / p.kchunk;
    return p;
}

template <int TM>
void launch_f32(int layout, dim3 g, long M, long N, long K, long kchunk, const float* A, long lda, const float* B, long ldb,
                const float* bias, const float* resid, float* C, long slab, float* asum, hipStream_t st) {
    if (layout == 0)
        gemm_f32_kernel<TM, true, true><<<g, NT, 0, st>>>(M, N, K, kchunk, A, lda, B, ldb, bias, resid, C, slab, nullptr);
    else if (layout == 1)
        gemm_f32_kernel<TM, true, false><<<g, NT, 0, st>>>(M, N, K, kchunk, A, lda, B, ldb, bias, resid, C, slab, nullptr);
    else
        gemm_f32_kernel<TM, false, false><<<g, NT, 0, st>>>(M, N, K, kchunk, A, lda, B, ldb, bias, resid, C, slab, asum);
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" size_t csu_gemm_f32_workspace(int layout, long M, int N, long K) {
    if (layout < 0 || layout > 2 || M < 1 || N < 1 || K < 1) return 0;
    const PlanF32 p = plan_f32(layout, M, N, K);
    return p.splits > 1 ? (size_t)p.splits * (M * N + M) * sizeof(float) : 0;
}

extern "C" int csu_gemm_f32(int layout, long M, int N, long K, const float* A, const float* B, const float* bias,
                            const float* resid, float* C, float* asum, void* workspace, size_t ws_bytes, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !A || !B || !C || layout < 0 || layout > 2)
        return fail(CSU_E_ARG, "gemm_f32: bad arguments");
    // vector loads along the contiguous dimension of each operand
    const long lda = layout == 2 ? M : K, ldb = layout == 0 ? K : N;
    if (lda % 4 || ldb % 4 || N % 4) return fail(CSU_E_ARG, "gemm_f32: row lengths must be multiples of 4");
    if (layout != 0 && (bias || resid)) return fail(CSU_E_ARG, "gemm_f32: bias / residual only in layout 0");
    if (layout != 2 && asum) return fail(CSU_E_ARG, "gemm_f32: column sums only in layout 2");
    hipStream_t st = as_stream(stream);
    const PlanF32 p = plan_f32(layout, M, N, K);
    const dim3 g((unsigned)((N + p.tm - 1) / p.tm), (unsigned)((M + p.tm - 1) / p.tm), (unsigned)p.splits);
    const bool split = p.splits > 1;
    if (split && (!workspace || ws_bytes < csu_gemm_f32_workspace(layout, M, N, K)))
        return fail(CSU_E_WORKSPACE, "gemm_f32: workspace");
    float* dst = split ? (float*)workspace : C;
    float* sdst = split && asum ? (float*)workspace + p.splits * M * N : asum;
    const float* kb = split ? nullptr : bias;
    const float* kr = split ? nullptr : resid;
    if (p.tm == 128) launch_f32<128>(layout, g, M, N, K, p.kchunk, A, lda, B, ldb, kb, kr, dst, M * N, sdst, st);
    else launch_f32<64>(layout, g, M, N, K, p.kchunk, A, lda, B, ldb, kb, kr, dst, M * N, sdst, st);
    if (int e = check_launch("gemm_f32")) return e;
    if (split) {
        const long n4 = M * N / 4;
        const long nb = (n4 + NT - 1) / NT + (asum ? (M + NT - 1) / NT : 0);
        slab_sum<<<(unsigned)nb, NT, 0, st>>>(n4, N, (int)p.splits, M * N, (const float*)workspace, bias, resid, C,
                                              asum ? M : 0, sdst, asum);
        return check_launch("gemm_f32 slab sum");
    }
    return 0;
}
