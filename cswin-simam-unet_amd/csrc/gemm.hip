// Token GEMM with fused prologue/epilogue for gfx950 (bf16 operands, fp32 accumulation).
//
//   out[m][n] = epi( sum_k pro(A[m][k]) * B(n, k) )
//   B(n, k) = b[n][k] (b_trans = 0, nn.Linear weight (N, K): forward)  or  b[k][n] (b_trans = 1,
//   the same weight read as (K, N): input gradient dX = dY W).
//   pro  = identity | exact GELU (fc2 consumes gelu(h) straight from fc1's pre-activation h)
//   epi  = + bias[n]  ->  * gelu'(aux[m][n]) (GELU backward)  ->  + resid[m][n] (residual add)
// Replaces, on the bf16 path, the nn.Linear GEMMs of CSWinBlock/Mlp (cswin:185-195, 314-368) and the
// separate GELU / GELU-backward / residual-add passes around them.  M = tokens (up to 4M), N, K <= 2048:
// memory-bound tiles, 128 x BN per workgroup, 4 waves in 2x2, v_mfma_f32_32x32x16_bf16; the next
// 32-deep K slice is prefetched into registers while the current one is multiplied from LDS.
// A and row-major B slices live in 64-B-row LDS images with 16-B chunks XOR-swizzled by row>>2
// (conflict-free 16-B fragment reads); a (K, N) B slice is read with ds_read_b64_tr_b16.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int BM = 128;
constexpr int BK = 32;

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int swz64(int row, int col) {   // [row][32] bf16 image, swizzled chunks
    return row * BK + ((((col >> 3) ^ (row >> 2)) & 3) << 3) + (col & 7);
}

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
    return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

template <int BN, bool BT>
struct Smem {
    static constexpr int BROW = BN + (BN == 128 ? 32 : 32);   // (K, N) image row stride (elements)
    static constexpr int A_EL = BM * BK;
    static constexpr int B_EL = BT ? BK * BROW : BN * BK;
};

template <int BN, bool BT, bool GELU_A, typename TOUT>
__global__ __launch_bounds__(NT) void gemm_kernel(long M, int N, int K, const bf16* __restrict__ A, int lda,
                                                  const bf16* __restrict__ Bm, int ldb, const float* __restrict__ bias,
                                                  const bf16* __restrict__ gaux, const float* __restrict__ resid,
                                                  TOUT* __restrict__ out, int ldc) {
    using S = Smem<BN, BT>;
    constexpr int WN = BN / 2;           // columns per wave
    constexpr int TN = WN / 32;          // 32-wide MFMA tiles per wave along n (1 or 2)
    constexpr int TMW = 2;               // 32-row tiles per wave along m (64 rows)
    __shared__ __attribute__((aligned(16))) bf16 As[S::A_EL];
    __shared__ __attribute__((aligned(16))) bf16 Bs[S::B_EL];
    const long m0 = (long)blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * WN;

    // ---- global -> register staging of one K slice ----
    // A: 128 rows x 4 chunks = 512 chunks, 2 per thread; chunk c -> row c >> 2, chunk c & 3
    bf16x8 ra[2], rbv[BN * BK / 8 / NT > 0 ? BN * BK / 8 / NT : 1];
    constexpr int BCH = BN * BK / 8 / NT;   // B chunks per thread (1 or 2)
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = threadIdx.x + NT * i, row = c >> 2, ch = c & 3;
            const long m = m0 + row;
            const int k = k0 + ch * 8;
            ra[i] = (m < M && k < K) ? *reinterpret_cast<const bf16x8*>(A + m * lda + k) : bf16x8{};
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int c = threadIdx.x + NT * i;
            if constexpr (!BT) {            // b[n][k]: BN rows x 4 chunks
                const int row = c >> 2, ch = c & 3;
                const int n = n0 + row, k = k0 + ch * 8;
                rbv[i] = (n < N && k < K) ? *reinterpret_cast<const bf16x8*>(Bm + (long)n * ldb + k) : bf16x8{};
            } else {                        // b[k][n]: 32 rows x BN/8 chunks
                constexpr int CPR = BN / 8;
                const int row = c / CPR, ch = c % CPR;
                const int k = k0 + row, n = n0 + ch * 8;
                rbv[i] = (k < K && n < N) ? *reinterpret_cast<const bf16x8*>(Bm + (long)k * ldb + n) : bf16x8{};
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = threadIdx.x + NT * i, row = c >> 2, ch = c & 3;
            bf16x8 v = ra[i];
            if constexpr (GELU_A) {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (bf16)gelu_f((float)v[j]);
            }
            *reinterpret_cast<bf16x8*>(As + swz64(row, ch * 8)) = v;
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int c = threadIdx.x + NT * i;
            if constexpr (!BT) {
                const int row = c >> 2, ch = c & 3;
                *reinterpret_cast<bf16x8*>(Bs + swz64(row, ch * 8)) = rbv[i];
            } else {
                constexpr int CPR = BN / 8;
                const int row = c / CPR, ch = c % CPR;
                *reinterpret_cast<bf16x8*>(Bs + row * S::BROW + ch * 8) = rbv[i];
            }
        }
    };

    f32x16 acc[TMW][TN];
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

    load(0);
    for (int k0 = 0; k0 < K; k0 += BK) {
        __syncthreads();
        store();
        __syncthreads();
        if (k0 + BK < K) load(k0 + BK);
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            bf16x8 af[TMW], bfg[TN];
#pragma unroll
            for (int i = 0; i < TMW; ++i)
                af[i] = *reinterpret_cast<const bf16x8*>(As + swz64(wm + 32 * i + r, 16 * s + 8 * h));
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (!BT) {
                    bfg[j] = *reinterpret_cast<const bf16x8*>(Bs + swz64(wn + 32 * j + r, 16 * s + 8 * h));
                } else {   // transposing read of rows k = 16s + 8h + {0..3}, {4..7}, column n = lane's r
                    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
                    const int col = wn + 32 * j + 16 * (grp & 1) + 4 * p;
                    const int row = 16 * s + 8 * (grp >> 1) + q;
                    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) v4s*)(Bs + row * S::BROW + col));
                    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (__attribute__((address_space(3))) v4s*)(Bs + (row + 4) * S::BROW + col));
                    const v4s v[2] = {lo, hi};
                    __builtin_memcpy(&bfg[j], v, 16);
                }
            }
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
        }
    }
    // ---- epilogue: acc[i][j][reg] = out[m0 + wm + 32 i + crow(reg, h)][n0 + wn + 32 j + r] ----
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn + 32 * j + r;
        if (n >= N) continue;
        const float bv = bias ? bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const long m = m0 + wm + 32 * i + crow(reg, h);
                if (m >= M) continue;
                float v = acc[i][j][reg] + bv;
                if (gaux) v *= gelu_grad((float)gaux[m * ldc + n]);
                if (resid) v += resid[m * ldc + n];
                out[m * ldc + n] = from_f<TOUT>(v);
            }
    }
}

template <int BN, bool BT, bool GA>
int launch_t(long M, int N, int K, const bf16* A, int lda, const bf16* B, int ldb, const float* bias, const bf16* gaux,
             const float* resid, void* out, int ldc, int odt, hipStream_t st) {
    const dim3 grid((unsigned)((M + BM - 1) / BM), (N + BN - 1) / BN);
    if (odt == CSU_BF16)
        gemm_kernel<BN, BT, GA, bf16><<<grid, NT, 0, st>>>(M, N, K, A, lda, B, ldb, bias, gaux, resid, (bf16*)out, ldc);
    else
        gemm_kernel<BN, BT, GA, float><<<grid, NT, 0, st>>>(M, N, K, A, lda, B, ldb, bias, gaux, resid, (float*)out, ldc);
    return check_launch("gemm");
}

// ---- v3: b[n][k] operand only, 64-deep K slices, double-buffered LDS (one barrier per slice),
// tile BM x BN in {64, 128}^2 chosen per shape for >= 2 workgroups per CU, LDS-staged epilogue
// writing 16-B row vectors (bias / GELU' / residual applied there with vector loads).
__device__ __forceinline__ int swz128g(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }

// erf(|x|/sqrt2) by Abramowitz-Stegun 7.1.26 (|abs err| < 1.5e-7): one rcp, one exp, 6 FMAs.
__device__ __forceinline__ float erf_as(float z) {   // z >= 0
    const float t = __frcp_rn(1.f + 0.3275911f * z);
    const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
    return 1.f - p * __expf(-z * z);
}
__device__ __forceinline__ float gelu_fast(float x) {
    const float e = erf_as(fabsf(x) * 0.70710678118654752f);
    return 0.5f * x * (1.f + (x >= 0.f ? e : -e));
}
__device__ __forceinline__ float gelu_grad_fast(float x) {
    const float e = erf_as(fabsf(x) * 0.70710678118654752f);
    return 0.5f * (1.f + (x >= 0.f ? e : -e)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

// STG = LDS stages (1 when K <= 64: a single slice, no prefetch).  The epilogue runs in two
// row halves so its fp32 staging tile fits in the (smaller) stage buffers: with one stage a
// 128 x 128 tile needs 34 KB of LDS and four workgroups share a CU.
template <int BM, int BN, int STG, bool GELU_A, typename TOUT>
__global__ __launch_bounds__(NT) void gemm3_kernel(long M, int N, int K, const bf16* __restrict__ A, int lda,
                                                   const bf16* __restrict__ Bm, int ldb, const float* __restrict__ bias,
                                                   const bf16* __restrict__ gaux, const float* __restrict__ resid,
                                                   TOUT* __restrict__ out, bf16* __restrict__ gout, int ldc) {
    constexpr int BK3 = 64;
    constexpr int TMW = BM / 64, TN = BN / 64;     // 32x32 MFMA tiles per wave (waves 2 x 2)
    constexpr int CA = BM / 32, CB = BN / 32;      // 16-B staging chunks per thread
    constexpr int STAGE = STG * (BM + BN) * BK3;   // bf16 elements
    constexpr int HB = BM / 2;                     // epilogue rows per half
    constexpr int CS = BN + 4;                     // fp32 row stride of the epilogue tile
    constexpr int EPI = HB * CS * 2;               // in bf16 units
    constexpr int LDS = STAGE > EPI ? STAGE : EPI;
    __shared__ __attribute__((aligned(16))) bf16 smem[LDS];
    bf16* As = smem;                       // [STG][BM * 64]
    bf16* Bs = smem + STG * BM * BK3;      // [STG][BN * 64]
    const int nbn = (N + BN - 1) / BN;     // n fastest: the N tiles of one A panel share an XCD's L2
    const long t = xcd_tile(blockIdx.x, gridDim.x);
    const long m0 = (t / nbn) * BM;
    const int n0 = (int)(t % nbn) * BN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = (wave >> 1) * HB, wn = (wave & 1) * (BN / 2);
    const int ch = threadIdx.x & 7, rb = threadIdx.x >> 3;
    bf16x8 ra[CA], rbv[CB];
    auto load = [&](int k0) {
        const int k = k0 + 8 * ch;
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const long m = m0 + rb + 32 * i;
            ra[i] = (m < M && k < K) ? *reinterpret_cast<const bf16x8*>(A + m * lda + k) : bf16x8{};
        }
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int n = n0 + rb + 32 * j;
            rbv[j] = (n < N && k < K) ? *reinterpret_cast<const bf16x8*>(Bm + (long)n * ldb + k) : bf16x8{};
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            bf16x8 v = ra[i];
            if constexpr (GELU_A) {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (bf16)gelu_fast((float)v[j]);
            }
            *reinterpret_cast<bf16x8*>(As + buf * BM * BK3 + swz128g(rb + 32 * i, ch)) = v;
        }
#pragma unroll
        for (int j = 0; j < CB; ++j)
            *reinterpret_cast<bf16x8*>(Bs + buf * BN * BK3 + swz128g(rb + 32 * j, ch)) = rbv[j];
    };
    f32x16 acc[TMW][TN];
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
    load(0);
    store(0);
    __syncthreads();
    int buf = 0;
    for (int k0 = 0; k0 < K; k0 += BK3) {
        const bool more = STG > 1 && k0 + BK3 < K;
        if (more) load(k0 + BK3);
        const bf16* Ab = As + buf * BM * BK3;
        const bf16* Bb = Bs + buf * BN * BK3;
#pragma unroll
        for (int s = 0; s < BK3 / 16; ++s) {
            bf16x8 af[TMW], bfg[TN];
#pragma unroll
            for (int i = 0; i < TMW; ++i) af[i] = *reinterpret_cast<const bf16x8*>(Ab + swz128g(wm + 32 * i + r, 2 * s + h));
#pragma unroll
            for (int j = 0; j < TN; ++j) bfg[j] = *reinterpret_cast<const bf16x8*>(Bb + swz128g(wn + 32 * j + r, 2 * s + h));
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
        }
        if (more) store(buf ^ 1);
        __syncthreads();
        if constexpr (STG > 1) buf ^= 1;
    }
    // ---- epilogue, per row half: prefetch bias/aux/resid vectors -> accumulators to the fp32 LDS
    // tile [HB][BN + 4] -> 8-column row vectors with the fused ops, 16-B stores ----
    float* Ct = reinterpret_cast<float*>(smem);
    constexpr int VPR = BN / 8;                    // 8-column vectors per row
    constexpr int EV = HB * VPR / NT;              // vectors per thread per half (>= 1)
    static_assert(EV >= 1 && HB * VPR % NT == 0, "epilogue split");
    const int c8 = (threadIdx.x % VPR) * 8;
    const int n = n0 + c8;
    float bv[8];
    if (bias && n < N) load8(bias + n, bv);
    else
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        float pre[EV][8];
#pragma unroll
        for (int v = 0; v < EV; ++v) {
            const int row = (threadIdx.x + v * NT) / VPR;
            const long m = m0 + half * HB + row;
            const bool ok = m < M && n < N;
#pragma unroll
            for (int e = 0; e < 8; ++e) pre[v][e] = 0.f;
            if (gaux && ok) load8(gaux + m * ldc + n, pre[v]);
            else if (resid && ok) load8(resid + m * ldc + n, pre[v]);
        }
        if ((wave >> 1) == half) {
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg)
                        Ct[(32 * i + crow(reg, h)) * CS + wn + 32 * j + r] = acc[i][j][reg];
        }
        __syncthreads();
#pragma unroll
        for (int v = 0; v < EV; ++v) {
            const int row = (threadIdx.x + v * NT) / VPR;
            const long m = m0 + half * HB + row;
            if (m >= M || n >= N) continue;
            float o[8];
            const f32x4 lo = *reinterpret_cast<const f32x4*>(Ct + row * CS + c8);
            const f32x4 hi = *reinterpret_cast<const f32x4*>(Ct + row * CS + c8 + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[e] = lo[e] + bv[e];
                o[e + 4] = hi[e] + bv[e + 4];
            }
            if (gaux) {
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] *= gelu_grad_fast(pre[v][e]);
            } else if (resid) {
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] += pre[v][e];
            }
            store8(out + m * ldc + n, o);
            if (gout) {
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = gelu_fast(o[e]);
                store8(gout + m * ldc + n, o);
            }
        }
        __syncthreads();
    }
}

template <int BM, int BN, int STG, bool GA>
int launch3_s(long M, int N, int K, const bf16* A, int lda, const bf16* B, int ldb, const float* bias, const bf16* gaux,
              const float* resid, void* out, bf16* gout, int ldc, int odt, hipStream_t st) {
    const dim3 grid((unsigned)(((M + BM - 1) / BM) * ((N + BN - 1) / BN)));
    if (odt == CSU_BF16)
        gemm3_kernel<BM, BN, STG, GA, bf16><<<grid, NT, 0, st>>>(M, N, K, A, lda, B, ldb, bias, gaux, resid, (bf16*)out, gout, ldc);
    else
        gemm3_kernel<BM, BN, STG, GA, float><<<grid, NT, 0, st>>>(M, N, K, A, lda, B, ldb, bias, gaux, resid, (float*)out, gout, ldc);
    return check_launch("gemm3");
}

template <int BM, int BN, bool GA>
int launch3_t(long M, int N, int K, const bf16* A, int lda, const bf16* B, int ldb, const float* bias, const bf16* gaux,
              const float* resid, void* out, bf16* gout, int ldc, int odt, hipStream_t st) {
    if (K <= 64) return launch3_s<BM, BN, 1, GA>(M, N, K, A, lda, B, ldb, bias, gaux, resid, out, gout, ldc, odt, st);
    return launch3_s<BM, BN, 2, GA>(M, N, K, A, lda, B, ldb, bias, gaux, resid, out, gout, ldc, odt, st);
}

// tile choice (measured on the CSWin-UNet token shapes, tools/gemm_probe3.py): 128 x 64 for a
// plain / bias epilogue; 64 x 64 when the epilogue streams a second tensor (GELU' aux, residual,
// h + gelu(h)) -- more workgroups per CU overlap those epilogue loads/stores with other tiles'
// main loops; 64 x 64 as well when 128 x 64 would leave fewer than one workgroup per CU.
int pick_cfg(long M, int N, bool heavy_epilogue) {
    const long wgs2 = ((M + 127) / 128) * (long)((N + 63) / 64);
    if (heavy_epilogue || wgs2 < 256) return 0;
    return 2;
}

int launch3(int cfg, long M, int N, int K, const bf16* A, int lda, const bf16* B, int ldb, const float* bias,
            const bf16* g, const float* resid, void* out, bf16* gout, int ldc, int odt, bool ga, hipStream_t st) {
#define CSU_G3(BM_, BN_)                                                                                       \
    return ga ? launch3_t<BM_, BN_, true>(M, N, K, A, lda, B, ldb, bias, g, resid, out, gout, ldc, odt, st)   \
              : launch3_t<BM_, BN_, false>(M, N, K, A, lda, B, ldb, bias, g, resid, out, gout, ldc, odt, st)
    switch (cfg) {
        case 3: CSU_G3(128, 128);
        case 2: CSU_G3(128, 64);
        case 1: CSU_G3(64, 128);
        default: CSU_G3(64, 64);
    }
#undef CSU_G3
}

}  // namespace

int gemm4_run(int cfg, int epi, int odt, long M, int N, int K, const bf16* A, int lda, const bf16* W, int ldw,
              const float* bias, const bf16* gaux, const float* resid, void* out, bf16* gout, int ldc, hipStream_t st);
}  // namespace csu

using namespace csu;

extern "C" int csu_gemm_ex(const csu_gemm_desc* d, void* stream);

extern "C" int csu_gemm(long M, int N, int K, const void* a, int lda, const void* b, int ldb, int b_trans, int a_gelu,
                        const float* bias, const void* gelu_aux, const float* resid, void* out, int ldc, int out_dtype,
                        void* stream) {
    csu_gemm_desc d{};
    d.M = M; d.N = N; d.K = K; d.a = a; d.b = b; d.lda = lda; d.ldb = ldb; d.b_trans = b_trans; d.a_gelu = a_gelu;
    d.bias = bias; d.gelu_aux = gelu_aux; d.resid = resid; d.out = out; d.gelu_out = nullptr; d.ldc = ldc;
    d.out_dtype = out_dtype; d.cfg = -1;
    return csu_gemm_ex(&d, stream);
}

extern "C" int csu_gemm_ex(const csu_gemm_desc* d, void* stream) {
    if (!d) return fail(CSU_E_ARG, "gemm: null descriptor");
    const long M = d->M;
    const int N = d->N, K = d->K, lda = d->lda, ldb = d->ldb, ldc = d->ldc, out_dtype = d->out_dtype;
    const int b_trans = d->b_trans, a_gelu = d->a_gelu;
    const float* bias = d->bias;
    const float* resid = d->resid;
    void* out = d->out;
    int cfg = d->cfg;
    if (M < 1 || N < 1 || K < 1 || !d->a || !d->b || !out) return fail(CSU_E_ARG, "gemm: bad args");
    if (K % 8 || lda % 8 || ldb % 8 || (b_trans && N % 8)) return fail(CSU_E_ARG, "gemm: K, lda, ldb (and N when b_trans) must be multiples of 8");
    if (out_dtype != CSU_BF16 && out_dtype != CSU_F32) return fail(CSU_E_ARG, "gemm: bad out dtype");
    if (resid && out_dtype != CSU_F32) return fail(CSU_E_ARG, "gemm: residual epilogue needs an fp32 output");
    if (d->gelu_out && (out_dtype != CSU_BF16 || d->gelu_aux || resid || b_trans || N % 8 || ldc % 8))
        return fail(CSU_E_ARG, "gemm: gelu_out needs a bf16 output, b_trans = 0, no gelu_aux/resid, N and ldc % 8 == 0");
    hipStream_t st = as_stream(stream);
    const bf16* A = (const bf16*)d->a;
    const bf16* B = (const bf16*)d->b;
    const bf16* g = (const bf16*)d->gelu_aux;
    // gemm4 (LDS-DMA staging, register epilogue): weight (N, K) operand, K % 64 == 0, no GELU prologue.
    // cfg -1 = auto, 10..15 force a gemm4 configuration, 0..3 force a gemm3 tile.
    const bool g4_ok = !b_trans && !a_gelu && K % 64 == 0 && N % 8 == 0 && M * (long)lda < (1L << 30) && (long)N * ldb < (1L << 30) && ldc % 8 == 0 &&
                       !(d->gelu_out && out_dtype != CSU_BF16) && !(d->gelu_aux && d->gelu_out) &&
                       !(resid && (d->gelu_aux || d->gelu_out));
    if (g4_ok && (cfg < 0 || cfg >= 10)) {
        const int epi = d->gelu_out ? 1 : d->gelu_aux ? 2 : resid ? 3 : 0;
        return gemm4_run(cfg < 0 ? -1 : cfg - 10, epi, out_dtype, M, N, K, A, lda, B, ldb, bias, g, resid, out,
                         (bf16*)d->gelu_out, ldc, st);
    }
    if (cfg >= 10) cfg = -1;
    if (!b_trans && N % 8 == 0 && ldc % 8 == 0) {
        if (cfg < 0 || cfg > 3) cfg = pick_cfg(M, N, d->gelu_out || d->gelu_aux || resid);
        return launch3(cfg, M, N, K, A, lda, B, ldb, bias, g, resid, out, (bf16*)d->gelu_out, ldc, out_dtype,
                       a_gelu != 0, st);
    }
    const bool wide = N > 64;
#define CSU_GEMM_CASE(BN, BT, GA) return launch_t<BN, BT, GA>(M, N, K, A, lda, B, ldb, bias, g, resid, out, ldc, out_dtype, st)
    if (wide) {
        if (b_trans) { if (a_gelu) CSU_GEMM_CASE(128, true, true); CSU_GEMM_CASE(128, true, false); }
        if (a_gelu) CSU_GEMM_CASE(128, false, true);
        CSU_GEMM_CASE(128, false, false);
    }
    if (b_trans) { if (a_gelu) CSU_GEMM_CASE(64, true, true); CSU_GEMM_CASE(64, true, false); }
    if (a_gelu) CSU_GEMM_CASE(64, false, true);
    CSU_GEMM_CASE(64, false, false);
#undef CSU_GEMM_CASE
}
