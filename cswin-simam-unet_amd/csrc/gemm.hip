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

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_gemm(long M, int N, int K, const void* a, int lda, const void* b, int ldb, int b_trans, int a_gelu,
                        const float* bias, const void* gelu_aux, const float* resid, void* out, int ldc, int out_dtype,
                        void* stream) {
    if (M < 1 || N < 1 || K < 1 || !a || !b || !out) return fail(CSU_E_ARG, "gemm: bad args");
    if (K % 8 || lda % 8 || ldb % 8 || (b_trans && N % 8)) return fail(CSU_E_ARG, "gemm: K, lda, ldb (and N when b_trans) must be multiples of 8");
    if (out_dtype != CSU_BF16 && out_dtype != CSU_F32) return fail(CSU_E_ARG, "gemm: bad out dtype");
    if (resid && out_dtype != CSU_F32) return fail(CSU_E_ARG, "gemm: residual epilogue needs an fp32 output");
    hipStream_t st = as_stream(stream);
    const bf16* A = (const bf16*)a;
    const bf16* B = (const bf16*)b;
    const bf16* g = (const bf16*)gelu_aux;
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
