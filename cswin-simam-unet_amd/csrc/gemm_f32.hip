// fp32 GEMMs for the fp32 (non-autocast) training path on gfx950 MFMA (v_mfma_f32_32x32x2_f32):
// the token Linear forward, its input gradient and its weight gradient (nn.Linear cswin:185/187/
// 314/323/568/581/592 in fp32, BASELINE config 2), replacing the platform BLAS on that path.
//
//   layout 0 (NT): C[m][n] = sum_k A[m][k] B[n][k]   (+ bias[n], + resid[m][n])   forward  y = x W^T + b
//   layout 1 (NN): C[m][n] = sum_k A[m][k] B[k][n]                                input gradient dx = dy W
//   layout 2 (TN): C[m][n] = sum_k A[k][m] B[k][n]                                weight gradient dW = dy^T x
//
// 128x128 output tiles, 4 waves of 64x64 (2x2 MFMA tiles of 32x32), K staged 16 at a time through
// a double-buffered LDS image stored k-major ([k][m] and [k][n]): the MFMA operand of lane (r, h)
// is one float at [k0 + h][r], conflict-free ds_read_b32.  Global loads are 16-B vectors along
// whichever dimension is contiguous (k for A in layouts 0/1 and B in layout 0, m / n otherwise),
// one K tile ahead in registers.  The fp32 MFMA peak is 157 TFLOP/s; at AI = 2MNK / 4(MK+NK+MN)
// bytes every shape of the model is MFMA-bound.
//
// Layout 2 contracts over the token dimension (10^4..10^5): split over tokens into fixed chunks,
// each writing its own fp32 slab, then one reduction sums the slabs in chunk order (deterministic,
// no atomics).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int BM = 128, BN = 128, BK = 16, PAD = 4;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 128 x 16 tile of operand X into regs: element (i, k) of X at X[i * ld + k] (KC) or X[k * ld + i]
template <bool KC>
__device__ __forceinline__ void load_tile(const float* X, long ld, long i0, long ni, long k0, long k1, int tid, f32x4* v) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = tid + u * NT;
        long i, k;
        if constexpr (KC) { i = i0 + (f >> 2); k = k0 + 4 * (f & 3); }
        else { k = k0 + (f >> 5); i = i0 + 4 * (f & 31); }
        const bool ok = i < ni && k < k1;   // the contiguous dimension is a multiple of 4
        v[u] = ok ? *reinterpret_cast<const f32x4*>(X + (KC ? i * ld + k : k * ld + i)) : f32x4{};
    }
}

template <bool KC, int W>
__device__ __forceinline__ void store_tile(float (*S)[W], int tid, const f32x4* v) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = tid + u * NT;
        if constexpr (KC) {
            const int i = f >> 2, k = 4 * (f & 3);
#pragma unroll
            for (int e = 0; e < 4; ++e) S[k + e][i] = v[u][e];
        } else {
            const int k = f >> 5, i = 4 * (f & 31);
            *reinterpret_cast<f32x4*>(&S[k][i]) = v[u];
        }
    }
}

// AK: A(m, k) k-contiguous; BK: B(n, k) k-contiguous.  grid (n tiles, m tiles, k splits)
template <bool AK, bool BKc>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(long M, long N, long K, long kchunk, const float* __restrict__ A,
                                                      long lda, const float* __restrict__ B, long ldb,
                                                      const float* __restrict__ bias, const float* __restrict__ resid,
                                                      float* __restrict__ C, long slab) {
    __shared__ __attribute__((aligned(16))) float As[2][BK][BM + PAD];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + PAD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const long m0 = (long)blockIdx.y * BM, n0 = (long)blockIdx.x * BN;
    const long kb = (long)blockIdx.z * kchunk, ke = min(K, kb + kchunk);
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    f32x16 acc[2][2] = {};
    f32x4 va[2], vb[2];
    load_tile<AK>(A, lda, m0, M, kb, ke, tid, va);
    load_tile<BKc>(B, ldb, n0, N, kb, ke, tid, vb);
    store_tile<AK>(As[0], tid, va);
    store_tile<BKc>(Bs[0], tid, vb);
    __syncthreads();
    int cur = 0;
    for (long k0 = kb; k0 < ke; k0 += BK) {
        const bool more = k0 + BK < ke;
        if (more) {   // next K tile in flight during this tile's MFMAs
            load_tile<AK>(A, lda, m0, M, k0 + BK, ke, tid, va);
            load_tile<BKc>(B, ldb, n0, N, k0 + BK, ke, tid, vb);
        }
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const float a0 = As[cur][kk + h][wm + r], a1 = As[cur][kk + h][wm + 32 + r];
            const float b0 = Bs[cur][kk + h][wn + r], b1 = Bs[cur][kk + h][wn + 32 + r];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (more) {
            store_tile<AK>(As[cur ^ 1], tid, va);
            store_tile<BKc>(Bs[cur ^ 1], tid, vb);
        }
        __syncthreads();
        cur ^= 1;
    }
    // epilogue: lane holds column n = n0 + wn + 32 tj + r, rows 8 (v / 4) + 4 h + v % 4 of each tile
    float* Cz = C + (long)blockIdx.z * slab;
#pragma unroll
    for (int tj = 0; tj < 2; ++tj) {
        const long n = n0 + wn + 32 * tj + r;
        if (n >= N) continue;
        const float bn = bias ? bias[n] : 0.f;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
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

// out[e] = sum_z slab[z][e] in z order (+ bias broadcast over rows of width N when given)
__global__ __launch_bounds__(NT) void slab_sum(long n4, int splits, long slab, const float* __restrict__ part,
                                               float* __restrict__ out) {
    const long e = ((long)blockIdx.x * NT + threadIdx.x) * 4;
    if (e >= n4 * 4) return;
    f32x4 s = *reinterpret_cast<const f32x4*>(part + e);
    for (int z = 1; z < splits; ++z) s += *reinterpret_cast<const f32x4*>(part + (long)z * slab + e);
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

// token splits of a layout-2 product: about two workgroups per CU, >= 512 tokens per split
long splits_of(long M, long N, long K) {
    const long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    long s = (2 * num_cus_f32() + tiles - 1) / tiles;
    const long maxs = (K + 511) / 512;
    if (s > maxs) s = maxs;
    return s < 1 ? 1 : s;
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" size_t csu_gemm_f32_workspace(int layout, long M, int N, long K) {
    if (layout != 2 || M < 1 || N < 1 || K < 1) return 0;
    const long s = splits_of(M, N, K);
    return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

extern "C" int csu_gemm_f32(int layout, long M, int N, long K, const float* A, const float* B, const float* bias,
                            const float* resid, float* C, void* workspace, size_t ws_bytes, void* stream) {
    if (M < 1 || N < 1 || K < 1 || !A || !B || !C || layout < 0 || layout > 2)
        return fail(CSU_E_ARG, "gemm_f32: bad arguments");
    // vector loads along the contiguous dimension of each operand
    const long lda = layout == 2 ? M : K, ldb = layout == 0 ? K : N;
    if (lda % 4 || ldb % 4 || N % 4) return fail(CSU_E_ARG, "gemm_f32: row lengths must be multiples of 4");
    hipStream_t st = as_stream(stream);
    const dim3 g2((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM));
    if (layout == 0) {
        gemm_f32_kernel<true, true><<<g2, NT, 0, st>>>(M, N, K, K, A, lda, B, ldb, bias, resid, C, 0);
        return check_launch("gemm_f32 NT");
    }
    if (bias || resid) return fail(CSU_E_ARG, "gemm_f32: bias / residual only in layout 0");
    if (layout == 1) {
        gemm_f32_kernel<true, false><<<g2, NT, 0, st>>>(M, N, K, K, A, lda, B, ldb, nullptr, nullptr, C, 0);
        return check_launch("gemm_f32 NN");
    }
    const long s = splits_of(M, N, K);
    const long kchunk = ((K + s - 1) / s + BK - 1) / BK * BK;
    const long splits = (K + kchunk - 1) / kchunk;
    if (splits == 1) {
        gemm_f32_kernel<false, false><<<g2, NT, 0, st>>>(M, N, K, kchunk, A, lda, B, ldb, nullptr, nullptr, C, 0);
        return check_launch("gemm_f32 TN");
    }
    if (!workspace || ws_bytes < csu_gemm_f32_workspace(2, M, N, K)) return fail(CSU_E_WORKSPACE, "gemm_f32: workspace");
    float* part = (float*)workspace;
    const long slab = M * N;
    gemm_f32_kernel<false, false><<<dim3(g2.x, g2.y, (unsigned)splits), NT, 0, st>>>(M, N, K, kchunk, A, lda, B, ldb,
                                                                                        nullptr, nullptr, part, slab);
    if (int e = check_launch("gemm_f32 TN split")) return e;
    const long n4 = slab / 4;
    slab_sum<<<(unsigned)((n4 + NT - 1) / NT), NT, 0, st>>>(n4, (int)splits, slab, part, C);
    return check_launch("gemm_f32 slab sum");
}
