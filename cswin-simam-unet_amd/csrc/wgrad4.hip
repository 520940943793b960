// wgrad4: Linear weight + bias gradient over token rows, bf16 in, fp32 out (gfx950).
//
//   dW[n][k] = sum_m dY[m][n] * X[m][k],   db[n] = sum_m dY[m][n]      (m = the B*L tokens)
//
// Backward of every token nn.Linear (qkv / proj / fc1 / fc2 cswin:185-195, 314-368, concat_linear
// cswin:568-592, the CARAFE 1x1 convs cswin:396-399).  The reduction runs over the token rows, so
// both operands are read row-major and transposed on the way into the MFMA:
//  * workgroup = (dW tile TN x TK, token chunk); 4 waves in 2 x 2, each (TN/2) x (TK/2);
//  * 64-token slices of dY[:, n0:n0+TN] and X[:, k0:k0+TK] go global -> LDS by buffer_load ... lds
//    (lane-linear 1 KB per wave instruction; rows past the chunk read as 0 by the hardware range
//    check) into an S-stage ring; the next slices stay in flight across the barrier (counted vmcnt);
//  * MFMA operands (8 consecutive tokens of one feature) are gathered with ds_read_b64_tr_b16 from
//    the row-major images, whose 16-B chunks are XOR-swizzled by row so the transposing reads of
//    4 rows hit 4 different bank quarters;
//  * db comes from one extra MFMA per step against a ones fragment (k-tile 0 workgroups only);
//  * each workgroup writes its partial tile into a [chunk][N*K + N] slab reduced in chunk order
//    by csu_colsum (deterministic: no float atomics).
#include <cstdlib>

#include "common.hpp"

namespace csu {
namespace {

constexpr int W4_NT = 256;
constexpr int W4_TM = 64;   // tokens per slice

typedef short v4s __attribute__((ext_vector_type(4)));

template <int T>   // swizzle of the 16-B chunk index of row `row` in a [64][T] bf16 image
__device__ __forceinline__ int w4_swz(int row) {
    return T == 128 ? (row & 3) << 2 : ((row >> 1) & 1) << 2;
}
template <int T>
__device__ __forceinline__ int w4_off(int row, int col) {   // element offset
    return row * T + ((((col >> 3) ^ w4_swz<T>(row))) << 3) + (col & 7);
}

template <int T>   // per-lane byte offsets (relative to the slice origin) of the DMA of a [64][T] slice
__device__ __forceinline__ void w4_voff(int ld, int wave, int lane, unsigned* voff) {
    constexpr int RPI = 1024 / (T * 2);          // rows per wave instruction
    constexpr int NI = W4_TM / RPI / 4;          // instructions per wave
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int row = (wave * NI + i) * RPI + lane / (T / 8);
        const int slot = lane % (T / 8);
        voff[i] = (unsigned)row * ld * 2 + ((slot ^ w4_swz<T>(row)) << 4);
    }
}
template <int T>
__device__ __forceinline__ void w4_dma(__amdgpu_buffer_rsrc_t rs, const unsigned* voff, unsigned soff, bf16* img, int wave) {
    constexpr int RPI = 1024 / (T * 2);
    constexpr int NI = W4_TM / RPI / 4;
#pragma unroll
    for (int i = 0; i < NI; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + (wave * NI + i) * RPI * T),
                                                 16, voff[i], soff, 0, 0);
}

// 32x32x16 operand fragment: 8 consecutive tokens (16 s + 8 h' ..) of feature column c0 + (lane & 31)
template <int T>
__device__ __forceinline__ bf16x8 w4_frag(const bf16* img, int c0, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = 16 * s + 8 * (grp >> 1) + q;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + w4_off<T>(row, col)));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(img + w4_off<T>(row + 4, col)));
    const v4s v[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

template <int N> __device__ __forceinline__ void w4_vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int TN, int TK, int S, int OCC>
__global__ __launch_bounds__(W4_NT, OCC) void wgrad4_kernel(long M, int N, int K, long R, int nt, int kt,
                                                            const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            float* __restrict__ part) {
    constexpr int STAGE = W4_TM * (TN + TK);          // bf16 elements per stage
    constexpr int DN = W4_TM / (1024 / (TN * 2)) / 4, DK = W4_TM / (1024 / (TK * 2)) / 4;
    constexpr int D = DN + DK;                         // DMA instructions per wave per slice
    constexpr int P = S - 1;
    constexpr int AN = TN / 64, AK = TK / 64;          // 32x32 tiles per wave
    __shared__ __attribute__((aligned(1024))) bf16 smem[S * STAGE];
    const long id = xcd_tile(blockIdx.x, gridDim.x);  // tiles of one chunk adjacent: the chunk is read once per XCD
    const int chunk = (int)(id / (nt * kt)), tile = (int)(id % (nt * kt));
    const int n0 = (tile / kt) * TN, k0 = (tile % kt) * TK;
    const long mb = (long)chunk * R;
    const long rows = M - mb < R ? M - mb : R;
    const int steps = (int)((rows + W4_TM - 1) / W4_TM);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave >> 1) * (TN / 2), wk = (wave & 1) * (TK / 2);
    const bool do_bias = k0 == 0 && wk == 0;

    unsigned voffN[DN], voffK[DK];
    w4_voff<TN>(N, wave, lane, voffN);
    w4_voff<TK>(K, wave, lane, voffK);
    auto issue = [&](int u) {   // slice min(u, steps - 1) into stage u % S (exactly D DMA ops)
        const int uu = u < steps ? u : steps - 1;
        const long m = mb + (long)uu * W4_TM, left = rows - (long)uu * W4_TM;   // resource = the slice's rows
        bf16* st = smem + (u % S) * STAGE;
        w4_dma<TN>(buf_rsrc(dy + m * N + n0, left * N * 2 - (long)n0 * 2), voffN, 0, st, wave);
        w4_dma<TK>(buf_rsrc(x + m * K + k0, left * K * 2 - (long)k0 * 2), voffK, 0, st + W4_TM * TN, wave);
    };

    f32x16 acc[AN][AK], accb[AN];
#pragma unroll
    for (int a = 0; a < AN; ++a) {
        accb[a] = f32x16{};
#pragma unroll
        for (int b = 0; b < AK; ++b) acc[a][b] = f32x16{};
    }
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;

#pragma unroll
    for (int p = 0; p < P; ++p) issue(p);
    for (int u = 0; u < steps; ++u) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        w4_vmwait<D * P - D>();          // slice u landed; P - 1 later slices stay in flight
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue(u + P);
        const bf16* Ns = smem + (u % S) * STAGE;
        const bf16* Ks = Ns + W4_TM * TN;
#pragma unroll
        for (int s = 0; s < W4_TM / 16; ++s) {
            bf16x8 fa[AN], fb[AK];
#pragma unroll
            for (int a = 0; a < AN; ++a) fa[a] = w4_frag<TN>(Ns, wn + 32 * a, s, lane);
#pragma unroll
            for (int b = 0; b < AK; ++b) fb[b] = w4_frag<TK>(Ks, wk + 32 * b, s, lane);
#pragma unroll
            for (int a = 0; a < AN; ++a) {
#pragma unroll
                for (int b = 0; b < AK; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
                if (do_bias) accb[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a], ones, accb[a], 0, 0, 0);
            }
        }
    }
    w4_vmwait<0>();
    // acc[a][b][reg] = dW[n0 + wn + 32a + crow(reg, h)][k0 + wk + 32b + r]: two 128-B row segments per store
    const long slab = (long)N * K + N;
    const auto rs_o = buf_rsrc(part + chunk * slab, slab * 4);
#pragma unroll
    for (int a = 0; a < AN; ++a)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int n = n0 + wn + 32 * a + crow(reg, h);
#pragma unroll
            for (int b = 0; b < AK; ++b) {
                const int k = k0 + wk + 32 * b + r;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[a][b][reg]), rs_o,
                                                      (n < N && k < K) ? (unsigned)(n * K + k) * 4 : kOOB, 0, 0);
            }
            if (do_bias && r == 0 && n < N) part[chunk * slab + (long)N * K + n] = accb[a][reg];
        }
}

struct W4Plan {
    int cfg, tn, tk, nt, kt, chunks;
    long R;
};

// cfg: 0 = 64x64 tiles, 4-stage ring, 2 workgroups/CU; 1 = 128x128, 3 stages, 1/CU;
//      2 = 128x64, 3 stages, 2/CU.  Chunks are sized for ~`target` workgroups of >= 256 tokens.
int w4_cfg_env() {
    static int v = -2;
    if (v == -2) {
        const char* e = getenv("CSU_W4CFG");
        v = e ? atoi(e) : -1;
    }
    return v;
}

W4Plan w4plan(long M, int N, int K) {
    W4Plan p;
    p.cfg = w4_cfg_env();
    if (p.cfg < 0 || p.cfg > 2) p.cfg = 0;
    p.tn = p.cfg == 0 ? 64 : 128;
    p.tk = p.cfg == 1 ? 128 : 64;
    p.nt = (N + p.tn - 1) / p.tn;
    p.kt = (K + p.tk - 1) / p.tk;
    const long target = p.cfg == 1 ? 512 : 1024;
    long want = (target + p.nt * p.kt - 1) / (p.nt * p.kt);
    const long maxc = (M + 255) / 256;
    if (want > maxc) want = maxc;
    if (want < 1) want = 1;
    p.R = ((M + want - 1) / want + W4_TM - 1) / W4_TM * W4_TM;
    p.chunks = (int)((M + p.R - 1) / p.R);
    return p;
}

template <int TN, int TK, int S, int OCC>
int w4_launch(const W4Plan& p, long M, int N, int K, const bf16* dy, const bf16* x, float* part, hipStream_t st) {
    const unsigned grid = (unsigned)(p.nt * p.kt * p.chunks);
    wgrad4_kernel<TN, TK, S, OCC><<<grid, W4_NT, 0, st>>>(M, N, K, p.R, p.nt, p.kt, dy, x, part);
    return check_launch("wgrad4");
}

}  // namespace

bool wgrad4_ok(long M, int N, int K) {
    return N % 8 == 0 && K % 8 == 0 && N >= 64 && K >= 64 && M * (long)(N > K ? N : K) < (1L << 30);
}

size_t wgrad4_workspace(long M, int N, int K) {
    const W4Plan p = w4plan(M, N, K);
    const long slab = (long)N * K + N;
    return p.chunks > 1 ? (size_t)p.chunks * slab * sizeof(float) + colsum_workspace(p.chunks, slab, CSU_F32) : 0;
}

// dw_db = [dW (N*K) | db (N)] fp32
int wgrad4_run(long M, int N, int K, const bf16* dy, const bf16* x, float* dw_db, void* ws, hipStream_t st) {
    const W4Plan p = w4plan(M, N, K);
    const long slab = (long)N * K + N;
    float* part = p.chunks > 1 ? (float*)ws : dw_db;
    int e;
    if (p.cfg == 1) e = w4_launch<128, 128, 3, 1>(p, M, N, K, dy, x, part, st);
    else if (p.cfg == 2) e = w4_launch<128, 64, 3, 2>(p, M, N, K, dy, x, part, st);
    else e = w4_launch<64, 64, 4, 2>(p, M, N, K, dy, x, part, st);
    if (e || p.chunks == 1) return e;
    return colsum_launch(p.chunks, slab, CSU_F32, part, dw_db, part + (size_t)p.chunks * slab, st);
}

}  // namespace csu
