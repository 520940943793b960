// Implicit-GEMM NHWC convolution for gfx950 (bf16 or fp32 operands, fp32 accumulation).
//
// Replaces the convolutions of the path: patch embed Conv2d(3,64,7,4,2) (cswin:505), Merge_Block
// Conv2d(C,2C,3,2,1) (cswin:376), the CARAFE encoder Conv2d(C/4, 9 s^2, 3, 1, 1) (cswin:397/446)
// and the plain-UNet DoubleConv 3x3 / ConvTranspose2d(k2, s2) stages (unet:182-211; a transposed
// conv is this file's input-gradient operator).  Activations stay NHWC (= the (B, L, C) tokens), so
// no im2col buffer and no layout transposes:
//   forward : out[m = (b,oy,ox)][n]      = bias[n] + sum_{k=(ky,kx,c)} x[b, oy*s-p+ky, ox*s-p+kx, c] * Wf[n][k]
//   dgrad   : dx [m = (b,iy,ix)][c]      = sum_{k=(ky,kx,n)} dy[b, (iy+p-ky)/s, (ix+p-kx)/s, n] * Wd[c][k]
//             (terms whose division is inexact or out of range are zero)
//   wgrad   : dW [n][k = (ky,kx,c)]      = sum_m dy[m][n] * x[pixel(m, ky, kx)][c],  db[n] = sum_m dy[m][n]
// Wf = weight permuted to [n][ky][kx][c] (OHWI), Wd = [c][ky][kx][n] (IHWO); both prepared by the caller.
// Tiles: 64 x 64 outputs per 256-thread workgroup, 4 waves of one 32x32 MFMA tile, 32-deep K slices
// gathered per 8-channel chunk (16-B loads when the gathered channel count is a multiple of 8).
#include <cstdlib>

#include "common.hpp"
#include "lds_dma.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int TBM = 64, TBN = 64, TBK = 32;

template <typename T> struct CT;
template <> struct CT<bf16> { static constexpr int AS = TBK; };        // swizzled 64-B rows
template <> struct CT<float> { static constexpr int AS = TBK + 4; };   // padded 144-B rows

__device__ __forceinline__ int cswz(int row, int col) {
    return row * TBK + ((((col >> 3) ^ (row >> 2)) & 3) << 3) + (col & 7);
}

struct Geo {
    int B, H, W, C, OH, OW, N, KH, KW, s, p;
};

// element index of the gathered operand for GEMM row m, reduction index k (or -1 when zero)
template <int MODE>   // 0 forward (rows = output pixels, k = (ky,kx,c) over x); 1 dgrad (rows = input pixels, k = (ky,kx,n) over dy)
__device__ __forceinline__ long gather_index(const Geo& g, long m, int k, long Mrows) {
    if (m >= Mrows) return -1;
    if (MODE == 0) {
        const int KC = g.C;
        if (k >= g.KH * g.KW * KC) return -1;
        const int tap = k / KC, c = k - tap * KC;
        const int ky = tap / g.KW, kx = tap - ky * g.KW;
        const int ox = (int)(m % g.OW);
        const long t = m / g.OW;
        const int oy = (int)(t % g.OH), b = (int)(t / g.OH);
        const int iy = oy * g.s - g.p + ky, ix = ox * g.s - g.p + kx;
        if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W) return -1;
        return (((long)b * g.H + iy) * g.W + ix) * g.C + c;
    } else {
        const int KN = g.N;
        if (k >= g.KH * g.KW * KN) return -1;
        const int tap = k / KN, n = k - tap * KN;
        const int ky = tap / g.KW, kx = tap - ky * g.KW;
        const int ix = (int)(m % g.W);
        const long t = m / g.W;
        const int iy = (int)(t % g.H), b = (int)(t / g.H);
        const int ny = iy + g.p - ky, nx = ix + g.p - kx;
        if (ny < 0 || nx < 0 || ny % g.s || nx % g.s) return -1;
        const int oy = ny / g.s, ox = nx / g.s;
        if (oy >= g.OH || ox >= g.OW) return -1;
        return (((long)b * g.OH + oy) * g.OW + ox) * g.N + n;
    }
}

// 8 consecutive reduction indices k..k+7 of row m -> v (zeros where out of range)
template <int MODE, typename T, bool VEC>
__device__ __forceinline__ void gather8(const Geo& g, const T* src, long m, int k, long Mrows, float* v) {
    if constexpr (VEC) {
        const long idx = gather_index<MODE>(g, m, k, Mrows);
        if (idx >= 0) load8(src + idx, v);
        else
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = 0.f;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const long idx = gather_index<MODE>(g, m, k + j, Mrows);
            v[j] = idx >= 0 ? to_f(src[idx]) : 0.f;
        }
    }
}

// out[m][n] = bias[n] + sum_k A(m, k) * Bw[n][k];  Bw row-major (Ncols x Kdim)
template <typename T, int MODE, bool VEC>
__global__ __launch_bounds__(NT) void conv_gemm(Geo g, long Mrows, int Ncols, int Kdim, const T* __restrict__ src,
                                                const T* __restrict__ Bw, const float* __restrict__ bias,
                                                T* __restrict__ out) {
    constexpr int AS = CT<T>::AS;
    __shared__ __attribute__((aligned(16))) T As[TBM * AS];
    __shared__ __attribute__((aligned(16))) T Bs[TBN * AS];
    const long m0 = (long)blockIdx.x * TBM;
    const int n0 = blockIdx.y * TBN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    f32x16 acc = {};
    const bool bvec = Kdim % 8 == 0;   // 16-B aligned weight rows
    // staging: 64 rows x 4 chunks of 8 per operand = 256 chunks -> one per thread
    const int srow = threadIdx.x >> 2, sch = threadIdx.x & 3;
    auto put = [&](T* img, int row, int ch, const float* v) {
        if constexpr (sizeof(T) == 2) store8(img + cswz(row, ch * 8), v);
        else store8(img + row * AS + ch * 8, v);
    };
    for (int k0 = 0; k0 < Kdim; k0 += TBK) {
        float va[8], vb[8];
        gather8<MODE, T, VEC>(g, src, m0 + srow, k0 + sch * 8, Mrows, va);
        {
            const int n = n0 + srow, k = k0 + sch * 8;
            if (bvec && n < Ncols && k + 8 <= Kdim) load8(Bw + (long)n * Kdim + k, vb);
            else
#pragma unroll
                for (int j = 0; j < 8; ++j) vb[j] = (n < Ncols && k + j < Kdim) ? to_f(Bw[(long)n * Kdim + k + j]) : 0.f;
        }
        __syncthreads();
        put(As, srow, sch, va);
        put(Bs, srow, sch, vb);
        __syncthreads();
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(As + cswz(wm + r, 16 * s + 8 * h));
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(Bs + cswz(wn + r, 16 * s + 8 * h));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t)
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[(wm + r) * AS + 16 * h + t], Bs[(wn + r) * AS + 16 * h + t],
                                                           acc, 0, 0, 0);
        }
    }
    const int n = n0 + wn + r;
    if (n >= Ncols) return;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const long m = m0 + wm + crow(reg, h);
        if (m < Mrows) out[m * Ncols + n] = from_f<T>(acc[reg] + bv);
    }
}

// weight-gradient grids are (n tile, k tile, token chunk): the tiles of one chunk read the same dy rows
// and input pixels, so they run on one XCD (consecutive logical ids, xcd_block) and share its L2 --
// in hardware order consecutive workgroups go to different XCDs and each re-fetched the chunk
#ifndef CW_XCD
#define CW_XCD 1
#endif
struct Blk3 { int x, y, z; };
__device__ __forceinline__ Blk3 wg_block() {
    if (!CW_XCD) return {(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const int t = __builtin_amdgcn_readfirstlane((int)xcd_block());
    const int gx = gridDim.x, gy = gridDim.y;
    return {t % gx, (t / gx) % gy, t / (gx * gy)};
}

// dW partial slabs: workgroup (n tile, k tile, m chunk) accumulates dY^T X_gather over its rows.
// Operands staged transposed ([n][m], [k][m]) in LDS; db from the k-tile-0 workgroups.
template <typename T, bool VEC>
__global__ __launch_bounds__(NT) void conv_wgrad_kernel(Geo g, long Mrows, int Ncols, int Kdim, long rows_per_chunk,
                                                        const T* __restrict__ x, const T* __restrict__ dy,
                                                        float* __restrict__ part) {
    constexpr int TM = 64;               // rows per step: two row groups per thread, both loads in flight
    constexpr int RG = TM / 32;
    constexpr int S = TM + (sizeof(T) == 2 ? 8 : 4);
    __shared__ __attribute__((aligned(16))) T At[TBN * S];   // dy^T [n][m]
    __shared__ __attribute__((aligned(16))) T Bt[TBN * S];   // X^T  [k][m]
    const Blk3 wb = wg_block();
    const int n0 = wb.x * TBN, k0 = wb.y * TBN;
    const long mb = (long)wb.z * rows_per_chunk, me = min(Mrows, mb + rows_per_chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave >> 1) * 32, wk = (wave & 1) * 32;
    const bool do_bias = wb.y == 0;
    f32x16 acc = {};
    float bsum = 0.f;
    // staging: RG x (32 rows x 8 chunks) = RG chunks per operand per thread, all loads issued
    // before the LDS stores (one memory round trip per TM rows)
    const int srow = threadIdx.x >> 3, sch = threadIdx.x & 7;
    // VEC: this thread's 8 reduction indices are one (ky, kx) tap and 8 channels of one pixel,
    // fixed for the whole loop -- decomposed once; rows are decomposed with 32-bit arithmetic
    // (the generic gather8 spent ~4 64-bit divisions per load)
    const int kk = k0 + sch * 8;
    const bool kval = kk < Kdim;
    const int ktap = kk / g.C, kc = kk - ktap * g.C;
    const int kdy = ktap / g.KW - g.p, kdx = ktap % g.KW - g.p;
    for (long m0 = mb; m0 < me; m0 += TM) {
        float va[RG][8], vb[RG][8];
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            const long m = m0 + 32 * q + srow;
            const int n = n0 + sch * 8;
            if (Ncols % 8 == 0 && m < me && n + 8 <= Ncols) load8(dy + m * Ncols + n, va[q]);
            else
#pragma unroll
                for (int j = 0; j < 8; ++j) va[q][j] = (m < me && n + j < Ncols) ? to_f(dy[m * Ncols + n + j]) : 0.f;
            if constexpr (VEC) {
                const int mi = (int)m;             // M < 2^31 (check_geo)
                const int ox = mi % g.OW, t = mi / g.OW;
                const int oy = t % g.OH, b = t / g.OH;
                const int iy = oy * g.s + kdy, ix = ox * g.s + kdx;
                if (kval && m < me && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
                    load8(x + (((long)b * g.H + iy) * g.W + ix) * g.C + kc, vb[q]);
                else
#pragma unroll
                    for (int j = 0; j < 8; ++j) vb[q][j] = 0.f;
            } else {
                gather8<0, T, VEC>(g, x, m, k0 + sch * 8, me, vb[q]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RG; ++q)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                At[(sch * 8 + j) * S + 32 * q + srow] = from_f<T>(va[q][j]);
                Bt[(sch * 8 + j) * S + 32 * q + srow] = from_f<T>(vb[q][j]);
            }
        __syncthreads();
        if (do_bias && threadIdx.x < TBN) {
#pragma unroll
            for (int j = 0; j < TM; ++j) bsum += to_f(At[threadIdx.x * S + j]);
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
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(At[(wn + r) * S + 2 * t + h], Bt[(wk + r) * S + 2 * t + h],
                                                           acc, 0, 0, 0);
        }
    }
    const long slab = ((long)Ncols * Kdim + Ncols + 3) & ~3L;   // 16-B aligned slab rows for colsum
    float* out = part + (long)wb.z * slab;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int n = n0 + wn + crow(reg, h), k = k0 + wk + r;
        if (n < Ncols && k < Kdim) out[(long)n * Kdim + k] = acc[reg];
    }
    if (do_bias && threadIdx.x < TBN && n0 + threadIdx.x < Ncols) out[(long)Ncols * Kdim + n0 + threadIdx.x] = bsum;
}

// bf16 weight gradient, v2 (C % 8 == 0): operand tiles staged ROW-major in LDS ([m][n] of dy,
// [m][k] of the gathered x) with 16-B stores, MFMA fragments gathered by the gfx950 transposing
// read ds_read_b64_tr_b16 (as wgrad.hip) -- the v1 kernel above stores both tiles transposed with
// 2-B LDS writes, 64 per thread per step, most of them bank conflicts.  64 rows per step, both
// row groups' global loads in flight together; the thread's tap is decomposed once.
typedef short cv4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ cv4s ctr_read(const bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) cv4s*)(p));
}
template <int RS>
__device__ __forceinline__ bf16x8 ctr_frag(const bf16* img, int c0, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = 16 * s + 8 * (grp >> 1) + q;
    const cv4s v[2] = {ctr_read(img + row * RS + col), ctr_read(img + (row + 4) * RS + col)};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

// N4: Ncols % 8 == 4 (the 36-channel CARAFE encoders): each thread's 8 dy columns as two 8-B loads
template <bool N4>
__global__ __launch_bounds__(NT) void conv_wgrad_bf16(Geo g, long Mrows, int Ncols, int Kdim, long rows_per_chunk,
                                                      const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                      float* __restrict__ part) {
    constexpr int TM = 64, RG = TM / 32;
    constexpr int RS = TBN + 32;          // 64 data + 64 B pad: conflict-free transposing reads
    __shared__ __attribute__((aligned(16))) bf16 At[TM * RS];   // dy tile [m][n]
    __shared__ __attribute__((aligned(16))) bf16 Bt[TM * RS];   // x  tile [m][k] (gathered)
    const Blk3 wb = wg_block();
    const int n0 = wb.x * TBN, k0 = wb.y * TBN;
    const long mb = (long)wb.z * rows_per_chunk, me = min(Mrows, mb + rows_per_chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5;
    const int wn = (wave >> 1) * 32, wk = (wave & 1) * 32;
    const bool do_bias = wb.y == 0;
    f32x16 acc = {};
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int srow = threadIdx.x >> 3, sch = threadIdx.x & 7;
    const int kk = k0 + sch * 8;
    const bool kval = kk < Kdim;
    const int ktap = kk / g.C, kc = kk - ktap * g.C;
    const int kdy = ktap / g.KW - g.p, kdx = ktap % g.KW - g.p;
    const int n = n0 + sch * 8;
    const bool nval = (N4 ? n + 4 : n + 8) <= Ncols, nval2 = n + 8 <= Ncols;   // Ncols % 4 == 0 on this path
    // branch-free gathers (raw buffer loads, out-of-range offsets read 0): the next step's loads
    // stay in flight across this step's LDS stores and MFMAs
    const __amdgpu_buffer_rsrc_t rs_dy = buf_rsrc(dy, Mrows * Ncols * 2);
    const __amdgpu_buffer_rsrc_t rs_x = buf_rsrc(x, (long)g.B * g.H * g.W * g.C * 2);
    bf16x8 va[RG], vb[RG];
    auto load = [&](long m0) {
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            const long m = m0 + 32 * q + srow;
            const bool mv = m < me;
            const unsigned mi = (unsigned)(mv ? m : 0);   // M < 2^31 (check_geo)
            const unsigned t = mi / (unsigned)g.OW, b = t / (unsigned)g.OH;
            const int ox = (int)(mi - t * (unsigned)g.OW), oy = (int)(t - b * (unsigned)g.OH);
            const int iy = oy * g.s + kdy, ix = ox * g.s + kdx;
            const unsigned offa = (mv && nval) ? (unsigned)((m * Ncols + n) * 2) : kOOB;
            const unsigned offb = (kval && mv && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
                                      ? (unsigned)(((((int)b * g.H + iy) * g.W + ix) * g.C + kc) * 2) : kOOB;
            u32x4 a4;
            if constexpr (N4) {   // 8-B aligned row segments: columns n..n+3, n+4..n+7
                const unsigned offa2 = (mv && nval2) ? offa + 8u : kOOB;
                const u32x2 lo = __builtin_amdgcn_raw_buffer_load_b64(rs_dy, offa, 0, 0);
                const u32x2 hi = __builtin_amdgcn_raw_buffer_load_b64(rs_dy, offa2, 0, 0);
                a4 = u32x4{lo[0], lo[1], hi[0], hi[1]};
            } else {
                a4 = __builtin_amdgcn_raw_buffer_load_b128(rs_dy, offa, 0, 0);
            }
            const u32x4 b4 = __builtin_amdgcn_raw_buffer_load_b128(rs_x, offb, 0, 0);
            __builtin_memcpy(&va[q], &a4, 16);
            __builtin_memcpy(&vb[q], &b4, 16);
        }
    };
    load(mb);
    for (long m0 = mb; m0 < me; m0 += TM) {
        __syncthreads();   // the previous step's MFMAs are done with the LDS tiles
#pragma unroll
        for (int q = 0; q < RG; ++q) {
            *reinterpret_cast<bf16x8*>(At + (32 * q + srow) * RS + sch * 8) = va[q];
            *reinterpret_cast<bf16x8*>(Bt + (32 * q + srow) * RS + sch * 8) = vb[q];
            if (do_bias)
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[j] += (float)va[q][j];
        }
        __syncthreads();
        load(m0 + TM);   // past the chunk: out-of-range offsets, zeros (never stored)
#pragma unroll
        for (int s = 0; s < TM / 16; ++s)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ctr_frag<RS>(At, wn, s, lane), ctr_frag<RS>(Bt, wk, s, lane),
                                                          acc, 0, 0, 0);
    }
    const long slab = ((long)Ncols * Kdim + Ncols + 3) & ~3L;   // 16-B aligned slab rows for colsum
    float* out = part + (long)wb.z * slab;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int nn = n0 + wn + crow(reg, h), k = k0 + wk + (lane & 31);
        if (nn < Ncols && k < Kdim) out[(long)nn * Kdim + k] = acc[reg];
    }
    if (do_bias) {   // column sums: 8 columns per thread, 32 row-threads per column group
        __shared__ float bcol[32][TBN + 1];
#pragma unroll
        for (int j = 0; j < 8; ++j) bcol[srow][sch * 8 + j] = bsum[j];
        __syncthreads();
        if (threadIdx.x < TBN && n0 + threadIdx.x < Ncols) {
            float sacc = 0.f;
            for (int r = 0; r < 32; ++r) sacc += bcol[r][threadIdx.x];
            out[(long)Ncols * Kdim + n0 + threadIdx.x] = sacc;
        }
    }
}

// ---- bf16 weight gradient, v3 (C % 8 == 0, N % 8 == 0): LDS-DMA gathers, S-stage ring ------------
// One TN x TK tile of dW over the rows of one chunk, 64 rows (output pixels m) per step.  Both
// operand images are row-major [m][columns] and filled by buffer_load ... lds: the dy image straight
// from the (rows, N) matrix (rows past the chunk end fall outside the step's resource and land as
// zeros), the x image gathered per lane -- column k = (tap, c) of row m is the input pixel under tap
// (ky, kx) of output pixel m, 8 channels per lane, out-of-image taps at an out-of-range offset.
// The tap and channel of each lane's columns are fixed for the whole loop; only the pixel moves.
// MFMA fragments are transposing reads (ds_read_b64_tr_b16) of the [m][...] images (trfrag); the
// row swizzle is applied to the DMA source columns.  db (k tile 0) sums the dy fragments the MFMAs
// read anyway.  Partial slabs per chunk as the v2 kernel: [chunk][N*K + N], reduced by colsum.
template <int TN, int TK, int S, int WN, int WK>
__global__ __launch_bounds__(64 * WN * WK, 1) void conv_wgrad_dma(Geo g, long Mrows, int Ncols, int Kdim, long rpc,
                                                                  const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                                  float* __restrict__ part) {
    constexpr int NWV = WN * WK;
    constexpr int RM = 64;                          // rows per step
    constexpr int RBA = TN * 2, RBB = TK * 2;       // image row bytes
    constexpr int STAGE = RM * (TN + TK);           // bf16 elements per ring stage
    constexpr int NA = RM * RBA / (1024 * NWV), NB = RM * RBB / (1024 * NWV);
    constexpr int D = NA + NB;                      // DMA instructions per wave per step
    constexpr int P = S - 1;
    constexpr int TNW = TN / (32 * WN), TKW = TK / (32 * WK);
    static_assert(NA >= 1 && NB >= 1 && TNW >= 1 && TKW >= 1 && (P - 1) * D <= 63, "conv_wgrad_dma layout");
    __shared__ __attribute__((aligned(1024))) bf16 smem[S * STAGE];
    const Blk3 wb = wg_block();
    const int n0 = wb.x * TN, k0 = wb.y * TK;
    const long mb = (long)wb.z * rpc, me = min(Mrows, mb + rpc);
    const int nsteps = (int)((me - mb + RM - 1) / RM);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int wn = (wave / WK) * (TN / WN), wk = (wave % WK) * (TK / WK);
    const bool do_bias = wb.y == 0 && wave % WK == 0;

    // dy image: lane's row and 16-B column chunk per instruction (fixed), byte offset within a step
    unsigned voffA[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int p = (wave * NA + i) * 1024 + lane * 16;
        const int row = p / RBA, slot = (p % RBA) >> 4;
        const int n = n0 + 8 * (slot ^ mkey<RBA>(row));
        voffA[i] = n < Ncols ? (unsigned)(row * Ncols + n) * 2u : kOOB;
    }
    // x image: row, and the tap offsets / channel of the lane's 8 columns (fixed)
    int brow[NB], bdy[NB], bdx[NB], bc[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int p = (wave * NB + i) * 1024 + lane * 16;
        const int row = p / RBB, slot = (p % RBB) >> 4;
        const int k = k0 + 8 * (slot ^ mkey<RBB>(row));
        const int tap = k / g.C, c = k - tap * g.C;
        brow[i] = row;
        bdy[i] = k < Kdim ? tap / g.KW - g.p : -(1 << 29);   // invalid column: never inside the image
        bdx[i] = tap % g.KW - g.p;
        bc[i] = c;
    }
    const i32x4 rsX = rsrc4(x, (long)g.B * g.H * g.W * g.C * 2);
    auto issue = [&](int u) {   // step u (steps past the chunk: every offset out of range, zeros)
        const long m0 = mb + (long)u * RM;
        bf16* stg = smem + (u % S) * STAGE;
        const long rows = me - m0;
        dma<NA>(rsrc4(dy + (rows > 0 ? m0 : 0) * Ncols, rows > 0 ? rows * Ncols * 2 : 0), voffA, 0u, stg, wave);
        unsigned vb[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const long m = m0 + brow[i];
            const bool mv = m < me;
            const unsigned mu = (unsigned)(mv ? m : 0);   // < 2^31 (check_geo)
            const unsigned t = mu / (unsigned)g.OW, b = t / (unsigned)g.OH;
            const int ox = (int)(mu - t * (unsigned)g.OW), oy = (int)(t - b * (unsigned)g.OH);
            const int iy = oy * g.s + bdy[i], ix = ox * g.s + bdx[i];
            const bool ok = mv && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
            vb[i] = ok ? (unsigned)(((((int)b * g.H + iy) * g.W + ix) * g.C + bc[i]) * 2) : kOOB;
        }
        dma<NB>(rsX, vb, 0u, stg + RM * TN, wave);
    };
    f32x16 acc[TNW][TKW];
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
        for (int i = 0; i < TKW; ++i) acc[j][i] = f32x16{};
    float bsum[TNW];
#pragma unroll
    for (int j = 0; j < TNW; ++j) bsum[j] = 0.f;
    auto mma = [&](int u) {
        const bf16* As = smem + (u % S) * STAGE;
        const bf16* Bs = As + RM * TN;
#pragma unroll
        for (int s = 0; s < RM / 16; ++s) {
            bf16x8 af[TNW], bfr[TKW];
#pragma unroll
            for (int j = 0; j < TNW; ++j) af[j] = trfrag<RBA>(As, wn + 32 * j, s, lane);
#pragma unroll
            for (int i = 0; i < TKW; ++i) bfr[i] = trfrag<RBB>(Bs, wk + 32 * i, s, lane);
#pragma unroll
            for (int j = 0; j < TNW; ++j)
#pragma unroll
                for (int i = 0; i < TKW; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[j], bfr[i], acc[j][i], 0, 0, 0);
            if (do_bias)
#pragma unroll
                for (int j = 0; j < TNW; ++j)
#pragma unroll
                    for (int e = 0; e < 8; ++e) bsum[j] += (float)af[j][e];
        }
    };
#pragma unroll
    for (int p = 0; p < P; ++p) issue(p);
    for (int u = 0; u < nsteps; ++u) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        vmwait<(P - 1) * D>();             // step u landed (only the P - 1 later steps' DMAs in flight)
        __builtin_amdgcn_s_barrier();      // ... for every wave; stage (u - 1) % S is free
        __builtin_amdgcn_sched_barrier(0);
        issue(u + P);
        mma(u);
    }
    vmwait<0>();   // drain the prefetch past the chunk before the LDS is released
    const long slab = ((long)Ncols * Kdim + Ncols + 3) & ~3L;
    float* out = part + (long)wb.z * slab;
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
        for (int i = 0; i < TKW; ++i)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = n0 + wn + 32 * j + crow(reg, h), k = k0 + wk + 32 * i + (lane & 31);
                if (n < Ncols && k < Kdim) out[(long)n * Kdim + k] = acc[j][i][reg];
            }
    if (do_bias) {   // lanes r and r + 32 hold the two row halves of column wn + 32 j + r
#pragma unroll
        for (int j = 0; j < TNW; ++j) {
            const float v = bsum[j] + __shfl_xor(bsum[j], 32, 64);
            const int n = n0 + wn + 32 * j + (lane & 31);
            if (h == 0 && n < Ncols) out[(long)Ncols * Kdim + n] = v;
        }
    }
}

// ---- bf16 weight gradient of a 3x3 / stride 1 / pad 1 conv, halo form (OW % 64 == 0, C % 64 == 0,
// N % 64 == 0) ------------------------------------------------------------------------------------
// dW[n][ky][kx][c] = sum_m dy[m][n] * x[m + (ky - 1, kx - 1)][c].  A step is one 64-pixel segment of
// an output row: the dy image [64 px][NS] and, per tap row ky, ONE halo image of the 66 input pixels
// under the segment [ox0 - 1, ox0 + 64] x 64 channels; tap kx is the halo image read from row kx on
// (transposing fragment reads at a row offset).  The x bytes staged per step are 3 x 66 rows instead
// of the 9 x 64 of a gathered im2col image, and the workgroup keeps the whole (NS x 64-channel x 9
// taps) weight-gradient block in its accumulators, so dy is staged once per pixel.  Wave (nt, ct)
// owns n rows nt*32.. and channels ct*32.. of all 9 taps (9 accumulator tiles).
constexpr int kHaloRows = 72;   // 66 halo rows padded to whole 1-KB DMA blocks (9 per image)

template <int RB>
__device__ __forceinline__ bf16x8 trfrag_at(const bf16* img, int row0, int c0, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = row0 + 16 * s + 8 * (grp >> 1) + q;
    return cat8(tr4(img + moff<RB>(row, col)), tr4(img + moff<RB>(row + 4, col)));
}

template <int NS, int S>
__global__ __launch_bounds__(64 * NS / 16, 1) void conv3_wgrad_halo(Geo g, long nseg, long spc, const bf16* __restrict__ x,
                                                                    const bf16* __restrict__ x2, int csplit,
                                                                    const bf16* __restrict__ dy, float* __restrict__ part) {
    constexpr int NTW = NS / 32;                    // n tiles
    constexpr int NWV = NTW * 2;                    // waves: n tile x channel half
    constexpr int RBD = NS * 2;                     // dy image row bytes
    constexpr int XIMG = kHaloRows * 64;            // bf16 per halo image
    constexpr int DIMG = 64 * NS;                   // bf16 per dy image
    constexpr int XBLK = XIMG * 2 / 1024;           // 1-KB DMA blocks per halo image (9)
    constexpr int NBLK = 3 * XBLK + DIMG * 2 / 1024;
    constexpr int NI = (NBLK + NWV - 1) / NWV;      // DMA instructions per wave per step
    constexpr int STAGE = NI * NWV * 512;           // bf16 per stage (spare blocks included)
    constexpr int P = S - 1;
    static_assert((P - 1) * NI <= 63, "conv3_wgrad_halo ring");
    __shared__ __attribute__((aligned(1024))) bf16 smem[S * STAGE];
    const Blk3 wb = wg_block();
    const int n0 = wb.x * NS, c0 = wb.y * 64;
    const long sb = (long)wb.z * spc, se = min(nseg, sb + spc);
    const int nsteps = (int)(se - sb);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const int nt = wave % NTW, ct = wave / NTW;
    const bool do_bias = wb.y == 0 && ct == 0;
    const int spr = g.OW / 64;                      // segments per output row
    // per instruction: the lane's image row and channel / n column (block-aligned regions: the
    // region -- halo image ky or the dy image -- is uniform per instruction)
    int irow[NI], icol[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int j = wave * NI + i;
        if (j < 3 * XBLK) {
            const int row = (j % XBLK) * 8 + (lane >> 3);
            irow[i] = row;
            icol[i] = 8 * ((lane & 7) ^ mkey<128>(row));
        } else {
            const int q = (j - 3 * XBLK) * 1024 + lane * 16;
            const int row = q / RBD;
            irow[i] = row;
            icol[i] = 8 * (((q % RBD) >> 4) ^ mkey<RBD>(row));
        }
    }
    // two sources (csplit > 0, % 64): this workgroup's 64-channel slice lies in one of them
    const bool sec = csplit > 0 && c0 >= csplit;
    const int xst = csplit ? (sec ? g.C - csplit : csplit) : g.C, xc0 = sec ? c0 - csplit : c0;
    const i32x4 rsX = sec ? rsrc4(x2, (long)g.B * g.H * g.W * xst * 2) : rsrc4(x, (long)g.B * g.H * g.W * xst * 2);
    const i32x4 rsD = rsrc4(dy, (long)g.B * g.OH * g.OW * g.N * 2);
    auto issue = [&](int u) {   // segment sb + u (past the chunk: every offset out of range, zeros)
        const long seg = sb + u;
        const bool sv = seg < se;
        const unsigned su = (unsigned)(sv ? seg : 0);   // < 2^31 / 64 (check_geo)
        const unsigned trow = su / (unsigned)spr, b = trow / (unsigned)g.OH;
        const int ox0 = (int)(su - trow * (unsigned)spr) * 64, oy = (int)(trow - b * (unsigned)g.OH);
        bf16* stg = smem + (u % S) * STAGE;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int j = wave * NI + i;
            unsigned off = kOOB;
            if (j < 3 * XBLK) {
                const int iy = oy + j / XBLK - 1, ix = ox0 - 1 + irow[i];
                const bool ok = sv && irow[i] < 66 && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
                if (ok) off = (unsigned)(((((int)b * g.H + iy) * g.W + ix) * xst + xc0 + icol[i]) * 2);
                dma1_u(rsX, off, 0u, stg + j * 512);
            } else {
                if (sv && j < NBLK)
                    off = (unsigned)((((((int)b * g.OH + oy) * g.OW + ox0 + irow[i]) * g.N) + n0 + icol[i]) * 2);
                dma1_u(rsD, off, 0u, stg + j * 512);
            }
        }
    };
    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f32x16{};
    float bsum = 0.f;
    auto mma = [&](int u) {
        const bf16* st = smem + (u % S) * STAGE;
        const bf16* dimg = st + 3 * XIMG;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const bf16x8 a = trfrag<RBD>(dimg, nt * 32, s2, lane);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx)
                    acc[ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        a, trfrag_at<128>(st + ky * XIMG, kx, ct * 32, s2, lane), acc[ky * 3 + kx], 0, 0, 0);
            if (do_bias)
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum += (float)a[e];
        }
    };
#pragma unroll
    for (int p = 0; p < P; ++p) issue(p);
    for (int u = 0; u < nsteps; ++u) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        vmwait<(P - 1) * NI>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue(u + P);
        mma(u);
    }
    vmwait<0>();
    const long K = 9L * g.C;
    const long slab = ((long)g.N * K + g.N + 3) & ~3L;
    float* out = part + (long)wb.z * slab;
    const int c = c0 + ct * 32 + (lane & 31);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int n = n0 + nt * 32 + crow(reg, h);
            out[(long)n * K + t * g.C + c] = acc[t][reg];
        }
    if (do_bias) {
        const float v = bsum + __shfl_xor(bsum, 32, 64);
        if (h == 0) out[(long)g.N * K + n0 + nt * 32 + (lane & 31)] = v;
    }
}

struct WDCfg { int tn, tk, s, wn, wk; };
#ifdef WD_PROBE256   // probe build only (tools/probes/wgrad_tile_probe.py): slot 4 = the 256 x 256 tile, 8 waves
constexpr WDCfg kWDCfgs[] = {{128, 128, 3, 2, 2}, {64, 256, 3, 1, 4}, {128, 128, 2, 2, 2}, {256, 128, 2, 4, 2}, {256, 256, 2, 2, 4}};
#else
constexpr WDCfg kWDCfgs[] = {{128, 128, 3, 2, 2}, {64, 256, 3, 1, 4}, {128, 128, 2, 2, 2}, {256, 128, 2, 4, 2}, {64, 128, 4, 1, 4}};
#endif
constexpr int kWDNCfg = 5;

// ---- bf16 implicit GEMM, v2: 128/256 x BN tiles, 64-deep K slices, double-buffered LDS ----------
// One problem description covers the forward conv and each stride phase of the input gradient:
//   row (b, ry, rx) gathers source pixel (ry*ay + by + ty*sty, rx*ax + bx + tx*stx) for tap (ty, tx),
//   weight column ((ty*wty + w0y)*KWf + tx*wtx + w0x)*Cs + c, output pixel (ry*oya + oyb, rx*oxa + oxb).
// Input gradient of a stride-s conv is split into s*s phases (input pixel parity), each a dense conv
// over only the taps that hit it (3x3/s2: 1, 2 or 4 taps instead of 9 mostly-zero ones).
struct IG {
    int Hs, Ws, Cs;
    int RH, RW;
    int ay, by, ax, bx;
    int nty, ntx, sty, stx;
    int ldw, KWf, wty, w0y, wtx, w0x;
    int OHo, OWo, oya, oyb, oxa, oxb;
    int B, Ncols, Kd;
    long M;
    // two-source gathers / two-destination outputs (the channel concat of UNet Up, unet:213-216,
    // without materialising it): channels [0, csplit) of the gathered operand come from src
    // (csplit per pixel), [csplit, Cs) from src2 (Cs - csplit per pixel); output columns [0, nsplit)
    // go to out (nsplit per pixel), [nsplit, Ncols) to out2.  0: one source / one output.
    int csplit, nsplit;
    const bf16* src2;
    bf16* out2;
};

// gathered-channel slice c0 (64-aligned, one tap): the source holding it, its channel stride and the
// channel inside it
struct CSel {
    bool second;
    int stride, c;
};
__device__ __forceinline__ CSel csel(const IG& g, int c0) {
    if (g.csplit == 0) return CSel{false, g.Cs, c0};
    const bool sec = c0 >= g.csplit;
    return CSel{sec, sec ? g.Cs - g.csplit : g.csplit, sec ? c0 - g.csplit : c0};
}
// output byte offset of column n of output pixel opix (out or out2), kOOB passes through
__device__ __forceinline__ unsigned obyte(const IG& g, unsigned opix, int n) {
    if (opix == kOOB) return kOOB;
    if (g.nsplit == 0) return (opix * (unsigned)g.Ncols + (unsigned)n) * 2u;
    return n < g.nsplit ? (opix * (unsigned)g.nsplit + (unsigned)n) * 2u
                        : (opix * (unsigned)(g.Ncols - g.nsplit) + (unsigned)(n - g.nsplit)) * 2u;
}

__device__ __forceinline__ int swz128(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }

// up to 4 independent problems in one launch (blockIdx.z): the stride phases of an input gradient
// run concurrently instead of as 1-4 small launches each (a 16x16x512 -> 32x32x256 input gradient
// is 4 launches of 128 workgroups)
struct IG4 {
    IG g[4];
    // split-K (one problem, few tiles): blockIdx.z = K part of kper gathered columns (a multiple of
    // 64); each part writes its fp32 partial tile to slab + z * M * Ncols, summed by conv_split_reduce
    int ksplit, kper;
    float* slab;
};

template <int BN, int VW>
__global__ __launch_bounds__(NT) void igemm_bf16(IG4 gs, const bf16* __restrict__ src, const bf16* __restrict__ Bw,
                                                 const float* __restrict__ bias, bf16* __restrict__ out) {
    constexpr int WN = BN / 32, WM = 4 / WN, BM = WM * 64, BK = 64;
    constexpr int ACH = BM * 8 / NT, BCH = BN * 8 / NT, NP = 8 / VW;
    __shared__ __attribute__((aligned(16))) bf16 As[2][BM * BK];
    __shared__ __attribute__((aligned(16))) bf16 Bs[2][BN * BK];
    __shared__ unsigned ooff[BM];   // output pixel of each tile row (kOOB: none)
    // problem of this z-slice (selects, not a dynamic index into the kernel-argument struct)
    const int z = blockIdx.z;
    const bool split = gs.ksplit > 1;
    const IG g = split || z == 0 ? gs.g[0] : z == 1 ? gs.g[1] : z == 2 ? gs.g[2] : gs.g[3];
    const long m0 = (long)blockIdx.x * BM;
    if (m0 >= g.M) return;   // phases differ in size: the grid covers the largest
    const int kb = split ? z * gs.kper : 0;                       // this workgroup's K range
    const int ke = split ? min(g.Kd, kb + gs.kper) : g.Kd;
    const int n0 = blockIdx.y * BN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wn = (wave % WN) * 32, wm = (wave / WN) * 64;
    const int ch = threadIdx.x & 7, rbase = threadIdx.x >> 3;

    // per staging row: image base pixel row and source base coordinates
    int rb[ACH], ryb[ACH], rxb[ACH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
        const long m = m0 + rbase + 32 * i;
        if (m < g.M) {   // 32-bit decomposition (check_geo: < 2^31 pixels)
            const unsigned mu = (unsigned)m, t = mu / (unsigned)g.RW;
            const int rx = (int)(mu - t * (unsigned)g.RW);
            const unsigned b = t / (unsigned)g.RH;
            const int ry = (int)(t - b * (unsigned)g.RH);
            rb[i] = (int)b * g.Hs;
            ryb[i] = ry * g.ay + g.by;
            rxb[i] = rx * g.ax + g.bx;
        } else {
            rb[i] = 0;
            ryb[i] = -(1 << 29);   // never in range
            rxb[i] = 0;
        }
    }
    // two register sets: the loads of K slice k + 2 are issued while slice k is multiplied and slice
    // k + 1 (loaded one step earlier) is stored to LDS -- two steps of MFMA work hide each load
    bf16x8 ra2[2][ACH], rbw2[2][BCH];
    // (pixel offsets fit 31 bits: check_geo bounds the pixel count, launch_ig the byte size)
    // branch-free gathers: raw buffer loads whose out-of-image / out-of-range lanes get an offset
    // past the resource (read as 0), so hipcc keeps every load of a slice in flight (a predicated
    // load makes it wait vmcnt(0) at the join and the register prefetch is lost)
    const int cs1 = g.csplit ? g.csplit : g.Cs;
    const __amdgpu_buffer_rsrc_t rs_src = buf_rsrc(src, (long)g.B * g.Hs * g.Ws * cs1 * 2);
    const __amdgpu_buffer_rsrc_t rs_src2 = buf_rsrc(g.src2, g.csplit ? (long)g.B * g.Hs * g.Ws * (g.Cs - g.csplit) * 2 : 0);
    const __amdgpu_buffer_rsrc_t rs_w = buf_rsrc(Bw, (long)g.Ncols * g.ldw * 2);
    auto load = [&](int k0, bf16x8* ra, bf16x8* rbw) {
        // two sources (csplit % 64 == 0, Cs % 64 == 0): the slice's side is uniform
        const CSel sl = csel(g, k0 % g.Cs);
        const int cadj = g.csplit && sl.second ? g.csplit : 0;
        const __amdgpu_buffer_rsrc_t rs_a = sl.second ? rs_src2 : rs_src;
#pragma unroll
        for (int pc = 0; pc < NP; ++pc) {
            const int k = k0 + 8 * ch + VW * pc;
            const bool kin = k < ke;
            const int t = kin ? k / g.Cs : 0, c = k - t * g.Cs;
            const int ty = t / g.ntx, tx = t - ty * g.ntx;
            const int oy = ty * g.sty, ox = tx * g.stx;
            const int wcol = ((ty * g.wty + g.w0y) * g.KWf + tx * g.wtx + g.w0x) * g.Cs + c;
#pragma unroll
            for (int i = 0; i < ACH; ++i) {
                const int y = ryb[i] + oy, x = rxb[i] + ox;
                const bool ok = kin && y >= 0 && y < g.Hs && x >= 0 && x < g.Ws;
                const unsigned off = ok ? (unsigned)((((rb[i] + y) * g.Ws + x) * sl.stride + c - cadj) * 2) : kOOB;
                if constexpr (VW == 8) {
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_a, off, 0, 0);
                    __builtin_memcpy(&ra[i], &v, 16);
                } else {
                    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_a, off, 0, 0);
                    bf16x4 b;
                    __builtin_memcpy(&b, &v, 8);
#pragma unroll
                    for (int j = 0; j < 4; ++j) ra[i][4 * pc + j] = b[j];
                }
            }
#pragma unroll
            for (int j = 0; j < BCH; ++j) {
                const int n = n0 + rbase + 32 * j;
                const bool ok = kin && n < g.Ncols;
                const unsigned off = ok ? (unsigned)((n * g.ldw + wcol) * 2) : kOOB;
                if constexpr (VW == 8) {
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_w, off, 0, 0);
                    __builtin_memcpy(&rbw[j], &v, 16);
                } else {
                    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs_w, off, 0, 0);
                    bf16x4 b;
                    __builtin_memcpy(&b, &v, 8);
#pragma unroll
                    for (int e = 0; e < 4; ++e) rbw[j][4 * pc + e] = b[e];
                }
            }
        }
    };
    auto store = [&](int buf, const bf16x8* ra, const bf16x8* rbw) {
#pragma unroll
        for (int i = 0; i < ACH; ++i) *reinterpret_cast<bf16x8*>(&As[buf][swz128(rbase + 32 * i, ch)]) = ra[i];
#pragma unroll
        for (int j = 0; j < BCH; ++j) *reinterpret_cast<bf16x8*>(&Bs[buf][swz128(rbase + 32 * j, ch)]) = rbw[j];
    };

    f32x16 acc[2] = {f32x16{}, f32x16{}};
    auto mfmas = [&](int buf) {
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Bs[buf][swz128(wn + r, 2 * s + h)]);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(&As[buf][swz128(wm + 32 * i + r, 2 * s + h)]);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
            }
        }
    };
    if (ke > kb) {
        load(kb, ra2[0], rbw2[0]);
        load(kb + BK, ra2[1], rbw2[1]);
        store(0, ra2[0], rbw2[0]);
    }
    __syncthreads();
    // step k: LDS buffer k & 1 holds slice k, register set (k + 1) & 1 slice k + 1 (in flight)
    for (int k0 = kb; k0 < ke; k0 += 2 * BK) {
        load(k0 + 2 * BK, ra2[0], rbw2[0]);   // past the end: all offsets out of range, zeros
        mfmas(0);
        if (k0 + BK < ke) store(1, ra2[1], rbw2[1]);
        __syncthreads();
        if (k0 + BK >= ke) break;
        load(k0 + 3 * BK, ra2[1], rbw2[1]);
        mfmas(1);
        if (k0 + 2 * BK < ke) store(0, ra2[0], rbw2[0]);
        __syncthreads();
    }
    if (split) {   // fp32 partial tile [row][Ncols] of K part z (rows / columns outside: dropped)
        const int n = n0 + wn + r;
        const __amdgpu_buffer_rsrc_t rs_s = buf_rsrc(gs.slab + (long)z * g.M * g.Ncols, g.M * g.Ncols * 4);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const long m = m0 + wm + 32 * i + crow(reg, h);
                const unsigned off = (n < g.Ncols && m < g.M) ? (unsigned)((m * g.Ncols + n) * 4) : kOOB;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][reg]), rs_s, off, 0, 0);
            }
        return;
    }
    // output pixel byte offsets of the BM rows (32-bit: launch_ig bounds the output to 2 GiB)
    for (int i = threadIdx.x; i < BM; i += NT) {
        const long m = m0 + i;
        unsigned o = kOOB;
        if (m < g.M) {
            const unsigned mu = (unsigned)m, t = mu / (unsigned)g.RW;
            const int rx = (int)(mu - t * (unsigned)g.RW);
            const unsigned b = t / (unsigned)g.RH;
            const int ry = (int)(t - b * (unsigned)g.RH);
            o = (unsigned)(((int)b * g.OHo + ry * g.oya + g.oyb) * g.OWo + rx * g.oxa + g.oxb);
        }
        ooff[i] = o;   // output pixel index (obyte maps it to out / out2)
    }
    __syncthreads();
    // branch-free epilogue: raw buffer stores, rows outside the problem / columns past N dropped by
    // the out-of-range offset.  acc[i][reg] = D[pixel wm + 32i + crow(reg, h)][feature wn + r]: per
    // store instruction 32 consecutive features of 2 rows (64-B segments).  Measured faster here than
    // 8-B feature-quad stores or an LDS-staged row-contiguous tile (profiles/r03v_conv_probe*.txt).
    const int n = n0 + wn + r;
    const bool nv = n < g.Ncols;
    const float bv = (bias && nv) ? bias[n] : 0.f;
    const long npix = (long)g.B * g.OHo * g.OWo;
    const __amdgpu_buffer_rsrc_t rs_o = buf_rsrc(out, npix * (g.nsplit ? g.nsplit : g.Ncols) * 2);
    const __amdgpu_buffer_rsrc_t rs_o2 = buf_rsrc(g.out2, g.nsplit ? npix * (g.Ncols - g.nsplit) * 2 : 0);
    const bool sec = g.nsplit && n >= g.nsplit;   // lanes may straddle nsplit: one store per destination
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const unsigned off = nv ? obyte(g, ooff[wm + 32 * i + crow(reg, h)], n) : kOOB;
            const unsigned short v = __builtin_bit_cast(unsigned short, (bf16)(acc[i][reg] + bv));
            __builtin_amdgcn_raw_buffer_store_b16(v, rs_o, sec ? kOOB : off, 0, 0);
            if (g.nsplit) __builtin_amdgcn_raw_buffer_store_b16(v, rs_o2, sec ? off : kOOB, 0, 0);
        }
}

// out = bf16(sum of the K parts' fp32 partials (fixed order) + bias), 4 columns per thread, the output
// pixel of each row as in igemm_bf16's epilogue (one problem, one destination; Ncols % 4 == 0)
__global__ __launch_bounds__(NT) void conv_split_reduce(IG g, int ksplit, const float* __restrict__ slab,
                                                        const float* __restrict__ bias, bf16* __restrict__ out) {
    const int nq = g.Ncols / 4;
    const long i = (long)blockIdx.x * NT + threadIdx.x;
    if (i >= g.M * nq) return;
    const long m = i / nq;
    const int n = (int)(i - m * nq) * 4;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) load4(bias + n, v);
    const long ms = (long)g.M * g.Ncols;
    f32x4 sum = *reinterpret_cast<const f32x4*>(slab + m * g.Ncols + n);
    for (int k = 1; k < ksplit; ++k) sum += *reinterpret_cast<const f32x4*>(slab + k * ms + m * g.Ncols + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += sum[e];
    const unsigned mu = (unsigned)m, t = mu / (unsigned)g.RW;
    const int rx = (int)(mu - t * (unsigned)g.RW);
    const unsigned b = t / (unsigned)g.RH;
    const int ry = (int)(t - b * (unsigned)g.RH);
    const long opix = ((long)b * g.OHo + ry * g.oya + g.oyb) * g.OWo + rx * g.oxa + g.oxb;
    store4(out + opix * g.Ncols + n, v);
}

// K split of a one-problem v2 launch: fewer than two workgroups per CU of tiles and >= 4 K slices ->
// parts of >= 2 slices, up to 8, so that the launch has about three workgroups per CU (1: no split)
struct KSplit {
    int ksplit, kper;
};
KSplit ksplit_plan(const IG& g, int cus) {
    const bool narrow = g.Ncols <= 32;
    const int BM = narrow ? 256 : 128, BN = narrow ? 32 : 64, BK = 64;
    const long tiles = ((g.M + BM - 1) / BM) * ((g.Ncols + BN - 1) / BN);
    const int nk = (g.Kd + BK - 1) / BK;
    // profiles/r06f_conv_probe.txt: pays for the CARAFE encoders' 32 / 128-tile forwards (26.5 -> 12.5,
    // 17.6 -> 14.9 us) and the 64-tile input gradient (15.4 -> 13.0), loses at 128 tiles of 6 slices
    if (g.csplit || g.nsplit || g.Ncols % 4 || tiles >= cus || (2 * tiles >= cus && nk < 8) || nk < 4) return KSplit{1, g.Kd};
    long want = (3L * cus + tiles - 1) / tiles;
    want = want < nk / 2 ? want : nk / 2;
    want = want < 8 ? want : 8;
    if (want < 2) return KSplit{1, g.Kd};
    const int kper = (int)((nk + want - 1) / want) * BK;
    const int n = (g.Kd + kper - 1) / kper;
    // the partials' round trip (2 x n x M x Ncols x 4 bytes) must stay small next to the work saved
    if ((long)n * g.M * g.Ncols * 4 > (32L << 20)) return KSplit{1, g.Kd};
    return KSplit{n, kper};
}
size_t ksplit_bytes(const IG& g, int cus) {
    const KSplit k = ksplit_plan(g, cus);
    return k.ksplit > 1 ? (size_t)k.ksplit * g.M * g.Ncols * 4 : 0;
}

// ---- bf16 implicit GEMM, v3 (Cs % 64 == 0, Ncols % BN == 0): persistent, LDS-DMA gathers ---------
// Both operand images are filled by buffer_load ... lds (no VGPR round trip, lds_dma.hpp): the
// A-image lanes gather their own 16 B (one pixel, one tap, 8 channels) through a per-lane offset --
// taps outside the image get an out-of-range offset and land as zeros -- and the weight image is a
// [BN][64] slice of the OHWI / IHWO matrix.  A 64-deep K slice lies inside one tap (Cs % 64 == 0), so
// the tap, the weight column and the validity of each row are per-slice scalars / per-lane selects.
// Workgroups are persistent and walk their tiles' K slices as one stream of units through an
// S-stage ring (the scheme of gemm4.hip): the gathers of the next tile overlap the last slices and
// the epilogue of the current one.  Tiles of one XCD are a contiguous range (xcd order), so the
// halo rows a 3x3 tap re-reads and the A panel shared by the N tiles stay in that XCD's L2.
// Accumulators hold [features][pixels] (the weight fragment is the MFMA A operand): lane (r, h) owns
// pixel r and features 8g + 4h .. + 3, written as 8-B vectors straight from registers.
constexpr int kIDMaxN = 1024;   // output columns of the LDS bias copy
template <int BM, int BN, int S, int WM, int WN, int OCC = 1>
__global__ __launch_bounds__(64 * WM * WN, OCC) void igemm_dma(IG g, const bf16* __restrict__ src, const bf16* __restrict__ Bw,
                                                             const float* __restrict__ bias, bf16* __restrict__ out) {
    constexpr int NWV = WM * WN;
    constexpr int TMW = BM / (32 * WM), TNW = BN / (32 * WN);   // 32x32 tiles per wave (pixels, features)
    constexpr int BK = 64;
    constexpr int STAGE = (BM + BN) * BK;                       // bf16 elements per ring stage
    constexpr int NA = BM / (8 * NWV), NB = BN / (8 * NWV);     // DMA instructions per wave per unit
    constexpr int D = NA + NB;
    constexpr int P = S - 1;
    constexpr int ST = TMW * TNW * 4;                           // epilogue stores per wave per tile
    static_assert(NA >= 1 && NB >= 1 && TMW >= 1 && TNW >= 1, "igemm_dma wave layout");
    __shared__ __attribute__((aligned(1024))) bf16 smem[S * STAGE];
    __shared__ __attribute__((aligned(16))) float sbias[kIDMaxN];
    const unsigned nbn = (unsigned)(g.Ncols / BN);
    const unsigned T = (unsigned)((g.M + BM - 1) / BM) * nbn;
    const unsigned x = blockIdx.x % kXcds, kk = blockIdx.x / kXcds, nloc = gridDim.x / kXcds;
    const unsigned q = T / kXcds, rem = T % kXcds;
    const unsigned lo = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    const unsigned cnt = q + (x < rem ? 1 : 0);
    const int mytiles = kk < cnt ? (int)((cnt - kk + nloc - 1) / nloc) : 0;
    if (mytiles == 0) return;
    const int nk = g.Kd / BK;
    const int U = mytiles * nk;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int wm = (wave / WN) * (BM / WM), wn = (wave % WN) * (BN / WN);
    // every output column's bias, once per workgroup (zeros without bias); vmcnt(0) here is before
    // the first DMA, and the first wait_unit's barrier publishes the LDS copy
    for (int n = threadIdx.x; n < g.Ncols; n += 64 * NWV) sbias[n] = bias ? bias[n] : 0.f;
    vmwait<0>();

    // DMA instruction i of this wave fills image rows (wave * N + i) * 8 .. + 7; lane l row + l / 8,
    // 16-B chunk position l & 7 holding source chunk (l & 7) ^ (row & 7) (XOR swizzle, g4 layout)
    unsigned achan[NA], voffW[NB];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int row = (wave * NA + i) * 8 + (lane >> 3);
        achan[i] = (unsigned)(((lane & 7) ^ (row & 7)) << 4);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int row = (wave * NB + i) * 8 + (lane >> 3);
        voffW[i] = (unsigned)row * g.ldw * 2 + (unsigned)(((lane & 7) ^ (row & 7)) << 4);
    }
    // gather bases of the lane's A rows for the tile being prefetched
    int arb[NA], ary[NA], arx[NA];
    unsigned ptile = 0xffffffffu;
    auto bases = [&](unsigned tile) {
        const long m0 = (long)(tile / nbn) * BM;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const long m = m0 + (wave * NA + i) * 8 + (lane >> 3);
            const bool mv = m < g.M;   // branch-free: rows past the end get a never-valid y
            const unsigned mu = (unsigned)(mv ? m : 0), t = mu / (unsigned)g.RW;   // 32-bit (check_geo)
            const int rx = (int)(mu - t * (unsigned)g.RW);
            const unsigned b = t / (unsigned)g.RH;
            const int ry = (int)(t - b * (unsigned)g.RH);
            arb[i] = (int)b * g.Hs;
            ary[i] = mv ? ry * g.ay + g.by : -(1 << 29);
            arx[i] = rx * g.ax + g.bx;
        }
    };
    const i32x4 rsA = rsrc4(src, (long)g.B * g.Hs * g.Ws * (g.csplit ? g.csplit : g.Cs) * 2);
    const i32x4 rsA2 = rsrc4(g.src2, g.csplit ? (long)g.B * g.Hs * g.Ws * (g.Cs - g.csplit) * 2 : 0);
    auto issue = [&](int u) {   // DMA of unit min(u, U - 1) into stage u % S
        const int uu = u < U ? u : U - 1;
        const unsigned tile = lo + kk + (unsigned)(uu / nk) * nloc;
        if (tile != ptile) {
            bases(tile);
            ptile = tile;
        }
        const int k0 = (uu % nk) * BK;
        const int t = k0 / g.Cs, c0 = k0 - t * g.Cs;
        const int ty = t / g.ntx, tx = t - ty * g.ntx;
        const int oy = ty * g.sty, ox = tx * g.stx;
        const int wcol = ((ty * g.wty + g.w0y) * g.KWf + tx * g.wtx + g.w0x) * g.Cs + c0;
        const CSel sl = csel(g, c0);
        unsigned va[NA];
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int y = ary[i] + oy, xx = arx[i] + ox;
            const bool ok = y >= 0 && y < g.Hs && xx >= 0 && xx < g.Ws;
            va[i] = ok ? (unsigned)((((arb[i] + y) * g.Ws + xx) * sl.stride + sl.c) * 2) + achan[i] : kOOB;
        }
        bf16* stg = smem + (u % S) * STAGE;
        dma<NA>(sl.second ? rsA2 : rsA, va, 0u, stg, wave);
        const long rw = (long)(tile % nbn) * BN;
        dma<NB>(rsrc4(Bw + rw * g.ldw, (long)(g.Ncols - rw) * g.ldw * 2), voffW, (unsigned)wcol * 2u, stg + BM * BK, wave);
    };
    auto wait_unit = [&](int u) {   // vector-memory ops issued after unit u's DMA (issued at step u - P)
        const int w = u - P;
        int c = (w >= 0 && w % nk == nk - 1) ? ST : 0;
        for (int v = w + 1; v < u; ++v) c += D + ((v >= 0 && v % nk == nk - 1) ? ST : 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        switch (c >= 63 ? 7 : c >> 3) {   // vmcnt(largest multiple of 8 <= c): waiting for more is safe
            case 0: vmwait<0>(); break;
            case 1: vmwait<8>(); break;
            case 2: vmwait<16>(); break;
            case 3: vmwait<24>(); break;
            case 4: vmwait<32>(); break;
            case 5: vmwait<40>(); break;
            case 6: vmwait<48>(); break;
            default: vmwait<56>(); break;
        }
        __builtin_amdgcn_s_barrier();   // unit u landed for every wave; stage (u - 1) % S is free
        __builtin_amdgcn_sched_barrier(0);
    };
    f32x16 acc[TMW][TNW];
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = f32x16{};
    auto mma = [&](int u) {
        const bf16* As = smem + (u % S) * STAGE;
        const bf16* Ws = As + BM * BK;
        bf16x8 af[2][TMW], wf[2][TNW];   // fragments of k-step s + 1 read while step s multiplies
        auto frags = [&](int s, int b) {
#pragma unroll
            for (int i = 0; i < TMW; ++i) af[b][i] = *reinterpret_cast<const bf16x8*>(As + swz128(wm + 32 * i + r, 2 * s + h));
#pragma unroll
            for (int j = 0; j < TNW; ++j) wf[b][j] = *reinterpret_cast<const bf16x8*>(Ws + swz128(wn + 32 * j + r, 2 * s + h));
        };
        frags(0, 0);
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            if (s + 1 < BK / 16) frags(s + 1, (s + 1) & 1);
#pragma unroll
            for (int i = 0; i < TMW; ++i)
#pragma unroll
                for (int j = 0; j < TNW; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s & 1][j], af[s & 1][i], acc[i][j], 0, 0, 0);
        }
    };
    const long npix = (long)g.B * g.OHo * g.OWo;
    const __amdgpu_buffer_rsrc_t rs_o = buf_rsrc(out, npix * (g.nsplit ? g.nsplit : g.Ncols) * 2);
    const __amdgpu_buffer_rsrc_t rs_o2 = buf_rsrc(g.out2, g.nsplit ? npix * (g.Ncols - g.nsplit) * 2 : 0);

#pragma unroll
    for (int p = 0; p < P; ++p) issue(p);
    int u = 0;
    for (int t = 0; t < mytiles; ++t) {
        for (int ks = 0; ks + 1 < nk; ++ks, ++u) {   // all but the tile's last K slice
            wait_unit(u);
            issue(u + P);
            mma(u);
        }
        wait_unit(u);
        const unsigned tile = lo + kk + (unsigned)t * nloc;
        const long m0 = (long)(tile / nbn) * BM;
        const int n0 = (int)(tile % nbn) * BN;
        unsigned orow[TMW];   // output pixel of rows wm + 32 i + r (kOOB: none)
#pragma unroll
        for (int i = 0; i < TMW; ++i) {
            const long m = m0 + wm + 32 * i + r;
            const bool mv = m < g.M;
            const unsigned mu = (unsigned)(mv ? m : 0), tq = mu / (unsigned)g.RW;
            const int rx = (int)(mu - tq * (unsigned)g.RW);
            const unsigned b = tq / (unsigned)g.RH;
            const int ry = (int)(tq - b * (unsigned)g.RH);
            const unsigned o = (unsigned)(((int)b * g.OHo + ry * g.oya + g.oyb) * g.OWo + rx * g.oxa + g.oxb);
            orow[i] = mv ? o : kOOB;
        }
        issue(u + P);
        mma(u);
        // bias from the LDS copy (lgkmcnt: the vmcnt accounting of the ring is untouched)
#pragma unroll
        for (int j = 0; j < TNW; ++j)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int nf = n0 + wn + 32 * j + 8 * gq + 4 * h;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + nf);
                const bool o2 = g.nsplit && n0 + wn + 32 * j + 8 * gq >= g.nsplit;   // nsplit % 8 == 0: uniform
#pragma unroll
                for (int i = 0; i < TMW; ++i) {
                    const float v[4] = {acc[i][j][4 * gq] + bv[0], acc[i][j][4 * gq + 1] + bv[1], acc[i][j][4 * gq + 2] + bv[2],
                                        acc[i][j][4 * gq + 3] + bv[3]};
                    buf_st4bf(o2 ? rs_o2 : rs_o, obyte(g, orow[i], nf), v);
                }
            }
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
            for (int j = 0; j < TNW; ++j) acc[i][j] = f32x16{};
        ++u;
    }
    vmwait<0>();   // drain the re-fetch DMAs before the workgroup's LDS is released
}

// ---- bf16 3x3 / stride 1 / pad 1 conv with 64 gathered and 64 output channels, halo form ----------
// (the UNet level-1 DoubleConv convs and their input gradients, unet:182-187: 64 -> 64 at full
// resolution).  Persistent workgroups own the whole 9 x 64 x 64 weight slab in LDS (loaded once) and
// walk items of two output rows x 64 pixels: per item the four input rows under them (66-pixel halo
// images, 64 channels) are staged once through a 2-stage ring and read by all 9 taps at row offsets
// (tap ky from halo row rr + ky, tap kx at pixel offset kx) -- 4 x 66 staged rows per 128 output
// pixels instead of 9 x 128 gathered ones.  8 waves: wave (rr, pixel half, n tile).  flip: the
// input gradient (IHWO weights, tap (ky, kx) = weight tap (2 - ky, 2 - kx)).
template <bool FLIP>
__global__ __launch_bounds__(512, 1) void conv3_halo64(int B, int H, int W, const bf16* __restrict__ src, const bf16* __restrict__ wt,
                                                       const float* __restrict__ bias, bf16* __restrict__ out) {
    constexpr int XIMG = kHaloRows * 64;    // bf16 per halo image (72 rows x 64 channels)
    constexpr int NBLK = 4 * XIMG * 2 / 1024;   // 36 DMA blocks per item
    constexpr int NI = (NBLK + 7) / 8;      // per wave (5)
    constexpr int STAGE = NI * 8 * 512;     // bf16 per ring stage (40 blocks)
    constexpr int WIMG = 64 * 64;           // bf16 per tap weight image [n][c]
    __shared__ __attribute__((aligned(1024))) bf16 wsm[9 * WIMG];
    __shared__ __attribute__((aligned(1024))) bf16 ring[2 * STAGE];
    __shared__ float sbias[64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;
    const int nt = wave & 1, ph = (wave >> 1) & 1, rr = wave >> 2;
    const int spr = W / 64, prs = H / 2;    // segments per row, row pairs per image
    const long items = (long)B * prs * spr;
    // this workgroup's items: a contiguous range per XCD, strided by the XCD's workgroups
    const long x = blockIdx.x % kXcds, kk = blockIdx.x / kXcds, nloc = gridDim.x / kXcds;
    const long q = items / kXcds, rem = items % kXcds;
    const long lo = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    const long cnt = q + (x < rem ? 1 : 0);
    const int my = kk < cnt ? (int)((cnt - kk + nloc - 1) / nloc) : 0;
    if (my == 0) return;
    if (threadIdx.x < 64) sbias[threadIdx.x] = bias ? bias[threadIdx.x] : 0.f;
    // weight slab: tap image t rows n, columns c (OHWI [n][t][c], or IHWO [c'][t'][n'] with t' = 8 - t)
    {
        const i32x4 rw = rsrc4(wt, 64L * 9 * 64 * 2);
#pragma unroll
        for (int i = 0; i < 9; ++i) {   // 72 blocks: 9 per wave
            const int j = wave * 9 + i, t = j / 8, row = (j % 8) * 8 + (lane >> 3);
            const int tw = FLIP ? 8 - t : t;
            const unsigned off = (unsigned)((row * 9 + tw) * 64 + 8 * ((lane & 7) ^ mkey<128>(row))) * 2u;
            dma1_u(rw, off, 0u, wsm + j * 512);
        }
    }
    const i32x4 rs = rsrc4(src, (long)B * H * W * 64 * 2);
    auto issue = [&](int u) {   // halo images of item lo + kk + u * nloc (past the last: zeros)
        const long it = lo + kk + (long)(u < my ? u : my - 1) * nloc;
        const bool iv = u < my;
        const long t1 = it / spr;
        const int ox0 = (int)(it - t1 * spr) * 64;
        const int b = (int)(t1 / prs), oy0 = (int)(t1 - (long)b * prs) * 2;
        bf16* stg = ring + (u & 1) * STAGE;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int j = wave * NI + i;
            const int img = j / 9, row = (j % 9) * 8 + (lane >> 3);
            const int iy = oy0 + img - 1, ix = ox0 - 1 + row;
            const bool ok = iv && j < NBLK && row < 66 && iy >= 0 && iy < H && ix >= 0 && ix < W;
            const unsigned off = ok ? (unsigned)(((((long)b * H + iy) * W + ix) * 64 + 8 * ((lane & 7) ^ mkey<128>(row))) * 2) : kOOB;
            dma1_u(rs, off, 0u, stg + j * 512);
        }
    };
    const __amdgpu_buffer_rsrc_t rso = buf_rsrc(out, (long)B * H * W * 64 * 2);
    issue(0);
    for (int u = 0; u < my; ++u) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (u == 0) vmwait<0>(); else vmwait<4>();   // item u landed (after its DMA: item u-1's 4 stores)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue(u + 1);
        const bf16* st = ring + (u & 1) * STAGE;
        f32x16 acc = f32x16{};
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const bf16* himg = st + (rr + ky) * XIMG;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const bf16* wimg = wsm + (ky * 3 + kx) * WIMG;
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) {
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(wimg + moff<128>(nt * 32 + r, 16 * s2 + 8 * h));
                    const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(himg + moff<128>(ph * 32 + r + kx, 16 * s2 + 8 * h));
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bfr, acc, 0, 0, 0);
                }
            }
        }
        // acc[4g + e] = out[pixel ph * 32 + r of row rr][n = nt * 32 + 8g + 4h + e]
        const long it = lo + kk + (long)u * nloc;
        const long t1 = it / spr;
        const int ox0 = (int)(it - t1 * spr) * 64;
        const int b = (int)(t1 / prs), oy = (int)(t1 - (long)b * prs) * 2 + rr;
        const unsigned pix = (unsigned)(((long)b * H + oy) * W + ox0 + ph * 32 + r);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int n = nt * 32 + 8 * g + 4 * h;
            const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + n);
            const float v[4] = {acc[4 * g] + bv[0], acc[4 * g + 1] + bv[1], acc[4 * g + 2] + bv[2], acc[4 * g + 3] + bv[3]};
            buf_st4bf(rso, (pix * 64u + (unsigned)n) * 2u, v);
        }
    }
    vmwait<0>();
}


// ---- few-channel 3x3 / stride 1 / pad 1 forward conv, 16 input channels, N outputs (N % 16 == 0):
// the CARAFE4 encoder Conv2d(16, 144, 3, 1, 1) (cswin:446) at 128 x 128 / 256 x 256 ----------------
// The generic implicit GEMM gathers the 16-channel input per tap into 64-deep K slices (a quarter of a
// slice per tap) and tiles N = 144 as 3 x 64; its time was ~7x the 75 MB the 144-channel output is.
// Here every wave holds the whole weight matrix as MFMA A fragments in registers (N x 160 k, k = tap *
// 16 + c, tap 9 zero: 45 fragments of v_mfma_f32_16x16x32_bf16), the workgroup walks 64-pixel row
// segments whose three 66-pixel input halo rows ([3][66][16] bf16, 7 DMA blocks) are fetched one item
// ahead (2 stages), wave w computes pixels 16 w .. 16 w + 15 x all N outputs (k-step = two taps x 16
// channels, 5 steps), and the 16 x N output tile goes through a wave-private LDS region so every
// pixel's N outputs leave as contiguous 16-B stores.  2 workgroups per CU.
template <int N>
__global__ __launch_bounds__(256, 2) void conv3_c16(int B, int H, int W, const bf16* __restrict__ src, const bf16* __restrict__ w_ohwi,
                                                    const float* __restrict__ bias, bf16* __restrict__ out) {
    constexpr int NT16 = N / 16;                 // 16-output tiles
    constexpr int HALO = 3 * 66 * 16;            // bf16 of a stage's halo image
    constexpr int STAGE = 7 * 512;               // bf16 per stage (7 DMA blocks of 1 KB)
    constexpr int EST = N + 8;                   // epilogue row stride (bf16)
    constexpr int NST = (16 * N / 8 + 63) / 64;  // 16-B stores per lane per segment
    static_assert(HALO <= STAGE, "halo image exceeds its stage");
    __shared__ __attribute__((aligned(1024))) bf16 ring[2 * STAGE];
    __shared__ __attribute__((aligned(16))) bf16 ep[4][16 * EST];
    __shared__ __attribute__((aligned(16))) float sbias[N];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int spr = W / 64;
    const long items = (long)B * H * spr;
    const long x = blockIdx.x % kXcds, kk = blockIdx.x / kXcds, nloc = gridDim.x / kXcds;
    const long q = items / kXcds, rem = items % kXcds;
    const long lo = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    const long cnt = q + (x < rem ? 1 : 0);
    const int my = kk < cnt ? (int)((cnt - kk + nloc - 1) / nloc) : 0;
    if (my == 0) return;
    const int l16 = lane & 15, kg = lane >> 4;
    // the weights as A fragments: lane (n = 16 t + l16, k-group kg) of k-step s = W[n][32 s + 8 kg .. + 7]
    // (OHWI [n][tap][c] = [n][k]; k >= 144 zero)
    bf16x8 aw[5][NT16];
    {
        const __amdgpu_buffer_rsrc_t rw = buf_rsrc(w_ohwi, (long)N * 144 * 2);
#pragma unroll
        for (int s2 = 0; s2 < 5; ++s2)
#pragma unroll
            for (int t = 0; t < NT16; ++t) {
                const int k = 32 * s2 + 8 * kg;
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, k < 144 ? (unsigned)(((16 * t + l16) * 144 + k) * 2) : kOOB, 0, 0);
                __builtin_memcpy(&aw[s2][t], &v, 16);
            }
    }
    for (int i = threadIdx.x; i < N; i += 256) sbias[i] = bias ? bias[i] : 0.f;
    const i32x4 rs = rsrc4(src, (long)B * H * W * 16 * 2);
    auto issue = [&](int u) {   // the 3 x 66-pixel halo of item lo + kk + u * nloc: blocks of 32 pixels
        const long it = lo + kk + (long)(u < my ? u : my - 1) * nloc;
        const bool iv = u < my;
        const long t1 = it / spr;
        const int ox0 = (int)(it - t1 * spr) * 64;
        const int b = (int)(t1 / H), oy = (int)(t1 - (long)b * H);
        bf16* stg = ring + (u & 1) * STAGE;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int j = wave * 2 + i;              // block j: halo pixels 32 j .. 32 j + 31 of [3][66]
            if (j < 7) {
                const int p = 32 * j + (lane >> 1), ky = p / 66, px = p - 66 * ky;
                const int iy = oy + ky - 1, ix = ox0 - 1 + px;
                const bool ok = iv && p < 3 * 66 && iy >= 0 && iy < H && ix >= 0 && ix < W;
                const unsigned off = ok ? (unsigned)(((((long)b * H + iy) * W + ix) * 16 + 8 * (lane & 1)) * 2) : kOOB;
                dma1_u(rs, off, 0u, stg + j * 512);
            }
        }
    };
    const __amdgpu_buffer_rsrc_t rso = buf_rsrc(out, (long)B * H * W * N * 2);
    issue(0);
    __syncthreads();   // bias in LDS
    for (int u = 0; u < my; ++u) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (u == 0) vmwait<0>(); else vmwait<NST>();   // item u landed (younger: item u-1's stores)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue(u + 1);
        const bf16* st = ring + (u & 1) * STAGE;
        f32x4 acc[NT16];
#pragma unroll
        for (int t = 0; t < NT16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 5; ++s2) {
            const int tap = 2 * s2 + (kg >> 1), tp = tap < 9 ? tap : 8;   // tap 9: zero weights (finite operand)
            const int ky = tp / 3, kx = tp % 3;
            const bf16x8 bx = *reinterpret_cast<const bf16x8*>(st + (ky * 66 + 16 * wave + l16 + kx) * 16 + 8 * (kg & 1));
#pragma unroll
            for (int t = 0; t < NT16; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s2][t], bx, acc[t], 0, 0, 0);
        }
        // acc[t][i] = out[pixel 16 wave + l16][n = 16 t + 4 kg + i]
        bf16* e = ep[wave];
#pragma unroll
        for (int t = 0; t < NT16; ++t) {
            const int n = 16 * t + 4 * kg;
            const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + n);
            const bf16x4 v = {(bf16)(acc[t][0] + bv[0]), (bf16)(acc[t][1] + bv[1]), (bf16)(acc[t][2] + bv[2]), (bf16)(acc[t][3] + bv[3])};
            *reinterpret_cast<bf16x4*>(e + l16 * EST + n) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's own LDS writes before its reads
        const long it = lo + kk + (long)u * nloc;
        const long t1 = it / spr;
        const int ox0 = (int)(it - t1 * spr) * 64;
        const long pix0 = t1 * W + ox0 + 16 * wave;             // (b * H + oy) * W + ox
#pragma unroll
        for (int k = 0; k < NST; ++k) {
            const int c = lane + 64 * k;                         // 16-B chunk: pixel c / (N / 8), chunk c % (N / 8)
            const int pp = c / (N / 8), ch = c % (N / 8);
            const bool ok = c < 16 * N / 8;
            u32x4 v = {};
            if (ok) v = *reinterpret_cast<const u32x4*>(e + pp * EST + 8 * ch);
            __builtin_amdgcn_raw_buffer_store_b128(v, rso, ok ? (unsigned)(((pix0 + pp) * N + 8 * ch) * 2) : kOOB, 0, 0);
        }
    }
    vmwait<0>();
}

bool c16_ok(const IG& g) {   // the forward 3x3 / stride 1 / pad 1 conv of a 16-channel input, N <= 144
    return g.Cs == 16 && g.Ncols == 144 && g.nty == 3 && g.ntx == 3 && g.csplit == 0 && g.nsplit == 0 && g.OHo == g.Hs &&
           g.OWo == g.Ws && g.Ws % 64 == 0 && g.RH == g.Hs && g.RW == g.Ws && g.sty == 1 && g.stx == 1 && g.ay == 1 &&
           g.ax == 1 && g.by == -1 && g.bx == -1;
}


// ---- its input gradient: 144 -> 16 channels, dx[p][c] = sum_{tap, n} dy[p + 1 - tap][n] W[n][tap][c] ----
// Same scheme with the roles of the channel counts swapped: the weights (IHWO [c][tap][n]) are the
// register-resident A fragments (16 rows c x 9 taps x 160 n, n >= 144 zero: 45 k-steps of 16x16x32),
// the 3 x 66-pixel halo of dy (144 channels, pixel stride 304 B = 19 16-B chunks, the 19th zero) is
// DMA'd one segment ahead, and wave w's 16 pixels x 16 channels leave as one contiguous 512-B store
// per wave instruction (lane (pixel, 4-channel group)).  One workgroup per CU (2 x 60 KB halo stages).
__global__ __launch_bounds__(256, 1) void conv3_c16d(int B, int H, int W, const bf16* __restrict__ dy, const bf16* __restrict__ w_ihwo,
                                                    bf16* __restrict__ dx) {
    constexpr int N = 144, PS = 152;             // dy channels, halo pixel stride (bf16)
    constexpr int NBLK = (3 * 66 * PS * 2 + 1023) / 1024;   // DMA blocks per stage (59)
    constexpr int STAGE = NBLK * 512;            // bf16 per stage
    constexpr int NI = (NBLK + 3) / 4;           // per wave
    __shared__ __attribute__((aligned(1024))) bf16 ring[2 * STAGE];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int spr = W / 64;
    const long items = (long)B * H * spr;
    const long x = blockIdx.x % kXcds, kk = blockIdx.x / kXcds, nloc = gridDim.x / kXcds;
    const long q = items / kXcds, rem = items % kXcds;
    const long lo = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    const long cnt = q + (x < rem ? 1 : 0);
    const int my = kk < cnt ? (int)((cnt - kk + nloc - 1) / nloc) : 0;
    if (my == 0) return;
    const int l16 = lane & 15, kg = lane >> 4;
    // A fragments: lane (c = l16, kg) of k-step (tap, chunk j) = Wi[c][tap][32 j + 8 kg .. + 7]
    bf16x8 aw[9][5];
    {
        const __amdgpu_buffer_rsrc_t rw = buf_rsrc(w_ihwo, 16L * 9 * N * 2);
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const int n = 32 * j + 8 * kg;
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rw, n < N ? (unsigned)(((l16 * 9 + t) * N + n) * 2) : kOOB, 0, 0);
                __builtin_memcpy(&aw[t][j], &v, 16);
            }
    }
    const i32x4 rs = rsrc4(dy, (long)B * H * W * N * 2);
    auto issue = [&](int u) {   // dy rows oy - 1 .. oy + 1, pixels ox0 - 1 .. ox0 + 64 of item u
        const long it = lo + kk + (long)(u < my ? u : my - 1) * nloc;
        const bool iv = u < my;
        const long t1 = it / spr;
        const int ox0 = (int)(it - t1 * spr) * 64;
        const int b = (int)(t1 / H), oy = (int)(t1 - (long)b * H);
        bf16* stg = ring + (u & 1) * STAGE;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int j = wave * NI + i;
            if (j < NBLK) {
                const int byte = 1024 * j + 16 * lane;
                const int P = byte / (2 * PS), chunk = (byte - P * 2 * PS) >> 4;
                const int ky = P / 66, px = P - 66 * ky;
                const int iy = oy + ky - 1, ix = ox0 - 1 + px;
                const bool ok = iv && P < 3 * 66 && chunk < N / 8 && iy >= 0 && iy < H && ix >= 0 && ix < W;
                const unsigned off = ok ? (unsigned)(((((long)b * H + iy) * W + ix) * N + 8 * chunk) * 2) : kOOB;
                dma1_u(rs, off, 0u, stg + j * 512);
            }
        }
    };
    const __amdgpu_buffer_rsrc_t rso = buf_rsrc(dx, (long)B * H * W * 16 * 2);
    issue(0);
    for (int u = 0; u < my; ++u) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (u == 0) vmwait<0>(); else vmwait<1>();   // item u landed (younger: item u-1's store)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue(u + 1);
        const bf16* st = ring + (u & 1) * STAGE;
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // two independent chains
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ky = t / 3, kx = t % 3;
            const bf16* row = st + ((2 - ky) * 66 + 16 * wave + l16 + 2 - kx) * PS;
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const int n = 32 * j + 8 * kg;
                const bf16x8 bx = *reinterpret_cast<const bf16x8*>(row + (n < N ? n : n - 16));   // n >= 144: zero weights
                acc[(t * 5 + j) & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[t][j], bx, acc[(t * 5 + j) & 1], 0, 0, 0);
            }
        }
        // acc[i] = dx[pixel 16 wave + l16][c = 4 kg + i]
        const long it = lo + kk + (long)u * nloc;
        const long t1 = it / spr;
        const int ox0 = (int)(it - t1 * spr) * 64;
        const long pix = t1 * W + ox0 + 16 * wave + l16;
        const float v[4] = {acc[0][0] + acc[1][0], acc[0][1] + acc[1][1], acc[0][2] + acc[1][2], acc[0][3] + acc[1][3]};
        buf_st4bf(rso, (unsigned)((pix * 16 + 4 * kg) * 2), v);
    }
    vmwait<0>();
}

bool c16d_ok(const IG& g) {   // the input gradient (flipped taps) of the 16 -> 144 3x3 stride-1 conv
    return g.Cs == 144 && g.Ncols == 16 && g.nty == 3 && g.ntx == 3 && g.csplit == 0 && g.nsplit == 0 && g.OHo == g.Hs &&
           g.OWo == g.Ws && g.Ws % 64 == 0 && g.RH == g.Hs && g.RW == g.Ws && g.sty == -1 && g.stx == -1 && g.by == 1 &&
           g.bx == 1 && g.wty == 1 && g.wtx == 1;
}

constexpr int kHalo64Cfg = 20;   // csu_conv2d_ex cfg selecting conv3_halo64
constexpr int kC16Cfg = 21;      // csu_conv2d_ex cfg selecting conv3_c16
bool halo64_ok(const IG& g, bool flip) {   // the forward conv (flip: its input gradient) this kernel takes
    return g.Cs == 64 && g.Ncols == 64 && g.nty == 3 && g.ntx == 3 && g.csplit == 0 && g.nsplit == 0 && g.OHo == g.Hs &&
           g.OWo == g.Ws && g.Hs % 2 == 0 && g.Ws % 64 == 0 && g.RH == g.Hs && g.RW == g.Ws &&
           (flip ? (g.sty == -1 && g.stx == -1 && g.by == 1 && g.bx == 1 && g.wty == 1 && g.wtx == 1)
                 : (g.sty == 1 && g.stx == 1 && g.ay == 1 && g.ax == 1 && g.by == -1 && g.bx == -1));
}

// occ: workgroups per CU of the persistent grid (2: the small-tile configurations for few-tile shapes,
// e.g. the CSWin merges, whose 128 x 64 tiles give one tile per CU)
struct IDCfg { int bm, bn, s, wm, wn, occ; };
constexpr IDCfg kIDCfgs[] = {{128, 128, 3, 2, 2, 1}, {256, 128, 2, 4, 2, 1}, {256, 128, 3, 4, 2, 1}, {128, 64, 4, 2, 2, 1},
                             {256, 64, 3, 4, 2, 1},  {128, 64, 3, 2, 2, 1},  {256, 256, 2, 2, 4, 1}, {256, 256, 2, 4, 2, 1},
                             {512, 64, 2, 8, 1, 1},  {64, 64, 4, 2, 2, 2},   {128, 64, 3, 2, 2, 2},  {64, 128, 3, 2, 2, 2}};
constexpr int kIDNCfg = 12;

int id_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        cus = (cus + kXcds - 1) / kXcds * kXcds;
    }
    return cus;
}

template <int C>
int id_launch(const IG& g, const void* src, const void* w, const float* bias, void* out, hipStream_t st) {
    constexpr IDCfg c = kIDCfgs[C];
    if (g.Ncols % c.bn) return fail(CSU_E_ARG, "conv2d: Ncols not a multiple of the tile's BN");
    igemm_dma<c.bm, c.bn, c.s, c.wm, c.wn, c.occ><<<dim3(c.occ * id_cus()), 64 * c.wm * c.wn, 0, st>>>(
        g, (const bf16*)src, (const bf16*)w, bias, (bf16*)out);
    return check_launch("conv2d (igemm_dma)");
}

// v3 eligibility and tile choice (tools/conv_probe.py on the UNet 512x512 B16 and CSWin merge shapes,
// profiles/r03q_conv_probe.txt): 256 x 256 tiles (MFMA busy 38-41 % at C >= 256) when they still give
// every CU a tile, else 256 x 128 (25-30 %); Ncols = 64 stays on the v2 kernel, which the 64-wide v3
// tiles do not beat (the A gathers dominate: 9 taps x 64 channels per 64 outputs).  -1: v2.
bool id_eligible(const IG& g) { return g.Cs % 64 == 0 && g.Kd >= 64 && g.Ncols <= kIDMaxN; }
int id_pick(const IG& g, bool single = false) {
    if (!id_eligible(g)) return -1;
    const long mt = (g.M + 255) / 256;
    if (g.Ncols % 256 == 0 && mt * (g.Ncols / 256) >= id_cus()) return 7;
    // fewer 256 x 128 tiles than CUs (the CSWin merges at 64^2 / 32^2, the stride phases of their
    // input gradients): the v2 kernel's 4x more 128 x 64 tiles win (profiles/r03v_conv_probe*.txt) --
    // except for a one-problem launch with a CU's worth of 64 x 128 tiles, which runs them two
    // workgroups per CU (the merges' forwards: 33.9 -> 28.0 / 48.6 -> 34.9 us,
    // profiles/r06f_conv_probe.txt; the 4-phase input gradients stay on v2)
    if (g.Ncols % 128 == 0 && mt * (g.Ncols / 128) >= id_cus()) return 2;
    if (single && g.Ncols % 128 == 0 && ((g.M + 63) / 64) * (g.Ncols / 128) >= id_cus()) return 11;
    return -1;
}

int id_run(int cfg, const IG& g, const void* src, const void* w, const float* bias, void* out, hipStream_t st) {
    switch (cfg) {
        case 0: return id_launch<0>(g, src, w, bias, out, st);
        case 1: return id_launch<1>(g, src, w, bias, out, st);
        case 2: return id_launch<2>(g, src, w, bias, out, st);
        case 3: return id_launch<3>(g, src, w, bias, out, st);
        case 4: return id_launch<4>(g, src, w, bias, out, st);
        case 5: return id_launch<5>(g, src, w, bias, out, st);
        case 6: return id_launch<6>(g, src, w, bias, out, st);
        case 7: return id_launch<7>(g, src, w, bias, out, st);
        case 8: return id_launch<8>(g, src, w, bias, out, st);
        case 9: return id_launch<9>(g, src, w, bias, out, st);
        case 10: return id_launch<10>(g, src, w, bias, out, st);
        case 11: return id_launch<11>(g, src, w, bias, out, st);
        default: return fail(CSU_E_ARG, "conv2d: bad igemm_dma configuration");
    }
}

// n problems with equal Ncols and channel count (the phases of one input gradient, or one forward)
// cfg: -1 per-shape choice (v3 where eligible), 0 the v2 kernel, 1 + k the v3 configuration k
int launch_ig(const IG* gv, int n, const void* src, const void* w, const float* bias, void* out, hipStream_t st,
              int cfg = -1, float* ws = nullptr, size_t ws_bytes = 0) {
    IG4 gs{};
    long maxm = 0;
    for (int i = 0; i < n; ++i) {
        gs.g[i] = gv[i];
        maxm = gv[i].M > maxm ? gv[i].M : maxm;
    }
    const IG& g = gv[0];
    if ((long)g.B * g.Hs * g.Ws * g.Cs * 2 >= (1L << 31) || (long)g.Ncols * g.ldw * 2 >= (1L << 31) ||
        (long)g.B * g.OHo * g.OWo * g.Ncols * 2 >= (1L << 31))
        return fail(CSU_E_UNSUPPORTED, "conv2d: operand larger than 2 GiB (32-bit buffer offsets)");
    if ((cfg < 0 || cfg == kHalo64Cfg) && n == 1) {   // 64 -> 64 channel 3x3 stride-1 conv: the halo kernel
        const bool flip = g.sty == -1;
        if (halo64_ok(g, flip)) {
            if (flip) conv3_halo64<true><<<dim3(id_cus()), 512, 0, st>>>(g.B, g.Hs, g.Ws, (const bf16*)src, (const bf16*)w, bias, (bf16*)out);
            else conv3_halo64<false><<<dim3(id_cus()), 512, 0, st>>>(g.B, g.Hs, g.Ws, (const bf16*)src, (const bf16*)w, bias, (bf16*)out);
            return check_launch("conv2d (halo64)");
        }
    }
    if (cfg == kHalo64Cfg) return fail(CSU_E_ARG, "conv2d: halo64 configuration not eligible");
    if ((cfg < 0 || cfg == kC16Cfg) && n == 1 && c16_ok(g)) {   // 16 -> 144 channel 3x3 conv (CARAFE4 encoder)
        conv3_c16<144><<<dim3(2 * id_cus()), 256, 0, st>>>(g.B, g.Hs, g.Ws, (const bf16*)src, (const bf16*)w, bias, (bf16*)out);
        return check_launch("conv2d (c16)");
    }
    if ((cfg < 0 || cfg == kC16Cfg) && n == 1 && c16d_ok(g)) {   // its input gradient (144 -> 16)
        conv3_c16d<<<dim3(id_cus()), 256, 0, st>>>(g.B, g.Hs, g.Ws, (const bf16*)src, (const bf16*)w, (bf16*)out);
        return check_launch("conv2d (c16d)");
    }
    if (cfg == kC16Cfg) return fail(CSU_E_ARG, "conv2d: c16 configuration not eligible");
    if (cfg > 0) {   // forced v3 configuration: every phase must be eligible for it
        const int k = cfg - 1;
        if (k >= kIDNCfg) return fail(CSU_E_ARG, "conv2d: bad igemm_dma configuration");
        for (int i = 0; i < n; ++i)
            if (!id_eligible(gv[i]) || gv[i].Ncols % kIDCfgs[k].bn) return fail(CSU_E_ARG, "conv2d: igemm_dma configuration not eligible");
        for (int i = 0; i < n; ++i)
            if (gv[i].M > 0)
                if (int e = id_run(k, gv[i], src, w, bias, out, st)) return e;
        return 0;
    }
    if (cfg < 0) {   // per-shape choice: v3 (each phase its own tile) when every phase has one
        int pk[4];
        bool all = true;
        for (int i = 0; i < n; ++i) all = all && (pk[i] = id_pick(gv[i], n == 1)) >= 0;
        if (all) {
            for (int i = 0; i < n; ++i)
                if (gv[i].M > 0)
                    if (int e = id_run(pk[i], gv[i], src, w, bias, out, st)) return e;
            return 0;
        }
    }
    const int vw = g.Cs % 8 == 0 ? 8 : 4;
    const bool narrow = g.Ncols <= 32;
    const int BM = narrow ? 256 : 128, BN = narrow ? 32 : 64;
    const KSplit ks = n == 1 && cfg < 0 && ws ? ksplit_plan(g, id_cus()) : KSplit{1, g.Kd};
    const bool split = ks.ksplit > 1 && ws_bytes >= (size_t)ks.ksplit * g.M * g.Ncols * 4;
    gs.ksplit = split ? ks.ksplit : 1;
    gs.kper = split ? ks.kper : g.Kd;
    gs.slab = split ? ws : nullptr;
    const dim3 grid((unsigned)((maxm + BM - 1) / BM), (g.Ncols + BN - 1) / BN, split ? ks.ksplit : n);
    const bf16* s = (const bf16*)src;
    const bf16* wb = (const bf16*)w;
    bf16* o = (bf16*)out;
    if (narrow) {
        if (vw == 8) igemm_bf16<32, 8><<<grid, NT, 0, st>>>(gs, s, wb, bias, o);
        else igemm_bf16<32, 4><<<grid, NT, 0, st>>>(gs, s, wb, bias, o);
    } else {
        if (vw == 8) igemm_bf16<64, 8><<<grid, NT, 0, st>>>(gs, s, wb, bias, o);
        else igemm_bf16<64, 4><<<grid, NT, 0, st>>>(gs, s, wb, bias, o);
    }
    if (split) {
        const long nthr = g.M * (g.Ncols / 4);
        conv_split_reduce<<<(unsigned)((nthr + NT - 1) / NT), NT, 0, st>>>(g, ks.ksplit, ws, bias, o);
    }
    return check_launch("conv2d (igemm)");
}
int launch_ig(const IG& g, const void* src, const void* w, const float* bias, void* out, hipStream_t st, int cfg = -1,
              float* ws = nullptr, size_t ws_bytes = 0) {
    return launch_ig(&g, 1, src, w, bias, out, st, cfg, ws, ws_bytes);
}
IG ig_forward(const csu_conv_geom& c) {
    IG g{};
    g.Hs = c.H; g.Ws = c.W; g.Cs = c.C;
    g.RH = c.OH; g.RW = c.OW;
    g.ay = c.stride; g.by = -c.pad; g.ax = c.stride; g.bx = -c.pad;
    g.nty = c.KH; g.ntx = c.KW; g.sty = 1; g.stx = 1;
    g.ldw = c.KH * c.KW * c.C; g.KWf = c.KW; g.wty = 1; g.w0y = 0; g.wtx = 1; g.w0x = 0;
    g.OHo = c.OH; g.OWo = c.OW; g.oya = 1; g.oyb = 0; g.oxa = 1; g.oxb = 0;
    g.B = c.B; g.Ncols = c.N; g.Kd = c.KH * c.KW * c.C;
    g.M = (long)c.B * c.OH * c.OW;
    return g;
}

// phase (ry_, rx_) of the input gradient: input pixels with (iy + pad) % s == ry_, taps ky = ry_ + s*ty
IG ig_dgrad_phase(const csu_conv_geom& c, int ry_, int rx_) {
    const int s = c.stride, p = c.pad;
    const int iy0 = ((ry_ - p) % s + s) % s, ix0 = ((rx_ - p) % s + s) % s;
    IG g{};
    g.Hs = c.OH; g.Ws = c.OW; g.Cs = c.N;
    g.RH = iy0 < c.H ? (c.H - iy0 + s - 1) / s : 0;
    g.RW = ix0 < c.W ? (c.W - ix0 + s - 1) / s : 0;
    g.ay = 1; g.by = (iy0 + p - ry_) / s; g.ax = 1; g.bx = (ix0 + p - rx_) / s;
    g.nty = ry_ < c.KH ? (c.KH - ry_ + s - 1) / s : 0;
    g.ntx = rx_ < c.KW ? (c.KW - rx_ + s - 1) / s : 0;
    g.sty = -1; g.stx = -1;
    g.ldw = c.KH * c.KW * c.N; g.KWf = c.KW; g.wty = s; g.w0y = ry_; g.wtx = s; g.w0x = rx_;
    g.OHo = c.H; g.OWo = c.W; g.oya = s; g.oyb = iy0; g.oxa = s; g.oxb = ix0;
    g.B = c.B; g.Ncols = c.C; g.Kd = g.nty * g.ntx * c.N;
    g.M = (long)c.B * g.RH * g.RW;
    return g;
}

int check_geo(const csu_conv_geom* g) {
    if (!g || g->B < 1 || g->H < 1 || g->W < 1 || g->C < 1 || g->OH < 1 || g->OW < 1 || g->N < 1 || g->KH < 1 ||
        g->KW < 1 || g->stride < 1 || g->pad < 0)
        return fail(CSU_E_ARG, "conv2d: bad geometry");
    if (g->OH != (g->H + 2 * g->pad - g->KH) / g->stride + 1 || g->OW != (g->W + 2 * g->pad - g->KW) / g->stride + 1)
        return fail(CSU_E_ARG, "conv2d: output size inconsistent with H, W, kernel, stride, pad");
    if ((long)g->B * g->H * g->W >= (1L << 31) || (long)g->B * g->OH * g->OW >= (1L << 31))
        return fail(CSU_E_UNSUPPORTED, "conv2d: more than 2^31 pixels");
    return 0;
}

Geo to_geo(const csu_conv_geom* g) {
    return Geo{g->B, g->H, g->W, g->C, g->OH, g->OW, g->N, g->KH, g->KW, g->stride, g->pad};
}

struct WPl {
    int chunks;
    long rpc;
};
constexpr int kConvWgs = 2048;   // target workgroups of the weight-gradient split
WPl wplan(long M, int N, int K) {
    const long tiles = (long)((N + TBN - 1) / TBN) * ((K + TBN - 1) / TBN);
    long want = (kConvWgs + tiles - 1) / tiles;
    const long maxc = (M + 255) / 256;
    if (want > maxc) want = maxc;
    if (want > 512) want = 512;
    if (want < 1) want = 1;
    WPl p;
    p.rpc = ((M + want - 1) / want + 63) / 64 * 64;
    p.chunks = (int)((M + p.rpc - 1) / p.rpc);
    return p;
}

// v3 weight-gradient plan: TN x TK tiles, chunks of >= 16 steps so that tiles x chunks ~ 2 rounds of
// the CUs (one 96-120 KB workgroup per CU)
WPl wplan_dma(long M, int N, int K, const WDCfg& c) {
    const long tiles = (long)((N + c.tn - 1) / c.tn) * ((K + c.tk - 1) / c.tk);
    long want = (2L * id_cus() + tiles - 1) / tiles;
    const long maxc = (M + 1023) / 1024;
    if (want > maxc) want = maxc;
    if (want > 512) want = 512;
    if (want < 1) want = 1;
    WPl p;
    p.rpc = ((M + want - 1) / want + 63) / 64 * 64;
    p.chunks = (int)((M + p.rpc - 1) / p.rpc);
    return p;
}

// halo plan (picks kHalo64 / kHalo128): 64-pixel segments per chunk, ~2 workgroup rounds
constexpr int kHalo64 = kWDNCfg, kHalo128 = kWDNCfg + 1;
bool halo_ok(const csu_conv_geom* gm, int ns) {
    return gm->KH == 3 && gm->KW == 3 && gm->stride == 1 && gm->pad == 1 && gm->OW % 64 == 0 && gm->C % 64 == 0 &&
           gm->N % ns == 0;
}
WPl wplan_halo(const csu_conv_geom* gm, int ns) {
    const long nseg = (long)gm->B * gm->OH * (gm->OW / 64);
    const long tiles = (long)(gm->N / ns) * (gm->C / 64);
    long want = (2L * id_cus() + tiles - 1) / tiles;
    const long maxc = (nseg + 15) / 16;
    if (want > maxc) want = maxc;
    if (want > 1024) want = 1024;
    if (want < 1) want = 1;
    WPl p;
    p.rpc = (nseg + want - 1) / want;
    p.chunks = (int)((nseg + p.rpc - 1) / p.rpc);
    return p;
}
WPl wplan_any(const csu_conv_geom* gm, int pick) {
    const long M = (long)gm->B * gm->OH * gm->OW;
    const int K = gm->KH * gm->KW * gm->C;
    if (pick == kHalo64) return wplan_halo(gm, 64);
    if (pick == kHalo128) return wplan_halo(gm, 128);
    return pick >= 0 ? wplan_dma(M, gm->N, K, kWDCfgs[pick]) : wplan(M, gm->N, K);
}

// weight-gradient kernel of a geometry: -1 the v2 kernel, else a kWDCfgs index or kHalo64 /
// kHalo128 (cfg: -1 auto, 0 v2, 1 + k forced; -2 when a forced configuration is not eligible)
int wd_pick(const csu_conv_geom* gm, int dtype, int cfg) {
    const bool ok = dtype == CSU_BF16 && gm->C % 8 == 0 && gm->N % 8 == 0 &&
                    (long)gm->B * gm->H * gm->W * gm->C * 2 < (1L << 31) && (long)gm->B * gm->OH * gm->OW * gm->N * 2 < (1L << 31);
    if (cfg == 0) return -1;
    if (cfg > 0) {
        const int k = cfg - 1;
        if (!ok || k > kHalo128) return -2;
        if (k == kHalo64 && !halo_ok(gm, 64)) return -2;
        if (k == kHalo128 && !halo_ok(gm, 128)) return -2;
        return k;
    }
    if (!ok) return -1;
    // tools/conv_wgrad_probe.py (profiles/r03r_wgrad_probe.txt, r03t_wgrad_probe.txt): the halo kernel
    // for the 3x3 stride-1 convs it takes (MFMA busy 31-34 % with 128 output channels per workgroup,
    // 20 % with 64, against 9-17 % for v2); otherwise the 8-wave 256 x 128 tile at N >= 256 (24-26 %),
    // the 2-stage 128 x 128 tile at N = 128 with C <= 64 (the ConvTranspose2d gradients); v2 for the
    // rest (64 output channels: both staged operands too narrow for the gathered DMA tiles), except
    // the few-channel inputs with a wide K (the CSWin patch embed 8 x 7 x 7 -> 64: 79.6 -> 72.6 us,
    // the CARAFE4 encoder 16 x 3 x 3 -> 144: 86.4 -> 73.2 us, profiles/r03v_wgrad_probe_cswin.txt),
    // which take the 128 x 128 tile
    if (halo_ok(gm, 128)) return kHalo128;
    if (halo_ok(gm, 64)) return kHalo64;
    if (gm->N >= 256 && gm->N % 128 == 0) return 3;
    if (gm->N == 128 && gm->C <= 64) return 2;
    if (gm->C <= 16 && gm->KH * gm->KW * gm->C >= 128) return 2;
    return -1;
}

size_t wgrad_ws(const csu_conv_geom* gm, int pick) {
    const int K = gm->KH * gm->KW * gm->C;
    const WPl p = wplan_any(gm, pick);
    const long slab = ((long)gm->N * K + gm->N + 3) & ~3L;
    const size_t stage = slab != (long)gm->N * K + gm->N ? slab * sizeof(float) : 0;   // padded colsum output
    return (size_t)p.chunks * slab * sizeof(float) + stage + colsum_workspace(p.chunks, slab, CSU_F32);
}

template <int C>
void wd_launch(const Geo& g, long M, int N, int K, const WPl& p, const void* x, const void* dy, float* part, hipStream_t st) {
    constexpr WDCfg c = kWDCfgs[C];
    const dim3 grid((N + c.tn - 1) / c.tn, (K + c.tk - 1) / c.tk, p.chunks);
    conv_wgrad_dma<c.tn, c.tk, c.s, c.wn, c.wk><<<grid, 64 * c.wn * c.wk, 0, st>>>(g, M, N, K, p.rpc, (const bf16*)x,
                                                                                 (const bf16*)dy, part);
}
void wd_run(int pick, const Geo& g, long M, int N, int K, const WPl& p, const void* x, const void* dy, float* part,
            hipStream_t st, const void* x2 = nullptr, int csplit = 0) {
    if (pick == kHalo64 || pick == kHalo128) {
        const long nseg = (long)g.B * g.OH * (g.OW / 64);
        const int ns = pick == kHalo64 ? 64 : 128;
        const dim3 grid(N / ns, g.C / 64, p.chunks);
        if (ns == 64)
            conv3_wgrad_halo<64, 3><<<grid, 256, 0, st>>>(g, nseg, p.rpc, (const bf16*)x, (const bf16*)x2, csplit, (const bf16*)dy, part);
        else
            conv3_wgrad_halo<128, 2><<<grid, 512, 0, st>>>(g, nseg, p.rpc, (const bf16*)x, (const bf16*)x2, csplit, (const bf16*)dy, part);
        return;
    }
    switch (pick) {
        case 0: wd_launch<0>(g, M, N, K, p, x, dy, part, st); break;
        case 1: wd_launch<1>(g, M, N, K, p, x, dy, part, st); break;
        case 2: wd_launch<2>(g, M, N, K, p, x, dy, part, st); break;
        case 3: wd_launch<3>(g, M, N, K, p, x, dy, part, st); break;
        default: wd_launch<4>(g, M, N, K, p, x, dy, part, st); break;
    }
}

template <typename T, int MODE>
int launch_gemm(const Geo& g, long M, int Ncols, int Kdim, const void* src, const void* w, const float* bias, void* out,
                bool vec, hipStream_t st) {
    const dim3 grid((unsigned)((M + TBM - 1) / TBM), (Ncols + TBN - 1) / TBN);
    if (vec)
        conv_gemm<T, MODE, true><<<grid, NT, 0, st>>>(g, M, Ncols, Kdim, (const T*)src, (const T*)w, bias, (T*)out);
    else
        conv_gemm<T, MODE, false><<<grid, NT, 0, st>>>(g, M, Ncols, Kdim, (const T*)src, (const T*)w, bias, (T*)out);
    return check_launch("conv2d");
}

}  // namespace
}  // namespace csu

using namespace csu;

static int conv_fwd_impl(const csu_conv_geom* gm, int dtype, const void* x, const void* w_ohwi, const float* bias, void* out,
                         int cfg, void* stream, void* ws = nullptr, size_t ws_bytes = 0) {
    if (int e = check_geo(gm)) return e;
    if (!x || !w_ohwi || !out) return fail(CSU_E_ARG, "conv2d_fwd: null buffer");
    const Geo g = to_geo(gm);
    const long M = (long)g.B * g.OH * g.OW;
    const int K = g.KH * g.KW * g.C;
    const bool vec = g.C % 8 == 0;
    hipStream_t st = as_stream(stream);
    if (dtype == CSU_BF16 && g.C % 4 == 0) return launch_ig(ig_forward(*gm), x, w_ohwi, bias, out, st, cfg, (float*)ws, ws_bytes);
    if (cfg > 0) return fail(CSU_E_ARG, "conv2d_fwd: igemm_dma needs bf16 with C % 64 == 0");
    if (dtype == CSU_BF16) return launch_gemm<bf16, 0>(g, M, g.N, K, x, w_ohwi, bias, out, vec, st);
    if (dtype == CSU_F32) return launch_gemm<float, 0>(g, M, g.N, K, x, w_ohwi, bias, out, vec, st);
    return fail(CSU_E_ARG, "conv2d_fwd: bad dtype");
}

static int conv_dgrad_impl(const csu_conv_geom* gm, int dtype, const void* dy, const void* w_ihwo, const float* bias, void* dx,
                           int cfg, void* stream, void* ws = nullptr, size_t ws_bytes = 0) {
    if (int e = check_geo(gm)) return e;
    if (!dy || !w_ihwo || !dx) return fail(CSU_E_ARG, "conv2d_dgrad: null buffer");
    const Geo g = to_geo(gm);
    const long M = (long)g.B * g.H * g.W;
    const int K = g.KH * g.KW * g.N;
    const bool vec = g.N % 8 == 0;
    hipStream_t st = as_stream(stream);
    if (dtype == CSU_BF16 && g.N % 4 == 0) {
        IG ph[4];
        int np = 0;
        for (int py = 0; py < g.s; ++py)
            for (int px = 0; px < g.s; ++px) {
                const IG ig = ig_dgrad_phase(*gm, py, px);
                if (ig.M == 0) continue;
                if (np == 4) {   // stride > 2: flush
                    if (int e = launch_ig(ph, np, dy, w_ihwo, bias, dx, st, cfg)) return e;
                    np = 0;
                }
                ph[np++] = ig;
            }
        if (np == 1) return launch_ig(ph, 1, dy, w_ihwo, bias, dx, st, cfg, (float*)ws, ws_bytes);
        return np ? launch_ig(ph, np, dy, w_ihwo, bias, dx, st, cfg) : 0;
    }
    if (cfg > 0) return fail(CSU_E_ARG, "conv2d_dgrad: igemm_dma needs bf16 with N % 64 == 0");
    if (dtype == CSU_BF16) return launch_gemm<bf16, 1>(g, M, g.C, K, dy, w_ihwo, bias, dx, vec, st);
    if (dtype == CSU_F32) return launch_gemm<float, 1>(g, M, g.C, K, dy, w_ihwo, bias, dx, vec, st);
    return fail(CSU_E_ARG, "conv2d_dgrad: bad dtype");
}

extern "C" int csu_conv2d_fwd(const csu_conv_geom* gm, int dtype, const void* x, const void* w_ohwi, const float* bias,
                              void* out, void* stream) {
    return conv_fwd_impl(gm, dtype, x, w_ohwi, bias, out, -1, stream);
}

extern "C" int csu_conv2d_dgrad(const csu_conv_geom* gm, int dtype, const void* dy, const void* w_ihwo,
                                const float* bias, void* dx, void* stream) {
    return conv_dgrad_impl(gm, dtype, dy, w_ihwo, bias, dx, -1, stream);
}

// workspace of the K-split v2 launches (one-problem bf16 convs with few tiles; 0: never split)
extern "C" size_t csu_conv2d_workspace(int op, const csu_conv_geom* gm, int dtype) {
    if (check_geo(gm) || dtype != CSU_BF16 || (op != 0 && op != 1)) return 0;
    if (op == 0) {
        if (gm->C % 4) return 0;
        const IG g = ig_forward(*gm);
        return id_pick(g, true) >= 0 ? 0 : ksplit_bytes(g, id_cus());
    }
    if (gm->N % 4 || gm->stride != 1) return 0;
    const IG g = ig_dgrad_phase(*gm, 0, 0);
    return id_pick(g, true) >= 0 ? 0 : ksplit_bytes(g, id_cus());
}

extern "C" int csu_conv2d_fwd_ws(const csu_conv_geom* gm, int dtype, const void* x, const void* w_ohwi, const float* bias,
                                 void* out, void* workspace, size_t ws_bytes, void* stream) {
    return conv_fwd_impl(gm, dtype, x, w_ohwi, bias, out, -1, stream, workspace, ws_bytes);
}

extern "C" int csu_conv2d_dgrad_ws(const csu_conv_geom* gm, int dtype, const void* dy, const void* w_ihwo, const float* bias,
                                   void* dx, void* workspace, size_t ws_bytes, void* stream) {
    return conv_dgrad_impl(gm, dtype, dy, w_ihwo, bias, dx, -1, stream, workspace, ws_bytes);
}

extern "C" int csu_conv2d_ex(int op, const csu_conv_geom* gm, int dtype, const void* src, const void* w, const float* bias,
                             void* out, int cfg, void* stream) {
    if (op == 0) return conv_fwd_impl(gm, dtype, src, w, bias, out, cfg, stream);
    if (op == 1) return conv_dgrad_impl(gm, dtype, src, w, bias, out, cfg, stream);
    return fail(CSU_E_ARG, "conv2d_ex: op must be 0 (forward) or 1 (input gradient)");
}

extern "C" size_t csu_conv2d_wgrad_workspace(const csu_conv_geom* gm) {
    if (check_geo(gm)) return 0;
    // dtype-independent: enough for the v2 plan and for the v3 plan the bf16 call picks
    const size_t a = wgrad_ws(gm, -1);
    const int pk = wd_pick(gm, CSU_BF16, -1);
    const size_t b = pk >= 0 ? wgrad_ws(gm, pk) : 0;
    return a > b ? a : b;
}

extern "C" size_t csu_conv2d_wgrad_workspace_ex(const csu_conv_geom* gm, int cfg) {
    if (check_geo(gm)) return 0;
    if (cfg < 0) return csu_conv2d_wgrad_workspace(gm);
    const int pk = wd_pick(gm, CSU_BF16, cfg);
    return pk == -2 ? 0 : wgrad_ws(gm, pk);
}

static int conv_wgrad_impl(const csu_conv_geom* gm, int dtype, const void* x, const void* dy, int creal, float* dw_db,
                           void* workspace, size_t ws_bytes, int cfg, void* stream, const void* x2 = nullptr, int csplit = 0) {
    if (int e = check_geo(gm)) return e;
    if (!x || !dy || !dw_db) return fail(CSU_E_ARG, "conv2d_wgrad: null buffer");
    const int pick = wd_pick(gm, dtype, cfg);
    if (pick == -2) return fail(CSU_E_ARG, "conv2d_wgrad: configuration not eligible (bf16, C % 8 == 0, N % 8 == 0)");
    if (csplit && pick != kHalo64 && pick != kHalo128)
        return fail(CSU_E_UNSUPPORTED, "conv2d_wgrad: two-source input needs the halo kernel");
    if (!workspace || ws_bytes < wgrad_ws(gm, pick)) return fail(CSU_E_WORKSPACE, "conv2d_wgrad: workspace");
    if (creal > gm->C) return fail(CSU_E_ARG, "conv2d_wgrad: c_real > C");
    const Geo g = to_geo(gm);
    const long M = (long)g.B * g.OH * g.OW;
    const int K = g.KH * g.KW * g.C;
    const WPl p = wplan_any(gm, pick);
    const long used = (long)g.N * K + g.N;
    const long slab = (used + 3) & ~3L;
    float* part = (float*)workspace;
    const dim3 grid((g.N + TBN - 1) / TBN, (K + TBN - 1) / TBN, p.chunks);
    const bool vec = g.C % 8 == 0;
    hipStream_t st = as_stream(stream);
    if (pick >= 0) {
        wd_run(pick, g, M, g.N, K, p, x, dy, part, st, x2, csplit);
    } else if (dtype == CSU_BF16) {
        const bool small = (long)g.B * g.H * g.W * g.C * 2 < (1L << 31) && M * g.N * 2 < (1L << 31);   // 32-bit offsets
        if (vec && g.N % 8 == 0 && small)
            conv_wgrad_bf16<false><<<grid, NT, 0, st>>>(g, M, g.N, K, p.rpc, (const bf16*)x, (const bf16*)dy, part);
        else if (vec && g.N % 4 == 0 && small)
            conv_wgrad_bf16<true><<<grid, NT, 0, st>>>(g, M, g.N, K, p.rpc, (const bf16*)x, (const bf16*)dy, part);
        else if (vec) conv_wgrad_kernel<bf16, true><<<grid, NT, 0, st>>>(g, M, g.N, K, p.rpc, (const bf16*)x, (const bf16*)dy, part);
        else conv_wgrad_kernel<bf16, false><<<grid, NT, 0, st>>>(g, M, g.N, K, p.rpc, (const bf16*)x, (const bf16*)dy, part);
    } else if (dtype == CSU_F32) {
        if (vec) conv_wgrad_kernel<float, true><<<grid, NT, 0, st>>>(g, M, g.N, K, p.rpc, (const float*)x, (const float*)dy, part);
        else conv_wgrad_kernel<float, false><<<grid, NT, 0, st>>>(g, M, g.N, K, p.rpc, (const float*)x, (const float*)dy, part);
    } else {
        return fail(CSU_E_ARG, "conv2d_wgrad: bad dtype");
    }
    if (int e = check_launch("conv2d_wgrad")) return e;
    if (creal > 0) {   // chunk sums written straight into torch's OIHW layout (+ db)
        const OutMap om{1, g.N, g.KH * g.KW, g.C, creal};
        return colsum_launch(p.chunks, slab, CSU_F32, part, dw_db, part + (size_t)p.chunks * slab, st, &om);
    }
    if (slab == used) return colsum_launch(p.chunks, slab, CSU_F32, part, dw_db, part + (size_t)p.chunks * slab, st);
    float* stage = part + (size_t)p.chunks * slab;
    if (int e = colsum_launch(p.chunks, slab, CSU_F32, part, stage, stage + slab, st)) return e;
    if (hipMemcpyAsync(dw_db, stage, used * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail(CSU_E_ARG, "conv2d_wgrad: copy-out failed");
    return 0;
}

extern "C" int csu_conv2d_wgrad(const csu_conv_geom* gm, int dtype, const void* x, const void* dy, float* dw_db,
                                void* workspace, size_t ws_bytes, void* stream) {
    return conv_wgrad_impl(gm, dtype, x, dy, 0, dw_db, workspace, ws_bytes, -1, stream);
}

extern "C" int csu_conv2d_wgrad_oihw(const csu_conv_geom* gm, int dtype, const void* x, const void* dy, int c_real,
                                     float* dw_db, void* workspace, size_t ws_bytes, void* stream) {
    if (c_real < 1) return fail(CSU_E_ARG, "conv2d_wgrad_oihw: c_real < 1");
    return conv_wgrad_impl(gm, dtype, x, dy, c_real, dw_db, workspace, ws_bytes, -1, stream);
}

extern "C" int csu_conv2d_wgrad_ex(const csu_conv_geom* gm, int dtype, const void* x, const void* dy, int c_real, float* dw_db,
                                   void* workspace, size_t ws_bytes, int cfg, void* stream) {
    if (c_real < 0) return fail(CSU_E_ARG, "conv2d_wgrad_ex: c_real < 0");
    return conv_wgrad_impl(gm, dtype, x, dy, c_real, dw_db, workspace, ws_bytes, cfg, stream);
}

// ---- two-source input (channel concat of UNet Up, unet:213-216, never materialised) -----------
extern "C" int csu_conv2d_split_ok(const csu_conv_geom* gm, int c_split) {
    if (check_geo(gm)) return 0;
    return c_split > 0 && c_split < gm->C && c_split % 64 == 0 && gm->C % 64 == 0 && gm->N % 64 == 0 &&
           (long)gm->B * gm->H * gm->W * gm->C * 2 < (1L << 31) && wd_pick(gm, CSU_BF16, -1) >= kHalo64;
}

extern "C" int csu_conv2d_fwd_split(const csu_conv_geom* gm, int dtype, const void* x, const void* x2, int c_split,
                                    const void* w_ohwi, const float* bias, void* y, void* stream) {
    if (int e = check_geo(gm)) return e;
    if (dtype != CSU_BF16 || !csu_conv2d_split_ok(gm, c_split)) return fail(CSU_E_UNSUPPORTED, "conv2d_fwd_split: not eligible");
    if (!x || !x2 || !w_ohwi || !y) return fail(CSU_E_ARG, "conv2d_fwd_split: null buffer");
    IG g = ig_forward(*gm);
    g.csplit = c_split;
    g.src2 = (const bf16*)x2;
    return launch_ig(g, x, w_ohwi, bias, y, as_stream(stream));
}

extern "C" int csu_conv2d_dgrad_split(const csu_conv_geom* gm, int dtype, const void* dy, const void* w_ihwo, void* dx, void* dx2,
                                      int c_split, void* stream) {
    if (int e = check_geo(gm)) return e;
    if (dtype != CSU_BF16 || !csu_conv2d_split_ok(gm, c_split)) return fail(CSU_E_UNSUPPORTED, "conv2d_dgrad_split: not eligible");
    if (!dy || !w_ihwo || !dx || !dx2) return fail(CSU_E_ARG, "conv2d_dgrad_split: null buffer");
    IG ph[4];
    int np = 0;
    for (int py = 0; py < gm->stride; ++py)
        for (int px = 0; px < gm->stride; ++px) {
            IG ig = ig_dgrad_phase(*gm, py, px);
            if (ig.M == 0) continue;
            ig.nsplit = c_split;
            ig.out2 = (bf16*)dx2;
            ph[np++] = ig;
        }
    return np ? launch_ig(ph, np, dy, w_ihwo, nullptr, dx, as_stream(stream)) : 0;
}

extern "C" int csu_conv2d_wgrad_split_oihw(const csu_conv_geom* gm, int dtype, const void* x, const void* x2, int c_split,
                                           const void* dy, float* dw_db, void* workspace, size_t ws_bytes, void* stream) {
    if (int e = check_geo(gm)) return e;
    if (dtype != CSU_BF16 || !csu_conv2d_split_ok(gm, c_split)) return fail(CSU_E_UNSUPPORTED, "conv2d_wgrad_split: not eligible");
    if (!x2) return fail(CSU_E_ARG, "conv2d_wgrad_split: null buffer");
    return conv_wgrad_impl(gm, dtype, x, dy, gm->C, dw_db, workspace, ws_bytes, -1, stream, x2, c_split);
}
