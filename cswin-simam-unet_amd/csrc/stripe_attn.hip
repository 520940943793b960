// Cross-shaped stripe attention + LePE for gfx950 (MI355X, CDNA4).
//
// Replaces LePEAttention.forward (train_cswinunet_segmentation.py cswin:271-298) together with
// its window layout (img2windows/windows2img cswin:199-217, im2cswin/get_lepe cswin:248-269)
// and the branch split/concat of CSWinBlock.forward (cswin:358-363).  No layout copies: every
// window token is gathered straight from the (B, L, 3C) qkv buffer and the result is written
// straight to its channels of the (B, L, C) output.
//
// Work decomposition: one 256-thread workgroup = one (branch, image, window, head, 128-row
// block); each of its 4 waves owns 32 rows.  The other operand streams through LDS in chunks of
// KC = 128 rows.  All products are 32x32 MFMA tiles:
//   bf16 storage: v_mfma_f32_32x32x16_bf16 (fp32 accumulate);
//   fp32 storage: v_mfma_f32_32x32x2_f32  (exact f32 fma chain -- the fp32 parity path).
// "Swapped" orientation: S^T = K Q^T puts the query on the lane and 16 keys in registers, so
// the softmax row statistics need one cross-half shuffle and the probabilities are already the
// B operand of O^T += V^T P^T (accumulator-as-operand, cdna_hip_programming.md §3).
//
// Backward = two kernels (query-owner: dQ and delta; key-owner: dK, dV including the LePE
// input gradient) plus a deterministic two-pass reduction for the LePE weight/bias gradient.
#include <cstdlib>

#include "common.hpp"
#include "rng.hpp"

#include <type_traits>

namespace csu {
namespace {

constexpr int HD = 32;     // head dim (fixed by the model: SURVEY §0.5)
constexpr int KC = 128;    // rows of the streamed operand per LDS chunk
constexpr int QR = 128;    // rows owned by one workgroup (4 waves x 32)
constexpr int NT = 256;

template <typename T> struct Cfg;
template <> struct Cfg<bf16> {
    static constexpr int KSTR = HD + 8;   // 80-B rows: conflict-free ds_read_b128 of row chunks
    static constexpr int VSTR = KC + 4;   // 264-B rows: conflict-free ds_read_b64 of transposed rows
};
template <> struct Cfg<float> {
    static constexpr int KSTR = HD + 4;   // 144-B rows
    static constexpr int VSTR = KC + 1;   // odd stride: conflict-free ds_read_b32 column reads
};

// select a branch without dynamic indexing of the kernel-argument struct (no scratch copy)
__device__ __forceinline__ const csu_stripe_branch& branch(const csu_stripe_args& a, int i) {
    return i ? a.br[1] : a.br[0];
}

struct Win {
    int br, b, h, wy, wx, blk;  // branch, image, head, window row/col, 128-row block
    int H_sp, W_sp, N;
    int chq;                    // channel of (branch, head) inside the C-wide Q/K/V slot
    float rW;                   // 1 / W_sp (correctly rounded): window row of a position, see wrow
};

// window row n / W_sp of window position n without an integer division (~20 VALU ops each):
// (n + 0.5) * (1 / W_sp) truncated -- exact for n < 4096, W_sp <= 1024 (checked exhaustively)
__device__ __forceinline__ int wrow(const Win& w, int n) {
    return (int)__fmul_rn(__fadd_rn((float)n, 0.5f), w.rW);
}

__device__ __forceinline__ Win decode_block(const csu_stripe_args& a) {
    Win w;
    w.br = blockIdx.y;
    const csu_stripe_branch& g = branch(a, w.br);
    w.H_sp = g.H_sp;
    w.W_sp = g.W_sp;
    w.rW = __frcp_rn((float)g.W_sp);
    w.N = w.H_sp * w.W_sp;
    const int nwx = a.reso / w.W_sp, nwin = (a.reso / w.H_sp) * nwx;
    const int nblk = (w.N + QR - 1) / QR;
    int id = blockIdx.x;
    w.blk = id % nblk; id /= nblk;
    w.h = id % a.heads; id /= a.heads;
    const int win = id % nwin;
    w.b = id / nwin;
    w.wy = win / nwx;
    w.wx = win % nwx;
    w.chq = g.ch_off + w.h * HD;
    return w;
}

// token index (inside its image) of window-local position n
__device__ __forceinline__ int tok_of(const Win& w, int reso, int n) {
    const int iy = wrow(w, n), ix = n - iy * w.W_sp;
    return (w.wy * w.H_sp + iy) * reso + w.wx * w.W_sp + ix;
}

// ---------------------------------------------------------------------------------------------
// Operand fragments of one 32-row tile: row r = lane & 31, half h = lane >> 5.
//   bf16: k-step s (16 wide) -> elements [16s + 8h, +8) of the row
//   f32 : k-step t (2 wide)  -> element 16h + t of the row (t = 0..15)
// Both A (rows from LDS) and B (rows from registers) use the same inner-index permutation.
// ---------------------------------------------------------------------------------------------
template <typename T> struct Frag;
template <> struct Frag<bf16> { bf16x8 v[2]; };
template <> struct Frag<float> { float v[16]; };

__device__ __forceinline__ void load_frag(Frag<bf16>& f, const bf16* row, int h, bool valid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        if (valid) f.v[s] = *reinterpret_cast<const bf16x8*>(row + 16 * s + 8 * h);
        else f.v[s] = bf16x8{};
    }
}
__device__ __forceinline__ void load_frag(Frag<float>& f, const float* row, int h, bool valid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f32x4 x = valid ? *reinterpret_cast<const f32x4*>(row + 16 * h + 4 * i) : f32x4{};
        f.v[4 * i] = x[0]; f.v[4 * i + 1] = x[1]; f.v[4 * i + 2] = x[2]; f.v[4 * i + 3] = x[3];
    }
}

// acc += A_lds(rows 32) * B_frag^T   (A rows are row-major [row][KSTR] in LDS)
__device__ __forceinline__ void mma_rows(f32x16& acc, const bf16* A, int r, int h, const Frag<bf16>& B) {
    constexpr int S = Cfg<bf16>::KSTR;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        bf16x8 a = *reinterpret_cast<const bf16x8*>(A + r * S + 16 * s + 8 * h);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, B.v[s], acc, 0, 0, 0);
    }
}
__device__ __forceinline__ void mma_rows(f32x16& acc, const float* A, int r, int h, const Frag<float>& B) {
    constexpr int S = Cfg<float>::KSTR;
    float a[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f32x4 x = *reinterpret_cast<const f32x4*>(A + r * S + 16 * h + 4 * i);
        a[4 * i] = x[0]; a[4 * i + 1] = x[1]; a[4 * i + 2] = x[2]; a[4 * i + 3] = x[3];
    }
#pragma unroll
    for (int t = 0; t < 16; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t], B.v[t], acc, 0, 0, 0);
}

// acc(d, col) += sum_k At[d][k0 + k] * X[k][col], X = 32x32 f32 accumulator tile of this wave
// (column on the lane, row k in registers).  At is a transposed [HD][VSTR] LDS image.
__device__ __forceinline__ void mma_acc_operand(f32x16& acc, const bf16* At, int k0, int r, int h, const f32x16& X) {
    constexpr int S = Cfg<bf16>::VSTR;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = (bf16)X[8 * s + j];
        const bf16* p = At + r * S + k0 + 16 * s + 4 * h;
        bf16x4 lo = *reinterpret_cast<const bf16x4*>(p);
        bf16x4 hi = *reinterpret_cast<const bf16x4*>(p + 8);
        bf16x8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
}
__device__ __forceinline__ void mma_acc_operand(f32x16& acc, const float* At, int k0, int r, int h, const f32x16& X) {
    constexpr int S = Cfg<float>::VSTR;
#pragma unroll
    for (int t = 0; t < 16; ++t)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(At[r * S + k0 + crow(t, h)], X[t], acc, 0, 0, 0);
}

// Cooperative gather of `nrows` window rows (rows >= valid_rows are zero) of one head into
//   nat: natural [KC][KSTR] image (optional) and tr: transposed [HD][VSTR] image (optional).
template <typename T>
__device__ __forceinline__ void stage_rows(const Win& w, int reso, const T* img, int rstride, int ch,
                                           int row0, int N, T* nat, T* tr) {
    constexpr int VEC = 16 / sizeof(T);
    constexpr int PER = HD / VEC;
    for (int it = threadIdx.x; it < KC * PER; it += NT) {
        const int rr = it / PER, d0 = (it % PER) * VEC;
        const int n = row0 + rr;
        float v[VEC];
        if (n < N) {
            const T* src = img + (size_t)tok_of(w, reso, n) * rstride + ch + d0;
            if constexpr (VEC == 8) load8(src, v); else load4(src, v);
        } else {
#pragma unroll
            for (int j = 0; j < VEC; ++j) v[j] = 0.f;
        }
        if (nat) {
            if constexpr (VEC == 8) store8(nat + rr * Cfg<T>::KSTR + d0, v);
            else store4(nat + rr * Cfg<T>::KSTR + d0, v);
        }
        if (tr) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) tr[(d0 + j) * Cfg<T>::VSTR + rr] = from_f<T>(v[j]);
        }
    }
}

// LePE (depthwise 3x3, window-local zero padding) of window position n for 4 consecutive head
// channels c0..c0+3; wts = [HD][9] weights + [HD] bias of this head in LDS.
// sign = +1: sum_t w[t] * img[n + off(t)] + bias (forward conv, cswin:244/265)
// sign = -1: sum_t w[t] * img[n - off(t)]        (transposed conv = input gradient)
template <typename T>
__device__ __forceinline__ void lepe4(const Win& w, int reso, const T* img, int rstride, int ch, int n,
                                      int c0, const float* wts, int sign, float* acc) {
    const int iy = wrow(w, n), ix = n - iy * w.W_sp;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = sign > 0 ? wts[HD * 9 + c0 + j] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int dy = sign * (t / 3 - 1), dx = sign * (t % 3 - 1);
        const int y = iy + dy, x = ix + dx;
        if (y < 0 || y >= w.H_sp || x < 0 || x >= w.W_sp) continue;
        float v[4];
        load4(img + (size_t)tok_of(w, reso, y * w.W_sp + x) * rstride + ch + c0, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += wts[(c0 + j) * 9 + t] * v[j];
    }
}

constexpr int LW_IT = (HD * 10 + NT - 1) / NT;
// the two halves of stage_lepe_weights for the whole-window kernels: issue the loads, and (after the
// window staging loads have been issued) write LDS -- the LDS write waits for its loads, and vmcnt
// counts in issue order, so writing right after the loads would drain everything issued before
__device__ __forceinline__ void lepe_weights_load(const csu_stripe_branch& g, int h, float* v) {
    const __amdgpu_buffer_rsrc_t rw = buf_rsrc(g.lepe_w + h * HD * 9, HD * 9 * 4), rb = buf_rsrc(g.lepe_b + h * HD, HD * 4);
#pragma unroll
    for (int k = 0; k < LW_IT; ++k) {
        const int i = threadIdx.x + k * NT;
        const float a = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, i < HD * 9 ? (unsigned)i * 4u : kOOB, 0, 0));
        const float b = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rb, (i >= HD * 9 && i < HD * 10) ? (unsigned)(i - HD * 9) * 4u : kOOB, 0, 0));
        v[k] = i < HD * 9 ? a : b;
    }
}
// whole-window kernels: LDS layout [tap][channel] (tap 9 = bias), so the 4 weights of a channel quad
// for one tap are one 16-B read (lepe4_lds)
__device__ __forceinline__ void lepe_weights_store(const float* v, float* wts) {
#pragma unroll
    for (int k = 0; k < LW_IT; ++k) {
        const int i = threadIdx.x + k * NT;   // source element: weight c * 9 + t, or bias HD * 9 + c
        const int c = i / 9, t = i - c * 9;
        if (i < HD * 9) wts[t * HD + c] = v[k];
        else if (i < HD * 10) wts[i] = v[k];
    }
}

__device__ __forceinline__ void stage_lepe_weights(const csu_stripe_branch& g, int h, float* wts) {
    constexpr int IT = (HD * 10 + NT - 1) / NT;
    float v[IT];
    // branch-free (raw buffer loads, masked lanes out of range): a predicated load here made hipcc
    // wait vmcnt(0) before the window staging loads that follow
    const __amdgpu_buffer_rsrc_t rw = buf_rsrc(g.lepe_w + h * HD * 9, HD * 9 * 4), rb = buf_rsrc(g.lepe_b + h * HD, HD * 4);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int i = threadIdx.x + k * NT;
        const float a = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, i < HD * 9 ? (unsigned)i * 4u : kOOB, 0, 0));
        const float b = __uint_as_float(
            __builtin_amdgcn_raw_buffer_load_b32(rb, (i >= HD * 9 && i < HD * 10) ? (unsigned)(i - HD * 9) * 4u : kOOB, 0, 0));
        v[k] = i < HD * 9 ? a : b;
    }
#pragma unroll
    for (int k = 0; k < IT; ++k)
        if (threadIdx.x + k * NT < HD * 10) wts[threadIdx.x + k * NT] = v[k];
}

__device__ __forceinline__ size_t stat_index(const csu_stripe_args& a, const Win& w, int tok) {
    const int L = a.reso * a.reso;
    return ((size_t)(w.br * a.B + w.b) * a.heads + w.h) * L + tok;
}

// ---- attention dropout (attn_drop on P, cswin:290) -------------------------------------------
// Element (query q, key k) of the window-head has index wbase + q * Npad + k (csu.h), Npad = N
// rounded up to 32, so every 32-key tile starts a group of 8 (rng.hpp: one Philox call = 8 keys).
struct ADrop {
    DropoutRng R;
    uint64_t wbase;
    int npad;
};

__device__ __forceinline__ ADrop attn_drop(const csu_stripe_args& a, const Win& w) {
    ADrop d;
    d.R = load_rng(a.drop_rng, a.drop_site + (unsigned)w.br, a.drop_p);
    d.npad = (w.N + 31) & ~31;
    const int nwx = a.reso / w.W_sp, nwin = (a.reso / w.H_sp) * nwx;
    d.wbase = (((uint64_t)w.b * nwin + (uint64_t)w.wy * nwx + w.wx) * a.heads + w.h) * (uint64_t)w.N * d.npad;
    return d;
}

// lane = query orientation: keep bits (bit i) of the 16 keys kt + crow(i, h) of query q (kt % 8 == 0)
__device__ __forceinline__ unsigned keep_q16(const ADrop& d, int q, int kt, int h) {
    return keep16_crow(d.R, (d.wbase + (uint64_t)q * d.npad + kt) >> 3, h);
}

// lane = key orientation: keep bits (bit i) of key kt + (lane & 31) for the 16 queries qb + crow(i, h)
// (kt % 8 == 0).  The tile's 32 queries x 4 key groups = 128 Philox calls are spread over the 64
// lanes and exchanged through `tbl`, 128 B of LDS private to this wave.
__device__ __forceinline__ unsigned keep_k16(const ADrop& d, int qb, int kt, int lane, unsigned char* tbl) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int c = 2 * lane + j, qq = c >> 2, g = c & 3;
        tbl[g * 32 + qq] = (unsigned char)keep8(d.R, ((d.wbase + (uint64_t)(qb + qq) * d.npad + kt) >> 3) + g);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int r = lane & 31, h = lane >> 5, b = r & 7;
    const unsigned* t32 = reinterpret_cast<const unsigned*>(tbl + (r >> 3) * 32 + 4 * h);
    unsigned m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const unsigned wd = t32[2 * j];   // queries crow(4j + t, h) = 8j + 4h + t, t = 0..3
#pragma unroll
        for (int t = 0; t < 4; ++t) m |= ((wd >> (8 * t + b)) & 1u) << (4 * j + t);
    }
    asm volatile("" ::: "memory");   // the reads stay ahead of the next tile's writes
    return m;
}

// =============================================================================================
// Forward
// =============================================================================================
template <typename T, bool DROP>
__global__ __launch_bounds__(NT) void stripe_fwd(csu_stripe_args a, const T* __restrict__ qkv,
                                                 T* __restrict__ out, float* __restrict__ lse) {
    __shared__ __attribute__((aligned(16))) T Ks[KC * Cfg<T>::KSTR];
    __shared__ __attribute__((aligned(16))) T Vt[HD * Cfg<T>::VSTR];
    __shared__ float wts[HD * 10];

    const Win w = decode_block(a);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const T* img = qkv + (size_t)w.b * L * C3;
    const int qn = w.blk * QR + wave * 32 + r;
    const bool qvalid = qn < w.N;
    const bool wave_active = w.blk * QR + wave * 32 < w.N;
    const int qtok = qvalid ? tok_of(w, a.reso, qn) : 0;

    stage_lepe_weights(branch(a, w.br), w.h, wts);
    Frag<T> qf;
    load_frag(qf, img + (size_t)qtok * C3 + w.chq, h, qvalid);

    const float c = a.scale * kLog2e;
    float m = -INFINITY, l = 0.f;
    f32x16 o = {};
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);

    for (int k0 = 0; k0 < w.N; k0 += KC) {
        __syncthreads();
        stage_rows<T>(w, a.reso, img, C3, C + w.chq, k0, w.N, Ks, nullptr);
        stage_rows<T>(w, a.reso, img, C3, 2 * C + w.chq, k0, w.N, nullptr, Vt);
        __syncthreads();
        if (!wave_active) continue;
        const int nk = min(KC, w.N - k0);
        for (int kb = 0; kb < nk; kb += 32) {
            f32x16 s = {};
            mma_rows(s, Ks + kb * Cfg<T>::KSTR, r, h, qf);
            float bm = -INFINITY;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool kv = k0 + kb + crow(i, h) < w.N;
                s[i] = kv ? s[i] * c : -INFINITY;
                bm = fmaxf(bm, s[i]);
            }
            bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
            const float mn = fmaxf(m, bm);
            const float alpha = exp2f(m - mn);
            m = mn;
            float ls = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s[i] = exp2f(s[i] - mn);
                ls += s[i];
            }
            l = l * alpha + ls;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] *= alpha;
            if constexpr (DROP) {   // the normaliser l keeps every key; O sees the dropped P
                const unsigned km = keep_q16(dr, qn, k0 + kb, h);
#pragma unroll
                for (int i = 0; i < 16; ++i) s[i] = ((km >> i) & 1u) ? s[i] * dr.R.scale : 0.f;
            }
            mma_acc_operand(o, Vt, kb, r, h, s);
        }
    }
    if (!qvalid) return;
    const float lt = l + __shfl_xor(l, 32, 64);
    const float inv = 1.f / lt;
    if (h == 0) lse[stat_index(a, w, qtok)] = (m + log2f(lt)) * kLn2;
    T* orow = out + ((size_t)w.b * L + qtok) * C + w.chq;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 8 * g4 + 4 * h;   // registers 4*g4..4*g4+3 hold channels d0..d0+3
        float lp[4];
        lepe4<T>(w, a.reso, img, C3, 2 * C + w.chq, qn, d0, wts, +1, lp);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = o[4 * g4 + j] * inv + lp[j];
        store4(orow + d0, v);
    }
}

// =============================================================================================
// Backward, query owner: delta = rowsum(dO * O_attn), dQ
// =============================================================================================
template <typename T, bool DROP>
__global__ __launch_bounds__(NT) void stripe_bwd_dq(csu_stripe_args a, const T* __restrict__ qkv,
                                                    const T* __restrict__ out, const T* __restrict__ dout,
                                                    const float* __restrict__ lse, float* __restrict__ delta,
                                                    T* __restrict__ dqkv) {
    __shared__ __attribute__((aligned(16))) T Ks[KC * Cfg<T>::KSTR];
    __shared__ __attribute__((aligned(16))) T Vs[KC * Cfg<T>::KSTR];
    __shared__ __attribute__((aligned(16))) T Kt[HD * Cfg<T>::VSTR];
    __shared__ float wts[HD * 10];

    const Win w = decode_block(a);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const T* img = qkv + (size_t)w.b * L * C3;
    const T* oimg = out + (size_t)w.b * L * C;
    const T* gimg = dout + (size_t)w.b * L * C;
    const int qn = w.blk * QR + wave * 32 + r;
    const bool qvalid = qn < w.N;
    const bool wave_active = w.blk * QR + wave * 32 < w.N;
    const int qtok = qvalid ? tok_of(w, a.reso, qn) : 0;

    stage_lepe_weights(branch(a, w.br), w.h, wts);
    Frag<T> qf, gf;
    load_frag(qf, img + (size_t)qtok * C3 + w.chq, h, qvalid);
    load_frag(gf, gimg + (size_t)qtok * C + w.chq, h, qvalid);
    __syncthreads();

    // delta over this lane's 16 channels (the dO fragment's channels), O_attn = out - lepe
    float dl = 0.f;
    if (qvalid) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = sizeof(T) == 2 ? 16 * (g4 >> 1) + 8 * h + 4 * (g4 & 1) : 16 * h + 4 * g4;
            float lp[4], ov[4];
            lepe4<T>(w, a.reso, img, C3, 2 * C + w.chq, qn, d0, wts, +1, lp);
            load4(oimg + (size_t)qtok * C + w.chq + d0, ov);
            float gv[4];
            load4(gimg + (size_t)qtok * C + w.chq + d0, gv);
#pragma unroll
            for (int j = 0; j < 4; ++j) dl += gv[j] * (ov[j] - lp[j]);
        }
    }
    dl += __shfl_xor(dl, 32, 64);
    const size_t si = stat_index(a, w, qtok);
    if (qvalid && h == 0) delta[si] = dl;
    const float lq = qvalid ? lse[si] * kLog2e : 0.f;

    const float c = a.scale * kLog2e;
    f32x16 dq = {};
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);
    for (int k0 = 0; k0 < w.N; k0 += KC) {
        __syncthreads();
        stage_rows<T>(w, a.reso, img, C3, C + w.chq, k0, w.N, Ks, Kt);
        stage_rows<T>(w, a.reso, img, C3, 2 * C + w.chq, k0, w.N, Vs, nullptr);
        __syncthreads();
        if (!wave_active) continue;
        const int nk = min(KC, w.N - k0);
        for (int kb = 0; kb < nk; kb += 32) {
            f32x16 s = {}, dp = {};
            mma_rows(s, Ks + kb * Cfg<T>::KSTR, r, h, qf);
            mma_rows(dp, Vs + kb * Cfg<T>::KSTR, r, h, gf);
            unsigned km = 0xffffu;
            if constexpr (DROP) km = keep_q16(dr, qn, k0 + kb, h);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bool kv = k0 + kb + crow(i, h) < w.N;
                const float p = kv ? exp2f(s[i] * c - lq) : 0.f;
                float g = dp[i];
                if constexpr (DROP) g = ((km >> i) & 1u) ? g * dr.R.scale : 0.f;   // dP through the mask
                s[i] = p * (g - dl);   // dS^T
            }
            mma_acc_operand(dq, Kt, kb, r, h, s);
        }
    }
    if (!qvalid) return;
    T* drow = dqkv + ((size_t)w.b * L + qtok) * C3 + w.chq;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 8 * g4 + 4 * h;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = dq[4 * g4 + j] * a.scale;
        store4(drow + d0, v);
    }
}

// =============================================================================================
// Backward, key owner: dK, dV (+ LePE input gradient)
// =============================================================================================
template <typename T, bool DROP>
__global__ __launch_bounds__(NT) void stripe_bwd_dkdv(csu_stripe_args a, const T* __restrict__ qkv,
                                                      const T* __restrict__ dout, const float* __restrict__ lse,
                                                      const float* __restrict__ delta, T* __restrict__ dqkv) {
    __shared__ __attribute__((aligned(16))) T Qs[KC * Cfg<T>::KSTR];
    __shared__ __attribute__((aligned(16))) T Gs[KC * Cfg<T>::KSTR];
    __shared__ __attribute__((aligned(16))) T Qt[HD * Cfg<T>::VSTR];
    __shared__ __attribute__((aligned(16))) T Gt[HD * Cfg<T>::VSTR];
    __shared__ float lse_s[KC], dl_s[KC];
    __shared__ __attribute__((aligned(16))) float wts[HD * 10];
    __shared__ __attribute__((aligned(16))) unsigned char dtbl[4][128];

    const Win w = decode_block(a);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const T* img = qkv + (size_t)w.b * L * C3;
    const T* gimg = dout + (size_t)w.b * L * C;
    const int kn = w.blk * QR + wave * 32 + r;
    const bool kvalid = kn < w.N;
    const bool wave_active = w.blk * QR + wave * 32 < w.N;
    const int ktok = kvalid ? tok_of(w, a.reso, kn) : 0;

    stage_lepe_weights(branch(a, w.br), w.h, wts);
    Frag<T> kf, vf;
    load_frag(kf, img + (size_t)ktok * C3 + C + w.chq, h, kvalid);
    load_frag(vf, img + (size_t)ktok * C3 + 2 * C + w.chq, h, kvalid);

    const float c = a.scale * kLog2e;
    f32x16 dk = {}, dv = {};
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);
    for (int q0 = 0; q0 < w.N; q0 += KC) {
        __syncthreads();
        stage_rows<T>(w, a.reso, img, C3, w.chq, q0, w.N, Qs, Qt);
        stage_rows<T>(w, a.reso, gimg, C, w.chq, q0, w.N, Gs, Gt);
        for (int i = threadIdx.x; i < KC; i += NT) {
            const int n = q0 + i;
            const bool v = n < w.N;
            const size_t si = stat_index(a, w, v ? tok_of(w, a.reso, n) : 0);
            lse_s[i] = v ? lse[si] * kLog2e : INFINITY;   // +inf -> p = 0 for padded queries
            dl_s[i] = v ? delta[si] : 0.f;
        }
        __syncthreads();
        if (!wave_active) continue;
        const int nq = min(KC, w.N - q0);
        for (int qb = 0; qb < nq; qb += 32) {
            f32x16 s = {}, dp = {};
            mma_rows(s, Qs + qb * Cfg<T>::KSTR, r, h, kf);    // S[q][key]
            mma_rows(dp, Gs + qb * Cfg<T>::KSTR, r, h, vf);   // dP[q][key]
            unsigned km = 0xffffu;
            if constexpr (DROP) km = keep_k16(dr, q0 + qb, w.blk * QR + wave * 32, lane, dtbl[wave]);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int qi = qb + crow(i, h);
                const float p = exp2f(s[i] * c - lse_s[qi]);
                float ps = p, g = dp[i];
                if constexpr (DROP) {
                    const float ms = ((km >> i) & 1u) ? dr.R.scale : 0.f;
                    ps = p * ms;
                    g *= ms;
                }
                s[i] = ps;                         // dropped P: dV^T += dO^T P_drop
                dp[i] = p * (g - dl_s[qi]);        // dS
            }
            mma_acc_operand(dv, Gt, qb, r, h, s);    // dV^T += dO^T P
            mma_acc_operand(dk, Qt, qb, r, h, dp);   // dK^T += Q^T dS
        }
    }
    if (!kvalid) return;
    T* drow = dqkv + ((size_t)w.b * L + ktok) * C3 + w.chq;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 8 * g4 + 4 * h;
        float vk[4], vv[4], lp[4];
        lepe4<T>(w, a.reso, gimg, C, w.chq, kn, d0, wts, -1, lp);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            vk[j] = dk[4 * g4 + j] * a.scale;
            vv[j] = dv[4 * g4 + j] + lp[j];
        }
        store4(drow + C + d0, vk);
        store4(drow + 2 * C + d0, vv);
    }
}

// =============================================================================================
// LePE weight/bias gradient: dW[c][t] = sum_q dout[q][c] * V[q + off(t)][c], db[c] = sum_q dout
// (window-local zero padding).  Pass 1: grid-stride over (image row, XR-token run) units with a
// fixed channel quad per thread: each unit issues all its loads at once (V of the 3 x (XR+2)
// neighbourhood and dout of the XR tokens; clamped addresses and 0/1 masks instead of branches, so
// the loads stay in flight together), then 40 FMAs per token.  Per-block partials are combined in
// thread order; pass 2 sums the block partials in a fixed order (deterministic).
// =============================================================================================
constexpr int XR = 4;            // tokens per run
constexpr int LW_MAXBLK = 512;   // pass-1 blocks per branch

template <typename T> struct Raw4;   // 4 channels as loaded (8 B bf16 / 16 B fp32)
template <> struct Raw4<bf16> {
    typedef bf16x4 type;
    static __device__ __forceinline__ float at(const type& v, int j) { return (float)v[j]; }
};
template <> struct Raw4<float> {
    typedef f32x4 type;
    static __device__ __forceinline__ float at(const type& v, int j) { return v[j]; }
};

template <typename T>
__global__ __launch_bounds__(NT, 4) void lepe_wgrad_partial(csu_stripe_args a, const T* __restrict__ qkv,
                                                         const T* __restrict__ dout, float* __restrict__ part) {
    typedef typename Raw4<T>::type R4;
    __shared__ float red[4][64][11];
    const int br = blockIdx.y;
    const csu_stripe_branch& g = branch(a, br);
    const int Cb = a.heads * HD, nq = Cb / 4;       // power of two dividing NT (checked by the caller)
    const int reso = a.reso, L = reso * reso, C = a.C, C3 = 3 * C;
    const int nseg = (reso + XR - 1) / XR;
    const long runs = (long)a.B * reso * nseg;
    const int per_blk = NT / nq;
    const int cq = threadIdx.x % nq;
    const int c0 = g.ch_off + 4 * cq;
    float acc[40];   // [k][j]: tap k (9 = bias) x channel j of the quad
#pragma unroll
    for (int i = 0; i < 40; ++i) acc[i] = 0.f;
    // XCD-aware: consecutive logical blocks (adjacent image rows, which share V neighbourhood rows)
    // run on one XCD
    const long lb = xcd_tile(blockIdx.x, gridDim.x);
    for (long ri = lb * per_blk + threadIdx.x / nq; ri < runs; ri += (long)gridDim.x * per_blk) {
        const int seg = (int)(ri % nseg);
        const long r2 = ri / nseg;
        const int y = (int)(r2 % reso), b = (int)(r2 / reso);
        const int x0 = seg * XR, iy = y % g.H_sp;
        const T* vimg = qkv + (size_t)b * L * C3 + 2 * C + c0;
        const T* gimg = dout + (size_t)b * L * C + c0;
        R4 vw[3][XR + 2], gv[XR];
        unsigned mask = 0;   // bit dy*(XR+2)+cx: V neighbour inside the image; bit 30-XR+tx: token inside
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const int yy = y + dy - 1;
            const bool yok = iy + dy - 1 >= 0 && iy + dy - 1 < g.H_sp;
            const int yc = min(max(yy, 0), reso - 1);
#pragma unroll
            for (int cx = 0; cx < XR + 2; ++cx) {
                const int xx = x0 - 1 + cx;
                vw[dy][cx] = *reinterpret_cast<const R4*>(vimg + (size_t)(yc * reso + min(max(xx, 0), reso - 1)) * C3);
                mask |= (yok && xx >= 0 && xx < reso) ? 1u << (dy * (XR + 2) + cx) : 0u;
            }
        }
#pragma unroll
        for (int tx = 0; tx < XR; ++tx)
            gv[tx] = *reinterpret_cast<const R4*>(gimg + (size_t)(y * reso + min(x0 + tx, reso - 1)) * C);
#pragma unroll
        for (int tx = 0; tx < XR; ++tx) {
            const int x = x0 + tx, ix = x % g.W_sp;
            if (x >= reso) break;
            const float mx[3] = {ix > 0 ? 1.f : 0.f, 1.f, ix + 1 < g.W_sp ? 1.f : 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float gj = Raw4<T>::at(gv[tx], j);
                acc[36 + j] += gj;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const float m = ((mask >> (dy * (XR + 2) + tx + dx)) & 1u) ? mx[dx] : 0.f;
                        acc[(dy * 3 + dx) * 4 + j] += gj * m * Raw4<T>::at(vw[dy][tx + dx], j);
                    }
            }
        }
    }
    // threads sharing a quad: lanes l ^ (nq, 2nq, ..) inside a wave (fixed xor tree), then the 4
    // waves through LDS, 10 values per pass
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int m = nq; m < 64; m <<= 1)
#pragma unroll
        for (int i = 0; i < 40; ++i) acc[i] += __shfl_xor(acc[i], m, 64);
    const int slots = nq < 64 ? nq : 64;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (lane < slots)
#pragma unroll
            for (int e = 0; e < 10; ++e) red[wave][lane][e] = acc[p * 10 + e];
        __syncthreads();
        for (int o = threadIdx.x; o < nq * 10; o += NT) {
            const int q = o / 10, e = o % 10, l = q % 64;
            float sum = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w)
                if ((w * 64 + l) % nq == q) sum += red[w][l][e];
            const int kj = p * 10 + e, k = kj >> 2, c = 4 * q + (kj & 3);
            part[((size_t)br * Cb * 10 + c * 10 + k) * gridDim.x + blockIdx.x] = sum;   // [branch][value][block]
        }
        __syncthreads();
    }
}

// LePE weight gradient, tiled (bf16 / fp32): block = (image b, TY image rows, one head's 32
// channels of one branch).  The rows' dout and the V rows with a one-row halo are staged in LDS
// with 16-B loads (each token's head slice is one contiguous 64 / 128-B piece), then thread
// (quad q, token lane) accumulates dW[c][tap] += dout[q][c] * V[q + off(tap)][c] (window-local
// zero padding) and db[c] += dout[q][c] for 4 channels over the tile's tokens from LDS; the 32
// token lanes of a quad are reduced by a fixed xor tree + the 4 waves in order.  Partial layout
// [branch][c * 10 + tap][block] as lepe_wgrad_partial's, block = b * nty + row tile.
template <typename T>
__global__ __launch_bounds__(NT) void lepe_wgrad_tiles(csu_stripe_args a, int ty_rows, int rows_blk,
                                                      const T* __restrict__ qkv, const T* __restrict__ dout,
                                                      float* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lw_smem[];
    __shared__ float red[4][8][40];
    typedef typename Raw4<T>::type R4;
    constexpr int CPT = HD * (int)sizeof(T) / 16;   // 16-B chunks per token slice
    const int br = blockIdx.z, head = blockIdx.y;
    const csu_stripe_branch& g = branch(a, br);
    const int reso = a.reso, L = reso * reso, C = a.C, C3 = 3 * C;
    const int nrb = (reso + rows_blk - 1) / rows_blk;   // row blocks per image
    const int b = blockIdx.x / nrb, yb = (blockIdx.x % nrb) * rows_blk, ye = min(reso, yb + rows_blk);
    const int ch = g.ch_off + head * HD;
    T* Vt = reinterpret_cast<T*>(lw_smem);                       // [(ty + 2)][reso][HD]
    T* Gt = Vt + (size_t)(ty_rows + 2) * reso * HD;             // [ty][reso][HD]
    const int vrows = ty_rows + 2;
    const int nchunk = (vrows + ty_rows) * reso * CPT;
    const int q = threadIdx.x & 7, tl = threadIdx.x >> 3;
    float acc[40];
#pragma unroll
    for (int i = 0; i < 40; ++i) acc[i] = 0.f;
    for (int y0 = yb; y0 < ye; y0 += ty_rows) {   // row tiles of this block, one reduction at the end
    constexpr int IT = 8;   // 16-B loads in flight per thread before their LDS stores
    for (int base = 0; base < nchunk; base += IT * NT) {
        u32x4 v[IT];
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int i = base + u * NT + threadIdx.x;
            const int part_ = i % CPT, tok = (i / CPT) % reso, row = i / (CPT * reso);
            const bool isv = row < vrows;
            const int y = isv ? y0 - 1 + row : y0 + row - vrows;
            v[u] = u32x4{0, 0, 0, 0};
            if (i < nchunk && y >= 0 && y < reso) {
                const T* src = isv ? qkv + ((size_t)b * L + (size_t)y * reso + tok) * C3 + 2 * C + ch
                                   : dout + ((size_t)b * L + (size_t)y * reso + tok) * C + ch;
                v[u] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned char*>(src) + 16 * part_);
            }
        }
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int i = base + u * NT + threadIdx.x;
            if (i >= nchunk) break;
            const int part_ = i % CPT, tok = (i / CPT) % reso, row = i / (CPT * reso);
            T* dst = row < vrows ? Vt + ((size_t)row * reso + tok) * HD : Gt + ((size_t)(row - vrows) * reso + tok) * HD;
            *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(dst) + 16 * part_) = v[u];
        }
    }
    __syncthreads();
    const int ntok = ty_rows * reso;
    for (int t = tl; t < ntok; t += NT / 8) {
        const int yy = t / reso, x = t - yy * reso, y = y0 + yy;
        if (y >= ye) break;
        const int iy = y % g.H_sp, ix = x % g.W_sp;
        const R4 gq = *reinterpret_cast<const R4*>(Gt + ((size_t)yy * reso + x) * HD + 4 * q);
        // all 9 neighbour reads issued unconditionally (clamped columns; the halo rows are staged,
        // zero outside the image), window-local padding applied as a 0 / 1 factor
        const int xs[3] = {max(x - 1, 0), x, min(x + 1, reso - 1)};
        R4 vq[3][3];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
                vq[dy][dx] = *reinterpret_cast<const R4*>(Vt + ((size_t)(yy + dy) * reso + xs[dx]) * HD + 4 * q);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const bool yok = iy + dy - 1 >= 0 && iy + dy - 1 < g.H_sp;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const float m = (yok && ix + dx - 1 >= 0 && ix + dx - 1 < g.W_sp) ? 1.f : 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[(dy * 3 + dx) * 4 + j] += Raw4<T>::at(gq, j) * (m * Raw4<T>::at(vq[dy][dx], j));
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[36 + j] += Raw4<T>::at(gq, j);
    }
    __syncthreads();   // the next row tile overwrites the images
    }
    // token lanes of a quad: lane bits 3..5 inside the wave, then the 4 waves in order
#pragma unroll
    for (int m = 8; m < 64; m <<= 1)
#pragma unroll
        for (int i = 0; i < 40; ++i) acc[i] += __shfl_xor(acc[i], m, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane < 8)
#pragma unroll
        for (int i = 0; i < 40; ++i) red[wave][lane][i] = acc[i];
    __syncthreads();
    const int Cb = a.heads * HD, nblk = a.B * nrb;
    for (int o = threadIdx.x; o < 8 * 40; o += NT) {
        const int qq = o / 40, i = o % 40;
        const float sum = ((red[0][qq][i] + red[1][qq][i]) + red[2][qq][i]) + red[3][qq][i];
        const int k = i >> 2, c = head * HD + 4 * qq + (i & 3);
        part[((size_t)br * Cb * 10 + c * 10 + k) * nblk + blockIdx.x] = sum;
    }
}

// rows per LePE tile so that the staged V (+halo) and dout fit 64 KiB of dynamic LDS (two blocks
// per CU); 0: use the untiled kernel
int lepe_tile_rows(const csu_stripe_args& a, int dtype) {
    const size_t es = dtype == CSU_BF16 ? 2 : 4;
    for (int ty : {4, 2, 1})
        if ((size_t)(2 * ty + 2) * a.reso * HD * es <= 64 * 1024) return ty;
    return 0;
}

// rows per LePE block (a multiple of the tile rows): about 512 blocks per launch, so each block
// amortises its reduction over several row tiles
int lepe_rows_blk(const csu_stripe_args& a, int ty) {
    const long per_img = (long)a.B * a.heads * a.nbranch;
    long nrb = 512 / per_img;
    const long nty = (a.reso + ty - 1) / ty;
    if (nrb > nty) nrb = nty;
    if (nrb < 1) nrb = 1;
    const long rows = (a.reso + nrb - 1) / nrb;
    return (int)((rows + ty - 1) / ty * ty);
}

// one wave per (branch, value): lanes stride over the block partials (contiguous), then a fixed
// xor-shuffle tree -- deterministic
// 16 lanes per value (the block partials are 32..128 per value at the model's sizes: a wave per value
// left lanes idle and launched 4x the waves); shared with lepe_reduce_batch, so the deferred batched
// reduction is bitwise equal to this one
// (nblk % 4 == 0: 16-B loads of 4 consecutive partials, four in flight per lane -- the fused
// backward leaves B * windows = 256..2048 partials per value, ~60 MB per step at 512x512 B16)
__device__ __forceinline__ float lepe_value_sum(const float* __restrict__ src, int nblk, int sub) {
    float s;
    if ((nblk & 3) == 0) {
        f32x4 a0 = {}, a1 = {}, a2 = {}, a3 = {};
        auto ld = [&](int j) { return *reinterpret_cast<const f32x4*>(src + j); };
        int j = 4 * sub;
        for (; j + 192 < nblk; j += 256) {
            a0 += ld(j);
            a1 += ld(j + 64);
            a2 += ld(j + 128);
            a3 += ld(j + 192);
        }
        for (; j < nblk; j += 64) a0 += ld(j);
        const f32x4 t = (a0 + a1) + (a2 + a3);
        s = (t[0] + t[1]) + (t[2] + t[3]);
    } else {
        s = strided_sum<16>(src, nblk, sub);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
}

__global__ __launch_bounds__(256) void lepe_wgrad_reduce(csu_stripe_args a, int nblk, const float* __restrict__ part) {
    const int Cb = a.heads * HD, vt = a.nbranch * Cb * 10;
    const int v = blockIdx.x * 16 + (threadIdx.x >> 4), sub = threadIdx.x & 15;
    const float s = lepe_value_sum(part + (size_t)(v < vt ? v : vt - 1) * nblk, nblk, sub);
    if (sub == 0 && v < vt) {
        const int br = v / (Cb * 10), i = v % (Cb * 10);
        const csu_stripe_branch& g = branch(a, br);
        const int c = i / 10, k = i % 10;
        if (k < 9) g.lepe_dw[c * 9 + k] = s;
        else g.lepe_db[c] = s;
    }
}

int wgrad_blocks(const csu_stripe_args& a) {
    const long items = (long)a.B * a.reso * ((a.reso + XR - 1) / XR) * (a.heads * HD / 4);
    const long blk = (items + NT - 1) / NT;
    return (int)(blk < LW_MAXBLK ? blk : LW_MAXBLK);
}

// =============================================================================================
// v2 (bf16, window <= 1024 tokens -- every stage of the 512x512 and 1024x1024 models): the whole
// window of the head is resident in LDS (images sized WM = 256 / 512 / 1024 tokens per launch).  Images are "natural" [token][32] rows of 64 B whose 16-B chunks are
// XOR-swizzled by (row >> 2) & 3, which makes the 32-row ds_read_b128 fragment reads AND the
// gfx950 transposing reads (ds_read_b64_tr_b16) used for the V^T / K^T / Q^T / dO^T operands
// bank-conflict free; LePE neighbours are read from the same images.  One image serves both
// orientations, so nothing is ever written transposed.
// =============================================================================================
constexpr int WMAX = 1024;  // largest window held in LDS (K + V images: 128 KiB of the 160 KiB)

#ifdef WG_TIMING   // debug build only: per-workgroup phase stamps (100 MHz) of the last launch of each
                   // whole-window kernel (0 fwd, 1 dq, 2 dkdv): start, staged, end + hardware id
__device__ unsigned long long attn_ts[3][6][16384];
#define ATT_STAMP(kern, k) do { \
    const unsigned _b = blockIdx.x + blockIdx.y * gridDim.x; \
    if (threadIdx.x == 0 && _b < 16384) { \
        attn_ts[kern][k][_b + threadIdx.x] = __builtin_amdgcn_s_memrealtime(); \
        if (k == 0) attn_ts[kern][5][_b + threadIdx.x] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)); } } while (0)
#else
#define ATT_STAMP(kern, k) do {} while (0)
#endif
typedef float f2 __attribute__((ext_vector_type(2)));   // packed-f32 pairs (v_pk_fma/mul/add_f32)

__device__ __forceinline__ int swz(int row, int col) {   // element offset in a swizzled image
    return row * HD + ((((col >> 3) ^ (row >> 2)) & 3) << 3) + (col & 7);
}

typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4s tr_read(const bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}

// ---- branch-free global loads for the whole-window kernels: raw buffer loads whose masked lanes
// get an out-of-range offset (read as 0).  A predicated `cond ? *p : 0` load compiles to an
// exec-masked branch and hipcc waits vmcnt(0) at every join, which serialised the staging loads
// (10-12 full waits before the first barrier) instead of keeping them in flight together.
__device__ __forceinline__ bf16x8 ld8_rs(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    bf16x8 b;
    __builtin_memcpy(&b, &v, 16);
    return b;
}
__device__ __forceinline__ float ldf_rs(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
}
// fragment of row (element offset `row` of the resource), lane half h
__device__ __forceinline__ void load_frag_rs(Frag<bf16>& f, __amdgpu_buffer_rsrc_t rs, size_t row, int h, bool valid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) f.v[s] = ld8_rs(rs, valid ? (unsigned)((row + 16 * s + 8 * h) * 2) : kOOB);
}
// per-(branch, image, head) statistics (lse / delta) tensor of the launch
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stat_rsrc(const csu_stripe_args& a, const float* p) {
    return buf_rsrc(p, (long)a.nbranch * a.B * a.heads * a.reso * a.reso * 4);
}

// A operand of X^T-orientation products: lane (r = channel d, h) gets image[k][d] for
// k = kbase + 16s + 8(j>>2) + 4h + (j&3), the k order of an accumulator tile used as B operand.
__device__ __forceinline__ bf16x8 tr_frag_acc(const bf16* img, int kbase, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = 16 * (grp & 1) + 4 * p;
    const int row = kbase + 16 * s + 4 * (grp >> 1) + q;
    const v4s lo = tr_read(img + swz(row, col));
    const v4s hi = tr_read(img + swz(row + 8, col));
    const v4s v[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

// acc += A(32 rows of the image starting at row0) * B^T, A rows read as 16-B fragments
__device__ __forceinline__ void mma_rows_sw(f32x16& acc, const bf16* img, int row0, int r, int h, const Frag<bf16>& B) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(img + swz(row0 + r, 16 * s + 8 * h));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, B.v[s], acc, 0, 0, 0);
    }
}

__device__ __forceinline__ void mma_acc_sw(f32x16& acc, const bf16* img, int kbase, int lane, const f32x16& X) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        bf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = (bf16)X[8 * s + j];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_frag_acc(img, kbase, s, lane), b, acc, 0, 0, 0);
    }
}

// gather the window rows [0, npad) of one head's channels of two tensors into swizzled images
// (rows >= N zero).  All global loads of the thread are issued before the first LDS store, so the
// staging costs one memory latency instead of one per row group.
template <int NTH = NT>
__device__ __forceinline__ void stage_win2(const Win& w, int reso, const bf16* imgA, int strideA, int chA,
                                           const bf16* imgB, int strideB, int chB, int npad, bf16* dstA, bf16* dstB) {
    constexpr int IT = 4;   // NTH rows per pass: 8 x 16-B loads in flight per thread
    const long L = (long)reso * reso;
    const __amdgpu_buffer_rsrc_t rsA = buf_rsrc(imgA, L * strideA * 2), rsB = buf_rsrc(imgB, L * strideB * 2);
    for (int base = 0; base < npad * 4; base += IT * NTH) {
        bf16x8 va[IT], vb[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const int it = base + threadIdx.x + i * NTH;
            const int n = it >> 2, c = (it & 3) * 8;
            const bool ok = it < npad * 4 && n < w.N;
            const unsigned tok = ok ? (unsigned)tok_of(w, reso, n) : 0u;
            va[i] = ld8_rs(rsA, ok ? (tok * (unsigned)strideA + chA + c) * 2u : kOOB);
            vb[i] = ld8_rs(rsB, ok ? (tok * (unsigned)strideB + chB + c) * 2u : kOOB);
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const int it = base + threadIdx.x + i * NTH;
            if (it < npad * 4) {
                const int n = it >> 2, c = (it & 3) * 8;
                *reinterpret_cast<bf16x8*>(dstA + swz(n, c)) = va[i];
                *reinterpret_cast<bf16x8*>(dstB + swz(n, c)) = vb[i];
            }
        }
    }
}

// LePE of window position n, channels c0..c0+3, from a swizzled LDS image; wts in the [tap][channel]
// layout of lepe_weights_store
__device__ __forceinline__ void lepe4_lds(const Win& w, const bf16* img, int n, int c0, const float* wts, int sign,
                                          float* acc) {
    const int iy = wrow(w, n), ix = n - iy * w.W_sp;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(wts + HD * 9 + c0);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = sign > 0 ? bias[j] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int dy = sign * (t / 3 - 1), dx = sign * (t % 3 - 1);
        const int y = iy + dy, x = ix + dx;
        if (y < 0 || y >= w.H_sp || x < 0 || x >= w.W_sp) continue;
        const bf16x4 v = *reinterpret_cast<const bf16x4*>(img + swz(y * w.W_sp + x, c0));
        const f32x4 wt = *reinterpret_cast<const f32x4*>(wts + t * HD + c0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += wt[j] * (float)v[j];
    }
}

__device__ __forceinline__ Win decode_w(const csu_stripe_args& a, int split) {
    Win w;
    w.br = blockIdx.y;
    const csu_stripe_branch& g = branch(a, w.br);
    w.H_sp = g.H_sp;
    w.W_sp = g.W_sp;
    w.rW = __frcp_rn((float)g.W_sp);
    w.N = w.H_sp * w.W_sp;
    const int nwx = a.reso / w.W_sp, nwin = (a.reso / w.H_sp) * nwx;
    // XCD-aware order: the split partners of a window-head (consecutive logical ids) run on one
    // XCD, so the window's K/V gather is fetched into that XCD's L2 once
    int id = (int)xcd_tile(blockIdx.x, gridDim.x);
    w.blk = id % split; id /= split;
    w.h = id % a.heads; id /= a.heads;
    const int win = id % nwin;
    w.b = id / nwin;
    w.wy = win / nwx;
    w.wx = win % nwx;
    w.chq = g.ch_off + w.h * HD;
    return w;
}

template <int WM, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW) void stripe_fwd_w(csu_stripe_args a, int split, const bf16* __restrict__ qkv,
                                                        bf16* __restrict__ out, float* __restrict__ lse) {
    __shared__ __attribute__((aligned(16))) bf16 Ks[WM * HD];
    __shared__ __attribute__((aligned(16))) bf16 Vs[WM * HD];
    __shared__ __attribute__((aligned(16))) float wts[HD * 10];
    ATT_STAMP(0, 0);
    const Win w = decode_w(a, split);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const bf16* img = qkv + (size_t)w.b * L * C3;
    const int npad = (w.N + 31) & ~31;
    const int rows = (((npad + split - 1) / split) + 31) & ~31;   // query rows of this workgroup (32-aligned)
    const int qbeg = w.blk * rows, qend = min(npad, qbeg + rows);
    // this wave's first query fragment is loaded together with the K/V staging loads
    Frag<bf16> qnext;
    const __amdgpu_buffer_rsrc_t rs_img = buf_rsrc(img, (long)L * C3 * 2);
    {
        const int qn = qbeg + 32 * wave + r;
        const bool qv = qbeg + 32 * wave < qend && qn < w.N;
        load_frag_rs(qnext, rs_img, (size_t)(qv ? tok_of(w, a.reso, qn) : 0) * C3 + w.chq, h, qv);
    }
    float lw[LW_IT];
    lepe_weights_load(branch(a, w.br), w.h, lw);
    stage_win2<64 * NW>(w, a.reso, img, C3, C + w.chq, img, C3, 2 * C + w.chq, (npad + 63) & ~63, Ks, Vs);  // zero rows up to a 64-key step
    lepe_weights_store(lw, wts);
    __syncthreads();
    ATT_STAMP(0, 1);
    const float c = a.scale * kLog2e;
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);
    for (int q0 = qbeg + 32 * wave; q0 < qend; q0 += 32 * NW) {
        const int qn = q0 + r;
        const bool qvalid = qn < w.N;
        const int qtok = qvalid ? tok_of(w, a.reso, qn) : 0;
        const Frag<bf16> qf = qnext;
        if (q0 + 32 * NW < qend) {
            const int qn2 = q0 + 32 * NW + r;
            const bool qv2 = qn2 < w.N;
            load_frag_rs(qnext, rs_img, (size_t)(qv2 ? tok_of(w, a.reso, qn2) : 0) * C3 + w.chq, h, qv2);
        }
        float m = -INFINITY, l = 0.f;
        f32x16 o = {};
        // 64 keys per online-softmax step: two independent S^T tiles, one rescale of O.  VALU per
        // score: 1/2 v_max3, 1/2 v_pk_fma (scale and max shift folded), v_exp, 1/2 v_pk_add; the
        // key mask only on the tail step (uniform branch)
        auto step = [&](int kb, auto masked) {
            f32x16 s0 = {}, s1 = {};
            mma_rows_sw(s0, Ks, kb, r, h, qf);
            mma_rows_sw(s1, Ks, kb + 32, r, h, qf);
            if constexpr (decltype(masked)::value) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (kb + crow(i, h) >= w.N) s0[i] = -INFINITY;
                    if (kb + 32 + crow(i, h) >= w.N) s1[i] = -INFINITY;
                }
            }
            float mn = m;   // raw-score running max (scale applied in the exponent)
#pragma unroll
            for (int i = 0; i < 16; ++i) mn = fmaxf(mn, fmaxf(s0[i], s1[i]));
            mn = fmaxf(mn, __shfl_xor(mn, 32, 64));
            const float alpha = __builtin_amdgcn_exp2f((m - mn) * c);
            m = mn;
            const f2 cc = {c, c}, mc = {mn * c, mn * c};
            f2 ls = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                f2 a = f2{s0[i], s0[i + 1]} * cc - mc;
                f2 b = f2{s1[i], s1[i + 1]} * cc - mc;
                a = f2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
                b = f2{__builtin_amdgcn_exp2f(b.x), __builtin_amdgcn_exp2f(b.y)};
                s0[i] = a.x; s0[i + 1] = a.y;
                s1[i] = b.x; s1[i + 1] = b.y;
                ls += a + b;
            }
            l = l * alpha + (ls.x + ls.y);
            const f2 al = {alpha, alpha};
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const f2 ov = f2{o[i], o[i + 1]} * al;
                o[i] = ov.x; o[i + 1] = ov.y;
            }
            if constexpr (DROP) {   // the normaliser l keeps every key; O sees the dropped P
                const unsigned k0m = keep_q16(dr, qn, kb, h), k1m = keep_q16(dr, qn, kb + 32, h);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    s0[i] = ((k0m >> i) & 1u) ? s0[i] * dr.R.scale : 0.f;
                    s1[i] = ((k1m >> i) & 1u) ? s1[i] * dr.R.scale : 0.f;
                }
            }
            mma_acc_sw(o, Vs, kb, lane, s0);
            mma_acc_sw(o, Vs, kb + 32, lane, s1);
        };
        const int nfull = w.N & ~63;   // steps without a key tail: no mask at all
        for (int kb = 0; kb < nfull; kb += 64) step(kb, std::false_type{});
        if (nfull < w.N) step(nfull, std::true_type{});
        const float lt = l + __shfl_xor(l, 32, 64);
        if (!qvalid) continue;
        const float inv = 1.f / lt;
        if (h == 0) lse[stat_index(a, w, qtok)] = (m * c + log2f(lt)) * kLn2;   // m is the raw-score max
        bf16* orow = out + ((size_t)w.b * L + qtok) * C + w.chq;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 8 * g4 + 4 * h;
            float lp[4], v[4];
            lepe4_lds(w, Vs, qn, d0, wts, +1, lp);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = o[4 * g4 + j] * inv + lp[j];
            store4(orow + d0, v);
        }
    }
    ATT_STAMP(0, 2);
}

template <int WM, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW) void stripe_bwd_dq_w(csu_stripe_args a, int split, const bf16* __restrict__ qkv,
                                                      const bf16* __restrict__ out, const bf16* __restrict__ dout,
                                                      const float* __restrict__ lse, float* __restrict__ delta,
                                                      bf16* __restrict__ dqkv) {
    __shared__ __attribute__((aligned(16))) bf16 Ks[WM * HD];
    __shared__ __attribute__((aligned(16))) bf16 Vs[WM * HD];
    __shared__ __attribute__((aligned(16))) float wts[HD * 10];
    ATT_STAMP(1, 0);
    const Win w = decode_w(a, split);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const bf16* img = qkv + (size_t)w.b * L * C3;
    const bf16* oimg = out + (size_t)w.b * L * C;
    const bf16* gimg = dout + (size_t)w.b * L * C;
    const int npad = (w.N + 31) & ~31;
    const int rows = (((npad + split - 1) / split) + 31) & ~31;   // 32-aligned: mask groups start on 8
    const int qbeg = w.blk * rows, qend = min(npad, qbeg + rows);
    // the wave's query-block operands (Q, dO and O fragments, lse): the first block's are loaded
    // with the staging loads, so their latency overlaps the K/V staging; later blocks (only when a
    // workgroup owns > 128 query rows: the 1024x1024 stages) load at the top of their iteration
    Frag<bf16> qf, gf, of;
    float lq_raw;
    const __amdgpu_buffer_rsrc_t rs_img = buf_rsrc(img, (long)L * C3 * 2), rs_g = buf_rsrc(gimg, (long)L * C * 2),
                                 rs_o = buf_rsrc(oimg, (long)L * C * 2), rs_lse = stat_rsrc(a, lse);
    auto load_q = [&](int q0) {
        const int qn = q0 + r;
        const bool qv = q0 < qend && qn < w.N;
        const size_t t = qv ? tok_of(w, a.reso, qn) : 0;
        load_frag_rs(qf, rs_img, t * C3 + w.chq, h, qv);
        load_frag_rs(gf, rs_g, t * C + w.chq, h, qv);
        load_frag_rs(of, rs_o, t * C + w.chq, h, qv);
        lq_raw = ldf_rs(rs_lse, qv ? (unsigned)(stat_index(a, w, (int)t) * 4) : kOOB);
    };
    load_q(qbeg + 32 * wave);
    float lw[LW_IT];
    lepe_weights_load(branch(a, w.br), w.h, lw);
    stage_win2<64 * NW>(w, a.reso, img, C3, C + w.chq, img, C3, 2 * C + w.chq, npad, Ks, Vs);
    lepe_weights_store(lw, wts);
    __syncthreads();
    ATT_STAMP(1, 1);
    const float c = a.scale * kLog2e;
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);
    for (int q0 = qbeg + 32 * wave; q0 < qend; q0 += 32 * NW) {
        const int qn = q0 + r;
        const bool qvalid = qn < w.N;
        const int qtok = qvalid ? tok_of(w, a.reso, qn) : 0;
        if (q0 != qbeg + 32 * wave) load_q(q0);
        // delta = rowsum(dO * (O - LePE)) = rowsum(dO * attention output), over the fragment's 16
        // channels (16 s + 8 h + 0..7) of this lane, then the other half's
        float dl = 0.f;
        if (qvalid) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int p4 = 0; p4 < 2; ++p4) {
                    float lp[4];
                    lepe4_lds(w, Vs, qn, 16 * s2 + 8 * h + 4 * p4, wts, +1, lp);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        dl += (float)gf.v[s2][4 * p4 + j] * ((float)of.v[s2][4 * p4 + j] - lp[j]);
                }
        }
        dl += __shfl_xor(dl, 32, 64);
        const size_t si = stat_index(a, w, qtok);
        if (qvalid && h == 0) delta[si] = dl;
        const float lq = qvalid ? lq_raw * kLog2e : 0.f;
        f32x16 dq = {};
        const f2 cc = {c, c}, lq2 = {lq, lq}, dl2 = {dl, dl};
        for (int kb = 0; kb < npad; kb += 32) {
            f32x16 s = {}, dp = {};
            mma_rows_sw(s, Ks, kb, r, h, qf);
            mma_rows_sw(dp, Vs, kb, r, h, gf);
            if constexpr (DROP) {   // dP through the mask
                const unsigned km = keep_q16(dr, qn, kb, h);
#pragma unroll
                for (int i = 0; i < 16; ++i) dp[i] = ((km >> i) & 1u) ? dp[i] * dr.R.scale : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 16; i += 2) {   // dS = P dP - P delta, packed pairs
                f2 p = f2{s[i], s[i + 1]} * cc - lq2;
                p = f2{__builtin_amdgcn_exp2f(p.x), __builtin_amdgcn_exp2f(p.y)};
                const f2 t = p * f2{dp[i], dp[i + 1]} - p * dl2;
                s[i] = t.x; s[i + 1] = t.y;
            }
            // no key mask: keys >= N have zero K rows in LDS, so their dS rows add nothing to dQ
            mma_acc_sw(dq, Ks, kb, lane, s);
        }
        if (!qvalid) continue;
        bf16* drow = dqkv + ((size_t)w.b * L + qtok) * C3 + w.chq;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 8 * g4 + 4 * h;
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = dq[4 * g4 + j] * a.scale;
            store4(drow + d0, v);
        }
    }
    ATT_STAMP(1, 2);
}

template <int WM, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW) void stripe_bwd_dkdv_w(csu_stripe_args a, int split, const bf16* __restrict__ qkv,
                                                        const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                        const float* __restrict__ delta, bf16* __restrict__ dqkv) {
    __shared__ __attribute__((aligned(16))) bf16 Qs[WM * HD];
    __shared__ __attribute__((aligned(16))) bf16 Gs[WM * HD];
    __shared__ __attribute__((aligned(16))) float lse_s[WM], dl_s[WM];
    __shared__ __attribute__((aligned(16))) float wts[HD * 10];
    __shared__ __attribute__((aligned(16))) unsigned char dtbl[NW][128];
    ATT_STAMP(2, 0);
    const Win w = decode_w(a, split);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const bf16* img = qkv + (size_t)w.b * L * C3;
    const bf16* gimg = dout + (size_t)w.b * L * C;
    const int npad = (w.N + 31) & ~31;
    const int rows = (((npad + split - 1) / split) + 31) & ~31;   // 32-aligned: mask groups start on 8
    const int kbeg = w.blk * rows, kend = min(npad, kbeg + rows);
    // the wave's key-block fragments: the first block's are loaded with the staging loads; later
    // blocks (only when a workgroup owns > 128 key rows: the 1024x1024 stages) load at the top of
    // their iteration -- no second register set, so the kernel stays at <= 128 VGPRs (4 waves/SIMD)
    Frag<bf16> kf, vf;
    const __amdgpu_buffer_rsrc_t rs_img = buf_rsrc(img, (long)L * C3 * 2);
    {
        const int kn = kbeg + 32 * wave + r;
        const bool kv = kbeg + 32 * wave < kend && kn < w.N;
        const size_t t = kv ? tok_of(w, a.reso, kn) : 0;
        load_frag_rs(kf, rs_img, t * C3 + C + w.chq, h, kv);
        load_frag_rs(vf, rs_img, t * C3 + 2 * C + w.chq, h, kv);
    }
    float lw[LW_IT];
    lepe_weights_load(branch(a, w.br), w.h, lw);
    {   // per-query statistics of the window: loads issued with the staging loads
        const __amdgpu_buffer_rsrc_t rs_lse = stat_rsrc(a, lse), rs_dl = stat_rsrc(a, delta);
        constexpr int NTH = 64 * NW, SI = WM / NTH;   // WM >= npad rows, one stat per thread per pass
        static_assert(SI * NTH == WM, "stripe_bwd_dkdv_w: WM a multiple of the workgroup");
        float lv[SI], dv2[SI];
#pragma unroll
        for (int k = 0; k < SI; ++k) {
            const int i = threadIdx.x + k * NTH;
            const bool v = i < w.N;
            const unsigned off = v ? (unsigned)(stat_index(a, w, tok_of(w, a.reso, i)) * 4) : kOOB;
            lv[k] = ldf_rs(rs_lse, off);
            dv2[k] = ldf_rs(rs_dl, off);
        }
        stage_win2<NTH>(w, a.reso, img, C3, w.chq, gimg, C, w.chq, npad, Qs, Gs);
        lepe_weights_store(lw, wts);
#pragma unroll
        for (int k = 0; k < SI; ++k) {
            const int i = threadIdx.x + k * NTH;
            if (i < npad) {
                lse_s[i] = i < w.N ? lv[k] * kLog2e : INFINITY;
                dl_s[i] = dv2[k];
            }
        }
    }
    __syncthreads();
    ATT_STAMP(2, 1);
    const float c = a.scale * kLog2e;
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);
    for (int k0 = kbeg + 32 * wave; k0 < kend; k0 += 32 * NW) {
        const int kn = k0 + r;
        const bool kvalid = kn < w.N;
        const int ktok = kvalid ? tok_of(w, a.reso, kn) : 0;
        if (k0 != kbeg + 32 * wave) {
            const size_t t2 = kvalid ? tok_of(w, a.reso, kn) : 0;
            load_frag_rs(kf, rs_img, t2 * C3 + C + w.chq, h, kvalid);
            load_frag_rs(vf, rs_img, t2 * C3 + 2 * C + w.chq, h, kvalid);
        }
        f32x16 dk = {}, dv = {};
        const f2 cc = {c, c};
        for (int qb = 0; qb < npad; qb += 32) {
            f32x16 s = {}, dp = {};
            mma_rows_sw(s, Qs, qb, r, h, kf);
            mma_rows_sw(dp, Gs, qb, r, h, vf);
            unsigned km = 0xffffu;
            if constexpr (DROP) {
                km = keep_k16(dr, qb, k0, lane, dtbl[wave]);
#pragma unroll
                for (int i = 0; i < 16; ++i) dp[i] = ((km >> i) & 1u) ? dp[i] * dr.R.scale : 0.f;
            }
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {   // rows qb + 8 g4 + 4 h + 0..3: one 16-B LDS read each
                const f32x4 lq = *reinterpret_cast<const f32x4*>(lse_s + qb + 8 * g4 + 4 * h);
                const f32x4 dq4 = *reinterpret_cast<const f32x4*>(dl_s + qb + 8 * g4 + 4 * h);
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
                    const int i = 4 * g4 + e;
                    f2 p = f2{s[i], s[i + 1]} * cc - f2{lq[e], lq[e + 1]};
                    p = f2{__builtin_amdgcn_exp2f(p.x), __builtin_amdgcn_exp2f(p.y)};
                    const f2 t = p * (f2{dp[i], dp[i + 1]} - f2{dq4[e], dq4[e + 1]});
                    if constexpr (DROP) {   // dV sees the dropped P
                        s[i] = ((km >> i) & 1u) ? p.x * dr.R.scale : 0.f;
                        s[i + 1] = ((km >> (i + 1)) & 1u) ? p.y * dr.R.scale : 0.f;
                    } else {
                        s[i] = p.x; s[i + 1] = p.y;
                    }
                    dp[i] = t.x; dp[i + 1] = t.y;
                }
            }
            mma_acc_sw(dv, Gs, qb, lane, s);
            mma_acc_sw(dk, Qs, qb, lane, dp);
        }
        if (!kvalid) continue;
        bf16* drow = dqkv + ((size_t)w.b * L + ktok) * C3 + w.chq;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 8 * g4 + 4 * h;
            float vk[4], vv[4], lp[4];
            lepe4_lds(w, Gs, kn, d0, wts, -1, lp);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                vk[j] = dk[4 * g4 + j] * a.scale;
                vv[j] = dv[4 * g4 + j] + lp[j];
            }
            store4(drow + C + d0, vk);
            store4(drow + 2 * C + d0, vv);
        }
    }
    ATT_STAMP(2, 2);
}

// =============================================================================================
// v3 one-pass backward (bf16, windows of <= 256 tokens: every stage of the 512x512 model, stages
// 1-2 of the 1024x1024 one).  ONE workgroup per (branch, image, window, head) stages Q, K, V and
// dO of the whole window once (swizzled images, 4 x 16 KiB) and produces dQ, dK, dV, the LePE
// input gradient AND the LePE weight-gradient partials -- v2 needed two kernels that each staged
// the window and recomputed P, plus a third kernel re-reading V and dO for the LePE weights.
//   prologue: delta = rowsum(dO * (O - LePE(V))) and the per-window LePE weight-gradient partials
//             sum_q dO[q] * V[q + tap] from the V / dO images (thread = channel quad x row group)
//   main loop over 32-query tiles (all waves in step): the key is on the lane -- wave w owns key
//             tiles w, w + 4 (dK^T, dV^T of its 64 keys stay in accumulators).  S and dP start from
//             the row constants -lse/scale and -delta (no subtraction per score), P = exp2(c S),
//             dS = P dP; dV^T += dO^T P, dK^T += Q^T dS take the accumulators as operands.  dS
//             goes to LDS once ([key][query] image in the V image's space, which the prologue
//             freed); after a barrier each wave computes a 16 x 16 quadrant of dQ^T = K^T dS over
//             ALL keys (16x16x32 MFMAs, K^T fragments held in registers), so dQ needs no sum
//             across waves or workgroups and is written once, deterministic.
// Algorithmic bytes per launch are v2's minus the delta round trip and the LePE kernel's re-read.
// =============================================================================================
typedef float f32x4v __attribute__((ext_vector_type(4)));

// 16x16x32 operand from a [k][c] swizzled image read column-wise (T10): lane l gets
// image[kb + 8 (l >> 4) + j][cb + (l & 15)], j = 0..7 -- A[m = c][k] or B[k][n = c]
__device__ __forceinline__ bf16x8 tr_frag16(const bf16* img, int kb, int cb, int lane) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const v4s lo = tr_read(img + swz(kb + 8 * g + q, cb + 4 * p));
    const v4s hi = tr_read(img + swz(kb + 8 * g + 4 + q, cb + 4 * p));
    const v4s v[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

// the fused backward's four window images in ONE pass (one memory latency instead of two): Q, K and
// dO swizzled (swz), V into a PLAIN [row][32] image; rows [N, npad) zero.  All loads of the pass are
// issued before the first LDS store (16 IT VGPRs of staged data).
template <int NTH, int WM>
__device__ __forceinline__ void stage_win4(const Win& w, int reso, const bf16* img, int C, const bf16* gimg, int npad,
                                           bf16* Qs, bf16* Ks, bf16* Vs, bf16* Gs) {
    constexpr int IT = (WM * 4 + NTH - 1) / NTH;   // 16-B items per thread (npad <= WM)
    const long L = (long)reso * reso;
    const unsigned C3 = 3u * (unsigned)C;
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(img, L * C3 * 2), rg = buf_rsrc(gimg, L * C * 2);
    bf16x8 vq[IT], vk[IT], vv[IT], vg[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int it = threadIdx.x + i * NTH;
        const int n = it >> 2, c = (it & 3) * 8;
        const bool ok = it < npad * 4 && n < w.N;
        const unsigned tok = ok ? (unsigned)tok_of(w, reso, n) : 0u;
        const unsigned oq = (tok * C3 + w.chq + c) * 2u;
        vq[i] = ld8_rs(rs, ok ? oq : kOOB);
        vk[i] = ld8_rs(rs, ok ? oq + 2u * C : kOOB);
        vv[i] = ld8_rs(rs, ok ? oq + 4u * C : kOOB);
        vg[i] = ld8_rs(rg, ok ? (tok * (unsigned)C + w.chq + c) * 2u : kOOB);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const int it = threadIdx.x + i * NTH;
        if (it < npad * 4) {
            const int n = it >> 2, c = (it & 3) * 8;
            *reinterpret_cast<bf16x8*>(Qs + swz(n, c)) = vq[i];
            *reinterpret_cast<bf16x8*>(Ks + swz(n, c)) = vk[i];
            *reinterpret_cast<bf16x8*>(Vs + n * HD + c) = vv[i];
            *reinterpret_cast<bf16x8*>(Gs + swz(n, c)) = vg[i];
        }
    }
}

// LePE (sign +1) / its transpose (sign -1) of window position n, channels c0..c0+3, from a swizzled
// image whose row `zrow` is all zeros: out-of-window taps read that row instead of branching
__device__ __forceinline__ void lepe4_lds_z(const Win& w, const bf16* img, int n, int c0, const float* wts, int sign,
                                            int zrow, float* acc) {
    const int iy = wrow(w, n), ix = n - iy * w.W_sp;
    const bool ym = iy > 0, yp = iy + 1 < w.H_sp, xm = ix > 0, xp = ix + 1 < w.W_sp;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(wts + HD * 9 + c0);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = sign > 0 ? bias[j] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int dy = sign * (t / 3 - 1), dx = sign * (t % 3 - 1);
        const bool in = (dy < 0 ? ym : dy > 0 ? yp : true) && (dx < 0 ? xm : dx > 0 ? xp : true);
        const int row = in ? n + dy * w.W_sp + dx : zrow;
        const bf16x4 v = *reinterpret_cast<const bf16x4*>(img + swz(row, c0));
        const f32x4 wt = *reinterpret_cast<const f32x4*>(wts + t * HD + c0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += wt[j] * (float)v[j];
    }
}

// NW waves: 4, or 8 for the 512-token windows (one workgroup per CU: two waves per SIMD hide the MFMA /
// LDS latencies of the per-tile chains); with 8 waves the dQ quadrants are split over two key halves
// and the upper half's partials added through LDS.
template <int WM, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW, WM <= 256 ? 2 : 1) void stripe_bwd_fused_w(csu_stripe_args a, const bf16* __restrict__ qkv,
                                                            const bf16* __restrict__ out, const bf16* __restrict__ dout,
                                                            const float* __restrict__ lse, bf16* __restrict__ dqkv,
                                                            float* __restrict__ part) {
    static_assert(NW == 4 || NW == 8, "stripe_bwd_fused_w: 4 or 8 waves");
    constexpr int NTH = 64 * NW;
    constexpr int KT = WM / (32 * NW);    // key tiles per wave
    constexpr int RT = WM / 32;           // 32-row tiles of the image
    constexpr int RS = NTH / 8;           // prologue: row stride (8 channel-quad lanes per row)
    constexpr int PR = WM / RS;           // prologue rows per thread
    __shared__ __attribute__((aligned(16))) bf16 Qs[WM * HD];
    __shared__ __attribute__((aligned(16))) bf16 Ks[WM * HD];
    // V: PLAIN [row][32] image + a zero row at WM (the prologue); from the main loop on the first WM
    // rows hold the swizzled dS tile [key][q]
    __shared__ __attribute__((aligned(16))) bf16 Vs[(WM + 1) * HD];
    __shared__ __attribute__((aligned(16))) bf16 Gs[(WM + 1) * HD];   // dO (swizzled) + a zero row at WM
    __shared__ __attribute__((aligned(16))) float nlse_s[WM], dl_s[WM];
    __shared__ __attribute__((aligned(16))) float wts[HD * 10];
    __shared__ float red[NW][8][41];
    __shared__ __attribute__((aligned(16))) unsigned char dtbl[NW][128];
    __shared__ __attribute__((aligned(16))) f32x4v xq[NW == 8 ? 4 : 1][64];   // upper key half's dQ partials
    ATT_STAMP(1, 0);
    const Win w = decode_w(a, 1);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int L = a.reso * a.reso, C = a.C, C3 = 3 * C;
    const bf16* img = qkv + (size_t)w.b * L * C3;
    const bf16* gimg = dout + (size_t)w.b * L * C;
    const int npad = (w.N + 31) & ~31, ntile = npad >> 5;
    const int c4 = threadIdx.x & 7, rg = threadIdx.x >> 3;   // prologue: channel quad, row group

    // ---- staging: Q, K, V, dO images, the window's -lse * log2(e) (the exponent offsets)
    u32x2 orow[PR];   // O rows of the prologue, loaded with the staging loads (global latency once)
    {
        const __amdgpu_buffer_rsrc_t rs_lse = stat_rsrc(a, lse);
        constexpr int SI = (WM + NTH - 1) / NTH;   // window rows per thread
        float lv[SI];
#pragma unroll
        for (int k = 0; k < SI; ++k) {
            const int i = threadIdx.x + k * NTH;
            lv[k] = ldf_rs(rs_lse, i < w.N ? (unsigned)(stat_index(a, w, tok_of(w, a.reso, i)) * 4) : kOOB);
        }
        float lw[LW_IT];
        lepe_weights_load(branch(a, w.br), w.h, lw);
        {
            const __amdgpu_buffer_rsrc_t rs_o = buf_rsrc(out + (size_t)w.b * L * C, (long)L * C * 2);
#pragma unroll
            for (int k = 0; k < PR; ++k) {
                const int n = rg + RS * k;
                orow[k] = __builtin_amdgcn_raw_buffer_load_b64(
                    rs_o, n < w.N ? (unsigned)(((size_t)tok_of(w, a.reso, n) * C + w.chq + 4 * c4) * 2) : kOOB, 0, 0);
            }
        }
        stage_win4<NTH, WM>(w, a.reso, img, C, gimg, npad, Qs, Ks, Vs, Gs);
        lepe_weights_store(lw, wts);
        if (threadIdx.x < 8) {   // the zero rows
            const bf16x8 z = {};
            *reinterpret_cast<bf16x8*>((threadIdx.x < 4 ? Vs : Gs) + WM * HD + 8 * (threadIdx.x & 3)) = z;
        }
#pragma unroll
        for (int k = 0; k < SI; ++k) {
            const int i = threadIdx.x + k * NTH;
            if (i < npad) nlse_s[i] = i < w.N ? -lv[k] * kLog2e : -INFINITY;   // padded queries: P = 0
        }
    }
    __syncthreads();
    ATT_STAMP(1, 1);

    // ---- prologue: delta and the LePE weight-gradient partials (thread: channel quad c4, rows rg + RS k)
    // RP rows per iteration with all their LDS reads issued before any use (one LDS latency per
    // iteration; r07n: one row per iteration waited on four read batches and three ds_bpermute round
    // trips); the cross-lane sums are DPP / permlane-swap VALU ops, not LDS permutes.  RP = 1 at
    // WM = 128: a second row's V values would push the kernel past 168 VGPRs (3 waves per SIMD).
    {
        constexpr int RP = WM <= 128 ? 1 : 2;
        static_assert(PR % RP == 0, "prologue: whole row groups per thread");
        float wacc[40];
#pragma unroll
        for (int i = 0; i < 40; ++i) wacc[i] = 0.f;
        const f32x4 bias = *reinterpret_cast<const f32x4*>(wts + HD * 9 + 4 * c4);
        // the thread's 9 x 4 LePE weights are the same for all its rows: read once, kept in registers
        // (inside the row loop they were re-read per row in dependent batches of LDS round trips;
        // stripe_attn_bwd -6 / -17 us per step at 512 / 1024, profiles/r09k_att_wreg_ab.txt)
        f32x4 wreg[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) wreg[t] = *reinterpret_cast<const f32x4*>(wts + t * HD + 4 * c4);
        const bf16* vq = Vs + 4 * c4;                  // plain image: row n of this quad at vq + 32 n
        // the preloaded O rows rotate through orow[0..RP) so every register index stays static.
        // Out-of-window taps read the zero row.
#pragma unroll 1
        for (int n0 = rg; n0 < npad; n0 += RP * RS) {
            bf16x4 g4[RP], v4[RP][9];
            bool valid[RP];
            u32x2 oraw[RP];
#pragma unroll
            for (int p = 0; p < RP; ++p) {
                const int n = n0 + p * RS;
                valid[p] = n < w.N;                        // uniform over the 8 lanes of the row
                const int nn = valid[p] ? n : 0;
                oraw[p] = orow[p];
                const int iy = wrow(w, nn), ix = nn - iy * w.W_sp;
                const bool ym = iy > 0, yp = iy + 1 < w.H_sp, xm = ix > 0, xp = ix + 1 < w.W_sp;
                g4[p] = *reinterpret_cast<const bf16x4*>(Gs + swz(nn, 4 * c4));
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int dy = t / 3 - 1, dx = t % 3 - 1;
                    const bool in = (dy < 0 ? ym : dy > 0 ? yp : true) && (dx < 0 ? xm : dx > 0 ? xp : true);
                    const int row = in ? nn + dy * w.W_sp + dx : WM;
                    v4[p][t] = *reinterpret_cast<const bf16x4*>(vq + row * HD);
                }
            }
#pragma unroll
            for (int k = 0; k + RP < PR; ++k) orow[k] = orow[k + RP];
            __builtin_amdgcn_sched_barrier(0);             // every read above issues before the math
            float dl[RP];
#pragma unroll
            for (int p = 0; p < RP; ++p) {
                float gv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) gv[j] = valid[p] ? (float)g4[p][j] : 0.f;
                // scalar FMAs: a v_pk_fma_f32 issues as two (MI355X_MICROARCH 'vector-instruction ISSUE
                // cost') and its operand pairs cost v_movs
                float lp[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) lp[j] = bias[j];
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const f32x4 wt = wreg[t];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float v = (float)v4[p][t][j];
                        lp[j] = fmaf(wt[j], v, lp[j]);
                        wacc[4 * t + j] = fmaf(gv[j], v, wacc[4 * t + j]);
                    }
                }
                bf16x4 o4;
                __builtin_memcpy(&o4, &oraw[p], 8);
                float d = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    wacc[36 + j] += gv[j];
                    d = fmaf(gv[j], (float)o4[j] - lp[j], d);
                }
                dl[p] = sum8_dpp(d);
            }
            if (c4 == 0) {                                 // padded rows: 0
#pragma unroll
                for (int p = 0; p < RP; ++p)
                    if (n0 + p * RS < npad) dl_s[n0 + p * RS] = dl[p];
            }
        }
        ATT_STAMP(2, 0);   // (debug build: the prologue's sub-phases in the dkdv slots, unused here)
        if (part) {
            // sum over the wave's 8 row groups (lanes of equal c4 = lane & 7) as a reduce-scatter:
            // row_ror:8 pairs the two halves of each 16-lane row (40 values), then one permlane16_swap
            // of the pair (i, i + 20) leaves value i summed over a row pair in the even rows and value
            // i + 20 in the odd rows (20 values), one permlane32_swap of (j, j + 10) the same over the
            // half-waves (10 values): lane (row parity p, half q) ends with values i + 10 q + 20 p.
            // The same additions in the same pairing as a full all-reduce, half the VALU.
#pragma unroll
            for (int i = 0; i < 40; ++i) wacc[i] += dppf<0x128>(wacc[i]);
#pragma unroll
            for (int i = 0; i < 20; ++i) {
                const auto r2 = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, wacc[i]),
                                                                 __builtin_bit_cast(unsigned, wacc[i + 20]), false, false);
                wacc[i] = __builtin_bit_cast(float, (unsigned)r2[0]) + __builtin_bit_cast(float, (unsigned)r2[1]);
            }
#pragma unroll
            for (int i = 0; i < 10; ++i) {
                const auto r2 = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, wacc[i]),
                                                                 __builtin_bit_cast(unsigned, wacc[i + 10]), false, false);
                wacc[i] = __builtin_bit_cast(float, (unsigned)r2[0]) + __builtin_bit_cast(float, (unsigned)r2[1]);
            }
            if ((lane & 8) == 0) {
                const int i0 = 10 * (lane >> 5) + 20 * ((lane >> 4) & 1);
#pragma unroll
                for (int i = 0; i < 10; ++i) red[wave][lane & 7][i0 + i] = wacc[i];
            }
        }
    }
    ATT_STAMP(2, 1);
    // ---- registers for the main loop (loaded after the prologue, before the V image is overwritten):
    // the own key tiles' K and V rows (B operands of S and dP)
    Frag<bf16> kf[KT], vf[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        const int kt = wave + NW * j;
        const int row = (kt < ntile ? kt : 0) * 32 + r;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            kf[j].v[s] = *reinterpret_cast<const bf16x8*>(Ks + swz(row, 16 * s + 8 * h));
            vf[j].v[s] = *reinterpret_cast<const bf16x8*>(Vs + row * HD + 16 * s + 8 * h);
        }
    }
    __syncthreads();   // dl_s / red complete; every read of the V image is done (it becomes the dS tile)
    ATT_STAMP(2, 2);
    if (part) {
        const int nwx = a.reso / w.W_sp, nwin = (a.reso / w.H_sp) * nwx;
        const int Cb = a.heads * HD, nblk = a.B * nwin, blk = w.b * nwin + w.wy * nwx + w.wx;
        for (int o = threadIdx.x; o < 8 * 40; o += NTH) {
            const int qq = o / 40, i = o % 40;
            float sum = red[0][qq][i];
#pragma unroll
            for (int v = 1; v < NW; ++v) sum += red[v][qq][i];
            const int k = i >> 2, c = w.h * HD + 4 * qq + (i & 3);
            part[((size_t)w.br * Cb * 10 + c * 10 + k) * nblk + blk] = sum;
        }
    }

    // ---- main loop over query tiles.  Every LDS address of the loop is (tile base) + a per-lane offset
    // computed here once: the swizzle depends only on the row's position inside its 32-row tile.
    const float c = a.scale * kLog2e;
    ADrop dr;
    if constexpr (DROP) dr = attn_drop(a, w);
    f32x16 dk[KT], dv[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) { dk[j] = f32x16{}; dv[j] = f32x16{}; }
    bf16* const dS = Vs;
    const int dh = wave & 1, qh = (wave >> 1) & 1, kh = wave >> 2;   // dQ quadrant; key half (NW = 8)
    constexpr int KK = NW == 8 ? RT / 2 : RT;                      // key tiles per dQ quadrant pass
    int o_row[2], o_tr[2][2], o_ds[4], o_k16[2], o_d16[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        o_row[s2] = swz(r, 16 * s2 + 8 * h);                        // A rows (mma_rows_sw)
        const int grp = lane >> 4, l = lane & 15, q = l >> 2, p4 = l & 3;
        const int col = 16 * (grp & 1) + 4 * p4, row = 16 * s2 + 4 * (grp >> 1) + q;
        o_tr[s2][0] = swz(row, col);                                // transposed A (tr_frag_acc)
        o_tr[s2][1] = swz(row + 8, col);
        const int g16 = lane >> 4, i16 = lane & 15;
        o_k16[s2] = swz(8 * g16 + 4 * s2 + (i16 >> 2), 16 * dh + 4 * (i16 & 3));   // 16x16x32 operands
        o_d16[s2] = swz(8 * g16 + 4 * s2 + (i16 >> 2), 16 * qh + 4 * (i16 & 3));
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) o_ds[g] = swz(r, 8 * g + 4 * h);
    auto trA = [&](const bf16* base, int s2) {
        const v4s lo = tr_read(base + o_tr[s2][0]);
        const v4s hi = tr_read(base + o_tr[s2][1]);
        const v4s v[2] = {lo, hi};
        bf16x8 o;
        __builtin_memcpy(&o, v, 16);
        return o;
    };
    auto tr16 = [&](const bf16* base, const int* off) {
        const v4s lo = tr_read(base + off[0]);
        const v4s hi = tr_read(base + off[1]);
        const v4s v[2] = {lo, hi};
        bf16x8 o;
        __builtin_memcpy(&o, v, 16);
        return o;
    };
    ATT_STAMP(1, 2);
    for (int qt = 0; qt < ntile; ++qt) {
        const int qb = qt * 32;
        const bf16* qrow = Qs + qb * HD;
        const bf16* grow = Gs + qb * HD;
        f32x4 nl[4], dq4[4];                               // rows qb + 8 g4 + 4 h + 0..3
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            nl[g4] = *reinterpret_cast<const f32x4*>(nlse_s + qb + 8 * g4 + 4 * h);
            dq4[g4] = *reinterpret_cast<const f32x4*>(dl_s + qb + 8 * g4 + 4 * h);
        }
        // no early exit for key tiles past the window (ntile < RT): their results are discarded (dS rows
        // >= npad are never read, dK / dV never stored) -- straight-line code lets the compiler
        // interleave the two tiles' MFMA chains and VALU work
#pragma unroll
        for (int j = 0; j < KT; ++j) {
            const int kt = wave + NW * j;
            f32x16 s = {}, dp = {};
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(qrow + o_row[s2]), kf[j].v[s2],
                                                            s, 0, 0, 0);    // S   [q][key]
                dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(grow + o_row[s2]), vf[j].v[s2],
                                                             dp, 0, 0, 0);  // dP  [q][key]
            }
            unsigned km = 0xffffu;
            if constexpr (DROP) km = keep_k16(dr, qb, kt * 32, lane, dtbl[wave]);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int g4 = i >> 2, e = i & 3;
                const float p = __builtin_amdgcn_exp2f(fmaf(s[i], c, nl[g4][e]));
                float gdp = dp[i];
                if constexpr (DROP) gdp = ((km >> i) & 1u) ? gdp * dr.R.scale : 0.f;   // dP through the mask
                dp[i] = p * (gdp - dq4[g4][e]);             // dS
                if constexpr (DROP) s[i] = ((km >> i) & 1u) ? p * dr.R.scale : 0.f;   // dV sees the dropped P
                else s[i] = p;
            }
            bf16x8 pb[2], db[2];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    pb[s2][e] = (bf16)s[8 * s2 + e];
                    db[s2][e] = (bf16)dp[8 * s2 + e];
                }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                dv[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(grow, s2), pb[s2], dv[j], 0, 0, 0);   // dV^T += dO^T P
                dk[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trA(qrow, s2), db[s2], dk[j], 0, 0, 0);   // dK^T += Q^T dS
            }
            bf16* dst = dS + kt * 32 * HD;                 // dS -> [key][q] image: q = 8 g + 4 h + 0..3
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const bf16x4 x = {db[g >> 1][4 * (g & 1)], db[g >> 1][4 * (g & 1) + 1], db[g >> 1][4 * (g & 1) + 2],
                                  db[g >> 1][4 * (g & 1) + 3]};
                *reinterpret_cast<bf16x4*>(dst + o_ds[g]) = x;
            }
        }
        __syncthreads();
        // dQ^T[d][q] quadrant (d = 16 dh + 4 (lane >> 4) + i, q = qb + 16 qh + (lane & 15)) over all keys
        f32x4v acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // two independent MFMA chains
        if (NW == 4 && ntile == RT) {   // (8 waves: the extra live fragments spilled)
            // the whole window (the common case): no per-tile condition, so the fragment reads of the
            // next key tiles issue while this one's MFMA runs (with the condition every tile was a
            // branch: its reads, a full LDS wait, then its MFMA -- ~120 cycles per key tile).
            // stripe_attn_bwd -32 us/step at 512x512 B16 (profiles/r09n_att_dq_full_ab.txt)
#pragma unroll
            for (int k2 = 0; k2 < KK; ++k2) {
                const int kk = kh * KK + k2;
                acc2[k2 & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr16(Ks + kk * 32 * HD, o_k16),
                                                                      tr16(dS + kk * 32 * HD, o_d16), acc2[k2 & 1], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int k2 = 0; k2 < KK; ++k2) {
                const int kk = kh * KK + k2;
                if (kk < ntile)
                    acc2[k2 & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr16(Ks + kk * 32 * HD, o_k16),
                                                                          tr16(dS + kk * 32 * HD, o_d16), acc2[k2 & 1], 0, 0, 0);
            }
        }
        f32x4v acc = acc2[0] + acc2[1];
        if constexpr (NW == 8)
            if (kh) xq[wave & 3][lane] = acc;              // the lower half adds it after the barrier
        auto store_dq = [&](const f32x4v& v4) {
            const int qn = qb + 16 * qh + (lane & 15);
            if (qn < w.N) {
                const int d0 = 16 * dh + 4 * (lane >> 4);
                const float v[4] = {v4[0] * a.scale, v4[1] * a.scale, v4[2] * a.scale, v4[3] * a.scale};
                store4(dqkv + ((size_t)w.b * L + tok_of(w, a.reso, qn)) * C3 + w.chq + d0, v);
            }
        };
        if constexpr (NW == 4) store_dq(acc);
        __syncthreads();                                   // the dS tile is rewritten by the next query tile
        if constexpr (NW == 8)
            if (!kh) store_dq(acc + xq[wave][lane]);       // xq is rewritten only after the next tile's barrier
    }
    ATT_STAMP(1, 3);

    // ---- dK, dV (+ LePE input gradient: the transposed conv of dO) of the own key tiles
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        const int kt = wave + NW * j, kn = kt * 32 + r;
        if (kt >= ntile || kn >= w.N) continue;
        bf16* drow = dqkv + ((size_t)w.b * L + tok_of(w, a.reso, kn)) * C3 + w.chq;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 8 * g4 + 4 * h;
            float vk[4], vv[4], lp[4];
            lepe4_lds_z(w, Gs, kn, d0, wts, -1, WM, lp);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                vk[e] = dk[j][4 * g4 + e] * a.scale;
                vv[e] = dv[j][4 * g4 + e] + lp[e];
            }
            store4(drow + C + d0, vk);
            store4(drow + 2 * C + d0, vv);
        }
    }
    ATT_STAMP(1, 4);
}

// the one-pass backward handles the launch (bf16, window <= 512 tokens: WM = 512 holds the four
// window images in 128 KiB of LDS, one workgroup per CU)
bool use_fused_bwd(const csu_stripe_args& a, int dtype) {
    return dtype == CSU_BF16 && a.br[0].H_sp * a.br[0].W_sp <= 512;
}
int fused_nblk(const csu_stripe_args& a) {
    return a.B * (a.reso / a.br[0].H_sp) * (a.reso / a.br[0].W_sp);
}

template <int WM, int NW = 4>
void bwd_fused(const csu_stripe_args& a, const bf16* qkv, const bf16* out, const bf16* dout, const float* lse, bf16* dqkv,
               float* part, hipStream_t st) {
    const int nwin = (a.reso / a.br[0].H_sp) * (a.reso / a.br[0].W_sp);
    const dim3 g(a.B * nwin * a.heads, a.nbranch);
    if (a.drop_p > 0.f) stripe_bwd_fused_w<WM, true, NW><<<g, 64 * NW, 0, st>>>(a, qkv, out, dout, lse, dqkv, part);
    else stripe_bwd_fused_w<WM, false, NW><<<g, 64 * NW, 0, st>>>(a, qkv, out, dout, lse, dqkv, part);
}

// split factor of the whole-window kernels: workgroups per window-head, so that a launch has
// about 1024 workgroups, each owning at least 128 query (key) rows -- one 32-row pass per wave
// (512x512: 2 at stages 3/4; 1024x1024: 4 at stage 3 (N = 512), 8 at stage 4 (N = 1024))
#ifndef ATTN_SPLIT_WGS
#define ATTN_SPLIT_WGS 1024
#endif
int wsplit(const csu_stripe_args& a) {
    const int N = a.br[0].H_sp * a.br[0].W_sp;
    const int nwin = (a.reso / a.br[0].H_sp) * (a.reso / a.br[0].W_sp);
    const long wgs = (long)a.B * nwin * a.heads * a.nbranch;
    const int maxsp = (((N + 31) & ~31) + 127) / 128;
    const long want = (ATTN_SPLIT_WGS + wgs - 1) / wgs;
    return (int)(want < maxsp ? want : maxsp);
}

bool use_window_path(const csu_stripe_args& a, int dtype) {
    return dtype == CSU_BF16 && a.br[0].H_sp * a.br[0].W_sp <= WMAX;
}

// LDS image rows of a launch: the window rounded up to 256 / 512 / 1024 tokens
int wm_of(const csu_stripe_args& a) {
    const int N = a.br[0].H_sp * a.br[0].W_sp;
    return N <= 256 ? 256 : N <= 512 ? 512 : 1024;
}

// ATTN_FWD_WAVES = 8: the forward's split partners merged into one 8-wave workgroup (the window's
// K / V staged once per window-head instead of once per partner)
#ifndef ATTN_FWD_WAVES
#define ATTN_FWD_WAVES 8
#endif
#ifndef ATTN_BWD_WAVES
#define ATTN_BWD_WAVES 8
#endif
template <int WM>
void fwd_w(const csu_stripe_args& a, int sp, dim3 g, const bf16* qkv, bf16* out, float* lse, hipStream_t st) {
    if (ATTN_FWD_WAVES == 8 && sp % 2 == 0) {
        g.x /= 2;
        if (a.drop_p > 0.f) stripe_fwd_w<WM, true, 8><<<g, 512, 0, st>>>(a, sp / 2, qkv, out, lse);
        else stripe_fwd_w<WM, false, 8><<<g, 512, 0, st>>>(a, sp / 2, qkv, out, lse);
        return;
    }
    if (a.drop_p > 0.f) stripe_fwd_w<WM, true><<<g, NT, 0, st>>>(a, sp, qkv, out, lse);
    else stripe_fwd_w<WM, false><<<g, NT, 0, st>>>(a, sp, qkv, out, lse);
}

template <int WM>
void bwd_w(const csu_stripe_args& a, int sp, dim3 g, const bf16* qkv, const bf16* out, const bf16* dout,
           const float* lse, float* delta, bf16* dqkv, hipStream_t st) {
    // windows of >= 512 tokens (their K / V or Q / dO images bound residency): split partners merged
    // into 8-wave workgroups, as the forward (ATTN_FWD_WAVES)
    if constexpr (WM >= 512) {
        if (ATTN_BWD_WAVES == 8 && sp % 2 == 0) {
            g.x /= 2;
            if (a.drop_p > 0.f) {
                stripe_bwd_dq_w<WM, true, 8><<<g, 512, 0, st>>>(a, sp / 2, qkv, out, dout, lse, delta, dqkv);
                stripe_bwd_dkdv_w<WM, true, 8><<<g, 512, 0, st>>>(a, sp / 2, qkv, dout, lse, delta, dqkv);
            } else {
                stripe_bwd_dq_w<WM, false, 8><<<g, 512, 0, st>>>(a, sp / 2, qkv, out, dout, lse, delta, dqkv);
                stripe_bwd_dkdv_w<WM, false, 8><<<g, 512, 0, st>>>(a, sp / 2, qkv, dout, lse, delta, dqkv);
            }
            return;
        }
    }
    if (a.drop_p > 0.f) {
        stripe_bwd_dq_w<WM, true><<<g, NT, 0, st>>>(a, sp, qkv, out, dout, lse, delta, dqkv);
        stripe_bwd_dkdv_w<WM, true><<<g, NT, 0, st>>>(a, sp, qkv, dout, lse, delta, dqkv);
    } else {
        stripe_bwd_dq_w<WM, false><<<g, NT, 0, st>>>(a, sp, qkv, out, dout, lse, delta, dqkv);
        stripe_bwd_dkdv_w<WM, false><<<g, NT, 0, st>>>(a, sp, qkv, dout, lse, delta, dqkv);
    }
}

int validate(const csu_stripe_args* a, int dtype) {
    if (!a) return fail(CSU_E_ARG, "stripe_attn: null args");
    if (a->head_dim != HD) return fail(CSU_E_UNSUPPORTED, "stripe_attn: head_dim must be 32");
    if (dtype != CSU_F32 && dtype != CSU_BF16) return fail(CSU_E_ARG, "stripe_attn: bad dtype");
    if (a->nbranch < 1 || a->nbranch > 2 || a->B < 1 || a->reso < 1 || a->heads < 1)
        return fail(CSU_E_ARG, "stripe_attn: bad B/reso/heads/nbranch");
    if (a->C % 8) return fail(CSU_E_ARG, "stripe_attn: C must be a multiple of 8");
    for (int i = 0; i < a->nbranch; ++i) {
        const csu_stripe_branch& g = a->br[i];
        if (g.H_sp < 1 || g.W_sp < 1 || a->reso % g.H_sp || a->reso % g.W_sp)
            return fail(CSU_E_ARG, "stripe_attn: resolution not divisible by the stripe window (cswin:204)");
        if (g.ch_off < 0 || g.ch_off + a->heads * HD > a->C)
            return fail(CSU_E_ARG, "stripe_attn: branch channels outside C");
        if (i > 0 && g.H_sp * g.W_sp != a->br[0].H_sp * a->br[0].W_sp)
            return fail(CSU_E_ARG, "stripe_attn: branches must have equal window size");
        if (!g.lepe_w || !g.lepe_b) return fail(CSU_E_ARG, "stripe_attn: null LePE weights");
    }
    if (a->br[0].H_sp * a->br[0].W_sp > 4096 || a->br[0].W_sp > 1024 || (a->nbranch > 1 && a->br[1].W_sp > 1024))
        return fail(CSU_E_UNSUPPORTED, "stripe_attn: windows of <= 4096 tokens, <= 1024 wide");
    if (a->drop_p < 0.f || a->drop_p >= 1.f || (a->drop_p > 0.f && !a->drop_rng))
        return fail(CSU_E_ARG, "stripe_attn: attention dropout needs 0 <= p < 1 and an RNG snapshot");
    return 0;
}

template <typename T>
void bwd_generic(const csu_stripe_args& a, dim3 grid, const T* qkv, const T* out, const T* dout, const float* lse,
                 float* delta, T* dqkv, hipStream_t st) {
    if (a.drop_p > 0.f) {
        stripe_bwd_dq<T, true><<<grid, NT, 0, st>>>(a, qkv, out, dout, lse, delta, dqkv);
        stripe_bwd_dkdv<T, true><<<grid, NT, 0, st>>>(a, qkv, dout, lse, delta, dqkv);
    } else {
        stripe_bwd_dq<T, false><<<grid, NT, 0, st>>>(a, qkv, out, dout, lse, delta, dqkv);
        stripe_bwd_dkdv<T, false><<<grid, NT, 0, st>>>(a, qkv, dout, lse, delta, dqkv);
    }
}

dim3 grid_of(const csu_stripe_args& a) {
    const int N = a.br[0].H_sp * a.br[0].W_sp;
    const int nwin = (a.reso / a.br[0].H_sp) * (a.reso / a.br[0].W_sp);
    return dim3(a.B * nwin * a.heads * ((N + QR - 1) / QR), a.nbranch);
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_stripe_attn_fwd(const csu_stripe_args* a, int dtype, const void* qkv, void* out,
                                   float* lse, void* stream) {
    if (int e = validate(a, dtype)) return e;
    if (!qkv || !out || !lse) return fail(CSU_E_ARG, "stripe_attn_fwd: null buffer");
    if (use_window_path(*a, dtype)) {
        const int sp = wsplit(*a);
        const int nwin = (a->reso / a->br[0].H_sp) * (a->reso / a->br[0].W_sp);
        const dim3 g(a->B * nwin * a->heads * sp, a->nbranch);
        const hipStream_t st = as_stream(stream);
        switch (wm_of(*a)) {
            case 256: fwd_w<256>(*a, sp, g, (const bf16*)qkv, (bf16*)out, lse, st); break;
            case 512: fwd_w<512>(*a, sp, g, (const bf16*)qkv, (bf16*)out, lse, st); break;
            default: fwd_w<1024>(*a, sp, g, (const bf16*)qkv, (bf16*)out, lse, st); break;
        }
        return check_launch("stripe_attn_fwd");
    }
    const dim3 grid = grid_of(*a);
    const bool drop = a->drop_p > 0.f;
    if (dtype == CSU_BF16 && drop) stripe_fwd<bf16, true><<<grid, NT, 0, as_stream(stream)>>>(*a, (const bf16*)qkv, (bf16*)out, lse);
    else if (dtype == CSU_BF16) stripe_fwd<bf16, false><<<grid, NT, 0, as_stream(stream)>>>(*a, (const bf16*)qkv, (bf16*)out, lse);
    else if (drop) stripe_fwd<float, true><<<grid, NT, 0, as_stream(stream)>>>(*a, (const float*)qkv, (float*)out, lse);
    else stripe_fwd<float, false><<<grid, NT, 0, as_stream(stream)>>>(*a, (const float*)qkv, (float*)out, lse);
    return check_launch("stripe_attn_fwd");
}

// LePE weight-gradient partial blocks of a launch (tiled kernel if its tile fits, else untiled)
int lepe_nblk(const csu_stripe_args& a, int dtype) {
    const int ty = lepe_tile_rows(a, dtype);
    if (!ty) return wgrad_blocks(a);
    const int rb = lepe_rows_blk(a, ty);
    return a.B * ((a.reso + rb - 1) / rb);
}

// many LePE weight-gradient reductions in one launch (the end-of-backward batch): item table in the
// kernel arguments, 16-value workgroup -> (item, values) by a scan over the value prefix sums
constexpr int LPB_MAX = 32;
struct LpBatch {
    const float* part[LPB_MAX];
    float* dw[LPB_MAX][2];
    float* db[LPB_MAX][2];
    int nblk[LPB_MAX], cb[LPB_MAX], nbranch[LPB_MAX], v0[LPB_MAX + 1];
    int count;
};

// lanes as lepe_wgrad_reduce; each item's value range starts on a multiple of 16 (v0), so the
// workgroup's item is found by a uniform scan on blockIdx (scalar loads of the item table)
__global__ __launch_bounds__(256) void lepe_reduce_batch(LpBatch t) {
    const int w0 = blockIdx.x * 16;
    int i = 0;
    while (i + 1 < t.count && t.v0[i + 1] <= w0) ++i;
    const int nblk = t.nblk[i], Cb = t.cb[i], nv = t.nbranch[i] * Cb * 10;
    const int u = w0 - t.v0[i] + (threadIdx.x >> 4), sub = threadIdx.x & 15;
    const float s = lepe_value_sum(t.part[i] + (size_t)(u < nv ? u : nv - 1) * nblk, nblk, sub);
    if (sub == 0 && u < nv) {
        const int br = u / (Cb * 10), r = u % (Cb * 10), c = r / 10, k = r % 10;
        float* dw = br ? t.dw[i][1] : t.dw[i][0];
        float* db = br ? t.db[i][1] : t.db[i][0];
        if (k < 9) dw[c * 9 + k] = s;
        else db[c] = s;
    }
}

void lepe_wgrad_launch(const csu_stripe_args& a, int dtype, const void* qkv, const void* dout, float* part, hipStream_t st,
                       bool reduce = true) {
    const int ty = lepe_tile_rows(a, dtype);
    const int nblk = lepe_nblk(a, dtype);
    if (ty) {
        const size_t es = dtype == CSU_BF16 ? 2 : 4;
        const size_t lds = (size_t)(2 * ty + 2) * a.reso * HD * es;
        const dim3 g((unsigned)nblk, (unsigned)a.heads, (unsigned)a.nbranch);
        const int rb = lepe_rows_blk(a, ty);
        if (dtype == CSU_BF16) lepe_wgrad_tiles<bf16><<<g, NT, lds, st>>>(a, ty, rb, (const bf16*)qkv, (const bf16*)dout, part);
        else lepe_wgrad_tiles<float><<<g, NT, lds, st>>>(a, ty, rb, (const float*)qkv, (const float*)dout, part);
    } else if (dtype == CSU_BF16) {
        lepe_wgrad_partial<bf16><<<dim3(nblk, a.nbranch), NT, 0, st>>>(a, (const bf16*)qkv, (const bf16*)dout, part);
    } else {
        lepe_wgrad_partial<float><<<dim3(nblk, a.nbranch), NT, 0, st>>>(a, (const float*)qkv, (const float*)dout, part);
    }
    if (!reduce) return;
    const dim3 rgrid((a.nbranch * a.heads * HD * 10 + 15) / 16);
    lepe_wgrad_reduce<<<rgrid, 256, 0, st>>>(a, nblk, part);
}

extern "C" size_t csu_stripe_attn_bwd_workspace(const csu_stripe_args* a) {
    if (!a) return 0;
    // enough for either partial layout (dtype decided at launch)
    int n = wgrad_blocks(*a);
    for (int dt : {CSU_BF16, CSU_F32}) n = n > lepe_nblk(*a, dt) ? n : lepe_nblk(*a, dt);
    n = n > fused_nblk(*a) ? n : fused_nblk(*a);
    return (size_t)a->nbranch * n * a->heads * HD * 10 * sizeof(float);
}

extern "C" int csu_stripe_attn_bwd_ex(const csu_stripe_args* a, int dtype, const void* qkv, const void* out,
                                      const void* dout, const float* lse, float* delta, void* dqkv,
                                      void* workspace, size_t workspace_bytes, int lepe_deferred, void* stream);

extern "C" int csu_stripe_attn_bwd(const csu_stripe_args* a, int dtype, const void* qkv, const void* out,
                                   const void* dout, const float* lse, float* delta, void* dqkv,
                                   void* workspace, size_t workspace_bytes, void* stream) {
    return csu_stripe_attn_bwd_ex(a, dtype, qkv, out, dout, lse, delta, dqkv, workspace, workspace_bytes, 0, stream);
}

// partial blocks csu_stripe_attn_bwd_ex(lepe_deferred = 1) leaves in its workspace
extern "C" int csu_stripe_lepe_nblk(const csu_stripe_args* a, int dtype) {
    if (!a) return 0;
    return use_fused_bwd(*a, dtype) ? fused_nblk(*a) : lepe_nblk(*a, dtype);
}

extern "C" int csu_stripe_lepe_reduce_batch(const csu_lepe_reduce_item* items, int count, void* stream) {
    if (count < 0 || (count && !items)) return fail(CSU_E_ARG, "stripe_lepe_reduce_batch: bad args");
    LpBatch t;
    t.count = 0;
    t.v0[0] = 0;
    auto flush = [&]() -> int {
        if (!t.count) return 0;
        lepe_reduce_batch<<<(unsigned)((t.v0[t.count] + 15) / 16), 256, 0, as_stream(stream)>>>(t);
        t.count = 0;
        return check_launch("stripe_lepe_reduce_batch");
    };
    for (int i = 0; i < count; ++i) {
        const csu_lepe_reduce_item& it = items[i];
        if (!it.part || it.nblk < 1 || it.channels < 1 || it.nbranch < 1 || it.nbranch > 2) return fail(CSU_E_ARG, "stripe_lepe_reduce_batch: bad item");
        for (int b = 0; b < it.nbranch; ++b)
            if (!it.dw[b] || !it.db[b]) return fail(CSU_E_ARG, "stripe_lepe_reduce_batch: null gradient");
        if (t.count == LPB_MAX)
            if (int e = flush()) return e;
        const int k = t.count;
        t.part[k] = it.part;
        t.dw[k][0] = it.dw[0]; t.dw[k][1] = it.nbranch > 1 ? it.dw[1] : it.dw[0];
        t.db[k][0] = it.db[0]; t.db[k][1] = it.nbranch > 1 ? it.db[1] : it.db[0];
        t.nblk[k] = it.nblk;
        t.cb[k] = it.channels;
        t.nbranch[k] = it.nbranch;
        t.v0[k + 1] = t.v0[k] + (it.nbranch * it.channels * 10 + 15) / 16 * 16;
        t.count = k + 1;
    }
    return flush();
}

extern "C" int csu_stripe_attn_bwd_ex(const csu_stripe_args* a, int dtype, const void* qkv, const void* out,
                                      const void* dout, const float* lse, float* delta, void* dqkv,
                                      void* workspace, size_t workspace_bytes, int lepe_deferred, void* stream) {
    if (int e = validate(a, dtype)) return e;
    if (!qkv || !out || !dout || !lse || !delta || !dqkv) return fail(CSU_E_ARG, "stripe_attn_bwd: null buffer");
    // all LePE weight-gradient pointers NULL: skip that part (csu_stripe_lepe_wgrad, e.g. on another stream)
    int nnull = 0;
    for (int i = 0; i < a->nbranch; ++i) nnull += (!a->br[i].lepe_dw) + (!a->br[i].lepe_db);
    const bool do_lepe = nnull == 0;
    if (nnull && nnull != 2 * a->nbranch) return fail(CSU_E_ARG, "stripe_attn_bwd: null LePE grads");
    if (do_lepe && (workspace_bytes < csu_stripe_attn_bwd_workspace(a) || !workspace))
        return fail(CSU_E_WORKSPACE, "stripe_attn_bwd: workspace too small");
    {
        const int nq = a->heads * HD / 4;   // LePE weight-gradient layout: channel quads per branch
        if (NT % nq || (nq & (nq - 1)))
            return fail(CSU_E_UNSUPPORTED, "stripe_attn_bwd: heads per branch must be a power of two <= 32");
    }
    hipStream_t st = as_stream(stream);
    const dim3 grid = grid_of(*a);
    float* part = (float*)workspace;
    if (use_fused_bwd(*a, dtype)) {
        // one pass: dQ, dK, dV and (do_lepe) the LePE weight-gradient partials, reduced below or deferred
        const bf16 *q = (const bf16*)qkv, *o = (const bf16*)out, *go = (const bf16*)dout;
        float* pp = do_lepe ? part : nullptr;
        const int N = a->br[0].H_sp * a->br[0].W_sp;
        if (N <= 128) bwd_fused<128>(*a, q, o, go, lse, (bf16*)dqkv, pp, st);
        else if (N <= 256) bwd_fused<256>(*a, q, o, go, lse, (bf16*)dqkv, pp, st);
        else bwd_fused<512, 8>(*a, q, o, go, lse, (bf16*)dqkv, pp, st);
        if (do_lepe && !lepe_deferred) {
            const dim3 rgrid((a->nbranch * a->heads * HD * 10 + 15) / 16);
            lepe_wgrad_reduce<<<rgrid, 256, 0, st>>>(*a, fused_nblk(*a), part);
        }
        return check_launch("stripe_attn_bwd");
    }
    if (use_window_path(*a, dtype)) {
        const int sp = wsplit(*a);
        const int nwin = (a->reso / a->br[0].H_sp) * (a->reso / a->br[0].W_sp);
        const dim3 g(a->B * nwin * a->heads * sp, a->nbranch);
        const bf16 *q = (const bf16*)qkv, *o = (const bf16*)out, *go = (const bf16*)dout;
        switch (wm_of(*a)) {
            case 256: bwd_w<256>(*a, sp, g, q, o, go, lse, delta, (bf16*)dqkv, st); break;
            case 512: bwd_w<512>(*a, sp, g, q, o, go, lse, delta, (bf16*)dqkv, st); break;
            default: bwd_w<1024>(*a, sp, g, q, o, go, lse, delta, (bf16*)dqkv, st); break;
        }
    } else if (dtype == CSU_BF16) {
        bwd_generic<bf16>(*a, grid, (const bf16*)qkv, (const bf16*)out, (const bf16*)dout, lse, delta, (bf16*)dqkv, st);
    } else {
        bwd_generic<float>(*a, grid, (const float*)qkv, (const float*)out, (const float*)dout, lse, delta, (float*)dqkv, st);
    }
    if (do_lepe) lepe_wgrad_launch(*a, dtype, qkv, dout, part, st, !lepe_deferred);
    return check_launch("stripe_attn_bwd");
}

extern "C" int csu_stripe_lepe_wgrad(const csu_stripe_args* a, int dtype, const void* qkv, const void* dout,
                                     void* workspace, size_t workspace_bytes, void* stream) {
    if (int e = validate(a, dtype)) return e;
    if (!qkv || !dout) return fail(CSU_E_ARG, "stripe_lepe_wgrad: null buffer");
    for (int i = 0; i < a->nbranch; ++i)
        if (!a->br[i].lepe_dw || !a->br[i].lepe_db) return fail(CSU_E_ARG, "stripe_lepe_wgrad: null LePE grads");
    if (workspace_bytes < csu_stripe_attn_bwd_workspace(a) || !workspace)
        return fail(CSU_E_WORKSPACE, "stripe_lepe_wgrad: workspace too small");
    const int nq = a->heads * HD / 4;
    if (NT % nq || (nq & (nq - 1))) return fail(CSU_E_UNSUPPORTED, "stripe_lepe_wgrad: heads per branch must be a power of two <= 32");
    lepe_wgrad_launch(*a, dtype, qkv, dout, (float*)workspace, as_stream(stream));
    return check_launch("stripe_lepe_wgrad");
}

#ifdef WG_TIMING
extern "C" int csu_debug_attn_ts(unsigned long long* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(csu::attn_ts), sizeof(csu::attn_ts), 0, hipMemcpyDeviceToHost);
}
#endif
