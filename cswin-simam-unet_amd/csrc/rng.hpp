// Counter-based dropout masks for gfx950 kernels (attention dropout on P, Mlp dropout, DropPath,
// pos_drop of train_cswinunet_segmentation.py cswin:196/290/344/367-368/512).
//
// Philox4x32-7 (Salmon et al., SC'11; 7 rounds pass BigCrush): key = the 64-bit seed of the step, counter = (element
// group, site, step counter).  One call yields 4 x 32 random bits = 8 x 16-bit uniforms, so each
// call decides 8 consecutive elements of a site: element e of site s keeps iff
//   u16[e % 8] of philox({e / 8, s, ctr_lo, ctr_hi}, seed) < keep_threshold,
// keep_threshold = round((1 - p) * 65536) (p quantised to 1/65536).  Kept elements are scaled by
// 1 / (1 - p) (nn.Dropout semantics).  The same (seed, counter) snapshot is passed to the forward
// and backward kernels of a site, so the backward regenerates the forward's mask exactly; any
// kernel (and csu_dropout_mask, which materialises masks for tests) indexing the same element of
// the same site draws the same bit.
#pragma once
#include <stdint.h>

namespace csu {

__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                             uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
}

// 4 x 32 random bits of counter (c0..c3) under key (k0, k1), 7 rounds
__device__ __forceinline__ uint4 philox4x32_7(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                               uint32_t k1) {
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        philox_round(c0, c1, c2, c3, k0, k1);
        k0 += W0;
        k1 += W1;
    }
    return make_uint4(c0, c1, c2, c3);
}

// The per-step RNG snapshot a dropout site reads: [seed, counter] (two 64-bit words in HBM).
struct DropoutRng {
    uint32_t k0, k1, c2, c3;   // key = seed, counter words 2/3 = step counter
    uint32_t thr;              // keep iff u16 < thr  (thr = 65536 keeps everything)
    float scale;               // 1 / (1 - p)
    uint32_t site;
};

__device__ __forceinline__ DropoutRng load_rng(const uint64_t* state, uint32_t site, float p) {
    DropoutRng r;
    // p = 0 launches may pass no state (no element is ever masked then)
    const uint64_t seed = state ? state[0] : 0, ctr = state ? state[1] : 0;
    r.k0 = (uint32_t)seed;
    r.k1 = (uint32_t)(seed >> 32);
    r.c2 = (uint32_t)ctr;
    r.c3 = (uint32_t)(ctr >> 32);
    r.site = site;
    float t = (1.f - p) * 65536.f + 0.5f;
    r.thr = t >= 65536.f ? 65536u : (uint32_t)t;
    r.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
    return r;
}

// keep bits of the 8 elements [8g, 8g + 8) of the site: bit j = element 8g + j
__device__ __forceinline__ uint32_t keep8(const DropoutRng& r, uint64_t g) {
    const uint4 v = philox4x32_7((uint32_t)g, ((uint32_t)(g >> 32) << 12) ^ r.site, r.c2, r.c3, r.k0, r.k1);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        m |= (uint32_t)((w[i] & 0xffffu) < r.thr) << (2 * i);
        m |= (uint32_t)((w[i] >> 16) < r.thr) << (2 * i + 1);
    }
    return m;
}

// Keep bits (bit i) of the 16 elements base8 * 8 + crow(i, h) -- the layout of a 32x32 MFMA
// accumulator row as held by lane (r, h): 4 groups of 8 consecutive elements, lane half h owns
// elements 4h..4h+3 of each.  The lane pair (r, h = 0 / 1) splits the 4 Philox calls and swaps
// results (both lanes must execute this).
__device__ __forceinline__ uint32_t keep16_crow(const DropoutRng& r, uint64_t base8, int h) {
    const uint32_t ma = keep8(r, base8 + h), mb = keep8(r, base8 + 2 + h);
    const uint32_t pa = __shfl_xor(ma, 32, 64), pb = __shfl_xor(mb, 32, 64);
    const uint32_t m0 = h ? pa : ma, m1 = h ? ma : pa, m2 = h ? pb : mb, m3 = h ? mb : pb;
    const int sh = 4 * h;
    return ((m0 >> sh) & 15u) | (((m1 >> sh) & 15u) << 4) | (((m2 >> sh) & 15u) << 8) | (((m3 >> sh) & 15u) << 12);
}

// scale (0 or 1/(1-p)) of element e
__device__ __forceinline__ float drop_scale(const DropoutRng& r, uint64_t e) {
    return ((keep8(r, e >> 3) >> (e & 7)) & 1u) ? r.scale : 0.f;
}

}  // namespace csu
