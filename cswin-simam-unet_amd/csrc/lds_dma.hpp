// LDS-DMA staging helpers for gfx950 kernels (mlp.hip, wgrad5.hip): XOR-swizzled bf16 images
// filled by buffer_load ... lds with per-lane source offsets, counted vmcnt waits, and MFMA
// fragment reads (row reads and ds_read_b64_tr_b16 transposed reads) of those images.
#pragma once
#include "common.hpp"

// m0 is reserved (not saved around asm); the DMA asm sets it right before use and the kernels
// that include this header keep no live value in it
#pragma clang diagnostic ignored "-Winline-asm"

namespace csu {

// swizzle key of an image row.  RB = bytes per row.  64-B rows: four rows share a 256-B bank row,
// key = (row >> 2) & 3; 128-B rows: two rows share one, key = bitrev3((row >> 1) & 7); >= 256-B rows:
// key = bitrev4(row & 15).
template <int RB>
__device__ __forceinline__ int mkey(int row) {
    if constexpr (RB == 64) {
        return (row >> 2) & 3;
    } else if constexpr (RB == 128) {
        const int v = (row >> 1) & 7;
        return ((v & 1) << 2) | (v & 2) | ((v >> 2) & 1);
    } else {
        const int v = row & 15;
        return ((v & 1) << 3) | ((v & 2) << 1) | ((v >> 1) & 2) | ((v >> 3) & 1);
    }
}
// element offset of column `col` (bf16) of row `row` in a swizzled [rows][RB/2] image
template <int RB>
__device__ __forceinline__ int moff(int row, int col) {
    return row * (RB / 2) + ((((col >> 3) ^ mkey<RB>(row))) << 3) + (col & 7);
}

// DMA of an R-row image of RB-byte rows from a row-major bf16 matrix (leading dimension ld
// elements): wave instruction i of wave w fills image bytes [(w * NW + i) * 1024, +1024); lane l
// the 16 B at + 16 l = row p / RB, slot (p % RB) / 16, whose source chunk is slot ^ key(row).
template <int R, int RB, int WAVES = 4>
struct Dma {
    static constexpr int NW = R * RB / (1024 * WAVES);   // instructions per wave
    static_assert(NW >= 1 && R * RB % (1024 * WAVES) == 0, "image must be a multiple of WAVES KB");
    unsigned v[NW];
    __device__ __forceinline__ void init(int ld, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int p = (wave * NW + i) * 1024 + lane * 16;
            const int row = p / RB, slot = (p % RB) >> 4;
            v[i] = (unsigned)row * ld * 2 + ((slot ^ mkey<RB>(row)) << 4);
        }
    }
};

// buffer resource words (base, num_records, raw-buffer flags as buf_rsrc) for inline asm
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 rsrc4(const void* base, long bytes) {
    const unsigned long a = reinterpret_cast<unsigned long>(base);
    return i32x4{(int)(unsigned)a, (int)((a >> 32) & 0xffff), (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL), 0x00020000};
}

// Issue the DMA of image `img`: NW wave instructions at the per-lane offsets voff, k offset soff
// (bytes).  Inline asm, not __builtin_amdgcn_raw_ptr_buffer_load_lds: the compiler cannot tell the
// two ring stages apart and would put s_waitcnt vmcnt(0) before every later LDS read, exposing
// the whole prefetch; completion is tracked by the explicit vmwait<> instead.  (Also a free
// function: as a member of Dma, hipcc dropped the host stub of the kernel.)
template <int NW>
__device__ __forceinline__ void dma(i32x4 rs, const unsigned* voff, unsigned soff, bf16* img, int wave) {
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const unsigned lds = (unsigned)reinterpret_cast<unsigned long>(
            (__attribute__((address_space(3))) bf16*)(img + (wave * NW + i) * 512));
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lds), "v"(voff[i]), "s"(rs), "s"(soff) : "memory", "m0");
    }
}

// One DMA instruction into the 1-KB block at img, the LDS address forced uniform (readfirstlane):
// for kernels where hipcc cannot prove it (the address would land in a VGPR and the asm be
// invalid).  Not used in dma(): there the extra readfirstlanes cost the fused Mlp its registers.
__device__ __forceinline__ void dma1_u(i32x4 rs, unsigned voff, unsigned soff, bf16* img) {
    const unsigned lds = __builtin_amdgcn_readfirstlane(
        (unsigned)reinterpret_cast<unsigned long>((__attribute__((address_space(3))) bf16*)img));
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(lds), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
}

template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// every wave's LDS traffic and (already waited-for) DMA visible to the workgroup
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 frag(const bf16* img, int off) { return *reinterpret_cast<const bf16x8*>(img + off); }

typedef short v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4s tr4(const bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p));
}
__device__ __forceinline__ bf16x8 cat8(v4s lo, v4s hi) {
    const v4s v[2] = {lo, hi};
    bf16x8 out;
    __builtin_memcpy(&out, v, 16);
    return out;
}

// 32x32x16 operand fragment A[i = c0 + (lane & 31)][k = 16 s + 8 h .. + 7] from an image whose
// ROWS are k and COLUMNS are i (transposing read: lane 4q+p of a 16-lane group addresses row q,
// columns 4p..4p+3; lane i of the group receives column i of the 4 rows).
template <int RB>
__device__ __forceinline__ bf16x8 trfrag(const bf16* img, int c0, int s, int lane) {
    const int grp = lane >> 4, l = lane & 15, q = l >> 2, p = l & 3;
    const int col = c0 + 16 * (grp & 1) + 4 * p;
    const int row = 16 * s + 8 * (grp >> 1) + q;
    return cat8(tr4(img + moff<RB>(row, col)), tr4(img + moff<RB>(row + 4, col)));
}

}  // namespace csu
