// Shared device helpers for the gfx950 (CDNA4) kernels of libcsu_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "csu.h"

namespace csu {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---- error reporting (thread-local last error) ----------------------------------------------
void set_error(const std::string& s);
int fail(int code, const std::string& s);
int check_launch(const char* what);

// ---- scalar <-> storage conversion ------------------------------------------------------------
template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v) { return (T)v; }

// 4 consecutive elements <-> float[4]
__device__ __forceinline__ void load4(const float* p, float* v) {
    f32x4 x = *reinterpret_cast<const f32x4*>(p);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
__device__ __forceinline__ void load4(const bf16* p, float* v) {
    bf16x4 x = *reinterpret_cast<const bf16x4*>(p);
    v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3];
}
__device__ __forceinline__ void store4(float* p, const float* v) {
    f32x4 x = {v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p) = x;
}
__device__ __forceinline__ void store4(bf16* p, const float* v) {
    bf16x4 x = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    *reinterpret_cast<bf16x4*>(p) = x;
}
// 8 consecutive elements <-> float[8]
template <typename T> __device__ __forceinline__ void load8(const T* p, float* v) {
    load4(p, v); load4(p + 4, v + 4);
}
__device__ __forceinline__ void load8(const bf16* p, float* v) {
    bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <typename T> __device__ __forceinline__ void store8(T* p, const float* v) {
    store4(p, v); store4(p + 4, v + 4);
}
__device__ __forceinline__ void store8(bf16* p, const float* v) {
    bf16x8 x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (bf16)v[j];
    *reinterpret_cast<bf16x8*>(p) = x;
}

// ---- wave reductions (wave64) -----------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// sum of p[j], j = sub, sub + G, ... < n, four independent loads in flight per round trip (a one-load
// loop serialises on the load latency); fixed association -- deterministic
template <int G> __device__ __forceinline__ float strided_sum(const float* __restrict__ p, int n, int sub) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int j = sub;
    for (; j + 3 * G < n; j += 4 * G) {
        s0 += p[j];
        s1 += p[j + G];
        s2 += p[j + 2 * G];
        s3 += p[j + 3 * G];
    }
    for (; j < n; j += G) s0 += p[j];
    return (s0 + s1) + (s2 + s3);
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Row of the 32x32 MFMA accumulator register `reg` held by lane half `h` (C/D map, gfx950):
// row = (reg & 3) + 8 * (reg >> 2) + 4 * h, column = lane & 31.
__device__ __forceinline__ constexpr int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// deterministic column sum out[c] = sum_r in[r][c] (reduce.hip); ws of colsum_workspace() bytes.
// map (optional): write column c of a conv weight-gradient slab ([N][khw][C] weights + [N] bias) to
// torch's OIHW position ([N][creal][khw] + [N]; channels >= creal and columns past the bias dropped)
struct OutMap {
    int on, N, khw, C, creal;
};
size_t colsum_workspace(long rows, long cols, int dtype);
int colsum_launch(long rows, long cols, int dtype, const void* in, float* out, float* ws, hipStream_t st,
                  const OutMap* map = nullptr);

// XCD-aware tile order.  Workgroups are dispatched round-robin over the 8 XCDs (workgroup id i
// runs on XCD i % 8), each with its own L2.  Remap the hardware id so that XCD x walks a
// contiguous range of logical tiles: tiles that share an operand panel (consecutive logical ids)
// then run concurrently on one XCD and the panel is fetched from HBM once into that XCD's L2.
constexpr int kXcds = 8;
constexpr bool kRot = true;   // rotate the fused Mlp's hidden-chunk order (spreads concurrent L2 reads)
__device__ __forceinline__ long xcd_tile(long id, long total) {
    const long q = total / kXcds, rem = total % kXcds;
    const long x = id % kXcds, k = id / kXcds;
    return x < rem ? x * (q + 1) + k : rem * (q + 1) + (x - rem) * q + k;
}

// xcd_tile over the whole (x, y, z) grid: the logical id of this workgroup
__device__ __forceinline__ long xcd_block() {
    const long total = (long)gridDim.x * gridDim.y * gridDim.z;
    const long id = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);
    return xcd_tile(id, total);
}

// ---- raw buffer access: out-of-range offsets are dropped (stores) / read as 0 (loads) by the
// hardware, so bounds checks need no branches (a branch around a store makes hipcc wait
// vmcnt(0) at the join, serialising an epilogue's stores).
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                             0x00020000);
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t rs, unsigned off, const float* v) {   // 4 x f32
    u32x4 x = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 0);
}
__device__ __forceinline__ void buf_st4bf(__amdgpu_buffer_rsrc_t rs, unsigned off, const float* v) {   // 4 x bf16
    bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    u32x2 x;
    __builtin_memcpy(&x, &b, 8);
    __builtin_amdgcn_raw_buffer_store_b64(x, rs, off, 0, 0);
}
__device__ __forceinline__ void buf_st8bf(__amdgpu_buffer_rsrc_t rs, unsigned off, const float* v) {   // 8 x bf16
    bf16x8 b;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = (bf16)v[e];
    u32x4 x;
    __builtin_memcpy(&x, &b, 16);
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, off, 0, 0);
}
__device__ __forceinline__ void buf_ld8bf(__amdgpu_buffer_rsrc_t rs, unsigned off, float* v) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    bf16x8 b;
    __builtin_memcpy(&b, &x, 16);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)b[e];
}
__device__ __forceinline__ void buf_ld4(__amdgpu_buffer_rsrc_t rs, unsigned off, float* v) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    v[0] = __uint_as_float(x[0]); v[1] = __uint_as_float(x[1]); v[2] = __uint_as_float(x[2]); v[3] = __uint_as_float(x[3]);
}
__device__ __forceinline__ void buf_ld4bf(__amdgpu_buffer_rsrc_t rs, unsigned off, float* v) {
    const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
    bf16x4 b;
    __builtin_memcpy(&b, &x, 8);
    v[0] = (float)b[0]; v[1] = (float)b[1]; v[2] = (float)b[2]; v[3] = (float)b[3];
}

// GELU (exact-erf form of nn.GELU) with erf by Abramowitz-Stegun 7.1.26 (|abs err| < 1.5e-7):
// one v_exp + one v_rcp (the hardware 1-ulp reciprocal: __frcp_rn expands to the ~10-instruction
// correctly rounded division sequence).  gelu_pair_as returns gelu and gelu' sharing both.
__device__ __forceinline__ float erf_poly_as(float t) {
    return t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
}
__device__ __forceinline__ float erf_as(float z) {   // z >= 0
    const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * z);
    return 1.f - erf_poly_as(t) * __expf(-z * z);
}
__device__ __forceinline__ float gelu_as(float x) {
    const float e = erf_as(fabsf(x) * 0.70710678118654752f);
    return 0.5f * x * (1.f + (x >= 0.f ? e : -e));
}
__device__ __forceinline__ float gelu_grad_as(float x) {
    const float e = erf_as(fabsf(x) * 0.70710678118654752f);
    return 0.5f * (1.f + (x >= 0.f ? e : -e)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ void gelu_pair_as(float x, float& g, float& dg) {
    const float z = fabsf(x) * 0.70710678118654752f;
    const float ex = __expf(-z * z);                  // = exp(-x^2 / 2)
    const float e = 1.f - erf_poly_as(__builtin_amdgcn_rcpf(1.f + 0.3275911f * z)) * ex;
    const float phi2 = 0.5f * (1.f + (x >= 0.f ? e : -e));   // Phi(x)
    g = x * phi2;
    dg = phi2 + x * 0.3989422804014327f * ex;
}

// Cheaper GELU for the bf16 paths: 0.5 erfc(|x|/sqrt2) by Abramowitz-Stegun 7.1.25 (|err| <
// 1.25e-5 on Phi, far below bf16 resolution): one v_rcp, one v_exp, ~10 mostly packable ops.
__device__ __forceinline__ float half_erfc_as(float x, float& ex) {   // 0.5 erfc(|x| / sqrt2); ex = exp(-x^2/2)
    const float t = __builtin_amdgcn_rcpf(fmaf(0.33267904f, fabsf(x), 1.f));   // p = 0.47047 / sqrt2
    ex = __builtin_amdgcn_exp2f(-0.72134752f * (x * x));
    return t * (0.1740121f + t * (-0.0479399f + t * 0.3739278f)) * ex;
}
// cross-lane sums on the VALU: DPP moves (quad_perm / row_half_mirror / row_ror) and the CDNA4 permlane
// swaps (xsum16: rows 2i <-> 2i+1, xsum32: half-waves) -- no LDS round trip
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float sum8_dpp(float x) {   // sum over each aligned group of 8 lanes
    x += dppf<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dppf<0x4E>(x);    // quad_perm [2,3,0,1]
    return x + dppf<0x141>(x);   // row_half_mirror: lane i <- 7 - i of its 8-lane group
}
__device__ __forceinline__ float xsum16(float x) {   // x + x of lane ^ 16
    const unsigned u = __builtin_bit_cast(unsigned, x);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ float xsum32(float x) {   // x + x of lane ^ 32
    const unsigned u = __builtin_bit_cast(unsigned, x);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

__device__ __forceinline__ float gelu_fast(float x) {
    float ex;
    const float q = half_erfc_as(x, ex);
    return x * (x >= 0.f ? 1.f - q : q);
}
__device__ __forceinline__ void gelu_pair_fast(float x, float& g, float& dg) {
    float ex;
    const float q = half_erfc_as(x, ex);
    const float phi = x >= 0.f ? 1.f - q : q;
    g = x * phi;
    dg = fmaf(x * 0.3989422804014327f, ex, phi);
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace csu
