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
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Row of the 32x32 MFMA accumulator register `reg` held by lane half `h` (C/D map, gfx950):
// row = (reg & 3) + 8 * (reg >> 2) + 4 * h, column = lane & 31.
__device__ __forceinline__ constexpr int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// deterministic column sum out[c] = sum_r in[r][c] (reduce.hip); ws of colsum_workspace() bytes
size_t colsum_workspace(long rows, long cols, int dtype);
int colsum_launch(long rows, long cols, int dtype, const void* in, float* out, float* ws, hipStream_t st);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace csu
