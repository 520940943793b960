// Dropout / DropPath as one elementwise pass for gfx950 (nn.Dropout cswin:190/193/512, timm DropPath
// cswin:344/367-368 where they are not fused into a producing kernel):
//   out[i] = res[i] + row_scale[row / rows_per_sample] * keep(site, i) / (1 - p) * x[i]
// (res, row_scale optional; p = 0 -> no mask).  The backward of the same site is the same call
// with res = NULL and x = the incoming gradient: the mask is regenerated from the RNG snapshot
// (rng.hpp), nothing is stored.  8 elements per thread = one Philox call, 16/32-B vector accesses.
#include "common.hpp"
#include "rng.hpp"

namespace csu {
namespace {

constexpr int NT = 256;

template <typename TX, typename TO>
__global__ __launch_bounds__(NT) void dropout_apply(long n8, int cols, const TX* __restrict__ x,
                                                    const float* __restrict__ res, TO* __restrict__ out,
                                                    const float* __restrict__ row_scale, long rps,
                                                    const uint64_t* __restrict__ rng, uint32_t site, float p) {
    const DropoutRng r = load_rng(rng, site, p);
    for (long g = (long)blockIdx.x * NT + threadIdx.x; g < n8; g += (long)gridDim.x * NT) {
        const long e0 = g * 8;
        float v[8];
        load8(x + e0, v);
        float s = 1.f;
        if (row_scale) s = row_scale[(e0 / cols) / rps];
        uint32_t m = 0xffu;
        if (p > 0.f) {
            m = keep8(r, (uint64_t)g);
            s *= r.scale;
        }
        float o[8];
        if (res) load8(res + e0, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float t = ((m >> j) & 1u) ? s * v[j] : 0.f;
            o[j] = res ? o[j] + t : t;
        }
        store8(out + e0, o);
    }
}

__global__ __launch_bounds__(NT) void dropout_mask_kernel(long n, const uint64_t* __restrict__ rng, uint32_t site, float p,
                                                          uint8_t* __restrict__ out) {
    const DropoutRng r = load_rng(rng, site, p);
    for (long g = (long)blockIdx.x * NT + threadIdx.x; g * 8 < n; g += (long)gridDim.x * NT) {
        const uint32_t m = keep8(r, (uint64_t)g);
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (g * 8 + j < n) out[g * 8 + j] = (uint8_t)((m >> j) & 1u);
    }
}

// snap = state; state.counter += 1 -- the per-step snapshot every dropout site of one forward
// reads (and its backward re-reads); a device-side advance so a captured HIP graph draws fresh
// masks on every replay.
__global__ void rng_advance_kernel(uint64_t* __restrict__ state, uint64_t* __restrict__ snap) {
    if (threadIdx.x == 0) {
        const uint64_t seed = state[0], ctr = state[1];
        snap[0] = seed;
        snap[1] = ctr;
        state[1] = ctr + 1;
    }
}

// DropPath (timm drop_path, cswin:344/367-368): per-sample scale keep(site, b) / (1 - p)
__global__ __launch_bounds__(NT) void droppath_scale_kernel(long n, const uint64_t* __restrict__ rng, uint32_t site,
                                                            float p, float* __restrict__ out) {
    const DropoutRng r = load_rng(rng, site, p);
    for (long b = (long)blockIdx.x * NT + threadIdx.x; b < n; b += (long)gridDim.x * NT)
        out[b] = p > 0.f ? drop_scale(r, (uint64_t)b) : 1.f;
}

unsigned grid_for(long n8) {
    const long b = (n8 + NT - 1) / NT;
    return (unsigned)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_dropout_apply(long rows, int cols, int xdtype, const void* x, const float* res, int odtype, void* out,
                                 const float* row_scale, long rows_per_sample, const uint64_t* rng, unsigned site,
                                 float p, void* stream) {
    if (rows < 0 || cols < 1 || cols % 8 || !x || !out || p < 0.f || p >= 1.f || (p > 0.f && !rng) ||
        (row_scale && rows_per_sample < 1))
        return fail(CSU_E_ARG, "dropout: bad args (cols must be a multiple of 8, 0 <= p < 1)");
    const long n8 = rows * (long)cols / 8;
    if (!n8) return 0;
    hipStream_t st = as_stream(stream);
    const unsigned g = grid_for(n8);
#define DA(TX, TO) dropout_apply<TX, TO><<<g, NT, 0, st>>>(n8, cols, (const TX*)x, res, (TO*)out, row_scale, rows_per_sample, rng, site, p)
    if (xdtype == CSU_BF16 && odtype == CSU_BF16) DA(bf16, bf16);
    else if (xdtype == CSU_BF16 && odtype == CSU_F32) DA(bf16, float);
    else if (xdtype == CSU_F32 && odtype == CSU_F32) DA(float, float);
    else if (xdtype == CSU_F32 && odtype == CSU_BF16) DA(float, bf16);
    else return fail(CSU_E_ARG, "dropout: bad dtype");
#undef DA
    return check_launch("dropout_apply");
}

extern "C" int csu_dropout_mask(long n, const uint64_t* rng, unsigned site, float p, uint8_t* out, void* stream) {
    if (n < 0 || !rng || !out || p < 0.f || p >= 1.f) return fail(CSU_E_ARG, "dropout_mask: bad args");
    if (!n) return 0;
    dropout_mask_kernel<<<grid_for((n + 7) / 8), NT, 0, as_stream(stream)>>>(n, rng, site, p, out);
    return check_launch("dropout_mask");
}

extern "C" int csu_rng_advance(uint64_t* state, uint64_t* snap, void* stream) {
    if (!state || !snap) return fail(CSU_E_ARG, "rng_advance: null pointer");
    rng_advance_kernel<<<1, 64, 0, as_stream(stream)>>>(state, snap);
    return check_launch("rng_advance");
}

extern "C" int csu_droppath_scale(long n, const uint64_t* rng, unsigned site, float p, float* out, void* stream) {
    if (n < 0 || !out || p < 0.f || p >= 1.f || (p > 0.f && !rng)) return fail(CSU_E_ARG, "droppath_scale: bad args");
    if (!n) return 0;
    droppath_scale_kernel<<<grid_for((n + 7) / 8), NT, 0, as_stream(stream)>>>(n, rng, site, p, out);
    return check_launch("droppath_scale");
}
