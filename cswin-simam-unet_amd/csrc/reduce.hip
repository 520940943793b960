// Deterministic column sums for gfx950: out[c] = sum_r in[r][c] (fp32 accumulation).
//
// Used for the Linear bias gradient (sum of dY over all B*L tokens), the split-K weight-gradient
// partial slabs and the LayerNorm dgamma/dbeta partials.  Two passes, fixed summation order
// (bitwise reproducible): pass 1 sums row chunks of a column block with 16-B loads and combines
// the row lanes of a workgroup in LDS; pass 2 adds the chunk partials in chunk order.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;

// destination of column c of the final sums: identity, or (m.on) the conv weight-gradient slab
// [N][KH*KW][C] + [N] bias re-laid out as torch's OIHW [N][Creal][KH*KW] + [N] (channels >= Creal,
// the zero padding of few-channel inputs, and slab padding columns dropped: -1)
__device__ __forceinline__ long out_index(const OutMap& m, long c) {
    if (!m.on) return c;
    const long k = (long)m.khw * m.C, w = (long)m.N * k;
    if (c >= w) return c < w + m.N ? (long)m.N * m.khw * m.creal + (c - w) : -1;
    const long n = c / k, rr = c - n * k, t = rr / m.C, ch = rr - t * m.C;
    return ch < m.creal ? (n * m.creal + ch) * m.khw + t : -1;
}

template <typename T>
__global__ __launch_bounds__(NT) void colsum_pass1(long rows, long cols, int tpr, long rows_per_chunk,
                                                   const T* __restrict__ in, float* __restrict__ out, OutMap om) {
    constexpr int V = 16 / sizeof(T);
    __shared__ float red[NT][V + 1];
    const int cl = threadIdx.x % tpr, rl = threadIdx.x / tpr, rpi = NT / tpr;
    const long c0 = ((long)blockIdx.x * tpr + cl) * V;
    const long r0 = (long)blockIdx.y * rows_per_chunk;
    const long r1 = min(rows, r0 + rows_per_chunk);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    if (c0 < cols) {
        long r = r0 + rl;
        // four independent row streams per thread keep four 16-B loads in flight
        float a1[V], a2[V], a3[V];
#pragma unroll
        for (int j = 0; j < V; ++j) a1[j] = a2[j] = a3[j] = 0.f;
        for (; r + 3 * rpi < r1; r += 4 * rpi) {
            float v0[V], v1[V], v2[V], v3[V];
            if constexpr (V == 8) {
                load8(in + r * cols + c0, v0); load8(in + (r + rpi) * cols + c0, v1);
                load8(in + (r + 2 * rpi) * cols + c0, v2); load8(in + (r + 3 * rpi) * cols + c0, v3);
            } else {
                load4(in + r * cols + c0, v0); load4(in + (r + rpi) * cols + c0, v1);
                load4(in + (r + 2 * rpi) * cols + c0, v2); load4(in + (r + 3 * rpi) * cols + c0, v3);
            }
#pragma unroll
            for (int j = 0; j < V; ++j) { acc[j] += v0[j]; a1[j] += v1[j]; a2[j] += v2[j]; a3[j] += v3[j]; }
        }
        for (; r < r1; r += rpi) {
            float v[V];
            if constexpr (V == 8) load8(in + r * cols + c0, v); else load4(in + r * cols + c0, v);
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] += v[j];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += (a1[j] + a2[j]) + a3[j];
    }
#pragma unroll
    for (int j = 0; j < V; ++j) red[threadIdx.x][j] = acc[j];
    __syncthreads();
    if (rl == 0 && c0 < cols) {
        for (int q = 1; q < rpi; ++q)
#pragma unroll
            for (int j = 0; j < V; ++j) acc[j] += red[q * tpr + cl][j];
        if (om.on) {   // single chunk: the final sums, re-laid out
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const long d = c0 + j < cols ? out_index(om, c0 + j) : -1;
                if (d >= 0) out[d] = acc[j];
            }
        } else {
            float* o = out + (long)blockIdx.y * cols + c0;
#pragma unroll
            for (int j = 0; j < V; ++j)
                if (c0 + j < cols) o[j] = acc[j];
        }
    }
}

// 32 columns x 8 chunk lanes per workgroup; lanes combined in lane order in LDS
__global__ __launch_bounds__(NT) void colsum_pass2(long cols, int nchunks, const float* __restrict__ part,
                                                   float* __restrict__ out, OutMap om) {
    __shared__ float red[8][33];
    const int cl = threadIdx.x & 31, lane = threadIdx.x >> 5;
    const long c = (long)blockIdx.x * 32 + cl;
    float s0 = 0.f, s1 = 0.f;
    if (c < cols) {
        int k = lane;
        for (; k + 8 < nchunks; k += 16) {
            s0 += part[(long)k * cols + c];
            s1 += part[(long)(k + 8) * cols + c];
        }
        if (k < nchunks) s0 += part[(long)k * cols + c];
    }
    red[lane][cl] = s0 + s1;
    __syncthreads();
    if (lane == 0 && c < cols) {
        float s = red[0][cl];
        for (int l = 1; l < 8; ++l) s += red[l][cl];
        const long d = out_index(om, c);
        if (d >= 0) out[d] = s;
    }
}

struct Plan {
    int tpr, colblocks, chunks;
    long rpc;
};

// Latency-bound shapes (a few dozen slab rows x 10^5 columns) need many workgroups and few
// dependent loads per thread: at most 64 column threads per row group (>= 4 row lanes per
// workgroup) and ~8 rows per thread, i.e. two rounds of the 4-stream loop.
Plan plan(long rows, long cols, int V) {
    Plan p;
    const long vecs = (cols + V - 1) / V;
    p.tpr = (int)(vecs >= 64 ? 64 : vecs);
    int t = 1;                                  // round tpr up to a power of two dividing NT
    while (t < p.tpr) t <<= 1;
    p.tpr = t;
    p.colblocks = (int)((vecs + p.tpr - 1) / p.tpr);
    const int rpi = NT / p.tpr;
    long want = (rows + 8L * rpi - 1) / (8L * rpi);   // ~8 rows per thread
    if (want > 256) want = 256;
    if (want < 1) want = 1;
    p.chunks = (int)want;
    p.rpc = (rows + p.chunks - 1) / p.chunks;
    return p;
}

}  // namespace

size_t colsum_workspace(long rows, long cols, int dtype) {
    const Plan p = plan(rows, cols, dtype == CSU_BF16 ? 8 : 4);
    return p.chunks > 1 ? (size_t)p.chunks * cols * sizeof(float) : 0;
}

int colsum_launch(long rows, long cols, int dtype, const void* in, float* out, float* ws, hipStream_t st,
                  const OutMap* map) {
    const OutMap om = map ? *map : OutMap{0, 0, 0, 0, 0};
    const int V = dtype == CSU_BF16 ? 8 : 4;
    if (cols % V) return fail(CSU_E_ARG, "colsum: cols must be a multiple of 16 bytes");
    const Plan p = plan(rows, cols, V);
    float* dst = p.chunks > 1 ? ws : out;
    const dim3 grid(p.colblocks, p.chunks);
    if (dtype == CSU_BF16)
        colsum_pass1<bf16><<<grid, NT, 0, st>>>(rows, cols, p.tpr, p.rpc, (const bf16*)in, dst,
                                                             p.chunks > 1 ? OutMap{0, 0, 0, 0, 0} : om);
    else
        colsum_pass1<float><<<grid, NT, 0, st>>>(rows, cols, p.tpr, p.rpc, (const float*)in, dst,
                                                              p.chunks > 1 ? OutMap{0, 0, 0, 0, 0} : om);
    if (p.chunks > 1) colsum_pass2<<<(unsigned)((cols + 31) / 32), NT, 0, st>>>(cols, p.chunks, ws, out, om);
    return check_launch("colsum");
}

}  // namespace csu

using namespace csu;

extern "C" size_t csu_colsum_workspace(long rows, long cols, int dtype) { return colsum_workspace(rows, cols, dtype); }

extern "C" int csu_colsum(long rows, long cols, int dtype, const void* in, float* out, void* workspace,
                          size_t ws_bytes, void* stream) {
    if (rows < 1 || cols < 1 || !in || !out) return fail(CSU_E_ARG, "colsum: bad args");
    if (dtype != CSU_F32 && dtype != CSU_BF16) return fail(CSU_E_ARG, "colsum: bad dtype");
    if (ws_bytes < colsum_workspace(rows, cols, dtype) || (colsum_workspace(rows, cols, dtype) && !workspace))
        return fail(CSU_E_WORKSPACE, "colsum: workspace too small");
    return colsum_launch(rows, cols, dtype, in, out, (float*)workspace, as_stream(stream));
}
