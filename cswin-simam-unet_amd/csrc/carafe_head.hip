// Fused CARAFE4 + output head for the 1-class segmentation output (gfx950).
//
// The tail of CSWinTransformer (cswin:674-688) is upsample1 = CARAFE4(64, 64) followed by the
// bias-free 1x1 `output` conv and torch.sigmoid.  Everything after the CARAFE encoder is linear up
// to the sigmoid:
//   logit[P] = w_h . (W_o r[P] + b_o),   r[P] = sum_t m[P, t] x[nbr_t(p)]     (cswin:429-434, 680)
// so with u = W_o^T w_h (C-vector) and c = w_h . b_o (computed by the caller, differentiably),
//   logit[P] = sum_t m[P, t] z[nbr_t(p)] + c,   z[q] = u . x[q]   (z = 0 in the zero padding).
// The (B, 16 L, C) reassembled tensor, the `out` conv output and the head's re-read of it (three
// 0.5 GB bf16 tensors at 512x512, batch 16) are never formed: the forward reads x once (for z) and
// the encoder logits once; the backward reads them once more and writes d enc and d x.
//
// Indexing follows carafe.hip: enc is NHWC (B, H, W, 9 s^2) with channel t * s^2 + i * s + j for
// tap t = 3 ky + kx and sub-pixel (i, j); output pixel P = (b, s y + i, s x + j).
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;
constexpr int KT = 9;

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + __expf(-v)); }

// z[q] = sum_c u[c] x[q, c]; G = C / 8 lanes per token (power of two <= 64).
template <typename T>
__global__ __launch_bounds__(NT) void head_z(long P, int C, const T* __restrict__ x, const float* __restrict__ u,
                                             float* __restrict__ z) {
    const int G = C / 8;
    const long gid = (long)blockIdx.x * NT + threadIdx.x;
    const long q = gid / G;
    const int g = gid % G;
    float acc = 0.f;
    if (q < P) {
        float v[8], w[8];
        load8(x + q * C + 8 * g, v);
        load4(u + 8 * g, w);
        load4(u + 8 * g + 4, w + 4);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k] * w[k];
    }
    for (int o = G >> 1; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (q < P && g == 0) z[q] = acc;
}

// z of the 9 neighbours of (b, y, x) (0 in the zero padding): branch-free raw buffer loads, all 9
// in flight (a predicated load per tap made hipcc wait for each one)
__device__ __forceinline__ void neighbours(const float* __restrict__ z, int b, int y, int x, int B, int H, int W, float* zn) {
    const __amdgpu_buffer_rsrc_t rz = buf_rsrc(z, (long)B * H * W * 4);
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
        zn[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rz, in ? (unsigned)((((long)b * H + yy) * W + xx) * 4) : kOOB, 0, 0));
    }
}

// One thread per low-resolution pixel q = (b, y, x): its s x s output pixels.
template <typename T, int S>
__global__ __launch_bounds__(NT) void carafe_head_fwd(int B, int H, int W, const float* __restrict__ z,
                                                      const T* __restrict__ enc, const float* __restrict__ cb,
                                                      float* __restrict__ prob) {
    constexpr int S2 = S * S;
    const long q = (long)blockIdx.x * NT + threadIdx.x;
    if (q >= (long)B * H * W) return;
    const int x = q % W, y = (q / W) % H, b = q / ((long)H * W);
    float zn[KT];
    neighbours(z, b, y, x, B, H, W, zn);
    const float c = *cb;
    const T* e = enc + q * KT * S2;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        float lg[KT][S];
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            if constexpr (S == 4) load4(e + t * S2 + i * S, lg[t]);
            else {
#pragma unroll
                for (int j = 0; j < S; ++j) lg[t][j] = to_f(e[t * S2 + i * S + j]);
            }
        }
        float o[S];
#pragma unroll
        for (int j = 0; j < S; ++j) {
            float mx = lg[0][j];
#pragma unroll
            for (int t = 1; t < KT; ++t) mx = fmaxf(mx, lg[t][j]);
            float den = 0.f, acc = 0.f;
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                const float ex = __expf(lg[t][j] - mx);
                den += ex;
                acc += ex * zn[t];
            }
            o[j] = sigm(acc / den + c);
        }
        float* pr = prob + ((long)b * S * H + (long)S * y + i) * (S * W) + (long)S * x;
        if constexpr (S == 4) store4(pr, o);
        else {
#pragma unroll
            for (int j = 0; j < S; ++j) pr[j] = o[j];
        }
    }
}

// Backward, part 1 (one thread per low-res pixel q'): recompute m, then
//   dl[P] = dprob * p (1 - p);  d enc[q', t, sub] = dl m_t (z_t - sum_u m_u z_u);
//   tsum[q', t] = sum_sub dl m_t   (d z of neighbour t, gathered in part 2);  part[blk] = sum dl.
template <typename T, int S>
__global__ __launch_bounds__(NT) void carafe_head_bwd_enc(int B, int H, int W, const float* __restrict__ z,
                                                          const T* __restrict__ enc, const float* __restrict__ prob,
                                                          const float* __restrict__ dprob, T* __restrict__ denc,
                                                          float* __restrict__ tsum, float* __restrict__ part) {
    constexpr int S2 = S * S;
    __shared__ float red[NT / 64];
    const long q = (long)blockIdx.x * NT + threadIdx.x;
    float dls = 0.f;
    if (q < (long)B * H * W) {
        const int x = q % W, y = (q / W) % H, b = q / ((long)H * W);
        float zn[KT], tk[KT];
        neighbours(z, b, y, x, B, H, W, zn);
#pragma unroll
        for (int t = 0; t < KT; ++t) tk[t] = 0.f;
        const T* e = enc + q * KT * S2;
        T* de = denc + q * KT * S2;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            float lg[KT][S], pv[S], dp[S];
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                if constexpr (S == 4) load4(e + t * S2 + i * S, lg[t]);
                else {
#pragma unroll
                    for (int j = 0; j < S; ++j) lg[t][j] = to_f(e[t * S2 + i * S + j]);
                }
            }
            const long row = ((long)b * S * H + (long)S * y + i) * (S * W) + (long)S * x;
#pragma unroll
            for (int j = 0; j < S; ++j) {
                pv[j] = prob[row + j];
                dp[j] = dprob[row + j];
            }
#pragma unroll
            for (int j = 0; j < S; ++j) {
                float mx = lg[0][j];
#pragma unroll
                for (int t = 1; t < KT; ++t) mx = fmaxf(mx, lg[t][j]);
                float den = 0.f, acc = 0.f;
#pragma unroll
                for (int t = 0; t < KT; ++t) {
                    lg[t][j] = __expf(lg[t][j] - mx);
                    den += lg[t][j];
                    acc += lg[t][j] * zn[t];
                }
                const float inv = 1.f / den, mz = acc * inv;
                const float dl = dp[j] * pv[j] * (1.f - pv[j]);
                dls += dl;
#pragma unroll
                for (int t = 0; t < KT; ++t) {
                    const float m = lg[t][j] * inv;
                    tk[t] += dl * m;
                    lg[t][j] = dl * m * (zn[t] - mz);   // d enc logit
                }
            }
#pragma unroll
            for (int t = 0; t < KT; ++t) {
                if constexpr (S == 4) store4(de + t * S2 + i * S, lg[t]);
                else {
#pragma unroll
                    for (int j = 0; j < S; ++j) de[t * S2 + i * S + j] = from_f<T>(lg[t][j]);
                }
            }
        }
#pragma unroll
        for (int t = 0; t < KT; ++t) tsum[q * KT + t] = tk[t];
    }
    dls = wave_sum(dls);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dls;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) s += red[w];
        part[4 * blockIdx.x] = s;
        part[4 * blockIdx.x + 1] = 0.f;
        part[4 * blockIdx.x + 2] = 0.f;
        part[4 * blockIdx.x + 3] = 0.f;
    }
}

// Backward, part 2: dz[q] = sum_t tsum[q - off_t, t];  dx[q, :] = dz u;  du partial = sum_q dz x[q, :].
// G = C / 8 lanes per token, NT / G tokens in flight, RB tokens per workgroup.
template <typename T>
__global__ __launch_bounds__(NT) void carafe_head_bwd_x(int B, int H, int W, int C, long RB,
                                                        const float* __restrict__ tsum, const T* __restrict__ x,
                                                        const float* __restrict__ u, T* __restrict__ dx,
                                                        float* __restrict__ part) {
    __shared__ float red[NT * 8];
    const int G = C / 8, RPL = NT / G;
    const int g = threadIdx.x % G, rr = threadIdx.x / G;
    const long P = (long)B * H * W;
    const long q0 = (long)blockIdx.x * RB, q1 = q0 + RB < P ? q0 + RB : P;
    float uw[8], acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    load4(u + 8 * g, uw);
    load4(u + 8 * g + 4, uw + 4);
    const __amdgpu_buffer_rsrc_t rt = buf_rsrc(tsum, P * KT * 4);
    for (long q = q0 + rr; q < q1; q += RPL) {
        const int xq = q % W, y = (q / W) % H, b = q / ((long)H * W);
        float tv[KT];
#pragma unroll
        for (int t = 0; t < KT; ++t) {   // branch-free gathers, all 9 in flight
            const int yy = y - (t / 3 - 1), xx = xq - (t % 3 - 1);   // q = nbr_t(q')  <=>  q' = q - off_t
            const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
            tv[t] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rt, in ? (unsigned)(((((long)b * H + yy) * W + xx) * KT + t) * 4) : kOOB, 0, 0));
        }
        float dz = 0.f;
#pragma unroll
        for (int t = 0; t < KT; ++t) dz += tv[t];
        float v[8], o[8];
        load8(x + q * C + 8 * g, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc[k] += dz * v[k];
            o[k] = dz * uw[k];
        }
        store8(dx + q * C + 8 * g, o);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[rr * C + 8 * g + k] = acc[k];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) {
        float s = 0.f;
        for (int r = 0; r < RPL; ++r) s += red[r * C + c];
        part[(long)blockIdx.x * C + c] = s;
    }
}

struct HPlan {
    long P;
    int nb1;      // part-1 workgroups
    long rb;      // part-2 tokens per workgroup
    int nb2;      // part-2 workgroups
    size_t off_part1, off_part2, off_cs1, off_cs2, total;
};

size_t al(size_t v) { return (v + 255) & ~(size_t)255; }

HPlan hplan(int B, int H, int W, int C) {
    HPlan p;
    p.P = (long)B * H * W;
    p.nb1 = (int)((p.P + NT - 1) / NT);
    p.rb = (p.P + 1023) / 1024;
    if (p.rb < 64) p.rb = 64;
    p.nb2 = (int)((p.P + p.rb - 1) / p.rb);
    size_t o = al((size_t)p.P * KT * sizeof(float));
    p.off_part1 = o;
    o += al((size_t)p.nb1 * 4 * sizeof(float));
    p.off_part2 = o;
    o += al((size_t)p.nb2 * C * sizeof(float));
    p.off_cs1 = o;
    o += al(colsum_workspace(p.nb1, 4, CSU_F32));
    p.off_cs2 = o;
    o += al(colsum_workspace(p.nb2, C, CSU_F32));
    p.off_cs2 += 0;
    p.total = o + 256;   // + the 4-float d c staging row
    return p;
}

int check_head(int B, int H, int W, int C, int s) {
    if (B < 1 || H < 1 || W < 1 || (s != 2 && s != 4) || C < 8 || C > 512 || C % 8 || ((C / 8) & (C / 8 - 1)))
        return fail(CSU_E_ARG, "carafe_head: need s in {2, 4} and C = 8 * 2^k <= 512");
    return 0;
}

// Output-head weight folding (cswin:674-688): the CARAFE `out` 1x1 conv (O x C weight w_out, bias
// b_out) followed by the bias-free 1-class `output` conv (w_h, O) is linear, so the fused head
// uses u = w_out^T w_h (C) and cb = w_h . b_out.  One block: four o-quarters per column with 8
// loads in flight each (a serial per-thread loop over O paid one L2 round trip per term: 28 us),
// combined in a fixed order.  C <= 512 (check_head).
__global__ __launch_bounds__(NT) void head_fold_fwd(int O, int C, const float* __restrict__ w_out,
                                                    const float* __restrict__ b_out, const float* __restrict__ w_h,
                                                    float* __restrict__ u, float* __restrict__ cb) {
    __shared__ float red[4][512];
    __shared__ float rb[NT];
    const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int per = (O + 3) / 4, o0 = q * per, o1 = min(O, o0 + per);
    for (int c = l; c < C; c += 64) {
        float a = 0.f;
#pragma unroll 8
        for (int o = o0; o < o1; ++o) a = fmaf(w_out[(long)o * C + c], w_h[o], a);
        red[q][c] = a;
    }
    float bsum = 0.f;   // cb partial of thread t: o = t, t + NT, ...
    for (int o = threadIdx.x; o < O; o += NT) bsum = fmaf(w_h[o], b_out[o], bsum);
    rb[threadIdx.x] = bsum;
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) u[c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    if (threadIdx.x < 64) {   // fixed-order tree over the NT partials
        float v = (rb[threadIdx.x] + rb[threadIdx.x + 64]) + (rb[threadIdx.x + 128] + rb[threadIdx.x + 192]);
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (threadIdx.x == 0) cb[0] = v;
    }
}

// gradients of the folding from du (C) and dcb: dw_out[o][c] = w_h[o] du[c], db_out[o] = w_h[o] dcb,
// dw_h[o] = sum_c w_out[o][c] du[c] + b_out[o] dcb (four lanes per o, 8 loads in flight each,
// combined by fixed xor-shuffles)
__global__ __launch_bounds__(NT) void head_fold_bwd(int O, int C, const float* __restrict__ w_out,
                                                    const float* __restrict__ b_out, const float* __restrict__ w_h,
                                                    const float* __restrict__ du, const float* __restrict__ dcb,
                                                    float* __restrict__ dw_out, float* __restrict__ db_out,
                                                    float* __restrict__ dw_h) {
    const float g = dcb[0];
    for (long i = threadIdx.x; i < (long)O * C; i += NT) dw_out[i] = w_h[i / C] * du[i % C];
    const int part = threadIdx.x & 3, per = (C + 3) / 4, c0 = part * per, c1 = min(C, c0 + per);
    for (int ob = 0; ob < O; ob += NT / 4) {   // every lane runs every round (shuffles need the whole wave)
        const int o = ob + (threadIdx.x >> 2);
        float a = 0.f;
        if (o < O) {
#pragma unroll 8
            for (int c = c0; c < c1; ++c) a = fmaf(w_out[(long)o * C + c], du[c], a);
        }
        a += __shfl_xor(a, 1, 64);
        a += __shfl_xor(a, 2, 64);
        if (o < O && part == 0) {
            dw_h[o] = fmaf(b_out[o], g, a);
            db_out[o] = w_h[o] * g;
        }
    }
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_carafe_head_fwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                                   const float* u, const float* cb, float* z, float* prob, void* stream) {
    if (int e = check_head(B, H, W, C, s)) return e;
    if (!x || !enc || !u || !cb || !z || !prob) return fail(CSU_E_ARG, "carafe_head_fwd: null buffer");
    const long P = (long)B * H * W;
    hipStream_t st = as_stream(stream);
    const unsigned nz = (unsigned)((P * (C / 8) + NT - 1) / NT), np = (unsigned)((P + NT - 1) / NT);
#define CSU_HF(T, S) carafe_head_fwd<T, S><<<np, NT, 0, st>>>(B, H, W, z, (const T*)enc, cb, prob)
    if (dtype == CSU_BF16) {
        head_z<bf16><<<nz, NT, 0, st>>>(P, C, (const bf16*)x, u, z);
        if (s == 4) CSU_HF(bf16, 4); else CSU_HF(bf16, 2);
    } else if (dtype == CSU_F32) {
        head_z<float><<<nz, NT, 0, st>>>(P, C, (const float*)x, u, z);
        if (s == 4) CSU_HF(float, 4); else CSU_HF(float, 2);
    } else {
        return fail(CSU_E_ARG, "carafe_head_fwd: bad dtype");
    }
#undef CSU_HF
    return check_launch("carafe_head_fwd");
}

extern "C" size_t csu_carafe_head_bwd_workspace(int B, int H, int W, int C, int s) {
    if (check_head(B, H, W, C, s)) return 0;
    return hplan(B, H, W, C).total;
}

static int head_bwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc, const float* z,
                    const float* u, const float* prob, const float* dprob, void* dx, void* denc, float* du, float* dcb,
                    const csu_head_fold* fold, void* workspace, size_t ws_bytes, void* stream) {
    if (int e = check_head(B, H, W, C, s)) return e;
    if (!x || !enc || !z || !u || !prob || !dprob || !dx || !denc || !du || (!dcb && !fold))
        return fail(CSU_E_ARG, "carafe_head_bwd: null buffer");
    if (fold && (fold->O < 1 || !fold->w_out || !fold->b_out || !fold->w_h || !fold->dw_out || !fold->db_out || !fold->dw_h))
        return fail(CSU_E_ARG, "carafe_head_bwd: bad fold");
    const HPlan p = hplan(B, H, W, C);
    if (!workspace || ws_bytes < p.total) return fail(CSU_E_WORKSPACE, "carafe_head_bwd: workspace");
    char* ws = (char*)workspace;
    float* tsum = (float*)ws;
    float* part1 = (float*)(ws + p.off_part1);
    float* part2 = (float*)(ws + p.off_part2);
    float* dc4 = (float*)(ws + p.total - 256);
    hipStream_t st = as_stream(stream);
#define CSU_HB(T, S)                                                                                                \
    carafe_head_bwd_enc<T, S><<<p.nb1, NT, 0, st>>>(B, H, W, z, (const T*)enc, prob, dprob, (T*)denc, tsum, part1)
    if (dtype == CSU_BF16) {
        if (s == 4) CSU_HB(bf16, 4); else CSU_HB(bf16, 2);
        carafe_head_bwd_x<bf16><<<p.nb2, NT, 0, st>>>(B, H, W, C, p.rb, tsum, (const bf16*)x, u, (bf16*)dx, part2);
    } else if (dtype == CSU_F32) {
        if (s == 4) CSU_HB(float, 4); else CSU_HB(float, 2);
        carafe_head_bwd_x<float><<<p.nb2, NT, 0, st>>>(B, H, W, C, p.rb, tsum, (const float*)x, u, (float*)dx, part2);
    } else {
        return fail(CSU_E_ARG, "carafe_head_bwd: bad dtype");
    }
#undef CSU_HB
    if (int e = check_launch("carafe_head_bwd")) return e;
    if (int e = colsum_launch(p.nb2, C, CSU_F32, part2, du, (float*)(ws + p.off_cs2), st)) return e;
    if (int e = colsum_launch(p.nb1, 4, CSU_F32, part1, dc4, (float*)(ws + p.off_cs1), st)) return e;
    if (fold) {   // the head-weight gradients straight from du and the dcb partial sum
        head_fold_bwd<<<1, NT, 0, st>>>(fold->O, C, fold->w_out, fold->b_out, fold->w_h, du, dc4, fold->dw_out,
                                        fold->db_out, fold->dw_h);
        if (int e = check_launch("carafe_head_bwd: fold")) return e;
    }
    if (dcb && hipMemcpyAsync(dcb, dc4, sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return fail(CSU_E_ARG, "carafe_head_bwd: copy-out failed");
    return 0;
}

extern "C" int csu_carafe_head_bwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                                   const float* z, const float* u, const float* prob, const float* dprob, void* dx,
                                   void* denc, float* du, float* dcb, void* workspace, size_t ws_bytes, void* stream) {
    if (!dcb) return fail(CSU_E_ARG, "carafe_head_bwd: null dcb");
    return head_bwd(B, H, W, C, s, dtype, x, enc, z, u, prob, dprob, dx, denc, du, dcb, nullptr, workspace, ws_bytes,
                    stream);
}

extern "C" int csu_carafe_head_bwd_fold(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                                        const float* z, const float* u, const float* prob, const float* dprob, void* dx,
                                        void* denc, float* du, const csu_head_fold* fold, void* workspace,
                                        size_t ws_bytes, void* stream) {
    if (!fold) return fail(CSU_E_ARG, "carafe_head_bwd_fold: null fold");
    return head_bwd(B, H, W, C, s, dtype, x, enc, z, u, prob, dprob, dx, denc, du, nullptr, fold, workspace, ws_bytes,
                    stream);
}

extern "C" int csu_head_fold_fwd(int O, int C, const float* w_out, const float* b_out, const float* w_h, float* u,
                                 float* cb, void* stream) {
    if (O < 1 || C < 1 || !w_out || !b_out || !w_h || !u || !cb) return fail(CSU_E_ARG, "head_fold_fwd: bad args");
    head_fold_fwd<<<1, NT, 0, as_stream(stream)>>>(O, C, w_out, b_out, w_h, u, cb);
    return check_launch("head_fold_fwd");
}
