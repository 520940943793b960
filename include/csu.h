/*
 * csu.h -- C ABI of libcsu_hip.so, the MI355X (gfx950) kernels of the CSWin-(SimAM-)UNet
 * training path.  Plain pointers, int sizes and a hipStream_t passed as void*; no framework
 * types.  Every buffer is owned by the caller (the library never allocates); every call is
 * asynchronous on `stream` and reentrant.  Return 0 on success, a positive hipError_t, or a
 * negative CSU_E* code; csu_last_error_string() describes the last failure of the calling thread.
 *
 * Layout convention: activations are token-major "(B, L, C)" = NHWC with L = H*W, exactly the
 * reference's token layout (train_cswinunet_segmentation.py, the `B, L, C` tensors of
 * cswin:349-370), so no NCHW transposes are needed between ops.
 *
 * The reference has no FFI (it is pure PyTorch); each entry point below names the reference
 * operator it replaces (cswin:N = train_cswinunet_segmentation.py line N,
 * unet:N = train_unet_segmentation.py line N).  The Python binding is csu/_lib.py (ctypes).
 */
#ifndef CSU_H_
#define CSU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum csu_dtype { CSU_F32 = 0, CSU_BF16 = 1 };

enum csu_status {
    CSU_OK = 0,
    CSU_E_ARG = -1,       /* invalid argument (shape, dtype, null pointer) */
    CSU_E_UNSUPPORTED = -2,
    CSU_E_WORKSPACE = -3  /* workspace too small */
};

const char* csu_last_error_string(void);
/* Library version and the offload arch it was built for ("gfx950"). */
const char* csu_build_info(void);

/* Timing events for bench.py's per-kernel roofline ledger (measurement plumbing, not part of the
 * reference interface).  csu_event_record_ext: inside a stream capture it appends an event-record
 * NODE to the graph being captured (hipGraphAddEventRecordNode after the stream's current
 * dependencies, which it then replaces), so every replay re-stamps it and csu_event_elapsed_ms
 * gives each captured kernel's time in that replay (torch refuses external events on ROCm).
 * Outside a capture it is a plain hipEventRecord. */
int csu_event_create(void** event);
int csu_event_destroy(void* event);
int csu_event_record_ext(void* event, void* stream);
int csu_event_elapsed_ms(void* start, void* end, float* ms);

/* ---------------------------------------------------------------------------------------
 * Cross-shaped stripe attention with LePE (LePEAttention.forward, cswin:271-298, geometry
 * cswin:232-240, get_v depthwise 3x3 cswin:244/256-269; branch split + concat of
 * CSWinBlock.forward cswin:358-363).  One call runs every branch of a CSWinBlock: branch i
 * reads its Q/K/V channels [ch_off, ch_off + heads*head_dim) of the (B, L, 3C) qkv Linear
 * output and writes the same channels of the (B, L, C) output (the torch.cat is free).
 * ------------------------------------------------------------------------------------- */
typedef struct {
    int32_t H_sp, W_sp;      /* stripe window: idx0 (reso, sw), idx1 (sw, reso), idx-1 (reso, reso) */
    int32_t ch_off;          /* first channel of this branch inside C (0 or C/2) */
    int32_t _pad;
    const float* lepe_w;     /* get_v.weight (C_b, 1, 3, 3), fp32 master weight */
    const float* lepe_b;     /* get_v.bias (C_b), fp32 */
    float* lepe_dw;          /* backward: written (not accumulated) gradient of lepe_w */
    float* lepe_db;          /* backward: gradient of lepe_b */
} csu_stripe_branch;

typedef struct {
    int32_t B, reso, C;      /* L = reso*reso tokens; qkv rows are 3C wide, output rows C wide */
    int32_t heads;           /* heads per branch (num_heads/2, or num_heads for the last stage) */
    int32_t head_dim;        /* must be 32 (embed_dim is hard-wired to 64: SURVEY §0.5) */
    int32_t nbranch;         /* 1 (last stage, idx -1) or 2 (idx 0 and idx 1) */
    float scale;             /* qk_scale or head_dim**-0.5 (cswin:231) */
    int32_t _pad;
    csu_stripe_branch br[2];
    /* attention dropout on the softmax probabilities (attn_drop, cswin:290), p = 0: none.  rng =
     * device [seed, counter] snapshot of the step (uint64 x 2), the same for forward and backward;
     * branch i uses dropout site drop_site + i.  Mask element of (branch, image b, window win,
     * head hh, query q, key k): ((((b * nwin + win) * heads + hh) * N + q) * Npad + k) with
     * N = window tokens, Npad = N rounded up to 32 (csu_dropout_mask materialises it). */
    const uint64_t* drop_rng;
    uint32_t drop_site;
    float drop_p;
} csu_stripe_args;

/* out (B, L, C) dtype; lse fp32 [nbranch][B][heads][L] (softmax log-sum-exp, saved for bwd). */
int csu_stripe_attn_fwd(const csu_stripe_args* a, int dtype, const void* qkv, void* out,
                        float* lse, void* stream);

/* Workspace bytes csu_stripe_attn_bwd needs (fp32 partial sums of the LePE weight gradient). */
size_t csu_stripe_attn_bwd_workspace(const csu_stripe_args* a);

/* Gradient of the forward above.  out = forward output, dout = its gradient (B, L, C);
 * delta fp32 scratch shaped like lse; dqkv (B, L, 3C) is fully written (Q|K|V slots of every
 * branch's channels); lepe_dw / lepe_db of each branch are written. */
int csu_stripe_attn_bwd(const csu_stripe_args* a, int dtype, const void* qkv, const void* out,
                        const void* dout, const float* lse, float* delta, void* dqkv,
                        void* workspace, size_t workspace_bytes, void* stream);
/* LePE weight/bias gradient alone (csu_stripe_attn_bwd skips it when every lepe_dw / lepe_db of
 * the args is NULL): lets it run on a second stream, concurrently with the dQ / dK / dV kernels.
 * Workspace: csu_stripe_attn_bwd_workspace bytes. */
int csu_stripe_lepe_wgrad(const csu_stripe_args* a, int dtype, const void* qkv, const void* dout,
                          void* workspace, size_t workspace_bytes, void* stream);
/* Deferred LePE weight gradient: csu_stripe_attn_bwd_ex with lepe_deferred = 1 leaves the per-block
 * partials in `workspace` (csu_stripe_lepe_nblk(a, dtype) blocks) instead of reducing them; one
 * csu_stripe_lepe_reduce_batch launch later reduces many such workspaces (e.g. every block's at the
 * end of a backward pass).  channels = heads * 32 per branch; dw [channels][9], db [channels]. */
int csu_stripe_attn_bwd_ex(const csu_stripe_args* a, int dtype, const void* qkv, const void* out, const void* dout,
                           const float* lse, float* delta, void* dqkv, void* workspace, size_t workspace_bytes,
                           int lepe_deferred, void* stream);
int csu_stripe_lepe_nblk(const csu_stripe_args* a, int dtype);
typedef struct {
    const float* part;
    float* dw[2];
    float* db[2];
    int32_t nblk, channels, nbranch, _pad;
} csu_lepe_reduce_item;
int csu_stripe_lepe_reduce_batch(const csu_lepe_reduce_item* items, int count, void* stream);

/* ---------------------------------------------------------------------------------------
 * LayerNorm over the last dim C of (rows, C) (nn.LayerNorm: norm1/norm2 cswin:315/347,
 * Merge_Block.norm cswin:377, patch-embed LN cswin:507, norm/norm_up cswin:554/602).
 * x dtype = xdtype, y dtype = ydtype (bf16 output feeds the next GEMM directly), gamma/beta
 * fp32; mean/rstd fp32 [rows] are saved for backward.
 * ------------------------------------------------------------------------------------- */
int csu_layernorm_fwd(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                      const float* beta, int ydtype, void* y, float* mean, float* rstd, void* stream);
size_t csu_layernorm_bwd_workspace(int rows, int C);
/* dx (xdtype) written; dgamma/dbeta fp32 written (deterministic two-pass reduction). */
int csu_layernorm_bwd(int rows, int C, int xdtype, const void* x, const float* gamma,
                      const float* mean, const float* rstd, int dydtype, const void* dy,
                      void* dx, float* dgamma, float* dbeta, void* workspace, size_t ws_bytes,
                      void* stream);
/* Residual-junction backward of y = LN(x) inside x_out = x + f(y) (CSWinBlock cswin:367-368):
 * dx = dres + dLN(dy) in one pass (dres fp32 [rows][C] or NULL; x/dx fp32 when dres is given),
 * plus an optional bf16 copy dx_bf16 (the next GEMM's operand; NULL to skip).  Replaces the
 * autograd add of the two branches and the bf16 cast of the summed gradient. */
int csu_layernorm_bwd_ex(int rows, int C, int xdtype, const void* x, const float* gamma,
                         const float* mean, const float* rstd, int dydtype, const void* dy,
                         const float* dres, void* dx, void* dx_bf16, float* dgamma, float* dbeta,
                         void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * SimAM (parameter-free energy gate) on token rows (B, L, C), statistics per (b, c) over L.
 * NOT in the reference: public SimAM formula; parity unpinned vs the
 * reference.  stats fp32 [B][C][2] = (mean, 4*(var_unbiased + lambda)) saved for backward.
 * ------------------------------------------------------------------------------------- */
/* dgamma / dbeta from the per-block partials that csu_layernorm_bwd_ex left in `workspace` when
 * called with dgamma = dbeta = NULL (same rows / C): the parameter reduction can then run on a
 * second stream, off the input-gradient chain. */
int csu_layernorm_param_reduce(int rows, int C, const void* workspace, float* dgamma, float* dbeta, void* stream);
/* the same for many layers in one launch (the deferred end-of-backward reduction of every
 * LayerNorm's dgamma / dbeta): items is a HOST array, copied into the kernel arguments */
typedef struct {
    const void* workspace;
    float* dgamma;
    float* dbeta;
    int32_t rows, C;
    int32_t nblocks;   /* partial rows in the workspace; 0: those of csu_layernorm_bwd_ex for `rows` */
    int32_t _pad;
} csu_ln_param_item;
int csu_layernorm_param_reduce_batch(const csu_ln_param_item* items, int count, void* stream);

size_t csu_simam_workspace(int B, int L, int C);
/* y (ydtype, e.g. bf16 for the GEMM that consumes the gated skip) = SimAM(x); C % 4 == 0 */
int csu_simam_fwd(int B, int L, int C, float lambda, int xdtype, const void* x, int ydtype, void* y, float* stats,
                  void* workspace, size_t ws_bytes, void* stream);
/* dx (xdtype) from dy (gdtype) */
int csu_simam_bwd(int B, int L, int C, int xdtype, const void* x, const float* stats, int gdtype, const void* dy,
                  void* dx, void* workspace, size_t ws_bytes, void* stream);
/* The skip fork of the CSWin-SimAM-UNet encoder (an fp32 stage output feeding the Merge_Block conv
 * and, through SimAM, the decoder's concat_linear -- cswin:530-545 / 568-592 + the SimAM gate):
 * y = bf16(SimAM(x)) and xc = bf16(x) from the same passes (no separate cast of x). */
int csu_simam_fwd_fork(int B, int L, int C, float lambda, const float* x, void* y, void* xc, float* stats,
                       void* workspace, size_t ws_bytes, void* stream);
/* its backward: dx = g2 + (SimAM input gradient of dy), dxb = bf16(dx); g2 bf16 (the conv's input
 * gradient), dy gdtype -- the autograd sum and both casts in the gate-gradient pass */
int csu_simam_bwd_join(int B, int L, int C, const float* x, const float* stats, int gdtype, const void* dy,
                       const void* g2, float* dx, void* dxb, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * CARAFE content-aware reassembly (CARAFE/CARAFE4.forward cswin:401-437 / 450-486, from the
 * encoder logits to the input of the `out` 1x1 conv: pixel_shuffle + softmax over 9 taps +
 * unfold + (C x 9)@(9 x s^2) + pixel_shuffle, fused).  x (B, H*W, C) tokens, enc (B, H, W, 9*s*s)
 * NHWC logits with channel t*s*s + i*s + j, out (B, sH*sW, C); wsave fp32 (B, H, W, 9*s*s)
 * softmax weights written by fwd for bwd.  C = 8 * 2^k <= 512.
 * ------------------------------------------------------------------------------------- */
int csu_carafe_fwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                   void* out, float* wsave, void* stream);
/* dx (B, H*W, C) and denc (B, H, W, 9*s*s) written. */
int csu_carafe_bwd(int B, int H, int W, int C, int s, int dtype, const void* x, const float* wsave,
                   const void* dout, void* dx, void* denc, void* stream);

/* ---------------------------------------------------------------------------------------
 * 1-class output head: 1x1 conv without bias + sigmoid (CSWinTransformer.up_x4 `output`
 * cswin:603/680 and forward's torch.sigmoid cswin:688).  x (P, C) tokens, w (C) fp32,
 * prob (P) fp32.  C in {8, 16, 32, 64}.
 * ------------------------------------------------------------------------------------- */
int csu_head_fwd(long P, int C, int dtype, const void* x, const float* w, float* prob, void* stream);
size_t csu_head_bwd_workspace(long P, int C);
/* dprob -> dx (P, C) and dw (C) (deterministic two-pass reduction). */
int csu_head_bwd(long P, int C, int dtype, const void* x, const float* w, const float* prob,
                 const float* dprob, void* dx, float* dw, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused CARAFE4 + 1-class output head (CSWinTransformer.up_x4 + sigmoid, cswin:674-688):
 * everything after upsample1's encoder conv is linear up to the sigmoid, so with
 * u = W_out^T w_output (C fp32) and cb = w_output . b_out (1 fp32, device), computed by the caller,
 *   prob[b, s y + i, s x + j] = sigmoid(sum_t m[t] z[nbr_t(y, x)] + cb),  z[q] = u . x[q]
 * (m = softmax over the 9 taps of enc[b, y, x, t*s*s + i*s + j]; cswin:456-481).  x (B, H*W, C)
 * tokens, enc NHWC (B, H, W, 9 s^2), z fp32 (B*H*W) written for bwd, prob fp32 (B, sH, sW).
 * s in {2, 4}; C = 8 * 2^k <= 512.
 * ------------------------------------------------------------------------------------- */
int csu_carafe_head_fwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                        const float* u, const float* cb, float* z, float* prob, void* stream);
size_t csu_carafe_head_bwd_workspace(int B, int H, int W, int C, int s);
/* dprob -> dx (B, H*W, C), denc (B, H, W, 9 s^2), du (C) and dcb (1), fp32 reductions deterministic. */
int csu_carafe_head_bwd(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                        const float* z, const float* u, const float* prob, const float* dprob, void* dx,
                        void* denc, float* du, float* dcb, void* workspace, size_t ws_bytes, void* stream);
/* Head-weight folding (the `out` 1x1 conv w_out (O x C) + b_out (O) and the 1-class `output` conv
 * w_h (O), cswin:674-688): u = w_out^T w_h, cb = w_h . b_out (fp32, one launch, fixed order). */
int csu_head_fold_fwd(int O, int C, const float* w_out, const float* b_out, const float* w_h, float* u, float* cb,
                      void* stream);
typedef struct {
    int32_t O;
    const float* w_out;  /* (O, C) */
    const float* b_out;  /* (O) */
    const float* w_h;    /* (O) */
    float* dw_out;       /* (O, C) = w_h du^T */
    float* db_out;       /* (O) = w_h dcb */
    float* dw_h;         /* (O) = w_out du + b_out dcb */
} csu_head_fold;
/* csu_carafe_head_bwd with the folding's backward appended (gradients of w_out, b_out, w_h from du
 * and dcb inside the same call; dcb itself not returned) */
int csu_carafe_head_bwd_fold(int B, int H, int W, int C, int s, int dtype, const void* x, const void* enc,
                             const float* z, const float* u, const float* prob, const float* dprob, void* dx,
                             void* denc, float* du, const csu_head_fold* fold, void* workspace, size_t ws_bytes,
                             void* stream);

/* ---------------------------------------------------------------------------------------
 * Deterministic column sum out[c] = sum_r in[r][c], fp32 accumulation (rows x cols row-major,
 * dtype in; out fp32).  The bias gradient of every nn.Linear (cswin:185/187/314/323/568/581/592)
 * is the column sum of dY over the B*L tokens; also reduces split-K weight-gradient slabs.
 * ------------------------------------------------------------------------------------- */
size_t csu_colsum_workspace(long rows, long cols, int dtype);
int csu_colsum(long rows, long cols, int dtype, const void* in, float* out, void* workspace,
               size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Linear weight + bias gradient over M token rows (backward of every nn.Linear on tokens:
 * cswin:185/187/314/323/568/581/592 and the CARAFE 1x1 convs cswin:396/399).
 * dy (M, N), x (M, K) row-major, dtype in; dw_db fp32 [N*K + N] = dW (N, K) then db (N), written.
 * Split-K over M with MFMA tiles; the chunk partials are summed in a fixed order (bitwise
 * reproducible).  N, K multiples of 16 bytes.
 * ------------------------------------------------------------------------------------- */
size_t csu_linear_wgrad_workspace(long M, int N, int K);
int csu_linear_wgrad(long M, int N, int K, int dtype, const void* dy, const void* x, float* dw_db,
                     void* workspace, size_t ws_bytes, void* stream);
/* Deferred form (bf16): only the tile kernel runs now; when the plan splits the tokens
 * (item->chunks > 1) the chunk partials stay in `workspace` and dw_db is written later by
 * csu_wslab_reduce_batch over the returned items (one launch for many Linears, e.g. at the end of
 * a backward pass; workspace and dw_db must stay allocated until then).  item->chunks == 1: dw_db
 * is already written. */
typedef struct {
    const float* slab;
    float* dst;
    int32_t N, K, tn, tk, chunks, _pad;
} csu_wslab_item;
int csu_linear_wgrad_deferred(long M, int N, int K, const void* dy, const void* x, float* dw_db,
                              void* workspace, size_t ws_bytes, csu_wslab_item* item, void* stream);
int csu_wslab_reduce_batch(const csu_wslab_item* items, int count, void* stream);
/* Grouped weight gradients (bf16): the tile kernels of many Linears in one launch per tile size
 * (items: HOST array, copied into kernel arguments, <= 48 items per launch).  Each item's plan
 * (tile, token chunks) comes from csu_linear_wgrad_group_plan, which returns the slab workspace
 * bytes the item needs (0: dw_db is written directly); items with chunks > 1 are completed by
 * csu_wslab_reduce_batch with {slab, dw_db, N, K, tn, tk, chunks}.  M < 2^31 tokens. */
typedef struct {
    const void* dy;      /* (M, N) bf16 */
    const void* x;       /* (M, K) bf16 */
    float* dw_db;        /* N*K + N fp32 */
    float* slab;         /* workspace of csu_linear_wgrad_group_plan's size, or NULL if 0 */
    int64_t M;
    int32_t N, K;
} csu_wgrad_group_item;
size_t csu_linear_wgrad_group_plan(long M, int N, int K, int* tn, int* tk, int* chunks);
int csu_linear_wgrad_group(const csu_wgrad_group_item* items, int count, void* stream);
/* Same with the plan forced (tuning / tests): bf16 output tile tn x tk (64 or 128; 0 = auto) and
 * the number of token chunks (0 = auto).  The fp32 path ignores them. */
size_t csu_linear_wgrad_tuned_workspace(long M, int N, int K, int tn, int tk, int chunks);
int csu_linear_wgrad_tuned(long M, int N, int K, int dtype, const void* dy, const void* x, float* dw_db,
                           void* workspace, size_t ws_bytes, int tn, int tk, int chunks, void* stream);

/* ---------------------------------------------------------------------------------------
 * Token GEMM, bf16 operands, fp32 accumulation, fused prologue/epilogue (nn.Linear of
 * CSWinBlock/Mlp cswin:185-195, 314-368 plus the GELU, GELU-backward and residual-add passes):
 *   out[m][n] = ((sum_k pro(a[m][k]) * B(n,k)) + bias[n]) * gelu'(gelu_aux[m][n]) + resid[m][n]
 *   B(n,k) = b[n*ldb + k] (b_trans = 0) or b[k*ldb + n] (b_trans = 1); pro = gelu if a_gelu.
 * bias / gelu_aux (bf16, ld = ldc) / resid (fp32, ld = ldc) may be NULL; resid needs out fp32.
 * K, lda, ldb multiples of 8 (and N when b_trans).
 * ------------------------------------------------------------------------------------- */
int csu_gemm(long M, int N, int K, const void* a, int lda, const void* b, int ldb, int b_trans, int a_gelu,
             const float* bias, const void* gelu_aux, const float* resid, void* out, int ldc, int out_dtype,
             void* stream);
/* Extended form: everything csu_gemm takes plus
 *   gelu_out  bf16 (M, ldc) or NULL: also write gelu(out) (exact erf GELU) -- fc1's activation
 *             next to its pre-activation (needs out bf16, no gelu_aux/resid);
 *   cfg       tile configuration of the b_trans = 0 kernel (0: 64x64, 1: 64x128, 2: 128x64,
 *             3: 128x128; -1 = per-shape choice, what csu_gemm uses). */
typedef struct {
    int64_t M;
    int32_t N, K;
    const void* a;
    const void* b;
    int32_t lda, ldb;
    int32_t b_trans, a_gelu;
    const float* bias;
    const void* gelu_aux;
    const float* resid;
    void* out;
    void* gelu_out;
    int32_t ldc, out_dtype;
    int32_t cfg, _pad;
} csu_gemm_desc;
int csu_gemm_ex(const csu_gemm_desc* d, void* stream);

/* The proj Linear + residual of CSWinBlock (cswin:366-367, K = N = C in {64, 128, 256}) with the
 * block's norm2 LayerNorm (cswin:368 -> Mlp input) in the epilogue: out = resid + x W^T + bias (fp32,
 * as csu_gemm_ws with resid) and ln_out = bf16(LayerNorm(out; gamma, beta, eps)) + the per-token mean /
 * rstd (fp32) for its backward.  M % (64 or 128) == 0 (csu_gemm_ws_ln_supported). */
int csu_gemm_ws_ln_supported(long M, int C, int K);
int csu_gemm_ws_ln(long M, int C, const void* x, int ldx, const void* w_frag, const float* bias, const float* resid,
                   float* out, const float* gamma, const float* beta, float eps, void* ln_out, float* mean, float* rstd,
                   void* stream);

/* ---------------------------------------------------------------------------------------
 * Weight-streaming token GEMM (csrc/gemm_ws.hip): out (M, N) = x (M, K) @ W^T (+ bias) (+ resid),
 * for the CSWinBlock qkv / proj Linears (cswin:337, 366) and their input gradients at C = 128 / 256.
 * x bf16 with row stride ldx; w_frag = W (N, K) bf16 in FRAGMENT order (csu_frag_layout_batch);
 * bias fp32 (N) or NULL; resid fp32 (M, N) or NULL (then out_dtype must be CSU_F32); out_dtype
 * CSU_BF16 or CSU_F32, out (M, N) contiguous.  csu_gemm_ws_supported says whether (M, N, K, resid,
 * out_dtype) is instantiated (M % 64 == 0; (K, N) in {(128,384), (256,768), (384,128), (768,256),
 * (128,128), (256,256)}); other shapes return CSU_E_ARG.
 * ------------------------------------------------------------------------------------- */
int csu_gemm_ws_supported(long M, int N, int K, int resid, int out_dtype);
int csu_gemm_ws(long M, int N, int K, const void* x, int ldx, const void* w_frag, const float* bias, const float* resid,
                int out_dtype, void* out, void* stream);
/* The input gradient of a LayerNorm -> Linear pair (CSWinBlock norm1 -> qkv, cswin:357 / 337) with the
 * LayerNorm backward in the GEMM's epilogue: dh = dy (M, K) @ W^T-fragments (wt_frag: the (C, K) weight
 * transpose, fragment-ordered) is never written; instead dx (M, C) fp32 = dres + rstd (g - mean(g) -
 * xhat mean(g xhat)), g = dh * gamma, xhat = (x - mean) rstd, its bf16 copy dx_bf16, and the dgamma /
 * dbeta column partials of every 64-token block into part [M / 64][2C] (reduce them with
 * csu_layernorm_param_reduce_batch, nblocks = M / 64).  x fp32 (M, C); dres fp32 (M, C) or NULL.
 * Instantiated for (C, K) = (128, 384), (256, 768); M % 64 == 0 (csu_gemm_ws_lnbwd_supported). */
int csu_gemm_ws_lnbwd_supported(long M, int C, int K);
int csu_gemm_ws_lnbwd(long M, int C, int K, const void* dy, const void* wt_frag, const float* x, const float* gamma,
                      const float* mean, const float* rstd, const float* dres, float* dx, void* dx_bf16, float* part,
                      void* stream);
/* Fragment-ordered copy of a bf16 (rows x cols) matrix, rows % 32 == 0, cols % 16 == 0: 16-B chunk
 * q of row n (k = 8q .. 8q+7) goes to chunk ((n / 32) * (cols / 16) + q / 2) * 64 + n % 32 + 32 (q % 2),
 * i.e. [rows/32][cols/16][64 lanes][8] -- the MFMA 32x32x16 A-operand fragment of lane (n % 32, half).
 * items: DEVICE array sorted by chunk0 (first 16-B chunk of the item; chunk0[i+1] = chunk0[i] +
 * rows * cols / 8); total_chunks = the sum. */
typedef struct {
    const void* src;
    void* dst;
    int32_t rows, cols;
    int64_t chunk0;
} csu_frag_item;
int csu_frag_layout_batch(const csu_frag_item* items, int count, long total_chunks, void* stream);

/* e4m3 weights (BASELINE config 5, the fp8 format's qkv / proj Linears): csu_gemm_ws with W = q * s[n]
 * given as e4m3 bytes q in fragment order (csu_frag8_layout_batch: [N/32][K/16][64 lanes][8 bytes]) and
 * per-row power-of-two scales s (fp32, length N of the Linear).  scale_mode 1: out = x W^T (w_frag8 =
 * the fragments of q, s indexed by the output column); 2: out = dy W, the input gradient (w_frag8 = the
 * fragments of q^T, s indexed by the reduction index).  Bitwise equal to csu_gemm_ws on the dequantised
 * bf16 weight (power-of-two scales are applied exactly); same shapes / epilogues as csu_gemm_ws.
 * csu_gemm_ws_ln_e4m3: csu_gemm_ws_ln with e4m3 weights (scale_mode 1). */
int csu_gemm_ws_e4m3(long M, int N, int K, const void* x, int ldx, const void* w_frag8, const float* w_scale,
                     int scale_mode, const float* bias, const float* resid, int out_dtype, void* out, void* stream);
int csu_gemm_ws_ln_e4m3(long M, int C, const void* x, int ldx, const void* w_frag8, const float* w_scale,
                        const float* bias, const float* resid, float* out, const float* gamma, const float* beta,
                        float eps, void* ln_out, float* mean, float* rstd, void* stream);
/* e4m3 fragment order of an e4m3 (N x K) matrix src (transpose 0: of src itself, rows N; 1: of src^T,
 * rows K); N % 32 == 0, K % 32 == 0.  items: DEVICE array sorted by block0, the first 8x8-byte source
 * block of the item (block0[i+1] = block0[i] + N * K / 64); total_blocks = the sum. */
typedef struct {
    const void* src;
    void* dst;
    int32_t N, K;
    int32_t transpose, _pad;
    int64_t block0;
} csu_frag8_item;
int csu_frag8_layout_batch(const csu_frag8_item* items, int count, long total_blocks, void* stream);

/* ---------------------------------------------------------------------------------------
 * Batched weight cast: for each item, dst (rows, cols) bf16 = src fp32, and when dst_t is not
 * NULL also dst_t (cols, rows) bf16 = src^T.  items is a DEVICE array sorted by tile0, the first
 * 64x64-tile index of the item (tile0[i+1] = tile0[i] + ceil(rows/64) * ceil(cols/64));
 * total_tiles = the sum.  One launch per step refreshes every bf16 shadow weight.
 * ------------------------------------------------------------------------------------- */
typedef struct {
    const float* src;
    void* dst;
    void* dst_t;
    int32_t rows, cols;
    int64_t tile0;
    int32_t taps;   /* 0: matrix item.  > 0: conv weight src (rows=N, cols=C, taps=KH*KW) -> dst = OHWI
                       [N][KH][KW][C], dst_t = IHWO [C][KH][KW][N] (or NULL); ceil(N*C*taps/4096) tiles */
    int32_t cols_pad;   /* conv items: channel stride of dst (0 = C; > C: channel-padded OHWI whose
                           pad channels are left untouched, e.g. zeroed once by the caller) */
} csu_cast_item;
int csu_cast_bf16_batch(const csu_cast_item* items, int count, long total_tiles, void* stream);

/* fp8-e4m3 weights (BASELINE config 5): per item (rows x cols fp32 row-major, row = output feature),
 * per row the power-of-two scale s = 2^ceil(log2(amax/448)), q = e4m3fn(w / s) (RNE), and
 * dst = q * s in fp32 (exact in bf16: the cast cache then makes the kernels' bf16 shadows from it);
 * dst_q (optional) the e4m3 bytes, scales (optional) s per row.  items: DEVICE array sorted by
 * row0 (prefix sum of rows); one block per row of every item. */
typedef struct {
    const float* src;
    float* dst;
    uint8_t* dst_q;
    float* scales;
    int64_t row0;
    int32_t rows, cols;
} csu_fp8_item;
int csu_quant_e4m3_batch(const csu_fp8_item* items, int count, long total_rows, void* stream);
/* The same quantisation written straight into bf16 shadows: per item (rows x cols fp32, cols % 16 ==
 * 0), scales[row] = s (optional), q (optional) the e4m3 bytes, shadow (rows x cols bf16) = q * s exactly,
 * shadow_t (cols x rows bf16, optional) its transpose; q_perm / q_t / q_tp (optional; rows % 64 == 0 and
 * cols % 64 == 0) the fp8 fused Mlp's byte layouts of q.  items: DEVICE array sorted by blk0 (prefix sum of
 * ceil(rows / 64)); one 256-thread block per 64 rows of every item. */
typedef struct {
    const float* src;
    uint8_t* q;
    float* scales;
    void* shadow;
    void* shadow_t;
    uint8_t* q_perm;   /* optional: e4m3 bytes with columns permuted in 64-groups (dst 32h+16t+4g+i <- src 32t+8g+4h+i) */
    uint8_t* q_t;      /* optional: transposed e4m3 bytes (cols x rows) */
    uint8_t* q_tp;     /* optional: transposed, columns permuted as q_perm (the fp8 fused Mlp's W1^T layout) */
    int64_t blk0;
    int32_t rows, cols;
} csu_fp8_shadow_item;
int csu_quant_e4m3_shadow_batch(const csu_fp8_shadow_item* items, int count, long total_blocks, void* stream);

/* fp8-e4m3 token GEMM (BASELINE config 5 "fp8 MFMA weights"; replaces CSWinBlock.qkv, cswin:337,
 * on the norm1 output, cswin:357):  out[m][n] = bf16(sa[m] sw[n] sum_k aq[m][k] wq[n][k] + bias[n]),
 * aq (M x K) / wq (N x K) OCP e4m3fn bytes, sa / sw fp32 per-row scales, bias fp32 (or NULL),
 * out bf16 (M x N).  v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulation.  N % 64 == 0, K % 64 == 0. */
int csu_fp8_gemm(long M, int N, int K, const void* aq, const float* sa, const void* wq, const float* sw,
                 const float* bias, void* out, void* stream);
/* LayerNorm forward with an e4m3 output: yq = e4m3fn(LN(x) / s) (RNE), yscale[row] = s =
 * 2^ceil(log2(amax_row / 448)) (1 for an all-zero row); mean / rstd as csu_layernorm_fwd. */
int csu_layernorm_fwd_fp8(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                          const float* beta, void* yq, float* yscale, float* mean, float* rstd, void* stream);
/* the same, also writing ydq (bf16, rows x C, or NULL) = e4m3fn(yq) * yscale[row] exactly: the
 * operand the weight gradient of the consuming Linear reads */
int csu_layernorm_fwd_fp8_dq(int rows, int C, float eps, int xdtype, const void* x, const float* gamma,
                             const float* beta, void* yq, float* yscale, void* ydq, float* mean, float* rstd,
                             void* stream);
/* out (bf16, rows x cols) = e4m3fn(q) * scale[row]; cols % 8 == 0 */
int csu_dequant_e4m3_rows(long rows, int cols, const void* q, const float* scale, void* out, void* stream);
/* e4m3 byte layouts of quantised weights (the fp8 fused Mlp's operand images): per item, src is a
 * rows x cols byte matrix; mode bit 0 = transpose (dst is cols x rows), bit 1 = permute the dst
 * columns inside every 64-column block: dst column 32h + 16t + 4g + i (h, t in {0,1}, g, i in 0..3)
 * takes column 32t + 8g + 4h + i of the (transposed) source -- the k order in which a 32x32 MFMA
 * accumulator tile pair reaches an f8 operand lane.  Permuting modes need a dst column count
 * % 64 == 0; every mode needs dst columns % 4 == 0.  items: DEVICE array sorted by word0 (prefix sum
 * of the items' dst sizes in 4-byte words); one thread per dst word. */
typedef struct {
    const uint8_t* src;
    uint8_t* dst;
    int64_t word0;
    int32_t rows, cols;        /* of src */
    int32_t mode;
    int32_t pad;
} csu_e4m3_layout_item;
int csu_e4m3_layout_batch(const csu_e4m3_layout_item* items, int count, long total_words, void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused multi-tensor AdamW step (torch.optim.AdamW semantics, cswin:937-941): for every item,
 * param *= 1 - lr*wd; m = lerp(m, g, 1-beta1); v = beta2 v + (1-beta2) g^2;
 * param -= lr/(1-beta1^t) * m / (sqrt(v)/sqrt(1-beta2^t) + eps).  items: DEVICE array sorted
 * by chunk0 = first chunk index of the item (chunk0[i+1] = chunk0[i] + the item's chunk count,
 * see below); total_chunks = the sum.  lr_dev / step_dev: device scalars (HIP graph capture) or
 * NULL to use lr / step.  Replaces torch's fused AdamW launches.
 * Optional bf16 shadows of the UPDATED parameter, written in the same pass (the weight copies the
 * next forward's kernels read; they replace the csu_cast_bf16_batch refresh):
 *   shadow == NULL                : no shadow; ceil(numel / csu_adamw_chunk_elems()) chunks.
 *   taps == 0, shadow_t == NULL   : shadow = bf16 param (same layout); ceil(numel / chunk) chunks.
 *   taps == 0, shadow_t != NULL   : the param is a rows x cols matrix processed in 64 x 64 tiles
 *                                   (ceil(rows/64) * ceil(cols/64) chunks): shadow = bf16 W,
 *                                   shadow_t = bf16 W^T (cols x rows).
 *   taps > 0                      : conv weight [rows=N][cols=C][taps=KH*KW]: shadow = OHWI with
 *                                   channel stride cols_pad (>= C), shadow_t = IHWO (or NULL);
 *                                   ceil(numel / chunk) chunks.
 * ------------------------------------------------------------------------------------- */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    int64_t chunk0;
    void* shadow;
    void* shadow_t;
    int32_t rows, cols;
    int32_t taps, cols_pad;
} csu_adamw_item;
long csu_adamw_chunk_elems(void);
int csu_adamw_step(const csu_adamw_item* items, int count, long total_chunks, const float* lr_dev, float lr,
                   float beta1, float beta2, float eps, float weight_decay, const float* step_dev, float step,
                   void* stream);
/* The same step with torch.optim.Adam's coupled L2 decay (the plain UNet's optimizer,
 * unet:486-490): g += wd * param, no decoupled decay. */
int csu_adam_l2_step(const csu_adamw_item* items, int count, long total_chunks, const float* lr_dev, float lr,
                     float beta1, float beta2, float eps, float weight_decay, const float* step_dev, float step,
                     void* stream);

/* ---------------------------------------------------------------------------------------
 * Dropout / DropPath (nn.Dropout cswin:190/193/512, timm DropPath cswin:344/367-368) as one
 * elementwise pass where no producing kernel fuses it:
 *   out[i] = res[i] + row_scale[(i / cols) / rows_per_sample] * keep(site, i) / (1 - p) * x[i]
 * over (rows, cols) row-major, cols % 8 == 0; res (fp32) and row_scale (fp32 per sample: 0 or
 * 1/keep_prob of DropPath) may be NULL; p = 0: no mask.  keep(site, i): Philox4x32-7 counter-based
 * bits (csrc/rng.hpp) of the [seed, counter] snapshot `rng` (device uint64 x 2).  The backward of
 * a site is the same call with res = NULL on the incoming gradient.  csu_dropout_mask writes the
 * 0/1 keep mask of elements [0, n) of a site (tests feed it to the CPU oracle).
 * ------------------------------------------------------------------------------------- */
int csu_dropout_apply(long rows, int cols, int xdtype, const void* x, const float* res, int odtype, void* out,
                      const float* row_scale, long rows_per_sample, const uint64_t* rng, unsigned site, float p,
                      void* stream);
int csu_dropout_mask(long n, const uint64_t* rng, unsigned site, float p, uint8_t* out, void* stream);
/* snap[0..1] = state[0..1]; state[1] += 1 (one kernel: the per-forward RNG snapshot, graph-safe) */
int csu_rng_advance(uint64_t* state, uint64_t* snap, void* stream);
/* DropPath per-sample scale (timm drop_path, cswin:344/367-368): out[b] = keep(site, b) / (1 - p)
 * (element b of the site's mask, as csu_dropout_mask) -- the row_scale operand above. */
int csu_droppath_scale(long n, const uint64_t* rng, unsigned site, float p, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * fp32 GEMMs of the fp32 training path (token Linear forward / input / weight gradient, BASELINE
 * config 2), on the fp32 MFMA.  Row-major, C (M, N):
 *   layout 0: C = A (M,K) B(N,K)^T [+ bias (N)] [+ resid (M,N)]   (nn.Linear forward)
 *   layout 1: C = A (M,K) B(K,N)                                    (input gradient dy W)
 *   layout 2: C = A(K,M)^T B(K,N)                                   (weight gradient dy^T x; token
 *             splits reduced in a fixed order through `workspace`, csu_gemm_f32_workspace bytes)
 * Row lengths (K for A in layouts 0/1, M in layout 2, N, K of B in layout 0) multiples of 4.
 * asum (layout 2 only, or NULL): asum[m] = sum_k A[k][m] -- the bias gradient of dW = dy^T x.
 * ------------------------------------------------------------------------------------- */
size_t csu_gemm_f32_workspace(int layout, long M, int N, long K);
int csu_gemm_f32(int layout, long M, int N, long K, const float* A, const float* B, const float* bias,
                 const float* resid, float* C, float* asum, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Fused Mlp + residual (Mlp cswin:180-196 with the residual add of CSWinBlock cswin:368):
 * fc1 -> GELU -> fc2 with the 4C hidden layer kept on chip.  x (M, C) bf16; w1 (4C, C) and
 * w2 (C, 4C) bf16 nn.Linear weights; b1 (4C), b2 (C) fp32; res / out (M, C) fp32 (may alias).
 * Backward recomputes h = fc1(x) and writes dh = (dy w2) * gelu'(h) (M, 4C), g = gelu(h)
 * (M, 4C) for the weight gradients and dx = dh w1 (M, C), all bf16.  C in {64, 128, 256}.
 * ------------------------------------------------------------------------------------- */
int csu_mlp_supported(int C);
int csu_mlp_fwd(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                const float* res, float* out, void* stream);
int csu_mlp_bwd(long M, int C, const void* x, const void* dy, const void* w1, const float* b1, const void* w2,
                void* dh, void* g, void* dx, void* stream);
/* Dropout inside the fused Mlp (Mlp.drop cswin:190/193, DropPath cswin:368), train mode:
 *   g  = gelu(fc1(x)) * keep(site_hidden, m * 4C + f) / (1 - p)
 *   out = res + row_scale[m / rows_per_sample] * keep(site_out, m * C + c) / (1 - p) * fc2(g)
 * (keep(): rng.hpp's Philox mask of the snapshot rng = [seed, counter]; row_scale NULL = 1).
 * The backward regenerates the hidden mask: dy must already carry the output mask and DropPath
 * scale (csu_dropout_apply on the same site_out / row_scale), g is written dropped (dW2 operand)
 * and dh = (dy w2) * mask * gelu'(h). */
typedef struct {
    const uint64_t* rng;
    uint32_t site_hidden, site_out;
    float p;                   /* 0 <= p < 1 (p = 0: no element masks, row_scale still applies) */
    const float* row_scale;    /* per-sample DropPath scale (0 or 1/keep_prob), or NULL */
    int64_t rows_per_sample;
} csu_mlp_dropout;
int csu_mlp_fwd_dp(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                   const float* res, float* out, const csu_mlp_dropout* d, void* stream);
int csu_mlp_bwd_dp(long M, int C, const void* x, const void* dy, const void* w1, const float* b1, const void* w2,
                   void* dh, void* g, void* dx, const csu_mlp_dropout* d, void* stream);
/* csu_mlp_fwd_dp that also applies the NEXT CSWinBlock's norm1 LayerNorm (cswin:357) to its output
 * out (M, C) fp32 in the same launch: ln_out (M, C) bf16 = LN(out) * ln_gamma + ln_beta (eps
 * ln_eps), ln_mean / ln_rstd (M) fp32 as csu_layernorm_fwd writes them.  out must not alias res. */
int csu_mlp_fwd_ln(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                   const float* res, float* out, const csu_mlp_dropout* d, const float* ln_gamma, const float* ln_beta,
                   float ln_eps, void* ln_out, float* ln_mean, float* ln_rstd, void* stream);
/* the forward with an explicit kernel: cfg 0 = the per-panel kernel (csu_mlp_fwd_dp), 1 / 2 = the deep
 * weight ring (32-hidden chunks, several in flight, waves split by tokens; 2: another ring depth) */
int csu_mlp_fwd_ex(long M, int C, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                   const float* res, float* out, const csu_mlp_dropout* d, int cfg, void* stream);
/* the backward with an explicit kernel: cfg 0 = the per-panel kernels, 1 / 2 = the deep ring (csu_mlp_bwd_dp
 * runs cfg 1 at C = 128 and cfg 0 otherwise) */
int csu_mlp_bwd_ex(long M, int C, const void* x, const void* dy, const void* w1, const float* b1, const void* w2,
                   void* dh, void* g, void* dx, const csu_mlp_dropout* d, int cfg, void* stream);
/* fp8-e4m3 fused Mlp forward (BASELINE config 5, "fp8 MFMA weights"; same math and dropout as
 * csu_mlp_fwd_dp) on v_mfma_scale_f32_32x32x64_f8f6f4 with MX block scales:
 *   h   = x_q W1^T + b1, x_q = x quantised per (token, 32 consecutive channels): scale 2^e, e the
 *         smallest integer with amax <= 448 * 2^e, e4m3fn round-to-nearest-even;
 *   g   = gelu(h) (* hidden dropout), g_q = g quantised per (token, 32 consecutive features);
 *   out = res + (g_q W2^T + b2) (* output dropout, DropPath).
 * w1q: (4C, C) e4m3 rows with power-of-two row scales sw1 (4C); w2p: (C, 4C) e4m3 rows (scales sw2,
 * C) with the columns permuted as csu_e4m3_layout_batch mode 2.  C in {64, 128, 256}. */
int csu_mlp_fp8_supported(int C);
int csu_mlp_fp8_fwd(long M, int C, const void* x, const void* w1q, const float* sw1, const float* b1,
                    const void* w2p, const float* sw2, const float* b2, const float* res, float* out,
                    const csu_mlp_dropout* d, void* stream);
/* the same with the NEXT CSWinBlock's norm1 (cswin:357) on its output, as csu_mlp_fwd_ln (bf16 ln_out,
 * fp32 mean / rstd; out must not alias res) */
int csu_mlp_fp8_fwd_ln(long M, int C, const void* x, const void* w1q, const float* sw1, const float* b1,
                       const void* w2p, const float* sw2, const float* b2, const float* res, float* out,
                       const csu_mlp_dropout* d, const float* ln_gamma, const float* ln_beta, float ln_eps, void* ln_out,
                       float* ln_mean, float* ln_rstd, void* stream);
/* Its backward (straight-through for every quantisation): h recomputed exactly as the forward;
 *   dg = (dy * sw2)_q W2q: w2t = W2q^T (4C, C) e4m3 (layout mode 1), dy quantised per (token, 32
 *        consecutive channels) after the per-channel scale sw2 (W2's row scale lies along this sum);
 *   dh = dg * gelu'(h) (* hidden mask) -> dh (bf16, M x 4C); g = g_q of the forward (bf16, exact);
 *   dx = (dh * sw1)_q W1q: w1tp = W1q^T (C, 4C) with permuted columns (layout mode 3), dh * sw1
 *        quantised per (token, 32 consecutive features).  dx bf16 (M, C).  dy carries the output mask. */
int csu_mlp_fp8_bwd(long M, int C, const void* x, const void* dy, const void* w1q, const float* sw1,
                    const float* b1, const void* w2t, const float* sw2, const void* w1tp, void* dh, void* g,
                    void* dx, const csu_mlp_dropout* d, void* stream);

/* ---------------------------------------------------------------------------------------
 * Implicit-GEMM NHWC convolution (patch embed cswin:505, Merge_Block.conv cswin:376, CARAFE
 * encoder cswin:397/446, plain-UNet DoubleConv 3x3 unet:182/185 and ConvTranspose2d(k2,s2)
 * unet:211 = the dgrad operator).  x (B,H,W,C), y (B,OH,OW,N) channels-last; weights prepared by
 * the caller: w_ohwi = [N][KH][KW][C], w_ihwo = [C][KH][KW][N] (same dtype as activations).
 * ------------------------------------------------------------------------------------- */
typedef struct {
    int32_t B, H, W, C;        /* input (of the forward conv) */
    int32_t OH, OW, N;         /* output */
    int32_t KH, KW, stride, pad;
} csu_conv_geom;

/* y = conv(x) + bias (bias fp32 or NULL) */
int csu_conv2d_fwd(const csu_conv_geom* g, int dtype, const void* x, const void* w_ohwi, const float* bias,
                   void* y, void* stream);
/* dx = conv^T(dy) (+ bias, used when this operator is a ConvTranspose2d forward) */
int csu_conv2d_dgrad(const csu_conv_geom* g, int dtype, const void* dy, const void* w_ihwo, const float* bias,
                     void* dx, void* stream);
/* Either operator with an explicit kernel choice (op 0: csu_conv2d_fwd, 1: csu_conv2d_dgrad; src /
 * w as there).  cfg -1: the per-shape choice the plain entries make; 0: the register-staged v2
 * implicit GEMM; 1 + k: the persistent LDS-DMA kernel (bf16, gathered channels % 64 == 0) in tile
 * configuration k (0: 128x128 3-stage, 1: 256x128 2-stage 8 waves, 2: 256x128 3-stage 8 waves,
 * 3: 128x64 4-stage, 4: 256x64 3-stage 8 waves, 5: 128x64 3-stage, 6 / 7: 256x256 8 waves, 8:
 * 512x64 8 waves); 20: the halo kernel of 3x3 stride-1 pad-1 convs with 64 gathered and 64 output
 * channels (H % 2 == 0, W % 64 == 0); CSU_E_ARG when not eligible. */
int csu_conv2d_ex(int op, const csu_conv_geom* g, int dtype, const void* src, const void* w, const float* bias, void* out,
                  int cfg, void* stream);
/* The plain operators with a workspace (op 0: csu_conv2d_fwd, 1: csu_conv2d_dgrad): one-problem bf16
 * convolutions with fewer output tiles than two per CU (the CSWin CARAFE encoders at 16x16 / 32x32)
 * split their K range over workgroups, write fp32 partials into the workspace and sum them in fixed
 * order (+ bias) in a second kernel.  csu_conv2d_workspace: the bytes that split needs (0: no split
 * for this geometry; a NULL or smaller workspace runs unsplit). */
size_t csu_conv2d_workspace(int op, const csu_conv_geom* g, int dtype);
int csu_conv2d_fwd_ws(const csu_conv_geom* g, int dtype, const void* x, const void* w_ohwi, const float* bias, void* y,
                      void* workspace, size_t ws_bytes, void* stream);
int csu_conv2d_dgrad_ws(const csu_conv_geom* g, int dtype, const void* dy, const void* w_ihwo, const float* bias,
                        void* dx, void* workspace, size_t ws_bytes, void* stream);
size_t csu_conv2d_wgrad_workspace(const csu_conv_geom* g);
/* dw_db fp32 [N*KH*KW*C + N] = dW in [N][KH][KW][C] order, then db (sum of dy) */
int csu_conv2d_wgrad(const csu_conv_geom* g, int dtype, const void* x, const void* dy, float* dw_db,
                     void* workspace, size_t ws_bytes, void* stream);
/* the same gradient written in torch's Conv2d weight layout: dw_db fp32 [N*c_real*KH*KW + N] = dW
 * (N, c_real, KH, KW) then db; input channels >= c_real (zero padding of a few-channel input) are
 * dropped.  Same workspace. */
int csu_conv2d_wgrad_oihw(const csu_conv_geom* g, int dtype, const void* x, const void* dy, int c_real, float* dw_db,
                          void* workspace, size_t ws_bytes, void* stream);
/* Weight gradient with an explicit kernel choice: c_real 0 = csu_conv2d_wgrad's [N][KH][KW][C]
 * layout, > 0 = csu_conv2d_wgrad_oihw's.  cfg -1: the per-shape choice of the plain entries; 0: the
 * register-staged v2 kernel; 1 + k: the LDS-DMA kernel (bf16, C % 8 == 0, N % 8 == 0) in tile
 * configuration k (0: 128x128 3-stage, 1: 64x256 3-stage, 2: 128x128 2-stage, 3: 256x128 2-stage 8
 * waves, 4: 64x128 4-stage; 5 / 6: the halo kernel of 3x3 / stride 1 / pad 1 convs with OW % 64 == 0,
 * C % 64 == 0 and N % 64 (5) / N % 128 (6) == 0).  Its workspace: csu_conv2d_wgrad_workspace_ex(g, cfg) (0 when not
 * eligible). */
size_t csu_conv2d_wgrad_workspace_ex(const csu_conv_geom* g, int cfg);
/* Two-source input: the conv of UNet Up over cat([x2, x1], channels) (unet:213-216) without the
 * concatenated tensor.  x holds input channels [0, c_split) (c_split per pixel), x2 channels
 * [c_split, C) (C - c_split per pixel); the input gradient is written the same way (dx / dx2), and
 * the weight gradient reads both (torch OIHW layout + db, csu_conv2d_wgrad_oihw's workspace).
 * csu_conv2d_split_ok: 1 when a geometry / split is supported (bf16 only; 3x3 stride-1 pad-1 with
 * OW % 64 == 0, C, N and c_split multiples of 64); the three calls fail with CSU_E_UNSUPPORTED
 * otherwise (the caller then materialises the concatenation). */
int csu_conv2d_split_ok(const csu_conv_geom* g, int c_split);
int csu_conv2d_fwd_split(const csu_conv_geom* g, int dtype, const void* x, const void* x2, int c_split, const void* w_ohwi,
                         const float* bias, void* y, void* stream);
int csu_conv2d_dgrad_split(const csu_conv_geom* g, int dtype, const void* dy, const void* w_ihwo, void* dx, void* dx2,
                           int c_split, void* stream);
int csu_conv2d_wgrad_split_oihw(const csu_conv_geom* g, int dtype, const void* x, const void* x2, int c_split, const void* dy,
                                float* dw_db, void* workspace, size_t ws_bytes, void* stream);
int csu_conv2d_wgrad_ex(const csu_conv_geom* g, int dtype, const void* x, const void* dy, int c_real, float* dw_db,
                        void* workspace, size_t ws_bytes, int cfg, void* stream);

/* ---------------------------------------------------------------------------------------
 * Step glue (csrc/glue.hip), the elementwise passes between the kernels above:
 * grad_join: out (fp32, n) = a + b (b may be NULL), plus out_bf16 (bf16 copy, or NULL); a / b
 *   bf16 or fp32, n % 8 == 0; out NULL with out_bf16 set: a bf16 cast of a (+ b).  The gradient of an fp32 activation cast once to bf16 for two
 *   consumers (encoder skip cswin:530-545/568-592, CARAFE input cswin:408-432).
 * bce_loss: nn.BCELoss(reduction='mean') (cswin:935) on probabilities p and targets t (fp32, n):
 *   loss[0] = mean(-(t max(log p, -100) + (1-t) max(log(1-p), -100))), deterministic; backward
 *   dp = dloss[0] (p - t) / max((1-p) p, 1e-12) / n.
 * pack_nhwc_bf16: fp32 NCHW image (B, C, H, W) -> bf16 NHWC (B, H, W, Cp), channels >= C zero
 *   (the patch-embed conv input, cswin:505).
 * ------------------------------------------------------------------------------------- */
int csu_grad_join(long n, int adtype, const void* a, int bdtype, const void* b, float* out, void* out_bf16,
                  void* stream);
size_t csu_bce_loss_workspace(long n);
int csu_bce_loss_fwd(long n, const float* p, const float* t, float* loss, void* workspace, size_t ws_bytes,
                     void* stream);
/* the same loss plus the reference loop's per-step segmentation sums (cswin:789-795, pred = p > 0.5):
 * stats[0] = sum(pred * t), stats[1] = sum(pred), stats[2] = sum(t) (fp32, fixed order) */
int csu_bce_loss_fwd_stats(long n, const float* p, const float* t, float* loss, float* stats, void* workspace,
                           size_t ws_bytes, void* stream);
int csu_bce_loss_bwd(long n, const float* p, const float* t, const float* dloss, float* dp, void* stream);
int csu_pack_nhwc_bf16(int B, int C, int H, int W, int Cp, const float* x, void* y, void* stream);

/* ---------------------------------------------------------------------------------------
 * Mask-aligned batch augmentation (AugmentationTransform cswin:20-87 + the dataset's /255 and
 * HWC -> CHW, cswin:166-173), square S x S images: img uint8 (B, S, S, 3), mask uint8 (B, S, S),
 * params int32 (B, 7) on the device = {hflip, vflip, clockwise quarter turns 0..3, crop top,
 * crop left, crop height, crop width} (the crop taken from the flipped/rotated image and resized
 * back to S x S bilinearly, half-pixel centres, results rounded to uint8 like the reference's
 * uint8 resize); out_img fp32 (B, 3, S, S) = value / 255, out_mask fp32 (B, 1, S, S).
 * ------------------------------------------------------------------------------------- */
int csu_augment_batch(int B, int S, const void* img, const void* mask, const int* params, float* out_img,
                      float* out_mask, void* stream);

/* ---------------------------------------------------------------------------------------
 * Plain-UNet BatchNorm2d (+ ReLU) and MaxPool2d(2) on NHWC rows (DoubleConv / Down,
 * train_unet_segmentation.py unet:177-204; replaces F.batch_norm + F.relu + F.max_pool2d there).
 * x, y: M = B*H*W rows of C channels (C % 8 == 0), dtype bf16 or f32 (y and dx in x's dtype).
 * training: batch statistics (biased variance) -> save = (mean[C], rstd[C]); running_mean /
 * running_var (may both be NULL) updated with `momentum` and the unbiased variance; else the
 * running statistics normalise.  relu != 0 fuses the following ReLU (backward masks by y > 0,
 * recomputed).  Deterministic (fixed-order reductions); workspace csu_bn_workspace(M, C) bytes.
 * ------------------------------------------------------------------------------------- */
size_t csu_bn_workspace(long M, int C);
int csu_bn_relu_fwd(long M, int C, int dtype, const void* x, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, float momentum, float eps, int training, int relu,
                    float* save, void* y, void* workspace, size_t ws_bytes, void* stream);
/* dx, dgamma, dbeta (either may be NULL) from dy (gdtype) and the forward's save */
int csu_bn_relu_bwd(long M, int C, int dtype, const void* x, const float* gamma, const float* beta, const float* save,
                    int training, int relu, int gdtype, const void* dy, void* dx, float* dgamma, float* dbeta,
                    void* workspace, size_t ws_bytes, void* stream);
/* MaxPool2d(2) of NHWC x (B, H, W, C) -> y (B, H/2, W/2, C); the backward writes every dx element
 * of the pooled 2x2 windows (the first maximum in torch's scan order gets dy, NaN wins); rows /
 * columns past 2*(H/2), 2*(W/2) are not written. */
int csu_maxpool2_fwd(int B, int H, int W, int C, int dtype, const void* x, void* y, void* stream);
int csu_maxpool2_bwd(int B, int H, int W, int C, int dtype, const void* x, int gdtype, const void* dy, void* dx,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CSU_H_ */
