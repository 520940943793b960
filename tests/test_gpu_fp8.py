"""fp8-e4m3 weights (BASELINE config 5: "fp8-e4m3 weights, bf16 activations, fp32 accumulate").

* The quantiser (csu_quant_e4m3_batch) equals torch's float8_e4m3fn round-to-nearest-even under the
  same per-row power-of-two scales, bit for bit.
* The LayerNorm's e4m3 output mode (csu_layernorm_fwd_fp8: per-token power-of-two scale) equals
  torch's LayerNorm quantised by torch.float8_e4m3fn under the same rule.
* The e4m3 GEMM (csu_fp8_gemm, v_mfma_scale_f32_32x32x64_f8f6f4) equals an fp64 GEMM of the
  dequantised operands to bf16 output rounding plus the MFMA's summation error:
  |out - ref| <= 2^-8 |ref| + 2^-14 sum_k |a_k w_k| (the e4m3 products are exact; measured on
  gfx950 the f8f6f4 MFMA's internal sum is ~2^-17 of sum |a w| off an fp64 sum, above plain fp32
  accumulation's ~K 2^-24).
* The model in the fp8 weight format equals the fp64 oracle run with the dequantised weights and
  the per-token e4m3 rounding of the qkv input (oracle.cswin_ref.QKV_INPUT_QUANT), at the
  bf16-autocast tolerances (probabilities 1e-2, loss 1e-2 rel, grad norms 5e-2 rel), at
  256x256 with split [1,2,8,8] (stage-3 windows of 128 tokens; the 512/1024-token windows of the
  1024 config are covered kernel-wise by ATTN_CASES)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cswin_ref as O


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _ref_quant(w: torch.Tensor):
    """torch restatement: per row s = 2^ceil(log2(amax / 448)), q = e4m3fn(w / s) (RNE)."""
    w2 = w.reshape(w.shape[0], -1).double()
    amax = w2.abs().amax(1)
    s = torch.where(amax > 0, torch.exp2(torch.ceil(torch.log2(amax / 448.0))), torch.ones_like(amax))
    q = (w2 / s[:, None]).float().to(torch.float8_e4m3fn)
    return (q.float().double() * s[:, None]).float().reshape(w.shape), q.view(torch.uint8).reshape(w.shape), s.float()


def _pow2_scale(amax):
    return torch.where(amax > 0, torch.exp2(torch.ceil(torch.log2(amax / 448.0))), torch.ones_like(amax))


def _tok_quant(y: torch.Tensor) -> torch.Tensor:
    """Per-token e4m3 rounding of the qkv input, straight-through for autograd (the device's
    backward uses dY W and the quantised activation as the forward did)."""
    s = _pow2_scale(y.detach().abs().amax(-1, keepdim=True))
    q = (y.detach() / s).float().to(torch.float8_e4m3fn).to(y.dtype) * s
    return y + (q - y.detach())


def test_quantizer_matches_torch_e4m3fn():
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(0)
    ws = [torch.randn(192, 64, generator=g) * 0.02, torch.randn(64, 256, generator=g) * 3.0,
          torch.randn(7, 1, 3, 3, generator=g), torch.zeros(8, 16), torch.randn(1024, 256, generator=g) * 1e-3]
    ws[1][3, 5] = 447.9       # near the e4m3 range edge after scaling
    ps = [w.to(d) for w in ws]
    fp8 = ops.Fp8Weights(ps)
    deq = fp8.quantize()
    torch.cuda.synchronize()
    for w, dq, q, sc in zip(ws, deq, fp8.q, fp8.scales):
        rd, rq, rs = _ref_quant(w)
        assert torch.equal(sc.cpu(), rs)
        assert torch.equal(q.cpu(), rq)
        assert torch.equal(dq.cpu(), rd)
        assert torch.equal(dq.cpu().bfloat16().float(), rd)     # exact in bf16


def test_quantizer_into_cast_cache_shadows():
    """csu_quant_e4m3_shadow_batch (the model's per-step path): the same bytes and scales as the
    row quantiser, and the cast cache's bf16 shadows W and W^T equal the dequantised weights exactly
    (ragged row counts: partial 64-row blocks and transposed tails)."""
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(1)
    ws = [torch.randn(192, 64, generator=g) * 0.02, torch.randn(64, 256, generator=g) * 3.0,
          torch.randn(100, 32, generator=g), torch.randn(1024, 256, generator=g) * 1e-3, torch.randn(16, 64, generator=g),
          torch.randn(37, 48, generator=g)]
    ps = [w.to(d) for w in ws] + [torch.randn(64, device=d)]          # + a 1-D tensor: cast, not quantised
    fp8 = ops.Fp8Weights(ps)
    cache = ops.CastCache()
    cache.refresh(ps, torch.bfloat16, (), sources=fp8.sources())
    fp8.quantize(cache)
    torch.cuda.synchronize()
    for i, w in enumerate(ws):
        rd, rq, rs = _ref_quant(w)
        assert torch.equal(fp8.scales[i].cpu(), rs)
        assert torch.equal(fp8.q[i].cpu(), rq)
        assert torch.equal(cache.shadow[i].float().cpu(), rd)
        assert torch.equal(cache.shadow_t[i].float().cpu(), rd.t())
    assert torch.equal(cache.shadow[-1], ps[-1].bfloat16())


@pytest.mark.parametrize("fp8_qkv", [False, True])
def test_fp8_weight_model_vs_oracle_with_quantized_weights(monkeypatch, fp8_qkv):
    """fp8_qkv (ops.FP8_QKV): True -- every qkv on the fp8 MFMA (e4m3 norm1 output, the oracle's
    QKV_INPUT_QUANT); False (the default) -- qkv on the bf16 kernels with the exact dequantised weight
    (no activation quantisation).  Every Mlp at C = 64 / 128 / 256 on the fp8 kernels either way."""
    from csu import ops
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss
    d = dev()
    monkeypatch.setattr(ops, "FP8_QKV", fp8_qkv)
    cfg = O.CSWinConfig(img_size=256, split_size=(1, 2, 8, 8))
    p = O.recipe_params(cfg, seed=0)
    m = CSWinTransformer(img_size=256, split_size=[1, 2, 8, 8]).to(d).set_weight_format("fp8_e4m3")
    m.load_state_dict(p)
    x, t = ellipse_batch(np.random.default_rng(5), 1, 256)
    calls = []
    real = ops.fp8_gemm
    monkeypatch.setattr(ops, "fp8_gemm", lambda *a, **k: calls.append(1) or real(*a, **k))
    mcalls = []
    real_mlp = ops.mlp_fp8
    monkeypatch.setattr(ops, "mlp_fp8", lambda *a, **k: (lambda r: mcalls.append(r is not None) or r)(real_mlp(*a, **k)))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x.to(d))
    nblk = sum(1 for mod in m.modules() if type(mod).__name__ == "CSWinBlock")
    assert len(calls) == (nblk if fp8_qkv else 0)   # every qkv on fp8 MFMA, or none
    # every Mlp at C = 64 / 128 / 256 on the fp8 fused kernels
    assert sum(mcalls) == sum(1 for mod in m.modules() if type(mod).__name__ == "Mlp" and mod.fc1.in_features in (64, 128, 256))
    assert sum(mcalls) > 10
    loss = bce_loss(y, t.to(d))
    loss.backward()
    # the oracle on the dequantised e4m3 weights of exactly the tensors the fp8 format quantises
    quant = {n for n, q in zip([id(w) for w in m._linear_weights()], m._fp8.q) if q is not None}
    names = {id(v): k for k, v in m.named_parameters()}
    pq = dict(p)
    for w in m._linear_weights():
        k = names.get(id(w))
        if k is not None and id(w) in quant:
            pq[k] = _ref_quant(p[k])[0]
    assert sum(1 for w in m._linear_weights() if id(w) in quant) > 100
    pref = {k: v.double().requires_grad_(True) for k, v in pq.items()}
    if fp8_qkv:
        monkeypatch.setattr(O, "QKV_INPUT_QUANT", _tok_quant)
    # the Mlps at C = 64 / 128 / 256 run the fp8 fused kernels: their MX roundings (oracle/fp8_ref.py)
    from oracle import fp8_ref as Q

    def mlp_fp8(xx, pp, key, m_h):
        if xx.shape[-1] not in (64, 128, 256):
            return None
        s1 = Q.quant_rows(p[key + ".fc1.weight"])[2]
        s2 = Q.quant_rows(p[key + ".fc2.weight"])[2]
        return Q.fp8_mlp(xx, pp[key + ".fc1.weight"], pp[key + ".fc1.bias"], pp[key + ".fc2.weight"],
                         pp[key + ".fc2.bias"], s1, s2, m_h, bwd_fp8=xx.shape[-1] in ops.FP8_MLP_BWD_C)
    monkeypatch.setattr(O, "MLP_FP8", mlp_fp8)

    yr = O.cswin_forward(pref, x.double(), cfg)
    lr = O.bce_loss(yr, t.double())
    lr.backward()
    assert float((y.detach().double().cpu() - yr).abs().max()) < 1e-2
    assert abs(loss.item() - lr.item()) < 1e-2 * lr.item()
    gn = np.array([q.grad.double().norm().item() for _, q in m.named_parameters()])
    gr = np.array([pref[k].grad.norm().item() for k, _ in m.named_parameters()])
    big = gr >= 1e-3 * gr.max()
    names = [k for k, _ in m.named_parameters()]
    off = [(names[i], float(gn[i] / gr[i] - 1)) for i in range(len(names)) if big[i] and abs(gn[i] / gr[i] - 1) > 5e-2]
    assert not off, off
    # and the format matters: the bf16-weight model differs from the fp8 one
    m2 = CSWinTransformer(img_size=256, split_size=[1, 2, 8, 8]).to(d)
    m2.load_state_dict(p)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y2 = m2(x.to(d))
    assert float((y2 - y.detach()).abs().max()) > 1e-4


@pytest.mark.parametrize("C", [64, 128, 256, 512])
@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
def test_layernorm_fp8_output_matches_torch(C, xdt):
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(C)
    rows = 1031                                   # ragged: not a multiple of any rows-per-block
    x = (torch.randn(rows, C, generator=g) * 2 + 0.5).to(xdt)
    x[5] = 0                                      # all-zero row: LN output = beta
    w = torch.randn(C, generator=g) * 0.5 + 1
    b = torch.randn(C, generator=g) * 0.1
    q, s, mean, rstd = ops.layer_norm_fp8(x.to(d), w.to(d), b.to(d), 1e-5)
    torch.cuda.synchronize()
    y = torch.nn.functional.layer_norm(x.float(), (C,), w, b, 1e-5)
    rs = _pow2_scale(y.abs().amax(1))
    assert torch.equal(s.cpu(), rs)
    rq = (y / rs[:, None]).to(torch.float8_e4m3fn)
    mism = (q.cpu() != rq.view(torch.uint8))
    assert mism.float().mean().item() < 1e-3       # fp32 LN rounding can move a rare value across a tie
    deq = ops.dequant_e4m3_rows(q, s).float().cpu()
    ref = rq.float() * rs[:, None]
    assert (deq != ref).float().mean().item() < 1e-3
    assert torch.allclose(deq, ref, rtol=0.13, atol=float(rs.max()) * 2.0 ** -9)   # at most one e4m3 step apart
    torch.testing.assert_close(mean.cpu(), x.float().mean(1), rtol=1e-5, atol=1e-5)
    assert torch.allclose(deq[5], (b / rs[5]).to(torch.float8_e4m3fn).float() * rs[5])
    # the bf16 dequantised copy written by the same pass equals the dequantisation bitwise
    q2, s2, _, _, dq = ops.layer_norm_fp8(x.to(d), w.to(d), b.to(d), 1e-5, dq=True)
    torch.cuda.synchronize()
    assert torch.equal(q2, q) and torch.equal(s2, s)
    assert torch.equal(dq.cpu(), ops.dequant_e4m3_rows(q, s).cpu())


@pytest.mark.parametrize("M,N,K", [(1000, 192, 64), (129, 384, 128), (4096, 768, 256), (257, 1536, 512),
                                   (64, 64, 64)])
def test_fp8_gemm_matches_fp64_on_quantized_operands(M, N, K):
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g) * 3
    w = torch.randn(N, K, generator=g) * 0.05
    sa = _pow2_scale(a.abs().amax(1))
    sw = _pow2_scale(w.abs().amax(1))
    aq = (a / sa[:, None]).to(torch.float8_e4m3fn)
    wq = (w / sw[:, None]).to(torch.float8_e4m3fn)
    bias = torch.randn(N, generator=g)
    out = ops.fp8_gemm(aq.view(torch.uint8).to(d), sa.to(d), wq.view(torch.uint8).to(d), sw.to(d), bias.to(d))
    out0 = ops.fp8_gemm(aq.view(torch.uint8).to(d), sa.to(d), wq.view(torch.uint8).to(d), sw.to(d), None)
    torch.cuda.synchronize()
    ad = aq.double() * sa.double()[:, None]
    wd = wq.double() * sw.double()[:, None]
    ref = ad @ wd.t()
    asum = ad.abs() @ wd.abs().t()      # sum_k |a_k w_k|: the scale of the summation error
    for o, r in ((out, ref + bias.double()), (out0, ref)):
        err = (o.double().cpu() - r).abs()
        assert float((err - (2.0 ** -8) * r.abs() - (2.0 ** -14) * asum).max()) <= 0


def test_fp8_gemm_rejects_bad_shapes():
    from csu import ops
    from csu._lib import CsuError
    d = dev()
    aq = torch.zeros(16, 96, dtype=torch.uint8, device=d)
    wq = torch.zeros(64, 96, dtype=torch.uint8, device=d)
    with pytest.raises(CsuError):
        ops.fp8_gemm(aq, torch.ones(16, device=d), wq, torch.ones(64, device=d))


def _perm64(q: torch.Tensor) -> torch.Tensor:
    """columns permuted per 64-block: dst 32h + 16t + 4g + i <- src 32t + 8g + 4h + i"""
    idx = torch.empty(64, dtype=torch.long)
    for h in range(2):
        for t in range(2):
            for g in range(4):
                for i in range(4):
                    idx[32 * h + 16 * t + 4 * g + i] = 32 * t + 8 * g + 4 * h + i
    n = q.shape[1]
    full = (torch.arange(n // 64)[:, None] * 64 + idx[None, :]).reshape(-1)
    return q[:, full]


@pytest.mark.parametrize("C", [64, 128, 256])
def test_e4m3_mlp_layouts(C):
    """csu_e4m3_layout_batch and csu_quant_e4m3_shadow_batch: W2 with permuted columns, W2^T, W1^T with
    permuted columns, bytewise."""
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(C)
    w1 = (torch.randn(4 * C, C, generator=g) * 0.05).to(d)
    w2 = (torch.randn(C, 4 * C, generator=g) * 0.05).to(d)
    fp8 = ops.Fp8Weights([w1, w2], mlp_pairs=[(w1, w2)])
    fp8.quantize()
    w1q, sw1, w2p, sw2, w2t, w1tp = fp8.mlp_operands(w1, w2)
    torch.cuda.synchronize()
    q1, q2 = w1q.cpu(), fp8.q[1].cpu()
    assert torch.equal(w2p.cpu(), _perm64(q2))
    assert torch.equal(w2t.cpu(), q2.t().contiguous())
    assert torch.equal(w1tp.cpu(), _perm64(q1.t().contiguous()))
    # the model's per-step path: the shadow quantiser writes the same layouts in its own pass
    for t in (w2p, w2t, w1tp):
        t.zero_()
    cache = ops.CastCache()
    cache.refresh([w1, w2], torch.bfloat16, (), sources=fp8.sources())
    fp8.quantize(cache)
    torch.cuda.synchronize()
    assert torch.equal(fp8.q[0].cpu(), q1) and torch.equal(fp8.q[1].cpu(), q2)
    assert torch.equal(w2p.cpu(), _perm64(q2))
    assert torch.equal(w2t.cpu(), q2.t().contiguous())
    assert torch.equal(w1tp.cpu(), _perm64(q1.t().contiguous()))


def _mx_torch_check():
    """the oracle's MX rule on known values: block amax 448 -> e = 0, 449 -> 1, 1.75 * 2^-3 -> e = -11"""
    from oracle import fp8_ref as Q
    e = Q.block_exponent(torch.tensor([448.0, 449.0, 1.75 * 2 ** -3, 0.0, 1.0]))
    assert e.tolist() == [0, 1, -11, 0, -8]


@pytest.mark.parametrize("C,M,drop", [(128, 1000, False), (256, 4160, False), (256, 100, True), (128, 777, True),
                                      (64, 5000, False), (64, 333, True)])
def test_mlp_fp8_fused_vs_oracle(C, M, drop):
    """csu_mlp_fp8_fwd / csu_mlp_fp8_bwd vs the fp64 restatement of the same roundings
    (oracle/fp8_ref.py: x / g / dY / dh MX-quantised in blocks of 32 consecutive channels, e4m3
    weights with per-row scales).  Only the
    device's fast GELU (|err| < 1.3e-5) and fp32 accumulation differ from the oracle, which can flip
    a rare e4m3 rounding of g or dh by one step: the gates are relative L2 errors, and the device is
    required to sit far closer to the fp8 oracle than to the unrounded Mlp."""
    import ctypes
    from csu import ops, rng
    from csu._lib import check, lib, ptr, stream_ptr
    from oracle import fp8_ref as Q
    _mx_torch_check()
    d = dev()
    torch.manual_seed(C + M)
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = torch.randn(4 * C, C, device=d) * C ** -0.5
    w2 = torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5
    b1, b2 = torch.randn(4 * C, device=d) * 0.1, torch.randn(C, device=d) * 0.1
    res = torch.randn(M, C, device=d)
    dz = (torch.randn(M, C, device=d) * 1e-3).bfloat16()      # gradient of the (dropped) fc2 output
    fp8 = ops.Fp8Weights([w1, w2], mlp_pairs=[(w1, w2)])
    fp8.quantize()
    w1q, sw1, w2p, sw2, w2t, w1tp = fp8.mlp_operands(w1, w2)
    snap = _snap_t(d, 5, 2)
    if drop:
        rps = max(1, M // 3)
        rs = rng.droppath_scale(snap, 30, 0.3, -(-M // rps))
        md = ops.MlpDrop(snap, 21, 22, 0.3, rs, rps).c_struct()
    else:
        md = ops.MlpDrop(None, 0, 0, 0.0).c_struct()
        md.rows_per_sample = M
    st = stream_ptr(d)
    y = torch.empty(M, C, device=d)
    check(lib().csu_mlp_fp8_fwd(M, C, ptr(x), ptr(w1q), ptr(sw1), ptr(b1), ptr(w2p), ptr(sw2), ptr(b2), ptr(res), ptr(y),
                                ctypes.byref(md), st), "mlp_fp8_fwd")
    dh = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    gq = torch.empty_like(dh)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    check(lib().csu_mlp_fp8_bwd(M, C, ptr(x), ptr(dz), ptr(w1q), ptr(sw1), ptr(b1), ptr(w2t), ptr(sw2), ptr(w1tp),
                                ptr(dh), ptr(gq), ptr(dx), ctypes.byref(md), st), "mlp_fp8_bwd")
    torch.cuda.synchronize()
    W1d, _, S1 = Q.quant_rows(w1.cpu())
    W2d, _, S2 = Q.quant_rows(w2.cpu())
    assert torch.equal(S1.float(), sw1.cpu()) and torch.equal(S2.float(), sw2.cpu())
    X, B1, B2, R, DZ = (t.double().cpu() for t in (x, b1, b2, res, dz))
    if drop:
        mh = rng.dropout_mask(snap, 21, 0.3, M * 4 * C).view(M, 4 * C).double().cpu() / 0.7
        mo = rng.dropout_mask(snap, 22, 0.3, M * C).view(M, C).double().cpu() / 0.7
        rsr = rs.double().cpu()[torch.arange(M) // rps].view(M, 1)
        outm = mo * rsr
    else:
        mh, outm = None, torch.ones(M, 1, dtype=torch.float64)
    z = Q.fp8_mlp(X, W1d, B1, W2d, B2, S1, S2, mh)
    yref = R + outm * z

    def rel(a, b):
        return float((a.double().cpu() - b).norm() / b.norm())

    assert rel(y - res, yref - R) < 1e-2, rel(y - res, yref - R)
    # the roundings are modelled: the unrounded Mlp (same dequantised weights) is much further away
    h_plain = X @ W1d.T + B1
    g_plain = torch.nn.functional.gelu(h_plain) * (mh if mh is not None else 1)
    z_plain = g_plain @ W2d.T + B2
    assert rel(y - res, outm * z_plain) > 5 * rel(y - res, yref - R)
    # backward pieces
    h = Q.mx_quant(X) @ W1d.T + B1
    g = torch.nn.functional.gelu(h) * (mh if mh is not None else 1)
    gqr = Q.mx_quant(g)
    assert rel(gq, gqr) < 1e-2
    assert float((gq.double().cpu() != gqr).double().mean()) < 2e-3      # rare one-step rounding flips only
    q1, q2 = W1d / S1[:, None], W2d / S2[:, None]
    dg = Q.mx_quant(DZ * S2) @ q2
    dgelu = 0.5 * (1 + torch.erf(h / 2 ** 0.5)) + h * torch.exp(-0.5 * h * h) / (2 * torch.pi) ** 0.5
    dhr = dg * dgelu * (mh if mh is not None else 1)
    assert rel(dh, dhr) < 5e-3, rel(dh, dhr)
    dxr = Q.mx_quant(dhr * S1) @ q1
    assert rel(dx, dxr) < 1e-2, rel(dx, dxr)
    # the autograd form of the oracle gives the same input gradient
    Xg = X.clone().requires_grad_(True)
    Q.fp8_mlp(Xg, W1d, B1, W2d, B2, S1, S2, mh).backward(DZ)
    assert rel(dx, Xg.grad) < 1e-2


def _snap_t(d, seed, ctr):
    return torch.tensor([seed, ctr], dtype=torch.int64, device=d)


def test_fp8_mlp_ratio_not_4_falls_back_to_bf16_mlp(monkeypatch):
    """The fp8 fused Mlp kernels hard-code 4C hidden features: a model built with mlp_ratio 2 in the
    fp8 weight format registers no fp8 Mlp pair and runs its Mlps on the bf16 path."""
    from csu import ops
    from csu.model import CSWinTransformer
    d = dev()
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4], mlp_ratio=2.0).to(d).set_weight_format("fp8_e4m3")
    got = []
    real = ops.mlp_fp8
    monkeypatch.setattr(ops, "mlp_fp8", lambda *a, **k: (lambda r: got.append(r is not None) or r)(real(*a, **k)))
    x = torch.randn(2, 3, 128, 128, device=d)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.sum().backward()
    assert got and not any(got)
    assert not m._fp8.mlp
    assert torch.isfinite(y).all()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)
