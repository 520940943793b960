"""fp8-e4m3 weights (BASELINE config 5: "fp8-e4m3 weights, bf16 activations, fp32 accumulate").

* The quantiser (csu_quant_e4m3_batch) equals torch's float8_e4m3fn round-to-nearest-even under the
  same per-row power-of-two scales, bit for bit.
* The model in the fp8 weight format equals the fp32 oracle run with the dequantised weights, at the
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


def test_fp8_weight_model_vs_oracle_with_quantized_weights():
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss
    d = dev()
    cfg = O.CSWinConfig(img_size=256, split_size=(1, 2, 8, 8))
    p = O.recipe_params(cfg, seed=0)
    m = CSWinTransformer(img_size=256, split_size=[1, 2, 8, 8]).to(d).set_weight_format("fp8_e4m3")
    m.load_state_dict(p)
    x, t = ellipse_batch(np.random.default_rng(5), 1, 256)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x.to(d))
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
    yr = O.cswin_forward(pref, x.double(), cfg)
    lr = O.bce_loss(yr, t.double())
    lr.backward()
    assert float((y.detach().double().cpu() - yr).abs().max()) < 1e-2
    assert abs(loss.item() - lr.item()) < 1e-2 * lr.item()
    gn = np.array([q.grad.double().norm().item() for _, q in m.named_parameters()])
    gr = np.array([pref[k].grad.norm().item() for k, _ in m.named_parameters()])
    big = gr >= 1e-3 * gr.max()
    np.testing.assert_allclose(gn[big], gr[big], rtol=5e-2)
    # and the format matters: the bf16-weight model differs from the fp8 one
    m2 = CSWinTransformer(img_size=256, split_size=[1, 2, 8, 8]).to(d)
    m2.load_state_dict(p)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y2 = m2(x.to(d))
    assert float((y2 - y.detach()).abs().max()) > 1e-4
