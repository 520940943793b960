"""Train-mode dropout on the fused path (reference main() rates: drop_rate = attn_drop_rate =
drop_path_rate = 0.3, cswin:930-932) vs the oracle under IDENTICAL masks.

The device draws every mask from the counter-based Philox stream (csrc/rng.hpp; csu.rng): site s
of snapshot (seed, step) keeps element e iff u16(philox(e / 8, s, step; seed))[e % 8] < keep.
csu_dropout_mask materialises exactly those bits, so the oracle (oracle/cswin_ref.py drop
provider, whose placement is pinned against the reference by tests/golden/f9_dropout.npz) replays
the same masks.  Tolerances: fp32 -- as the dropout-free parity tests (1e-4 abs on activations,
2e-3 rel on gradient norms); bf16 -- 1e-2 (y), 5e-2 rel (grad norms of tensors >= 1e-3 max)."""
import copy
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cswin_ref as O


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _snap(d, seed, ctr):
    return torch.tensor([seed, ctr], dtype=torch.int64, device=d)


def test_mask_statistics_and_determinism():
    from csu import rng
    d = dev()
    n = 1 << 22
    for p in (0.1, 0.3, 0.5):
        m = rng.dropout_mask(_snap(d, 1234, 5), 3, p, n).double()
        keep = float(m.mean())
        assert abs(keep - (1 - p)) < 5 * math.sqrt(p * (1 - p) / n), (p, keep)
        # neighbours independent (the 8 lanes of one Philox call, and across calls)
        a = m - m.mean()
        for lag in (1, 7, 8, 64):
            c = float((a[:-lag] * a[lag:]).mean() / a.var())
            assert abs(c) < 5 / math.sqrt(n), (p, lag, c)
    a = rng.dropout_mask(_snap(d, 1234, 5), 3, 0.3, 4096)
    assert torch.equal(a, rng.dropout_mask(_snap(d, 1234, 5), 3, 0.3, 4096))        # deterministic
    for other in (rng.dropout_mask(_snap(d, 1234, 6), 3, 0.3, 4096),               # next step
                  rng.dropout_mask(_snap(d, 1234, 5), 4, 0.3, 4096),               # other site
                  rng.dropout_mask(_snap(d, 99, 5), 3, 0.3, 4096)):                # other seed
        assert 0.3 < float((a != other).double().mean()) < 0.55
    # a prefix of a longer mask is the shorter mask (element index, not launch shape, decides)
    assert torch.equal(rng.dropout_mask(_snap(d, 7, 0), 1, 0.3, 1000), rng.dropout_mask(_snap(d, 7, 0), 1, 0.3, 5000)[:1000])
    # the device counter advances once per snapshot
    rng.manual_seed(42, d)
    s0, s1 = rng.advance(d).cpu().tolist(), rng.advance(d).cpu().tolist()
    assert s0 == [42, 0] and s1 == [42, 1]


@pytest.mark.parametrize("xdt,odt", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                     (torch.bfloat16, torch.float32)])
def test_dropout_apply_and_droppath(xdt, odt):
    from csu import ops, rng
    d = dev()
    snap = _snap(d, 11, 3)
    B, L, C = 3, 100, 72
    x = torch.randn(B, L, C, device=d).to(xdt)
    res = torch.randn(B, L, C, device=d)
    m = rng.dropout_mask(snap, 9, 0.3, x.numel()).view(B, L, C).float() / 0.7
    y = ops.dropout(x, 0.3, 9, snap, out_dtype=odt)
    assert y.dtype == odt
    torch.testing.assert_close(y.float(), (x.float() * m).to(odt).float(), rtol=0, atol=0)
    rs = rng.droppath_scale(snap, 17, 0.5, B)
    bits = rng.dropout_mask(snap, 17, 0.5, B).float() * 2
    assert torch.equal(rs, bits)
    y2 = ops.dropout(x, 0.3, 9, snap, row_scale=rs, rows_per_sample=L, residual=res)
    ref = res + rs.view(B, 1, 1) * m * x.float()
    torch.testing.assert_close(y2, ref, rtol=1e-6, atol=1e-6)
    # backward regenerates the mask
    xr = x.clone().requires_grad_(True)
    g = torch.randn(B, L, C, device=d)
    ops.dropout(xr, 0.3, 9, snap, row_scale=rs, rows_per_sample=L).float().backward(g)
    gx = g.to(xdt).float()        # autograd hands the bf16 leaf's kernel a bf16 gradient
    torch.testing.assert_close(xr.grad.float(), (gx * rs.view(B, 1, 1) * m).to(xdt).float(), rtol=0, atol=0)


@pytest.mark.parametrize("C,M", [(64, 4096), (64, 37), (128, 1000), (256, 4160), (256, 100)])
def test_mlp_fused_dropout_vs_fp64(C, M):
    """csu_mlp_fwd_dp / csu_mlp_bwd_dp (hidden + output dropout and DropPath inside the fused
    Mlp) vs the fp64 composition under the same masks."""
    import ctypes
    from csu import _lib, rng
    from csu._lib import check, lib, ptr, stream_ptr
    from csu.ops import MlpDrop
    d = dev()
    torch.manual_seed(C + M)
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.randn(4 * C, device=d) * 0.1, torch.randn(C, device=d) * 0.1
    res = torch.randn(M, C, device=d)
    dz = torch.randn(M, C, device=d).bfloat16()      # gradient of the (dropped) fc2 output
    snap = _snap(d, 5, 2)
    rps = max(1, M // 3)
    nb = -(-M // rps)
    rs = rng.droppath_scale(snap, 30, 0.3, nb)
    md = MlpDrop(snap, 21, 22, 0.3, rs, rps)
    st = stream_ptr(d)
    y = torch.empty(M, C, device=d)
    check(lib().csu_mlp_fwd_dp(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y),
                               ctypes.byref(md.c_struct()), st), "mlp_fwd_dp")
    dh = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    g = torch.empty_like(dh)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    check(lib().csu_mlp_bwd_dp(M, C, ptr(x), ptr(dz), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx),
                               ctypes.byref(md.c_struct()), st), "mlp_bwd_dp")
    mh = rng.dropout_mask(snap, 21, 0.3, M * 4 * C).view(M, 4 * C).double().cpu() / 0.7
    mo = rng.dropout_mask(snap, 22, 0.3, M * C).view(M, C).double().cpu() / 0.7
    rsr = rs.double().cpu()[torch.arange(M) // rps].view(M, 1)
    torch.cuda.synchronize()
    X, W1, W2, B1, B2 = (t.double().cpu() for t in (x, w1, w2, b1, b2))
    F = torch.nn.functional
    h = X @ W1.T + B1
    gd = F.gelu(h) * mh
    yref = res.double().cpu() + rsr * mo * (gd @ W2.T + B2)
    tol = dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y.double().cpu(), yref, **tol)
    torch.testing.assert_close(g.double().cpu(), gd, **tol)
    hg = h.clone().requires_grad_(True)
    (F.gelu(hg) * mh).backward(dz.double().cpu() @ W2)
    torch.testing.assert_close(dh.double().cpu(), hg.grad, **tol)
    torch.testing.assert_close(dx.double().cpu(), hg.grad @ W1, rtol=2e-2, atol=5e-2)
    # the fused Mlp with p = 0 and no DropPath is the dropout-free kernel (bitwise)
    y0 = torch.empty_like(y)
    y1 = torch.empty_like(y)
    check(lib().csu_mlp_fwd(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y0), st), "f")
    check(lib().csu_mlp_fwd_dp(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y1),
                               ctypes.byref(MlpDrop(None, 0, 0, 0.0).c_struct()), st), "f0")
    assert torch.equal(y0, y1)


def _attn_provider(snap, site, p, nwin_heads_n):
    from csu import rng

    def mask(shape):
        Bw, H, N, N2 = shape
        npad = -(-N // 32) * 32
        m = rng.dropout_mask(snap, site, p, Bw * H * N * npad).view(Bw, H, N, npad)[..., :N]
        return m.double().cpu() / (1 - p)
    return mask


# (reso, C, heads, split, last): branch windows N = reso*split (two-branch) or reso^2 (last stage)
ATTN_CASES = [(16, 64, 2, 2, False), (8, 64, 2, 8, True), (14, 128, 4, 7, False), (7, 128, 4, 7, True),
              (32, 64, 2, 1, False), (16, 64, 2, 16, True), (64, 64, 2, 4, False),
              (64, 64, 2, 8, False), (24, 64, 2, 24, True), (32, 128, 4, 32, True)]


@pytest.mark.parametrize("case", ATTN_CASES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_stripe_attention_dropout_vs_oracle(case, dt):
    """Attention dropout on P inside the stripe kernels (fwd, dq, dkdv; all window sizes incl.
    ragged N and the wide-window kernels) vs the oracle's lepe_attention under the same masks."""
    from csu import ops
    d = dev()
    reso, C, heads, split, last = case
    torch.manual_seed(reso * 7 + C)
    B = 2
    L = reso * reso
    if last:
        branches = [(reso, reso, 0)]
        nh, cb = heads, C
    else:
        branches = [(reso, split, 0), (split, reso, C // 2)]
        nh, cb = heads // 2, C // 2
    scale = (cb // nh) ** -0.5
    geom = ops.StripeGeometry(reso, C, nh, branches, scale, head_dim=cb // nh)
    qkv = torch.randn(B, L, 3 * C, device=d)
    ws = [torch.randn(cb, 1, 3, 3, device=d) * 0.2 for _ in branches]
    bs = [torch.randn(cb, device=d) * 0.1 for _ in branches]
    snap = _snap(d, 77, 1)
    p = 0.3
    q = qkv.to(dt).requires_grad_(True)
    wr = [w.clone().requires_grad_(True) for w in ws]
    br = [b.clone().requires_grad_(True) for b in bs]
    out = ops.stripe_attention(q, geom, wr, br, ops.AttnDrop(snap, 40, p))
    g = torch.randn(B, L, C, device=d)
    out.float().backward(g)
    # oracle, fp64, same masks (branch i uses site 40 + i)
    Q = q.detach().double().cpu().requires_grad_(True)
    W = [w.detach().double().cpu().requires_grad_(True) for w in ws]
    Bb = [b.detach().double().cpu().requires_grad_(True) for b in bs]
    outs = []
    for i, (hs, wsp, off) in enumerate(branches):
        sl = slice(off, off + cb)
        outs.append(O.lepe_attention(Q[..., sl], Q[..., C + off:C + off + cb], Q[..., 2 * C + off:2 * C + off + cb],
                                     reso, hs, wsp, nh, W[i], Bb[i], scale,
                                     attn_mask=_attn_provider(snap, 40 + i, p, None)))
    ref = torch.cat(outs, -1)
    ref.backward(g.double().cpu())
    if dt == torch.float32:
        tol = dict(rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(out.double().cpu(), ref.detach(), **tol)
        torch.testing.assert_close(q.grad.double().cpu(), Q.grad, rtol=1e-3, atol=1e-3)
        for a, b in zip(wr + br, W + Bb):
            torch.testing.assert_close(a.grad.double().cpu(), b.grad, rtol=1e-3, atol=1e-3 * max(1, float(b.grad.abs().max())))
    else:
        def rel(a, b):
            return float((a.double().cpu() - b).norm() / b.norm())
        assert rel(out.detach(), ref.detach()) < 1e-2
        assert rel(q.grad, Q.grad) < 2e-2
        for a, b in zip(wr + br, W + Bb):
            assert rel(a.grad, b.grad) < 2e-2
    # and the mask is really applied: without dropout the output differs
    with torch.no_grad():
        o0 = ops.stripe_attention(q.detach(), geom, ws, bs)
    assert float((o0.float() - out.detach().float()).abs().max()) > 1e-2


def _model_provider(m, snap, device):
    """Oracle drop provider replaying the device masks of csu model `m` under `snap`."""
    from csu import rng
    from csu.model import CSWinBlock, DropPath
    blocks = {n: b for n, b in m.named_modules() if isinstance(b, CSWinBlock)}
    p_pos = m.pos_drop.p if hasattr(m, "pos_drop") else 0.0

    def bits(site, p, n):
        return rng.dropout_mask(snap, site, p, n).double().cpu() / (1 - p)

    def drop(name, shape):
        if name == "pos":
            return bits(rng.SITE_POS_DROP, p_pos, int(np.prod(shape))).view(shape) if p_pos > 0 else None
        bname, kind = name.rsplit(".", 1) if not name.endswith((".mlp.h", ".mlp.o")) else (name[:-6], name[-5:])
        blk = blocks[bname]
        base = blk._site_base
        if kind.startswith("attn"):
            p = blk.attns[0].attn_drop.p
            if p == 0:
                return None
            Bw, H, N, _ = shape
            npad = -(-N // 32) * 32
            i = int(kind[4:])
            return bits(base + rng.OFF_ATTN + i, p, Bw * H * N * npad).view(Bw, H, N, npad)[..., :N]
        if kind in ("mlp.h", "mlp.o"):
            p = blk.mlp.drop.p
            if p == 0:
                return None
            site = base + (rng.OFF_MLP_HIDDEN if kind == "mlp.h" else rng.OFF_MLP_OUT)
            return bits(site, p, int(np.prod(shape))).view(shape)
        if kind in ("dp_attn", "dp_mlp"):
            if not isinstance(blk.drop_path, DropPath):
                return None
            p = blk.drop_path.drop_prob
            site = base + (rng.OFF_DROPPATH_ATTN if kind == "dp_attn" else rng.OFF_DROPPATH_MLP)
            return rng.droppath_scale(snap, site, p, shape[0]).double().cpu()
        raise KeyError(name)
    return drop


@pytest.mark.parametrize("amp", [None, torch.bfloat16], ids=["fp32", "bf16"])
def test_block_dropout_vs_oracle(amp):
    """Standalone CSWinBlock (train mode, 0.3 / 0.3 / 0.3) vs the oracle block with its masks."""
    from csu import rng
    from csu.model import CSWinBlock
    d = dev()
    for dim, reso, heads, sw, last in ((64, 16, 2, 2, False), (128, 8, 4, 8, True), (512, 7, 16, 7, True)):
        torch.manual_seed(dim + reso)
        m = CSWinBlock(dim=dim, reso=reso, num_heads=heads, split_size=sw, qkv_bias=True, last_stage=last,
                       drop=0.3, attn_drop=0.3, drop_path=0.3).to(d).train()
        x = torch.randn(2, reso * reso, dim, device=d).requires_grad_(True)
        rng.manual_seed(5, d)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp is not None):
            y = m(x)
        snap = _snap(d, 5, 0)
        g = torch.randn_like(y)
        y.backward(g)
        p = {"blk." + k: v.detach().double().cpu().requires_grad_(True) for k, v in m.state_dict().items()}
        X = x.detach().double().cpu().requires_grad_(True)
        prov = _model_provider(_wrap(m), snap, d)
        yr = O.cswin_block(X, p, "blk", reso, heads, sw, last, drop=prov)
        yr.backward(g.double().cpu())
        if amp is None:
            torch.testing.assert_close(y.detach().double().cpu(), yr.detach(), rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(x.grad.double().cpu(), X.grad, rtol=1e-3, atol=1e-3)
        else:
            assert float((y.detach().double().cpu() - yr).norm() / yr.norm()) < 1e-2
            assert float((x.grad.double().cpu() - X.grad).norm() / X.grad.norm()) < 3e-2
        gn = np.array([q.grad.double().norm().item() for _, q in m.named_parameters()])
        gr = np.array([p["blk." + k].grad.norm().item() for k, _ in m.named_parameters()])
        big = gr >= 1e-3 * gr.max()
        np.testing.assert_allclose(gn[big], gr[big], rtol=2e-3 if amp is None else 5e-2)


def _wrap(block):
    """A module tree naming `block` "blk" (the provider keys blocks by module name)."""
    w = torch.nn.Module()
    w.blk = block
    w.pos_drop = torch.nn.Dropout(0.0)
    return w


@pytest.mark.parametrize("amp", [None, torch.bfloat16], ids=["fp32", "bf16"])
def test_model_dropout_vs_oracle(amp):
    """Whole CSWinTransformer at the reference main() rates (drop / attn / drop_path 0.3), one
    training forward + backward at 128x128 (split [1,2,4,4]) vs the fp64 oracle replaying the
    device's masks: probabilities, BCE loss and every gradient norm."""
    from csu import rng
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss
    d = dev()
    cfg = O.CSWinConfig(img_size=128, split_size=(1, 2, 4, 4))
    p = O.recipe_params(cfg, seed=0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4], drop_rate=0.3, attn_drop_rate=0.3,
                         drop_path_rate=0.3).to(d)
    m.load_state_dict(p)
    m.train()
    x, t = ellipse_batch(np.random.default_rng(5), 2, 128)
    rng.manual_seed(2024, d)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp is not None):
        y = m(x.to(d))
    loss = bce_loss(y, t.to(d))
    loss.backward()
    snap = _snap(d, 2024, 0)
    pref = {k: v.double().requires_grad_(True) for k, v in p.items()}
    yr = O.cswin_forward(pref, x.double(), cfg, drop=_model_provider(m, snap, d))
    lr = O.bce_loss(yr, t.double())
    lr.backward()
    gn = np.array([q.grad.double().norm().item() for _, q in m.named_parameters()])
    gr = np.array([pref[k].grad.norm().item() for k, _ in m.named_parameters()])
    big = gr >= 1e-3 * gr.max()
    if amp is None:
        torch.testing.assert_close(y.detach().double().cpu(), yr.detach(), rtol=1e-4, atol=1e-4)
        assert abs(loss.item() - lr.item()) < 1e-5 * lr.item() + 1e-6
        np.testing.assert_allclose(gn[big], gr[big], rtol=2e-3)
    else:
        assert float((y.detach().double().cpu() - yr).abs().max()) < 2e-2
        assert abs(loss.item() - lr.item()) < 1e-2 * lr.item()
        np.testing.assert_allclose(gn[big], gr[big], rtol=5e-2)
    # dropout changes the forward (vs eval mode on the same weights)
    m.eval()
    with torch.no_grad():
        ye = m(x.to(d))
    assert float((ye - y.detach()).abs().max()) > 1e-3


def test_graph_replays_draw_fresh_masks_and_reproduce():
    """A captured train step with dropout draws new masks on every replay (the device counter
    advances inside the graph) and two captures from the same seed replay bitwise equal."""
    from csu import rng
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    d = dev()
    torch.manual_seed(0)
    m0 = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4], drop_rate=0.3, attn_drop_rate=0.3,
                          drop_path_rate=0.3)
    xb, tb = (t.to(d) for t in ellipse_batch(np.random.default_rng(1), 4, 128))
    res = []
    for _ in range(2):
        m = copy.deepcopy(m0).to(d)
        rng.manual_seed(9, d)
        opt = make_optimizer(m, lr=0.0, weight_decay=0.0, capturable=True)   # lr 0: same weights every replay
        gs = GraphedTrainStep(m, opt, bce_loss, xb, tb, torch.bfloat16, warmup=2)
        losses = [float(gs(xb, tb)[0].item()) for _ in range(4)]
        torch.cuda.synchronize()
        res.append((losses, int(rng.state(d)[1].item())))
        del gs, opt
    assert res[0] == res[1]
    losses = res[0][0]
    assert len(set(losses)) == len(losses), losses          # fresh masks each replay
