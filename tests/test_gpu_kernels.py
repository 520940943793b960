"""Kernel-level parity on the MI355X: HIP path (through the C ABI) vs the CPU oracle.

Tolerances: fp32 kernels rtol 1e-4 / atol 1e-5 (relative to the tensor's max magnitude);
bf16 kernels are compared with the fp64 oracle on the same bf16-rounded inputs by relative L2
error <= 2e-2 and max-abs <= 3e-2 * max|ref| (SURVEY §8c calibration)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cswin_ref as O


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def assert_close(a, b, dtype):
    a, b = a.double().cpu(), b.double().cpu()
    scale = float(b.abs().max().clamp_min(1e-30))
    if dtype == torch.float32:
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * max(1.0, scale))
    else:
        assert rel_l2(a, b) < 2e-2, rel_l2(a, b)
        assert float((a - b).abs().max()) < 3e-2 * scale


# (reso, idx, sw, cb, heads, B): covers width-1 stripes, N % 32 != 0 (masking), N up to 1024
ATTN_CASES = [
    (16, 0, 1, 32, 1, 2), (16, 1, 1, 32, 1, 2), (16, 0, 2, 64, 2, 2), (16, 1, 4, 64, 2, 1),
    (8, -1, 8, 128, 4, 2), (14, 0, 7, 64, 2, 1), (7, -1, 7, 64, 2, 2), (32, 0, 8, 128, 4, 1),
    (16, -1, 16, 64, 2, 1), (32, -1, 32, 32, 1, 1), (64, 1, 2, 64, 2, 1), (56, 0, 1, 32, 1, 1),
    # 1024x1024-class windows held whole in LDS: 512 (stage 3, split 8), ragged 400 / 576, 1024 (stage 4)
    (64, 0, 8, 64, 2, 1), (20, -1, 20, 32, 1, 2), (24, -1, 24, 64, 2, 1), (32, -1, 32, 128, 4, 1),
    # the 512x512 headline's stage-1 (reso 128, width-1 stripes of 128 tokens, cswin:232-237) and stage-2 windows
    (128, 0, 1, 32, 1, 1), (128, 1, 1, 32, 1, 1), (64, 0, 2, 64, 2, 1),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ATTN_CASES)
def test_stripe_attention_vs_oracle(case, dtype):
    from csu import ops
    d = dev()
    reso, idx, sw, cb, heads, B = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    L = reso * reso
    qkv = torch.randn(B, L, 3 * cb, generator=g).to(dtype)
    w = torch.randn(cb, 1, 3, 3, generator=g) * 0.3
    b = torch.randn(cb, generator=g) * 0.1
    gout = torch.randn(B, L, cb, generator=g).to(dtype)
    hs, ws = O.stripe_geometry(reso, idx, sw)
    scale = (cb // heads) ** -0.5
    # oracle (fp64, on the same rounded inputs)
    q64 = qkv.double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = O.lepe_attention(q64[..., :cb], q64[..., cb:2 * cb], q64[..., 2 * cb:], reso, hs, ws, heads, w64, b64, scale)
    ref.backward(gout.double())
    # HIP
    qd = qkv.to(d).requires_grad_(True)
    wd, bd = w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    geom = ops.StripeGeometry(reso, cb, heads, [(hs, ws, 0)], scale)
    out = ops.stripe_attention(qd, geom, [wd], [bd])
    out.backward(gout.to(d))
    torch.cuda.synchronize()
    assert out.dtype == dtype
    assert_close(out, ref, dtype)
    assert_close(qd.grad, q64.grad, dtype)
    assert_close(wd.grad, w64.grad, dtype)
    assert_close(bd.grad, b64.grad, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_two_branch_fused_launch(dtype):
    """Both LePE branches of a CSWinBlock in one launch == two separate oracle branches + cat."""
    from csu import ops
    d = dev()
    reso, C, heads, sw, B = 32, 128, 4, 2, 2
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(B, reso * reso, 3 * C, generator=g).to(dtype)
    ws_ = [torch.randn(C // 2, 1, 3, 3, generator=g) * 0.3 for _ in range(2)]
    bs_ = [torch.randn(C // 2, generator=g) * 0.1 for _ in range(2)]
    scale = (C // heads) ** -0.5
    q = qkv.double()
    outs = []
    for i, sl in enumerate((slice(0, C // 2), slice(C // 2, C))):
        hs, wsp = O.stripe_geometry(reso, i, sw)
        outs.append(O.lepe_attention(q[..., :C][..., sl], q[..., C:2 * C][..., sl], q[..., 2 * C:][..., sl], reso, hs,
                                     wsp, heads // 2, ws_[i].double(), bs_[i].double(), scale))
    ref = torch.cat(outs, -1)
    geom = ops.StripeGeometry(reso, C, heads // 2, [(reso, sw, 0), (sw, reso, C // 2)], scale)
    out = ops.stripe_attention(qkv.to(d), geom, [w.to(d) for w in ws_], [b.to(d) for b in bs_])
    assert_close(out, ref, dtype)


@pytest.mark.parametrize("C", [64, 128, 256, 512])
@pytest.mark.parametrize("xdt,ydt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)])
def test_layernorm_vs_torch_fp64(C, xdt, ydt):
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(C)
    x = (torch.randn(3, 517, C, generator=g) * 2 + 0.5).to(xdt)
    w = torch.randn(C, generator=g)
    b = torch.randn(C, generator=g)
    dy = torch.randn(3, 517, C, generator=g).to(ydt)
    x64 = x.double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(x64, (C,), w64, b64, 1e-5)
    ref.backward(dy.double())
    xd = x.to(d).requires_grad_(True)
    wd, bd = w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    y = ops.layer_norm(xd, wd, bd, 1e-5, ydt)
    y.backward(dy.to(d))
    assert y.dtype == ydt
    tol_dt = torch.float32 if (xdt, ydt) == (torch.float32, torch.float32) else torch.bfloat16
    assert_close(y, ref, tol_dt)
    assert_close(xd.grad, x64.grad, tol_dt)
    assert_close(wd.grad, w64.grad, tol_dt)
    assert_close(bd.grad, b64.grad, tol_dt)


@pytest.mark.parametrize("C", [64, 128, 256, 512])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_layernorm_fork_residual_junction(C, gdt):
    """x -> (x, LN(x)) used as x + f(LN(x)): one-kernel dx = dres + dLN == torch fp64, and the bf16
    copy handed to the upstream GEMM equals the fp32 gradient rounded."""
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(C + 7)
    x = torch.randn(2, 1029, C, generator=g) * 2 + 0.5
    w, b = torch.randn(C, generator=g), torch.randn(C, generator=g)
    gres = torch.randn(2, 1029, C, generator=g)          # gradient through the residual branch
    gln = torch.randn(2, 1029, C, generator=g).to(gdt)    # gradient through the LayerNorm branch
    x64 = x.double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    y64 = torch.nn.functional.layer_norm(x64, (C,), w64, b64, 1e-5)
    ((x64 * gres.double()).sum() + (y64 * gln.double()).sum()).backward()
    seen = {}

    class Probe(torch.autograd.Function):   # upstream consumer: records the gradient object it receives
        @staticmethod
        def forward(ctx, t):
            return t.view_as(t)

        @staticmethod
        def backward(ctx, gt):
            seen["g"] = gt
            return gt

    x0 = x.to(d).requires_grad_(True)
    wd, bd = w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    xa, y = ops.layer_norm_fork(Probe.apply(x0), wd, bd, 1e-5, gdt)   # LN output dtype = its gradient's dtype
    assert y.dtype == gdt and xa.data_ptr() == x0.data_ptr()
    ((xa * gres.to(d)).sum() + (y.float() * gln.to(d).float()).sum()).backward()
    assert_close(x0.grad, x64.grad, torch.float32 if gdt == torch.float32 else torch.bfloat16)
    assert_close(wd.grad, w64.grad, torch.bfloat16)
    assert_close(bd.grad, b64.grad, torch.bfloat16)
    gb = getattr(seen["g"], "_csu_bf16", None)
    assert gb is not None and torch.equal(gb, seen["g"].to(torch.bfloat16))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 64, 32), (2, 1024, 64), (1, 4096, 128), (3, 17, 200), (16, 16384, 64),
                                   (2, 1000, 256)])
def test_simam_vs_formula(shape, dtype):
    """SimAM vs the float64 formula (parity unpinned vs the reference, which has no SimAM)."""
    from csu.simam import simam
    d = dev()
    g = torch.Generator().manual_seed(sum(shape))
    x = (torch.randn(*shape, generator=g) * 1.5 + 0.3).to(dtype)
    dy = torch.randn(*shape, generator=g).to(dtype)
    x64 = x.double().requires_grad_(True)
    ref = O.simam(x64)
    ref.backward(dy.double())
    xd = x.to(d).requires_grad_(True)
    y = simam(xd)
    y.backward(dy.to(d))
    assert_close(y, ref, dtype)
    assert_close(xd.grad, x64.grad, dtype)
    # bf16 output for the GEMM consumer (model path), bf16 incoming gradient, x's dtype for dx
    xb = x.to(d).requires_grad_(True)
    yb = simam(xb, out_dtype=torch.bfloat16)
    assert yb.dtype == torch.bfloat16
    yb.backward(dy.to(d).bfloat16())
    assert_close(yb, ref, torch.bfloat16)
    assert xb.grad.dtype == dtype
    assert_close(xb.grad, x64.grad, torch.bfloat16)


@pytest.mark.parametrize("shape", [(2, 4096, 64), (3, 1024, 128), (2, 256, 256)])
def test_simam_fork_vs_unfused(shape):
    """simam_fork (the encoder skip fork with SimAM: bf16 x for the Merge_Block conv + the gated bf16
    skip, one joined backward pass) equals the unfused form -- bf16 cast, simam(out_dtype=bf16),
    autograd's sum of the two input gradients: outputs bit for bit, the fp32 gradient within a few
    ulps, and its bf16 gradient copy is the cast of its fp32 gradient."""
    from csu.simam import simam, simam_fork
    d = dev()
    g = torch.Generator(device=d).manual_seed(sum(shape))
    x0 = torch.randn(*shape, device=d, generator=g) * 1.5 + 0.3
    g1 = torch.randn(*shape, device=d, generator=g).bfloat16()
    dy = torch.randn(*shape, device=d, generator=g).bfloat16()
    x = x0.clone().requires_grad_(True)
    xc, y = simam_fork(x)
    assert xc.dtype == y.dtype == torch.bfloat16
    captured = {}
    def hook(gr):
        captured["bf16"] = getattr(gr, "_csu_bf16", None)   # returns None: the gradient is unchanged
    x.register_hook(hook)
    torch.autograd.backward([xc, y], [g1, dy])
    xr = x0.clone().requires_grad_(True)
    xcr, yr = xr.to(torch.bfloat16), simam(xr, out_dtype=torch.bfloat16)
    torch.autograd.backward([xcr, yr], [g1, dy])
    assert torch.equal(xc, xcr) and torch.equal(y, yr)
    # fp32 gradient: the same terms, one more add in the joined pass (FMA contraction may differ): ulps
    err = float((x.grad - xr.grad).abs().max())
    assert err <= 2 ** -20 * float(xr.grad.abs().max()), err
    assert captured["bf16"] is not None and torch.equal(captured["bf16"], x.grad.bfloat16())


def test_cpu_tensor_fails_loudly():
    from csu import ops
    from csu._lib import CsuError
    geom = ops.StripeGeometry(8, 32, 1, [(8, 1, 0)], 32 ** -0.5)
    with pytest.raises(CsuError):
        ops.stripe_attention(torch.zeros(1, 64, 96), geom, [torch.zeros(32, 1, 3, 3)], [torch.zeros(32)])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,C,s", [(2, 8, 64, 2), (1, 16, 32, 4), (2, 4, 512, 2), (1, 7, 128, 2), (1, 5, 64, 4),
                                     (2, 6, 32, 2)])   # 4 lanes per pixel (S = 2)
def test_carafe_module_vs_oracle(B, H, C, s, dtype):
    """CARAFE / CARAFE4 module (HIP reassembly + conv/GEMM kernel prediction) vs the oracle."""
    from csu.model import CARAFE
    d = dev()
    torch.manual_seed(B * 100 + H * 10 + s)
    m = CARAFE(C, C // 2 if C > 32 else C, up_factor=s)
    x = torch.randn(B, H * H, C)
    gy = torch.randn(B, H * H * s * s, m.out.weight.shape[0])
    p64 = {"." + k: v.double().requires_grad_(True) for k, v in m.state_dict().items()}
    x64 = x.double().requires_grad_(True)
    ref = O.carafe(x64, p64, "", s)
    ref.backward(gy.double())
    md = m.to(d)
    xd = x.to(d).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        y = md(xd)
    y.float().backward(gy.to(d))
    assert_close(y.float(), ref, dtype)
    assert_close(xd.grad, x64.grad, dtype)
    for k, p in md.named_parameters():
        assert_close(p.grad, p64["." + k].grad, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,C,s", [(1, 5, 8, 2), (2, 4, 16, 2), (1, 6, 32, 2), (2, 5, 64, 2), (1, 3, 512, 2),
                                     (1, 4, 8, 4)])
def test_carafe_reassemble_lane_counts(B, H, C, s, dtype):
    """csu_carafe_fwd / _bwd alone (ops.carafe_reassemble) for every lane count per pixel (G = C / 8:
    1, 2 -- the all-reduce path -- and 4 .. 64, the S = 2 reduce-scatter) vs a float64 restatement of
    the reassembly (oracle.cswin_ref.carafe, cswin:410-432): out, d x, d logits."""
    from csu import ops
    d = dev()
    torch.manual_seed(B * 1000 + H * 10 + C + s)
    x = torch.randn(B, H * H, C)
    enc = torch.randn(B, H, H, 9 * s * s) * 2
    gy = torch.randn(B, H * H * s * s, C)
    x64, e64 = x.double().requires_grad_(True), enc.double().requires_grad_(True)
    xi = x64.transpose(1, 2).reshape(B, C, H, H)
    kern = e64.permute(0, 3, 1, 2).reshape(B, 9, s, s, H, H).softmax(dim=1)
    nb = torch.nn.functional.unfold(xi, 3, padding=1).reshape(B, C, 9, H, H)
    ref = torch.einsum("btijhw,bcthw->bchiwj", kern, nb).reshape(B, C, H * s * H * s).transpose(1, 2)
    ref.backward(gy.double())
    xd = x.to(d, dtype).requires_grad_(True)
    ed = enc.to(d, dtype).requires_grad_(True)
    y = ops.carafe_reassemble(xd, ed, H, H, s)
    y.float().backward(gy.to(d))
    assert_close(y.float(), ref, dtype)
    assert_close(xd.grad.float(), x64.grad, dtype)
    assert_close(ed.grad.float(), e64.grad, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,C,s", [(2, 8, 64, 4), (1, 5, 32, 4), (2, 6, 64, 2)])
def test_carafe_sigmoid_head_vs_oracle(B, H, C, s, dtype):
    """Fused CARAFE(4) + `out` conv + 1-class `output` conv + sigmoid (csu_carafe_head_*) vs the
    oracle's unfused chain in fp64 (cswin:450-486, 674-688)."""
    from csu.model import CARAFE, carafe_sigmoid_head
    d = dev()
    torch.manual_seed(B * 100 + H * 10 + s + C)
    m = CARAFE(C, C, up_factor=s)
    with torch.no_grad():
        m.out.bias.normal_(0, 0.3)
    wo = torch.randn(1, C, 1, 1) * 0.3
    x = torch.randn(B, H * H, C)
    dp = torch.randn(B, 1, s * H, s * H)
    p64 = {"." + k: v.double().requires_grad_(True) for k, v in m.state_dict().items()}
    x64, wo64 = x.double().requires_grad_(True), wo.double().requires_grad_(True)
    y = O.carafe(x64, p64, "", s)                                           # (B, s^2 L, C)
    ref = torch.sigmoid(y @ wo64.view(C)).view(B, 1, s * H, s * H)
    ref.backward(dp.double())
    md, wod = m.to(d), wo.to(d).requires_grad_(True)
    xd = x.to(d).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        p = carafe_sigmoid_head(md, wod, xd)
    p.backward(dp.to(d))
    assert p.dtype == torch.float32 and p.shape == ref.shape
    assert_close(p, ref, dtype)
    assert_close(xd.grad, x64.grad, dtype)
    assert_close(wod.grad, wo64.grad, dtype)
    for k, q in md.named_parameters():
        assert_close(q.grad, p64["." + k].grad, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sigmoid_head_vs_torch(dtype):
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, 4099, 64, generator=g).to(dtype)
    w = torch.randn(1, 64, 1, 1, generator=g) * 0.2
    dp = torch.randn(3, 4099, generator=g)
    x64, w64 = x.double().requires_grad_(True), w.double().requires_grad_(True)
    ref = torch.sigmoid(x64 @ w64.view(64))
    ref.backward(dp.double())
    xd, wd = x.to(d).requires_grad_(True), w.to(d).requires_grad_(True)
    p = ops.sigmoid_head(xd, wd)
    p.backward(dp.to(d))
    assert p.dtype == torch.float32
    assert_close(p, ref, dtype)
    assert_close(xd.grad, x64.grad, dtype)
    assert_close(wd.grad, w64.grad, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(1, 8), (262144, 64), (4096, 2048), (128, 12288), (7, 40), (100000, 200)])
def test_colsum_deterministic(rows, cols, dtype):
    from csu import ops
    d = dev()
    x = torch.randn(rows, cols, device=d).to(dtype)
    a, b = ops.colsum(x), ops.colsum(x)
    assert torch.equal(a, b)                      # bitwise reproducible
    ref = x.double().sum(0)
    torch.testing.assert_close(a.double(), ref, rtol=1e-5, atol=1e-3 * max(1.0, rows ** 0.5) * 1e-2)


def test_linear_splitk_matches_torch():
    from csu import ops
    d = dev()
    x = torch.randn(8, 4096, 64, device=d, requires_grad=True)
    w = torch.randn(256, 64, device=d, requires_grad=True)
    b = torch.randn(256, device=d, requires_grad=True)
    gy = torch.randn(8, 4096, 256, device=d)
    y = ops.linear(x, w, b)
    y.backward(gy)
    x2, w2, b2 = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    torch.nn.functional.linear(x2, w2, b2).backward(gy.double())
    for a_, r_ in ((y, torch.nn.functional.linear(x2, w2, b2)), (x.grad, x2.grad), (w.grad, w2.grad), (b.grad, b2.grad)):
        assert_close(a_, r_, torch.float32)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(262144, 256, 64), (4096, 512, 2048), (1000, 16, 64), (16384, 768, 256), (77, 64, 8),
                                   (3001, 136, 200), (130, 1024, 256), (65536, 128, 512), (4096, 2048, 512), (700, 64, 64)])
def test_linear_wgrad_kernel(M, N, K, dtype):
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K)
    dy = torch.randn(M, N, device=d, generator=g).to(dtype)
    x = torch.randn(M, K, device=d, generator=g).to(dtype)
    dw, db = ops.linear_wgrad(dy, x)
    dw2, db2 = ops.linear_wgrad(dy, x)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)       # deterministic
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    scale_w = float(ref_w.abs().max())
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert float((dw.double() - ref_w).abs().max()) <= tol * max(scale_w, M ** 0.5)
    assert float((db.double() - ref_b).abs().max()) <= tol * max(float(ref_b.abs().max()), M ** 0.5)


def _gelu(t):
    return torch.nn.functional.gelu(t)


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4099, 192, 64), (2048, 768, 256), (300, 128, 1024), (513, 256, 32),
                                   (65536, 128, 512), (1030, 520, 128)])
@pytest.mark.parametrize("b_trans", [False, True])
@pytest.mark.parametrize("mode", ["plain", "bias_gelu_a", "gelu_aux", "resid"])
def test_gemm_vs_torch(M, N, K, b_trans, mode):
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K)
    a = torch.randn(M, K, device=d, generator=g).bfloat16()
    w = (torch.randn(N, K, device=d, generator=g) * 0.1).bfloat16()       # nn.Linear weight (N, K)
    b = torch.randn(K, N, device=d, generator=g).bfloat16() * 0.1 if b_trans else w
    bias = torch.randn(N, device=d, generator=g) if mode == "bias_gelu_a" else None
    aux = torch.randn(M, N, device=d, generator=g).bfloat16() if mode == "gelu_aux" else None
    res = torch.randn(M, N, device=d, generator=g) if mode == "resid" else None
    odt = torch.float32 if mode == "resid" else torch.bfloat16
    out = ops.gemm(a, b, b_trans, odt, bias=bias, a_gelu=mode == "bias_gelu_a", gelu_aux=aux, resid=res)
    A = a.double()
    if mode == "bias_gelu_a":
        A = _gelu(a.float()).bfloat16().double()
    ref = A @ (b.double() if b_trans else b.double().t())
    if bias is not None:
        ref = ref + bias.double()
    if aux is not None:
        x = aux.double()
        ref = ref * (0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5)
    if res is not None:
        ref = ref + res.double()
    assert out.dtype == odt
    assert_close(out, ref, torch.bfloat16)


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19])
@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4099, 192, 128), (300, 520, 1024), (16384, 1024, 256)])
def test_gemm_tile_configs_and_gelu_out(M, N, K, cfg):
    """Every tile configuration of the b[n][k] kernel, with the dual (h, gelu(h)) epilogue."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K + cfg)
    a = torch.randn(M, K, device=d, generator=g).bfloat16()
    w = (torch.randn(N, K, device=d, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=d, generator=g)
    h, gh = ops.gemm(a, w, False, torch.bfloat16, bias=bias, cfg=cfg, gelu_out=True)
    ref = a.double() @ w.double().t() + bias.double()
    assert_close(h, ref, torch.bfloat16)
    assert_close(gh, _gelu(ref), torch.bfloat16)
    # the GELU output is computed from the fp32 accumulator (before the bf16 rounding of h)
    assert float((gh.float() - _gelu(h.float())).abs().max()) < 2e-2 * float(ref.abs().max())


def test_cast_cache_batch_kernel():
    """csu_cast_bf16_batch: bf16 shadows and (K, N) transposes of 2-D, 1-D and 4-D weights."""
    from csu import ops
    d = dev()
    torch.manual_seed(3)
    ps = [torch.randn(192, 64, device=d), torch.randn(70, device=d), torch.randn(16, 64, 1, 1, device=d),
          torch.randn(130, 333, device=d), torch.randn(5, device=d)]
    convs = [torch.randn(36, 16, 3, 3, device=d), torch.randn(64, 3, 7, 7, device=d), torch.randn(256, 128, 3, 3, device=d)]
    c = ops.CastCache()
    c.refresh(ps, torch.bfloat16, convs)
    assert c.items is not None
    for p in ps:
        torch.testing.assert_close(c.get(p, torch.bfloat16), p.bfloat16(), rtol=0, atol=0)
        if p.dim() > 1:
            v = p.reshape(p.shape[0], -1)
            torch.testing.assert_close(c.get_t(v, torch.bfloat16), v.t().bfloat16(), rtol=0, atol=0)
    for w in convs:   # channels-last conv layouts written by the same launch
        o, i = c.get_conv(w, torch.bfloat16)
        C = w.shape[1]
        if C % 8:     # few-channel conv (patch embed): OHWI zero-padded to 8 channels, no IHWO
            assert o.shape[-1] == 8 and i is None and not o[..., C:].any()
            assert torch.equal(o[..., :C], w.permute(0, 2, 3, 1).bfloat16())
            continue
        assert torch.equal(o, w.permute(0, 2, 3, 1).bfloat16()) and torch.equal(i, w.permute(1, 2, 3, 0).bfloat16())
    with torch.no_grad():
        ps[0].mul_(2)
        convs[1].mul_(3)
    c.refresh(ps, torch.bfloat16, convs)
    torch.testing.assert_close(c.get(ps[0], torch.bfloat16), ps[0].bfloat16(), rtol=0, atol=0)
    o = c.get_conv(convs[1], torch.bfloat16)[0]
    assert torch.equal(o[..., :3], convs[1].permute(0, 2, 3, 1).bfloat16()) and not o[..., 3:].any()


def test_fused_mlp_residual_matches_unfused():
    """mlp_residual / linear_residual (bf16 fused GEMMs) == the unfused autocast composition."""
    from csu import ops
    d = dev()
    torch.manual_seed(0)
    fc1, fc2, proj = torch.nn.Linear(128, 512).to(d), torch.nn.Linear(512, 128).to(d), torch.nn.Linear(128, 128).to(d)
    res = torch.randn(2, 1000, 128, device=d, requires_grad=True)
    xin = torch.randn(2, 1000, 128, device=d).bfloat16().requires_grad_(True)
    gy = torch.randn(2, 1000, 128, device=d)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.mlp_residual(ops.linear_residual(res, xin, proj.weight, proj.bias), xin, fc1, fc2)
    y.backward(gy)
    grads = [t.grad.clone() for t in (res, xin, fc1.weight, fc1.bias, fc2.weight, fc2.bias, proj.weight, proj.bias)]
    for t in (res, xin, fc1.weight, fc1.bias, fc2.weight, fc2.bias, proj.weight, proj.bias):
        t.grad = None
    r64, x64 = res.detach().double().requires_grad_(True), xin.detach().double().requires_grad_(True)
    ps = [p.detach().double().requires_grad_(True) for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias, proj.weight, proj.bias)]
    F = torch.nn.functional
    z = r64 + F.linear(x64, ps[4], ps[5])
    ref = z + F.linear(F.gelu(F.linear(x64, ps[0], ps[1])), ps[2], ps[3])
    ref.backward(gy.double())
    assert_close(y, ref, torch.bfloat16)
    for got, r in zip(grads, [r64.grad, x64.grad] + [p.grad for p in ps]):
        assert_close(got, r, torch.bfloat16)


@pytest.mark.parametrize("C,M", [(64, 4096), (64, 37), (128, 1000), (256, 4160), (256, 100)])
def test_mlp_fused_kernels_vs_fp64(C, M):
    """csu_mlp_fwd / csu_mlp_bwd (fc1 -> GELU -> fc2 + residual with the hidden layer on chip) vs
    the fp64 composition on the same bf16 inputs: y, and the backward's dh = (dy W2) gelu'(h),
    g = gelu(h), dx = dh W1.  Ragged M exercises the token tail of the last 64-token panel."""
    from csu._lib import check, lib, ptr, stream_ptr
    d = dev()
    torch.manual_seed(C + M)
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.randn(4 * C, device=d) * 0.1, torch.randn(C, device=d) * 0.1
    res = torch.randn(M, C, device=d)
    dy = torch.randn(M, C, device=d).bfloat16()
    y = torch.empty(M, C, device=d)
    st = stream_ptr(d)
    check(lib().csu_mlp_fwd(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), st), "mlp_fwd")
    dh = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    g = torch.empty_like(dh)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    check(lib().csu_mlp_bwd(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx), st), "mlp_bwd")
    torch.cuda.synchronize()
    X, W1, W2, B1, B2 = (t.double().cpu() for t in (x, w1, w2, b1, b2))
    F = torch.nn.functional
    h = X @ W1.T + B1
    gr = F.gelu(h)
    assert_close(y, res.double().cpu() + gr @ W2.T + B2, torch.bfloat16)
    assert_close(g, gr, torch.bfloat16)
    hg = h.clone().requires_grad_(True)
    F.gelu(hg).backward(dy.double().cpu() @ W2)
    assert_close(dh, hg.grad, torch.bfloat16)
    assert_close(dx, hg.grad @ W1, torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(16384, 1024, 256), (4099, 192, 64), (262144, 64, 128), (4096, 2048, 512), (700, 32, 128)])
@pytest.mark.parametrize("tn,tk,chunks", [(64, 64, 1), (128, 128, 0), (128, 64, 5), (64, 128, 37), (0, 0, 0), (128, 128, 300)])
def test_linear_wgrad_plans(M, N, K, tn, tk, chunks):
    """csu_linear_wgrad_tuned: every output tile (64/128 x 64/128) and split-K chunking (1 chunk =
    direct write; >1 = tile-local slabs + the fixed-order reduce) == fp64, bitwise reproducible."""
    from csu._lib import check, lib, ptr, stream_ptr
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K + tn + chunks)
    dy = torch.randn(M, N, device=d, generator=g).bfloat16()
    x = torch.randn(M, K, device=d, generator=g).bfloat16()
    L = lib()
    outs = []
    for _ in range(2):
        n = L.csu_linear_wgrad_tuned_workspace(M, N, K, tn, tk, chunks)
        ws = torch.full((max(n, 16) // 4,), float("nan"), device=d)      # poisoned workspace
        out = torch.full((N * K + N,), float("nan"), device=d)
        check(L.csu_linear_wgrad_tuned(M, N, K, 1, ptr(dy), ptr(x), ptr(out), ptr(ws), n, tn, tk, chunks, stream_ptr(d)),
              "linear_wgrad_tuned")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    dw, db = outs[0][:N * K].view(N, K), outs[0][N * K:]
    assert float((dw.double() - ref_w).abs().max()) <= 1e-2 * max(float(ref_w.abs().max()), M ** 0.5)
    assert float((db.double() - ref_b).abs().max()) <= 1e-2 * max(float(ref_b.abs().max()), M ** 0.5)


@pytest.mark.parametrize("M,N,K,chunks", [(16384, 1024, 256, 1), (16384, 768, 256, 5), (4096, 2048, 512, 3),
                                           (700, 256, 128, 2), (65536, 512, 128, 0)])
def test_linear_wgrad_8wave_tile(M, N, K, chunks):
    """The 8-wave 256 x 128 tile (the grouped path's choice for N % 256 == 0, K % 128 == 0) through
    csu_linear_wgrad_tuned: == fp64 (dW and db), bitwise reproducible, ragged token chunks."""
    from csu._lib import check, lib, ptr, stream_ptr
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K + chunks)
    dy = torch.randn(M, N, device=d, generator=g).bfloat16()
    x = torch.randn(M, K, device=d, generator=g).bfloat16()
    L = lib()
    outs = []
    for _ in range(2):
        n = L.csu_linear_wgrad_tuned_workspace(M, N, K, 256, 128, chunks)
        ws = torch.full((max(n, 16) // 4,), float("nan"), device=d)
        out = torch.full((N * K + N,), float("nan"), device=d)
        check(L.csu_linear_wgrad_tuned(M, N, K, 1, ptr(dy), ptr(x), ptr(out), ptr(ws), n, 256, 128, chunks, stream_ptr(d)),
              "linear_wgrad_tuned 256x128")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    dw, db = outs[0][:N * K].view(N, K), outs[0][N * K:]
    assert float((dw.double() - ref_w).abs().max()) <= 1e-2 * max(float(ref_w.abs().max()), M ** 0.5)
    assert float((db.double() - ref_b).abs().max()) <= 1e-2 * max(float(ref_b.abs().max()), M ** 0.5)
    assert L.csu_linear_wgrad_tuned(M, 192, K, 1, ptr(dy), ptr(x), ptr(out), ptr(ws), n, 256, 128, chunks,
                                    stream_ptr(d)) != 0   # N % 256 != 0: refused


def test_side_stream_wgrad_with_gradient_accumulation(monkeypatch):
    """Two backward passes without zeroing (gradient accumulation: AccumulateGrad adds in place on
    the launching stream) give bitwise the same .grad with the side stream on and off: a parameter
    that already holds a .grad takes its weight gradient inline (ops._param_safe).  (The grouped
    end-of-backward weight gradients use another token chunking -- equal to rounding, tested in
    test_linear_wgrad_grouped -- so they are off here.)"""
    from csu import ops
    monkeypatch.setattr(ops, "GROUP_WGRAD", False)
    d = dev()
    torch.manual_seed(0)
    res = {}
    for side in (True, False):
        old = ops.SIDE_WGRAD
        ops.SIDE_WGRAD = side
        try:
            torch.manual_seed(1)
            fc1, fc2 = torch.nn.Linear(256, 1024).to(d), torch.nn.Linear(1024, 256).to(d)
            x = torch.randn(4, 4096, 256, device=d)
            for _ in range(2):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    y = ops.mlp_residual(x, x.bfloat16(), fc1, fc2)
                y.float().square().mean().backward()
            torch.cuda.synchronize()
            res[side] = [p.grad.clone() for p in (fc1.weight, fc1.bias, fc2.weight, fc2.bias)]
        finally:
            ops.SIDE_WGRAD = old
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


CONV_CASES = [  # (B, H, C, N, k, stride, pad)
    (2, 32, 3, 64, 7, 4, 2),      # patch embed (cswin:505)
    (2, 16, 64, 128, 3, 2, 1),    # Merge_Block (cswin:376)
    (1, 8, 16, 144, 3, 1, 1),     # CARAFE4 encoder (cswin:446)
    (2, 64, 16, 144, 3, 1, 1),    # CARAFE4 encoder at a width the few-channel kernel takes (conv3_c16)
    (2, 9, 32, 36, 3, 1, 1),      # CARAFE encoder, odd size / N % 8 != 0 (bf16: K split in 2, ragged last part)
    (16, 16, 128, 36, 3, 1, 1),   # CARAFE encoder at 16x16 (512x512 decoder): 32 tiles -> K split (fwd and dgrad)
    (16, 32, 64, 36, 3, 1, 1),    # CARAFE encoder at 32x32: 128 tiles -> K split
    (1, 10, 32, 68, 3, 1, 1),     # N % 8 == 4 over two N tiles (weight gradient: 8-B dy loads, half-valid tail)
    (1, 12, 8, 24, 3, 1, 1),      # UNet DoubleConv-like
    (2, 6, 40, 16, 1, 1, 0),      # 1x1
    (2, 11, 64, 128, 3, 2, 1),    # stride 2 on an odd size (phase split of the input gradient)
    (1, 70, 64, 72, 3, 1, 1),     # several 128/256-row tiles, N tail
    (1, 13, 12, 20, 5, 3, 2),     # stride 3, 5x5: phases with 1-2 taps per axis
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_nhwc_vs_torch(case, dtype):
    from csu import ops
    d = dev()
    B, H, C, N, k, s, p = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(B, H, H, C, generator=g).to(dtype)
    w = torch.randn(N, C, k, k, generator=g) * (1.0 / (C * k * k) ** 0.5)
    b = torch.randn(N, generator=g) * 0.1
    x64, w64, b64 = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.nn.functional.conv2d(x64.permute(0, 3, 1, 2), w64, b64, stride=s, padding=p).permute(0, 2, 3, 1)
    gy = torch.randn(ref.shape, generator=g).to(dtype)
    ref.backward(gy.double())
    xd, wd, bd = x.to(d).requires_grad_(True), w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        y = ops.conv2d(xd, wd, bd, s, p)
    y.backward(gy.to(d).to(y.dtype))
    assert tuple(y.shape) == tuple(ref.shape)
    assert_close(y.float(), ref, dtype)
    assert_close(xd.grad, x64.grad, dtype)
    assert_close(wd.grad, w64.grad, dtype)
    assert_close(bd.grad, b64.grad, dtype)


# persistent LDS-DMA implicit GEMM (csu_conv2d_ex cfg 1 + k): BN of each tile configuration
IGEMM_DMA_BN = {1: 128, 2: 128, 3: 128, 4: 64, 5: 64, 6: 64, 7: 256, 8: 256, 9: 64, 10: 64, 11: 64, 12: 128}
DMA_CONV_CASES = [  # (B, H, C, N, k, stride, pad): 64-channel gathers, partial M tiles
    (1, 20, 64, 256, 3, 1, 1),     # UNet-like 3x3, M = 400 (partial 256-row tile), two N tiles of 128
    (2, 9, 128, 512, 3, 2, 1),     # stride 2 on an odd size: 4 input-gradient phases of 1-4 taps
    (1, 12, 256, 256, 2, 2, 0),    # ConvTranspose2d(k2, s2)-shaped
    (2, 7, 64, 64, 1, 1, 0),       # 1x1
]


@pytest.mark.parametrize("case", DMA_CONV_CASES)
def test_conv_igemm_dma_cfgs(case):
    """Every tile configuration of the LDS-DMA implicit GEMM (forward and input gradient, bf16
    operands, fp32 accumulation) vs float64 torch on the same bf16 operands; configurations whose
    BN does not divide the output channels must refuse (CSU_E_ARG)."""
    import ctypes
    from csu import ops
    from csu._lib import lib, CSU_BF16
    d = dev()
    B, H, C, N, k, s, p = case
    gm = ops._conv_geom(B, H, H, C, N, k, k, s, p)
    g = torch.Generator().manual_seed(sum(case) + 7)
    x = torch.randn(B, H, H, C, generator=g).bfloat16()
    w = (torch.randn(N, C, k, k, generator=g) / (C * k * k) ** 0.5).bfloat16()
    b = torch.randn(N, generator=g)
    dy = torch.randn(B, gm.OH, gm.OW, N, generator=g).bfloat16()
    ref_f = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), s, p).permute(0, 2, 3, 1)
    ref_d = torch.nn.functional.conv_transpose2d(dy.double().permute(0, 3, 1, 2), w.double(), None, s, p,
                                                 output_padding=H - ((gm.OH - 1) * s - 2 * p + k)).permute(0, 2, 3, 1)
    xd, dyd, bd = x.to(d), dy.to(d), b.to(d)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(d)
    w_ihwo = w.permute(1, 2, 3, 0).contiguous().to(d)
    st = torch.cuda.current_stream().cuda_stream
    for op, src, wt, bias, ncols, cs, ref in ((0, xd, w_ohwi, bd, N, C, ref_f), (1, dyd, w_ihwo, None, C, N, ref_d)):
        for cfg, bn in IGEMM_DMA_BN.items():
            out = torch.full(ref.shape, float("nan"), dtype=torch.bfloat16, device=d)
            e = lib().csu_conv2d_ex(op, ctypes.byref(gm), CSU_BF16, src.data_ptr(), wt.data_ptr(),
                                    bias.data_ptr() if bias is not None else None, out.data_ptr(), cfg, st)
            if ncols % bn or cs % 64:
                assert e != 0, (op, cfg)
                continue
            assert e == 0, (op, cfg, lib().csu_last_error_string())
            torch.cuda.synchronize()
            err = float((out.double().cpu() - ref).norm() / ref.norm())
            assert err < 4e-3, (op, cfg, err)   # bf16 output rounding (2^-9 relative) dominates


@pytest.mark.parametrize("B,H,W", [(2, 64, 64), (1, 6, 128), (1, 5, 64)])
def test_conv_halo64(B, H, W):
    """The halo kernel of the 64 -> 64 channel 3x3 stride-1 conv (csu_conv2d_ex cfg 20), forward and
    input gradient, vs float64 torch on the same bf16 operands; H odd is not eligible (CSU_E_ARG)."""
    import ctypes
    from csu import ops
    from csu._lib import lib, CSU_BF16
    d = dev()
    gm = ops._conv_geom(B, H, W, 64, 64, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(B * 1000 + H + W)
    x = torch.randn(B, H, W, 64, generator=g).bfloat16()
    w = (torch.randn(64, 64, 3, 3, generator=g) / 24.0).bfloat16()
    b = torch.randn(64, generator=g)
    dy = torch.randn(B, H, W, 64, generator=g).bfloat16()
    ref_f = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), 1, 1).permute(0, 2, 3, 1)
    ref_d = torch.nn.functional.conv_transpose2d(dy.double().permute(0, 3, 1, 2), w.double(), None, 1, 1).permute(0, 2, 3, 1)
    xd, dyd, bd = x.to(d), dy.to(d), b.to(d)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(d)
    w_ihwo = w.permute(1, 2, 3, 0).contiguous().to(d)
    st = torch.cuda.current_stream().cuda_stream
    for op, src, wt, bias, ref in ((0, xd, w_ohwi, bd, ref_f), (1, dyd, w_ihwo, None, ref_d)):
        out = torch.full(ref.shape, float("nan"), dtype=torch.bfloat16, device=d)
        e = lib().csu_conv2d_ex(op, ctypes.byref(gm), CSU_BF16, src.data_ptr(), wt.data_ptr(),
                                bias.data_ptr() if bias is not None else None, out.data_ptr(), 20, st)
        if H % 2:
            assert e != 0
            continue
        assert e == 0, lib().csu_last_error_string()
        torch.cuda.synchronize()
        err = float((out.double().cpu() - ref).norm() / ref.norm())
        assert err < 4e-3, (op, err)


@pytest.mark.parametrize("case", DMA_CONV_CASES + [(2, 16, 64, 128, 3, 2, 1), (1, 70, 64, 72, 3, 1, 1), (2, 9, 32, 64, 3, 1, 1),
                                  (1, 64, 64, 128, 3, 1, 1), (2, 64, 128, 64, 3, 1, 1)])   # halo-eligible (OW % 64 == 0)
def test_conv_wgrad_cfgs(case):
    """Weight + bias gradient by every csu_conv2d_wgrad_ex configuration (v2 and the LDS-DMA tile
    configurations) vs float64 torch on the same bf16 operands, in both output layouts."""
    import ctypes
    from csu import ops
    from csu._lib import lib, CSU_BF16
    d = dev()
    B, H, C, N, k, s, p = case
    gm = ops._conv_geom(B, H, H, C, N, k, k, s, p)
    g = torch.Generator().manual_seed(sum(case) + 11)
    x = torch.randn(B, H, H, C, generator=g).bfloat16()
    dy = torch.randn(B, gm.OH, gm.OW, N, generator=g).bfloat16()
    dw = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (N, C, k, k), dy.double().permute(0, 3, 1, 2),
                                     stride=s, padding=p)
    db = dy.double().sum((0, 1, 2))
    xd, dyd = x.to(d), dy.to(d)   # kept alive across the asynchronous calls
    st = torch.cuda.current_stream().cuda_stream
    halo = k == 3 and s == 1 and p == 1 and H % 64 == 0 and C % 64 == 0
    for cfg in range(0, 8):
        nws = lib().csu_conv2d_wgrad_workspace_ex(ctypes.byref(gm), cfg)
        if nws == 0:
            assert C % 8 or N % 8 or (cfg == 6 and not (halo and N % 64 == 0)) or (cfg == 7 and not (halo and N % 128 == 0))
            continue
        work = torch.empty(nws, dtype=torch.uint8, device=d)
        for creal, ref in ((0, torch.cat([dw.permute(0, 2, 3, 1).reshape(-1), db])), (C, torch.cat([dw.reshape(-1), db]))):
            out = torch.full((ref.numel(),), float("nan"), device=d)
            e = lib().csu_conv2d_wgrad_ex(ctypes.byref(gm), CSU_BF16, xd.data_ptr(), dyd.data_ptr(), creal,
                                          out.data_ptr(), work.data_ptr(), nws, cfg, st)
            assert e == 0, (cfg, lib().csu_last_error_string())
            torch.cuda.synchronize()
            err = float((out.double().cpu() - ref).norm() / ref.norm())
            assert err < 1e-5, (cfg, creal, err)   # fp32 accumulation of exact bf16 products


@pytest.mark.parametrize("B,H,Ca,Cb,N", [(1, 64, 64, 64, 64), (2, 64, 128, 64, 128), (1, 32, 64, 64, 64)])
def test_conv2d_cat_two_source(B, H, Ca, Cb, N):
    """UNet Up's conv over cat([x2, x1], channels) (unet:213-216) on the two-source kernels (no
    concatenated tensor; (1, 32, ...) is not eligible and runs on the materialised cat) vs float64
    torch: output, both input gradients, weight and bias gradients (bf16 autocast tolerances)."""
    import ctypes
    from csu import ops
    from csu._lib import lib
    d = dev()
    g = torch.Generator().manual_seed(B + H + Ca + Cb + N)
    xa = torch.randn(B, H, H, Ca, generator=g).bfloat16()
    xb = torch.randn(B, H, H, Cb, generator=g).bfloat16()
    w = torch.randn(N, Ca + Cb, 3, 3, generator=g) * (1.0 / (9 * (Ca + Cb)) ** 0.5)
    b = torch.randn(N, generator=g) * 0.1
    xa64, xb64 = xa.double().requires_grad_(True), xb.double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.nn.functional.conv2d(torch.cat([xa64, xb64], -1).permute(0, 3, 1, 2), w64, b64, 1, 1).permute(0, 2, 3, 1)
    gy = torch.randn(ref.shape, generator=g).bfloat16()
    ref.backward(gy.double())
    gm = ops._conv_geom(B, H, H, Ca + Cb, N, 3, 3, 1, 1)
    assert bool(lib().csu_conv2d_split_ok(ctypes.byref(gm), Ca)) == (H % 64 == 0)
    xad, xbd = xa.to(d).requires_grad_(True), xb.to(d).requires_grad_(True)
    wd, bd = w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.conv2d_cat(xad, xbd, wd, bd, 1)
    y.backward(gy.to(d))
    torch.cuda.synchronize()
    assert_close(y.float(), ref, torch.bfloat16)
    assert_close(xad.grad, xa64.grad, torch.bfloat16)
    assert_close(xbd.grad, xb64.grad, torch.bfloat16)
    assert_close(wd.grad, w64.grad, torch.bfloat16)
    assert_close(bd.grad, b64.grad, torch.bfloat16)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,H,Cin,Cout", [(2, 8, 64, 32), (1, 5, 128, 64)])
def test_conv_transpose2d_nhwc_vs_torch(B, H, Cin, Cout, dtype):
    """UNet Up.up = ConvTranspose2d(C, C/2, 2, 2) (unet:211)."""
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(B + H + Cin)
    x = torch.randn(B, H, H, Cin, generator=g).to(dtype)
    w = torch.randn(Cin, Cout, 2, 2, generator=g) * 0.1
    b = torch.randn(Cout, generator=g) * 0.1
    x64, w64, b64 = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = torch.nn.functional.conv_transpose2d(x64.permute(0, 3, 1, 2), w64, b64, stride=2).permute(0, 2, 3, 1)
    gy = torch.randn(ref.shape, generator=g).to(dtype)
    ref.backward(gy.double())
    xd, wd, bd = x.to(d).requires_grad_(True), w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
        y = ops.conv_transpose2d(xd, wd, bd, 2)
    y.backward(gy.to(d).to(y.dtype))
    assert_close(y.float(), ref, dtype)
    assert_close(xd.grad, x64.grad, dtype)
    assert_close(wd.grad, w64.grad, dtype)
    assert_close(bd.grad, b64.grad, dtype)


@pytest.mark.parametrize("capturable", [False, True])
def test_fused_adamw_matches_torch(capturable):
    """csu_adamw_step (one launch, all tensors) == torch.optim.AdamW over several steps, incl.
    ragged numels and a ReduceLROnPlateau-style lr change; bias corrections in fp32 -> rtol 1e-5."""
    from csu.optim import FusedAdamW
    d = dev()
    g = torch.Generator(device=d).manual_seed(0)
    shapes = [(256, 64), (64,), (3, 7, 11), (1,), (4099,), (512, 2048)]
    ps = [torch.randn(s, device=d, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [p.clone().requires_grad_(True) for p in ps]
    o_ref = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-2, foreach=False)
    o_mine = FusedAdamW(mine, lr=1e-3, weight_decay=1e-2, capturable=capturable)
    for it in range(6):
        if it == 3:
            for o in (o_ref, o_mine):
                o.param_groups[0]["lr"] = 5e-4
            o_mine.sync_lr()
        grads = [torch.randn(s, device=d, generator=g) for s in shapes]
        for p, q, gr in zip(ref, mine, grads):
            p.grad, q.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_mine.step()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-5, atol=1e-6)
    for p, q in zip(ref, mine):
        torch.testing.assert_close(o_mine.state[q]["exp_avg"], o_ref.state[p]["exp_avg"], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(o_mine.state[q]["exp_avg_sq"], o_ref.state[p]["exp_avg_sq"], rtol=5e-5, atol=1e-9)


def test_fused_adamw_writes_cast_cache_shadows(monkeypatch):
    """FusedAdamW writes the bf16 shadows a CastCache keeps (W, W^T in 64 x 64 tiles incl. ragged
    edges, 1-D copies, conv OHWI (channel-padded) / IHWO) from the updated weights, bit-equal to a
    fresh cast; the next refresh then launches nothing, and an in-place change of a weight (version
    bump) makes it re-cast."""
    from csu import ops
    from csu.optim import FusedAdamW
    d = dev()
    torch.manual_seed(4)
    ps = [torch.randn(192, 64, device=d), torch.randn(70, device=d), torch.randn(16, 64, 1, 1, device=d),
          torch.randn(130, 333, device=d), torch.randn(5, device=d), torch.randn(512, 2048, device=d)]
    convs = [torch.randn(36, 16, 3, 3, device=d), torch.randn(64, 3, 7, 7, device=d), torch.randn(256, 128, 3, 3, device=d)]
    allp = [p.requires_grad_(True) for p in ps + convs]
    plain = [p.detach().clone().requires_grad_(True) for p in allp]
    c = ops.CastCache()
    casts = []
    real = ops.CastCache._cast
    monkeypatch.setattr(ops.CastCache, "_cast", lambda self: casts.append(1) or real(self))
    c.refresh(ps, torch.bfloat16, convs)
    assert len(casts) == 1
    o1 = FusedAdamW(allp, lr=1e-2, weight_decay=1e-2)
    o2 = FusedAdamW(plain, lr=1e-2, weight_decay=1e-2)      # same update without shadows (other buffers)
    for _ in range(3):
        for p, q in zip(allp, plain):
            gr = torch.randn_like(p)
            p.grad, q.grad = gr, gr.clone()
        o1.step()
        o2.step()
        c.refresh(ps, torch.bfloat16, convs)
    assert len(casts) == 1                                   # the optimizer kept every shadow fresh
    for p, q in zip(allp, plain):
        assert torch.equal(p.detach(), q.detach())           # the shadow writes do not change the update
    for p in ps:
        assert torch.equal(c.get(p, torch.bfloat16), p.detach().bfloat16())
        if p.dim() > 1:
            v = p.detach().reshape(p.shape[0], -1)
            assert torch.equal(c.get_t(v, torch.bfloat16), v.t().bfloat16())
    for w in convs:
        o, i = c.get_conv(w, torch.bfloat16)
        C = w.shape[1]
        assert torch.equal(o[..., :C], w.detach().permute(0, 2, 3, 1).bfloat16())
        if C % 8:
            assert i is None and not o[..., C:].any()
        else:
            assert torch.equal(i, w.detach().permute(1, 2, 3, 0).bfloat16())
    with torch.no_grad():
        ps[3].mul_(2)                                        # a change the optimizer did not make
    c.refresh(ps, torch.bfloat16, convs)
    assert len(casts) == 2
    assert torch.equal(c.get(ps[3], torch.bfloat16), ps[3].detach().bfloat16())


@pytest.mark.gpu
def test_fused_adam_l2_matches_torch():
    """csu_adam_l2_step == torch.optim.Adam(weight_decay) (coupled L2: the plain UNet's optimizer,
    unet:486-490) over several steps, ragged numels."""
    from csu.optim import FusedAdam
    d = dev()
    g = torch.Generator(device=d).manual_seed(1)
    shapes = [(64, 3, 3, 3), (64,), (5, 13), (4099,)]
    ps = [torch.randn(s, device=d, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    mine = [p.clone().requires_grad_(True) for p in ps]
    o_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-4, foreach=False)
    o_mine = FusedAdam(mine, lr=1e-3, weight_decay=1e-4)
    for _ in range(5):
        grads = [torch.randn(s, device=d, generator=g) for s in shapes]
        for p, q, gr in zip(ref, mine, grads):
            p.grad, q.grad = gr.clone(), gr.clone()
        o_ref.step()
        o_mine.step()
    for p, q in zip(ref, mine):
        torch.testing.assert_close(q.detach(), p.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(o_mine.state[q]["exp_avg"], o_ref.state[p]["exp_avg"], rtol=1e-5, atol=1e-7)

@pytest.mark.gpu
@pytest.mark.parametrize("B,L,C,N", [(2, 4096, 64, 64), (2, 1024, 128, 128), (3, 256, 256, 256), (1, 100, 64, 64)])
def test_concat_linear_and_shared_cast_vs_fp64(B, L, C, N):
    """Decoder skip fusion without the cat (ops.concat_linear: two GEMMs on the weight halves) and
    the shared bf16 skip copy (ops.shared_cast) vs Linear(cat([skip, up])) in fp64 (cswin:568-592)."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(B * L + C)
    skip = torch.randn(B, L, C, device=d, generator=g, requires_grad=True)
    up = torch.randn(B, L, C, device=d, generator=g).bfloat16().requires_grad_(True)
    w = (torch.randn(N, 2 * C, device=d, generator=g) * 0.05).requires_grad_(True)
    b = torch.randn(N, device=d, generator=g).requires_grad_(True)
    gy = torch.randn(B, L, N, device=d, generator=g)
    gm = torch.randn(B, L, C, device=d, generator=g)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        sm, sk = ops.shared_cast(skip, torch.bfloat16)
        y = ops.concat_linear(sk, up, w, b)
    assert y.dtype == torch.float32 and sm.dtype == torch.bfloat16 and sm.data_ptr() == sk.data_ptr()
    # second consumer of the shared copy (stands in for Merge_Block's conv)
    (y * gy).sum().backward(retain_graph=True)
    (sm.float() * gm).sum().backward()
    s2, u2, w2, b2 = (t.detach().double().requires_grad_(True) for t in (skip, up, w, b))
    sb = s2.bfloat16().double()            # the bf16 rounding autocast applies to the GEMM input
    y2 = torch.nn.functional.linear(torch.cat([sb, u2], -1), w2.bfloat16().double(), b2)
    (y2 * gy.double()).sum().backward()
    gskip_ref = s2.grad + gm.double()
    for got, ref, name in ((y, y2, "y"), (skip.grad, gskip_ref, "dskip"), (up.grad, u2.grad, "dup"),
                           (w.grad, w2.grad, "dw"), (b.grad, b2.grad, "db")):
        ref = ref.detach()
        err = float((got.double() - ref).norm() / ref.norm().clamp_min(1e-30))
        assert err <= 2e-2, (name, err)


@pytest.mark.parametrize("layout,M,N,K", [(0, 4096, 192, 64), (0, 37, 64, 128), (0, 1000, 256, 1024), (1, 4096, 64, 192),
                                          (1, 300, 512, 128), (2, 192, 64, 32768), (2, 1024, 256, 4096), (2, 64, 16, 100)])
def test_gemm_f32_layouts(layout, M, N, K):
    """csu_gemm_f32 (fp32 MFMA: Linear forward / input gradient / weight gradient with ordered
    token splits) vs fp64; bias + residual epilogue on layout 0; bitwise repeatable."""
    from csu import ops
    d = dev()
    g = torch.Generator().manual_seed(M + N + K + layout)
    if layout == 0:
        a, b = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g)
        bias, res = torch.randn(N, generator=g), torch.randn(M, N, generator=g)
        ref = a.double() @ b.double().T + bias.double() + res.double()
        out = ops.gemm_f32(0, a.to(d), b.to(d), M, N, K, bias=bias.to(d), resid=res.to(d))
    elif layout == 1:
        a, b = torch.randn(M, K, generator=g), torch.randn(K, N, generator=g)
        ref = a.double() @ b.double()
        out = ops.gemm_f32(1, a.to(d), b.to(d), M, N, K)
    else:
        a, b = torch.randn(K, M, generator=g), torch.randn(K, N, generator=g)
        ref = a.double().T @ b.double()
        out, asum = ops.gemm_f32(2, a.to(d), b.to(d), M, N, K, with_asum=True)
        again, asum2 = ops.gemm_f32(2, a.to(d), b.to(d), M, N, K, with_asum=True)
        assert torch.equal(out, again) and torch.equal(asum, asum2)
        assert_close(asum, a.double().sum(0), torch.float32)
    assert_close(out, ref, torch.float32)


@pytest.mark.parametrize("n,adt,bdt", [(4096 * 64, torch.bfloat16, torch.bfloat16), (1000 * 8, torch.float32, torch.bfloat16),
                                       (4096, torch.bfloat16, None)])
def test_grad_join(n, adt, bdt):
    """csu_grad_join: a + b in fp32 (exact: fp32 sum of the two inputs) plus its bf16 copy."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(n)
    a = torch.randn(n // 64, 64, device=d, generator=g).to(adt)
    b = torch.randn(n // 64, 64, device=d, generator=g).to(bdt) if bdt is not None else None
    out = ops.grad_join(a, b, torch.float32)
    ref = a.float() + (b.float() if b is not None else 0)
    assert out.dtype == torch.float32 and torch.equal(out, ref)
    assert torch.equal(out._csu_bf16, ref.bfloat16())


@pytest.mark.parametrize("n", [16 * 512 * 512, 1000, 4 * 1024 + 3, 4000, 3 * 1024 * 1000])
def test_bce_loss_vs_torch(n):
    """ops.bce_loss (nn.BCELoss mean, cswin:935) vs torch on probabilities incl. exact 0 / 1
    (the -100 log clamp) and targets in {0, 1}; deterministic."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(n)
    p = torch.rand(n, device=d, generator=g)
    p[:7] = torch.tensor([0.0, 1.0, 1e-30, 1 - 1e-7, 0.5, 1.0, 0.0], device=d)
    t = (torch.rand(n, device=d, generator=g) > 0.5).float()
    t[:7] = torch.tensor([1.0, 0.0, 0.0, 1.0, 1.0, 1.0, 0.0], device=d)
    pa = p.clone().requires_grad_(True)
    pb = p.clone().requires_grad_(True)
    la = ops.bce_loss(pa, t)
    lb = torch.nn.functional.binary_cross_entropy(pb, t)
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=0)
    la.backward()
    lb.backward()
    torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-6, atol=0)
    assert torch.equal(ops.bce_loss(p, t), ops.bce_loss(p, t))


def test_bce_loss_tiny_probabilities():
    """p in 1e-9..1e-6 with target 0: ATen's log1p(-p) term is ~p, which logf(1 - p) rounds to 0 --
    a low-loss batch (a well-trained background) must not drift from torch's loss."""
    from csu import ops
    d = dev()
    p = torch.logspace(-9, -6, 4096, device=d)
    t = torch.zeros_like(p)
    t[::7] = 1.0
    p[::7] = 1.0 - p[::7]
    la = ops.bce_loss(p, t)
    lb = torch.nn.functional.binary_cross_entropy(p, t)
    assert float(lb) > 0
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=0)


def test_pack_nhwc_image():
    """csu_pack_nhwc_bf16: fp32 NCHW image -> bf16 NHWC, channels zero-padded to 8 (bit-exact)."""
    from csu import _lib, ops
    d = dev()
    x = torch.randn(3, 3, 37, 41, device=d)
    y = torch.empty(3, 37, 41, 8, dtype=torch.bfloat16, device=d)
    _lib.check(_lib.lib().csu_pack_nhwc_bf16(3, 3, 37, 41, 8, ops.ptr(x), ops.ptr(y), ops.stream_ptr(d)), "pack")
    assert torch.equal(y[..., :3], x.permute(0, 2, 3, 1).bfloat16()) and not y[..., 3:].any()


@pytest.mark.parametrize("M,N,K", [(16384, 1024, 256), (16384, 256, 1024), (65536, 384, 128), (4096, 512, 512),
                                   (262144, 192, 64), (100, 64, 64)])
def test_linear_wgrad_deferred_batch(M, N, K, monkeypatch):
    """Deferred slab sums (tile kernels now, ONE batched reduction at the end of backward) are
    bitwise equal to the inline reduction, across several Linears in one batch."""
    from csu import ops
    monkeypatch.setattr(ops, "GROUP_WGRAD", False)
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K)
    outs = []
    for rep in range(3):   # three Linears of the same shape in one batch
        dy = (torch.randn(M, N, device=d, generator=g) * 0.1).bfloat16()
        x = torch.randn(M, K, device=d, generator=g).bfloat16()
        dw, db = ops.linear_wgrad(dy, x)
        dwd, dbd = ops.linear_wgrad(dy, x, defer=True)
        outs.append((dw.clone(), db.clone(), dwd, dbd))
    ops._wgrad_flush()
    torch.cuda.synchronize()
    assert not ops._WG_PENDING
    for dw, db, dwd, dbd in outs:
        assert torch.equal(dw, dwd) and torch.equal(db, dbd)


def test_linear_wgrad_grouped():
    """Grouped end-of-backward weight gradients (one tile launch per tile size for Linears of mixed
    shapes, then the batched slab sums) vs the per-Linear kernel (fp32 sums in another chunk order:
    rel 1e-5) and vs themselves (bitwise reproducible)."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(7)
    shapes = [(16384, 768, 256), (16384, 256, 256), (16384, 1024, 256), (16384, 256, 1024), (262144, 192, 64),
              (65536, 384, 128), (4096, 512, 512), (100, 64, 64), (262144, 64, 64), (4096, 1536, 512),
              # the C = 64 fc1 / fc2 weight gradients on the rectangular 128x64 / 64x128 group tiles
              # (WG_RECT), full and with a ragged token count
              (262144, 256, 64), (262144, 64, 256), (99999, 256, 64), (65537, 64, 128)]
    ops_in = []
    for M, N, K in shapes:
        dy = (torch.randn(M, N, device=d, generator=g) * 0.1).bfloat16()
        x = torch.randn(M, K, device=d, generator=g).bfloat16()
        ops_in.append((dy, x))
    ref = [tuple(t.clone() for t in ops.linear_wgrad(dy, x)) for dy, x in ops_in]
    runs = []
    for _ in range(2):
        res = [ops.linear_wgrad(dy, x, defer=True) for dy, x in ops_in]
        assert len(ops._WG_DEFER) == len(shapes)
        ops._wgrad_flush()
        torch.cuda.synchronize()
        assert not ops._WG_DEFER and not ops._WG_PENDING
        runs.append([(a.clone(), b.clone()) for a, b in res])
    for (dw, db), (gw, gb), (hw, hb) in zip(ref, runs[0], runs[1]):
        assert torch.equal(gw, hw) and torch.equal(gb, hb)
        for got, want in ((gw, dw), (gb, db)):
            err = float((got.double() - want.double()).norm() / want.double().norm().clamp_min(1e-30))
            assert err < 1e-5, err


@pytest.mark.parametrize("reso,C,heads,sw", [(32, 256, 8, 8), (64, 128, 4, 2), (16, 512, 16, 16)])
def test_lepe_wgrad_deferred_reduce(reso, C, heads, sw, monkeypatch):
    """LePE weight gradients reduced at the end of backward by one batched launch (several attention
    calls in one backward) are bitwise equal to the per-call reduction."""
    from csu import ops
    d = dev()
    nb = 1 if sw == reso else 2
    brs = [(reso, sw, 0), (sw, reso, C // 2)] if nb == 2 else [(reso, reso, 0)]
    geom = ops.StripeGeometry(reso, C, heads // nb, brs, 32 ** -0.5)
    g = torch.Generator(device=d).manual_seed(reso + C)
    qkvs = [torch.randn(2, reso * reso, 3 * C, device=d, generator=g).bfloat16() for _ in range(3)]
    gys = [torch.randn(2, reso * reso, C, device=d, generator=g).bfloat16() for _ in range(3)]
    w0 = [[torch.randn(C // nb, 1, 3, 3, device=d, generator=g) * 0.1 for _ in range(nb)] for _ in range(3)]
    b0 = [[torch.randn(C // nb, device=d, generator=g) * 0.1 for _ in range(nb)] for _ in range(3)]
    res = {}
    for late in (False, True):
        monkeypatch.setattr(ops, "DEFER_WGRAD", late)
        ws = [[w.clone().requires_grad_(True) for w in ww] for ww in w0]
        bs = [[b.clone().requires_grad_(True) for b in bb] for bb in b0]
        loss = sum((ops.stripe_attention(q, geom, w, b).float() * gy.float()).sum()
                   for q, gy, w, b in zip(qkvs, gys, ws, bs))
        loss.backward()
        torch.cuda.synchronize()
        assert not ops._LEPE_PENDING
        res[late] = [t.grad.clone() for ww, bb in zip(ws, bs) for t in ww + bb]
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)
    # weights shared by the three calls (the engine sums their contributions as they arrive): never
    # deferred (use counts), same result as the inline path
    res2 = {}
    for late in (False, True):
        monkeypatch.setattr(ops, "DEFER_WGRAD", late)
        ws = [w.clone().requires_grad_(True) for w in w0[0]]
        bs = [b.clone().requires_grad_(True) for b in b0[0]]
        loss = sum((ops.stripe_attention(q, geom, ws, bs).float() * gy.float()).sum() for q, gy in zip(qkvs, gys))
        loss.backward()
        torch.cuda.synchronize()
        res2[late] = [t.grad.clone() for t in ws + bs]
    for a, b in zip(res2[False], res2[True]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,H,W", [(2, 64, 64), (1, 5, 128), (3, 7, 192)])
def test_conv_c16_carafe4_encoder(B, H, W):
    """The few-channel kernels of the CARAFE4 encoder Conv2d(16, 144, 3, 1, 1) (cswin:446; csu_conv2d_ex
    cfg 21, chosen by the default dispatch for W % 64 == 0): forward (conv3_c16) and input gradient
    (conv3_c16d) vs float64 torch on the same bf16 operands, bitwise equal to the default choice;
    W % 64 != 0 is not eligible (CSU_E_ARG)."""
    import ctypes
    from csu import ops
    from csu._lib import lib, CSU_BF16
    d = dev()
    gm = ops._conv_geom(B, H, W, 16, 144, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(B * 1000 + H + W)
    x = torch.randn(B, H, W, 16, generator=g).bfloat16()
    w = (torch.randn(144, 16, 3, 3, generator=g) / 12.0).bfloat16()
    b = torch.randn(144, generator=g)
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double(), 1, 1).permute(0, 2, 3, 1)
    xd, bd = x.to(d), b.to(d)
    w_ohwi = w.permute(0, 2, 3, 1).contiguous().to(d)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for cfg in (21, -1):
        out = torch.full(ref.shape, float("nan"), dtype=torch.bfloat16, device=d)
        e = lib().csu_conv2d_ex(0, ctypes.byref(gm), CSU_BF16, xd.data_ptr(), w_ohwi.data_ptr(), bd.data_ptr(),
                                out.data_ptr(), cfg, st)
        assert e == 0, lib().csu_last_error_string()
        outs.append(out)
    torch.cuda.synchronize()
    err = float((outs[0].double().cpu() - ref).norm() / ref.norm())
    assert err < 4e-3, err
    assert torch.equal(outs[0], outs[1])
    # the input gradient (144 -> 16, conv3_c16d)
    dy = torch.randn(B, H, W, 144, generator=g).bfloat16()
    ref_d = torch.nn.functional.conv_transpose2d(dy.double().permute(0, 3, 1, 2), w.double(), None, 1, 1).permute(0, 2, 3, 1)
    w_ihwo = w.permute(1, 2, 3, 0).contiguous().to(d)
    dyd = dy.to(d)
    outs = []
    for cfg in (21, -1):
        out = torch.full(ref_d.shape, float("nan"), dtype=torch.bfloat16, device=d)
        e = lib().csu_conv2d_ex(1, ctypes.byref(gm), CSU_BF16, dyd.data_ptr(), w_ihwo.data_ptr(), None, out.data_ptr(),
                                cfg, st)
        assert e == 0, lib().csu_last_error_string()
        outs.append(out)
    torch.cuda.synchronize()
    err = float((outs[0].double().cpu() - ref_d).norm() / ref_d.norm())
    assert err < 4e-3, err
    assert torch.equal(outs[0], outs[1])
    gm2 = ops._conv_geom(1, 8, 40, 16, 144, 3, 3, 1, 1)
    out = torch.empty(1, 8, 40, 144, dtype=torch.bfloat16, device=d)
    xs = torch.zeros(1, 8, 40, 16, dtype=torch.bfloat16, device=d)
    assert lib().csu_conv2d_ex(0, ctypes.byref(gm2), CSU_BF16, xs.data_ptr(), w_ohwi.data_ptr(), bd.data_ptr(),
                               out.data_ptr(), 21, st) != 0


@pytest.mark.parametrize("C,M", [(64, 4096), (128, 1000), (256, 4160), (256, 100)])
@pytest.mark.parametrize("cfg", [1, 2])
def test_mlp_fwd_deep_ring_vs_fp64(C, M, cfg):
    """csu_mlp_fwd_ex cfg 1 / 2 (the deep-ring forward: 32-hidden weight chunks, waves split by tokens)
    vs the fp64 Mlp + residual, without and with hidden / output dropout + DropPath (same masks as
    the oracle composition); and it agrees with the per-panel kernel to bf16 rounding."""
    import ctypes
    from csu import rng
    from csu._lib import check, lib, ptr, stream_ptr
    from csu.ops import MlpDrop
    d = dev()
    torch.manual_seed(C + M + cfg)
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.randn(4 * C, device=d) * 0.1, torch.randn(C, device=d) * 0.1
    res = torch.randn(M, C, device=d)
    st = stream_ptr(d)
    X, W1, W2, B1, B2, R = (t.double().cpu() for t in (x, w1, w2, b1, b2, res))
    F = torch.nn.functional
    for drop in (False, True):
        if drop:
            snap = torch.tensor([5, 2], dtype=torch.int64, device=d)
            rps = max(1, M // 3)
            rs = rng.droppath_scale(snap, 30, 0.3, -(-M // rps))
            md = MlpDrop(snap, 21, 22, 0.3, rs, rps).c_struct()
            mh = rng.dropout_mask(snap, 21, 0.3, M * 4 * C).view(M, 4 * C).double().cpu() / 0.7
            mo = rng.dropout_mask(snap, 22, 0.3, M * C).view(M, C).double().cpu() / 0.7
            outm = mo * rs.double().cpu()[torch.arange(M) // rps].view(M, 1)
        else:
            md = MlpDrop(None, 0, 0, 0.0).c_struct()
            md.rows_per_sample = M
            mh, outm = 1.0, 1.0
        ys = []
        for c in (cfg, 0):
            y = torch.empty(M, C, device=d)
            check(lib().csu_mlp_fwd_ex(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y),
                                       ctypes.byref(md), c, st), "mlp_fwd_ex")
            ys.append(y)
        torch.cuda.synchronize()
        ref = R + outm * ((F.gelu(X @ W1.T + B1) * mh) @ W2.T + B2)
        err = float((ys[0].double().cpu() - ref).norm() / (ref - R).norm())
        assert err < 1e-2, (drop, err)
        d01 = float((ys[0] - ys[1]).double().norm() / (ys[1] - res).double().norm())
        assert d01 < 1e-2, (drop, d01)


@pytest.mark.parametrize("C,M", [(64, 4096), (128, 1000), (256, 4160), (256, 100)])
@pytest.mark.parametrize("cfg", [1, 2])
def test_mlp_bwd_deep_ring_vs_fp64(C, M, cfg):
    """csu_mlp_bwd_ex cfg 1 / 2 (the deep-ring backward) vs the fp64 composition: dh = (dy W2)
    gelu'(h) m_h, g = gelu(h) m_h, dx = dh W1, without and with the hidden dropout mask; and it agrees
    with the per-panel backward (cfg 0) to bf16 rounding."""
    import ctypes
    from csu import rng
    from csu._lib import check, lib, ptr, stream_ptr
    from csu.ops import MlpDrop
    d = dev()
    torch.manual_seed(C + M + cfg + 7)
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1 = torch.randn(4 * C, device=d) * 0.1
    dy = torch.randn(M, C, device=d).bfloat16()
    st = stream_ptr(d)
    X, W1, W2, B1, DY = (t.double().cpu() for t in (x, w1, w2, b1, dy))
    F = torch.nn.functional
    for drop in (False, True):
        if drop:
            snap = torch.tensor([9, 4], dtype=torch.int64, device=d)
            md = MlpDrop(snap, 31, 32, 0.25).c_struct()
            md.rows_per_sample = max(1, M // 2)
            mh = rng.dropout_mask(snap, 31, 0.25, M * 4 * C).view(M, 4 * C).double().cpu() / 0.75
        else:
            md = MlpDrop(None, 0, 0, 0.0).c_struct()
            md.rows_per_sample = M
            mh = torch.ones(M, 4 * C, dtype=torch.float64)
        outs = []
        for c in (cfg, 0):
            dh = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
            g = torch.empty_like(dh)
            dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
            check(lib().csu_mlp_bwd_ex(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx),
                                       ctypes.byref(md), c, st), "mlp_bwd_ex")
            outs.append((dh, g, dx))
        torch.cuda.synchronize()
        h = (X @ W1.T + B1).requires_grad_(True)
        gr = F.gelu(h)
        gr.backward((DY @ W2) * mh)
        refs = (h.grad, gr.detach() * mh, h.grad @ W1)
        for name, got, other, ref in zip(("dh", "g", "dx"), outs[0], outs[1], refs):
            err = float((got.double().cpu() - ref).norm() / ref.norm())
            assert err < 1e-2, (drop, name, err)
            d01 = float((got - other).double().norm() / other.double().norm())
            assert d01 < 1e-2, (drop, name, d01)


def _frag_ref(w: torch.Tensor) -> torch.Tensor:
    """Fragment order of csu_frag_layout_batch (include/csu.h): [rows/32][cols/16][64 lanes][8],
    lane = row % 32 + 32 * ((k % 16) // 8)."""
    R, Cc = w.shape
    t = w.reshape(R // 32, 32, Cc // 16, 2, 8)          # [nt][r][s][half][8]
    return t.permute(0, 2, 3, 1, 4).reshape(-1)         # [nt][s][half][r][8] = [nt][s][lane][8]


@pytest.mark.parametrize("rows,cols", [(32, 16), (768, 256), (128, 384), (256, 768)])
def test_frag_layout_batch(rows, cols):
    import ctypes
    import numpy as np
    from csu._lib import lib
    d = dev()
    g = torch.Generator(device=d).manual_seed(rows + cols)
    ws = [torch.randn(rows, cols, device=d, generator=g).bfloat16(), torch.randn(64, 128, device=d, generator=g).bfloat16()]
    outs = [torch.empty_like(w).view(-1) for w in ws]
    rec = np.zeros(len(ws), dtype=[("src", "<u8"), ("dst", "<u8"), ("rows", "<i4"), ("cols", "<i4"), ("chunk0", "<i8")])
    c0 = 0
    for k, (w, o) in enumerate(zip(ws, outs)):
        rec[k] = (w.data_ptr(), o.data_ptr(), w.shape[0], w.shape[1], c0)
        c0 += w.numel() // 8
    items = torch.frombuffer(bytearray(rec.tobytes()), dtype=torch.uint8).to(d)
    assert lib().csu_frag_layout_batch(ctypes.c_void_p(items.data_ptr()), len(ws), c0, None) == 0
    torch.cuda.synchronize()
    for w, o in zip(ws, outs):
        assert torch.equal(o, _frag_ref(w))


GEMM_WS_SHAPES = [(16384, 768, 256), (16384, 256, 768), (16384, 256, 256), (1024, 384, 128), (65536, 128, 384),
                  (192, 128, 128),
                  # stage-1 shapes (C = 64): two 64-token groups per workgroup, direct fragment loads
                  (262144, 192, 64), (1024, 64, 64), (384, 192, 64)]


@pytest.mark.parametrize("M,N,K", GEMM_WS_SHAPES)
@pytest.mark.parametrize("mode", ["bf16_bias", "f32", "resid"])
def test_gemm_ws_vs_fp64(M, N, K, mode):
    """csu_gemm_ws (weight-streaming token GEMM) against an fp64 GEMM of the same bf16 operands:
    fp32 out within 1e-5 of max |ref| (fp32 accumulation), bf16 out within bf16 rounding."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K)
    ldx = K + 64 if M <= 1024 else K          # a strided token operand on the small shapes
    xfull = torch.randn(M, ldx, device=d, generator=g).bfloat16()
    x = xfull[:, :K]
    w = (torch.randn(N, K, device=d, generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=d, generator=g) if mode != "f32" else None
    resid = torch.randn(M, N, device=d, generator=g) if mode == "resid" else None
    odt = torch.bfloat16 if mode == "bf16_bias" else torch.float32
    out = ops.gemm_ws(x, _frag_ref(w).contiguous(), N, odt, bias=bias, resid=resid)
    torch.cuda.synchronize()
    ref = x.double() @ w.double().t()
    if bias is not None:
        ref = ref + bias.double()
    if resid is not None:
        ref = ref + resid.double()
    err = float((out.double() - ref).abs().max())
    scale = float(ref.abs().max())
    if odt == torch.float32:
        assert err <= 1e-5 * scale, (err, scale)
    else:
        assert err <= 2 ** -8 * scale + 1e-6, (err, scale)
    with pytest.raises(Exception):
        ops.gemm_ws(x[:M - 8], _frag_ref(w).contiguous(), N, odt)   # M % 64 != 0: refused
    if N in (64, 192):
        with pytest.raises(Exception):
            ops.gemm_ws(x[:M - 64], _frag_ref(w).contiguous(), N, odt)   # two token groups: M % 128 != 0


@pytest.mark.parametrize("M,C", [(16384, 256), (65536, 128), (262144, 64), (384, 64), (1024, 128)])
def test_gemm_ws_ln_vs_fp64(M, C):
    """csu_gemm_ws_ln (proj + residual with norm2 in the epilogue, cswin:366-368): the fp32 output
    equals csu_gemm_ws's residual epilogue bit for bit; the LayerNorm output / mean / rstd match an
    fp64 LayerNorm of that output to bf16 / fp32 rounding."""
    from csu import ops
    from csu._lib import lib, ptr, stream_ptr
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + C)
    x = torch.randn(M, C, device=d, generator=g).bfloat16()
    w = (torch.randn(C, C, device=d, generator=g) / C ** 0.5).bfloat16()
    bias = torch.randn(C, device=d, generator=g)
    res = torch.randn(M, C, device=d, generator=g) * 2 + 0.5
    gam = torch.randn(C, device=d, generator=g) * 0.5 + 1
    bet = torch.randn(C, device=d, generator=g) * 0.1
    wf = _frag_ref(w).contiguous()
    ref_y = ops.gemm_ws(x, wf, C, torch.float32, bias=bias, resid=res)
    assert lib().csu_gemm_ws_ln_supported(M, C, C)
    y = torch.empty(M, C, device=d)
    h = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    mean = torch.empty(M, device=d)
    rstd = torch.empty(M, device=d)
    rc = lib().csu_gemm_ws_ln(M, C, ptr(x), C, ptr(wf), ptr(bias), ptr(res), ptr(y), ptr(gam), ptr(bet), 1e-5, ptr(h),
                              ptr(mean), ptr(rstd), stream_ptr(x.device))
    torch.cuda.synchronize()
    assert rc == 0
    assert torch.equal(y, ref_y)
    y64 = y.double()
    mu = y64.mean(-1)
    var = y64.var(-1, unbiased=False)
    h64 = (y64 - mu[:, None]) / torch.sqrt(var[:, None] + 1e-5) * gam.double() + bet.double()
    assert float((mean.double() - mu).abs().max()) <= 1e-6 * float(y64.abs().max())
    assert float((rstd.double() / torch.rsqrt(var + 1e-5) - 1).abs().max()) <= 1e-5
    assert float((h.double() - h64).abs().max()) <= 2 ** -8 * float(h64.abs().max())
    assert not lib().csu_gemm_ws_ln_supported(M - 32, C, C)


def test_linear_residual_ln_next_matches_unfused(monkeypatch):
    """proj + residual with norm2 fused (ops.linear_residual(ln_next=...)) feeding layer_norm_fork:
    the same forward values (bf16 rounding) and gradients (fp32 sums) as the unfused launch pair."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(5)
    B, L, C = 2, 1024, 128
    res0 = torch.randn(B, L, C, device=d, generator=g)
    x0 = torch.randn(B, L, C, device=d, generator=g).bfloat16()
    lin = torch.nn.Linear(C, C).to(d)
    ln = torch.nn.LayerNorm(C).to(d)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    cache = ops.CastCache()
    cache.refresh([lin.weight], torch.bfloat16)
    cache.refresh_frag()
    assert cache.get_frag(lin.weight) is not None
    outs = {}
    try:
        ops.set_cast_cache(cache)
        for fused in (False, True):
            monkeypatch.setattr(ops, "FUSE_PROJ_LN", fused)
            for p in (*lin.parameters(), *ln.parameters()):
                p.grad = None
            res, x = res0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
            y = ops.linear_residual(res, x, lin.weight, lin.bias, ln_next=(ln.weight, ln.bias, ln.eps))
            assert hasattr(y, "_csu_ln") == fused
            yb, h = ops.layer_norm_fork(y, ln.weight, ln.bias, ln.eps, torch.bfloat16)
            loss = (h.float() * torch.linspace(-1, 1, C, device=d)).sum() + (yb.float() ** 2).sum() * 1e-3
            loss.backward()
            torch.cuda.synchronize()
            grads = [res.grad, x.grad, lin.weight.grad, lin.bias.grad, ln.weight.grad, ln.bias.grad]
            outs[fused] = (yb.detach(), h.detach(), [gr.detach().clone() for gr in grads])
    finally:
        ops.set_cast_cache(None)
    (y0, h0, g0), (y1, h1, g1) = outs[False], outs[True]
    assert torch.equal(y0, y1)
    assert float((h0.float() - h1.float()).abs().max()) <= 2 ** -7 * float(h0.float().abs().max())
    for a, b in zip(g0, g1):
        err = float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
        assert err < 2e-2, err


@pytest.mark.parametrize("C", [64, 128, 256])
@pytest.mark.parametrize("drop", [False, True])
def test_mlp_fwd_ln_next(C, drop):
    """csu_mlp_fwd_ln: the fused Mlp forward that also applies the next block's norm1 to its output
    (cswin:357): the output equals csu_mlp_fwd_dp's bit for bit, the LayerNorm output / mean / rstd
    equal an fp64 LayerNorm of that output to bf16 / fp32 rounding; layer_norm_fork then uses them
    without a LayerNorm launch."""
    from csu import ops, rng
    d = dev()
    g = torch.Generator(device=d).manual_seed(C + int(drop))
    B, L = 2, 1024
    x = torch.randn(B, L, C, device=d, generator=g).bfloat16()
    res = torch.randn(B, L, C, device=d, generator=g)
    fc1, fc2 = torch.nn.Linear(C, 4 * C).to(d), torch.nn.Linear(4 * C, C).to(d)
    ln = torch.nn.LayerNorm(C).to(d)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    md = None
    if drop:
        snap = rng.snapshot(d)
        md = ops.MlpDrop(snap, 7, 8, 0.2, torch.tensor([1.25, 0.0], device=d), L)
    y0 = ops.mlp_residual(res, x, fc1, fc2, md)
    y1 = ops.mlp_residual(res, x, fc1, fc2, md, ln_next=(ln.weight, ln.bias, ln.eps))
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    pre = y1._csu_ln
    yd = y1.double().view(-1, C)
    mu = yd.mean(-1)
    var = ((yd - mu[:, None]) ** 2).mean(-1)
    ref = (yd - mu[:, None]) / torch.sqrt(var[:, None] + ln.eps) * ln.weight.double() + ln.bias.double()
    torch.testing.assert_close(pre[4].double(), mu, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(pre[5].double(), 1 / torch.sqrt(var + ln.eps), rtol=1e-4, atol=0)
    assert float((pre[3].double().view(-1, C) - ref).abs().max()) <= 2 ** -7 * float(ref.abs().max())
    calls = []
    real = ops._launch
    ops._launch = lambda name, *a, **k: (calls.append(name), real(name, *a, **k))[1]
    try:
        xa, h = ops.layer_norm_fork(y1, ln.weight, ln.bias, ln.eps, torch.bfloat16)
    finally:
        ops._launch = real
    assert "layernorm_fwd" not in calls and torch.equal(h.view(-1), pre[3].view(-1))
    # an in-place change of the output after the launch invalidates the attached LayerNorm
    # (autograd itself forbids using an in-place-modified view output of a custom Function with grad
    # enabled; the stale-stash case is a no_grad one)
    calls.clear()
    ops._launch = lambda name, *a, **k: (calls.append(name), real(name, *a, **k))[1]
    try:
        with torch.no_grad():
            y1.detach().mul_(1.0)     # shares y1's version counter
            ops.layer_norm_fork(y1, ln.weight, ln.bias, ln.eps, torch.bfloat16)
    finally:
        ops._launch = real
    assert "layernorm_fwd" in calls


@pytest.mark.parametrize("C", [128, 256])
def test_ln_linear_ws_vs_unfused(C):
    """_LnLinearWsFn (norm1 -> qkv with the LayerNorm backward in csu_gemm_ws_lnbwd's epilogue) against
    the unfused layer_norm_fork + linear: outputs and every gradient (dx, dgamma, dbeta, dW, db) agree
    to bf16 rounding (the fused path feeds the LayerNorm backward dh in fp32, the unfused one rounds it
    to bf16 first)."""
    from csu import ops
    d = dev()
    torch.manual_seed(C)
    B, L = 2, 1024
    x0 = torch.randn(B, L, C, device=d)
    ln = torch.nn.LayerNorm(C).to(d)
    lin = torch.nn.Linear(C, 3 * C).to(d)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
        lin.bias.uniform_(-0.1, 0.1)
    G = torch.randn(B, L, 3 * C, device=d)
    R = torch.randn(B, L, C, device=d)

    def run(fused):
        for p in (*ln.parameters(), *lin.parameters()):
            p.grad = None
        x = x0.clone().requires_grad_(True)
        if fused:
            wc = lin.weight.detach().bfloat16()
            wf, wtf = _frag_ref(wc).contiguous(), _frag_ref(wc.t().contiguous()).contiguous()
            xa, y = ops._LnLinearWsFn.apply(x, ln.weight, ln.bias, lin.weight, lin.bias, ln.eps, wf, wtf, None)
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                xa, h = ops.layer_norm_fork(x, ln.weight, ln.bias, ln.eps, torch.bfloat16)
                y = ops.linear(h, lin.weight, lin.bias)
        ((y.float() * G).sum() + (xa * R).sum()).backward()
        torch.cuda.synchronize()
        return [y.detach().float(), x.grad, ln.weight.grad, ln.bias.grad, lin.weight.grad, lin.bias.grad]

    a, b = run(True), run(False)
    for name, u, v in zip(["y", "dx", "dgamma", "dbeta", "dW", "db"], a, b):
        rel = float((u - v).norm() / v.norm())
        assert rel < 1e-2, (name, rel)


def _e4m3_rows(w):
    """Per-row power-of-two e4m3 quantisation (the fp8 format's, oracle/fp8_ref.py): bytes q, scales s,
    and the exact bf16 dequantisation q * s."""
    amax = w.float().abs().amax(1).clamp_min(1e-30)
    s = torch.exp2(torch.ceil(torch.log2(amax / 448.0)))
    q = (w.float() / s[:, None]).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), s.contiguous(), (q.float() * s[:, None]).bfloat16()


def _frag8(q, transpose):
    """csu_frag8_layout_batch of one e4m3 (N, K) matrix."""
    import numpy as np
    from csu._lib import check, lib, ptr, stream_ptr
    N, K = q.shape
    out = torch.empty(N * K, dtype=torch.uint8, device=q.device)
    dt = np.dtype([("src", "<u8"), ("dst", "<u8"), ("N", "<i4"), ("K", "<i4"), ("transpose", "<i4"), ("pad", "<i4"),
                   ("block0", "<i8")])
    it = torch.frombuffer(bytearray(np.array([(q.data_ptr(), out.data_ptr(), N, K, int(transpose), 0, 0)], dtype=dt)
                                    .tobytes()), dtype=torch.uint8).to(q.device)
    check(lib().csu_frag8_layout_batch(ptr(it), 1, N * K // 64, stream_ptr(q.device)), "frag8")
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("M,N,K,mode", [(16384, 768, 256, "bf16_bias"), (4096, 256, 256, "resid"), (4096, 384, 128, "f32"),
                                        (8192, 192, 64, "bf16_bias"), (1024, 64, 64, "resid"),
                                        (4096, 256, 768, "dgrad"), (4096, 128, 384, "dgrad"), (2048, 128, 128, "dgrad"),
                                        (2048, 64, 64, "dgrad")])
def test_gemm_ws_e4m3_bitwise_vs_dequantised(M, N, K, mode):
    """fp8 weight format (BASELINE config 5): csu_gemm_ws_e4m3 streams e4m3 weight fragments and widens
    them to bf16 in registers -- bitwise equal to csu_gemm_ws on the exact bf16 dequantisation, for x W^T
    (scale_mode 1: per-column scales in the epilogue) and the input gradient dy W (scale_mode 2: the
    weight is W^T, per-k scales on the token panel)."""
    from csu import ops
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + N + K)
    x = torch.randn(M, K, device=d, generator=g).bfloat16()
    qa, _, _ = _e4m3_rows(torch.randn(N, K, device=d, generator=g))
    assert torch.equal(_frag8(qa, False), _frag_ref(qa)) and torch.equal(_frag8(qa, True), _frag_ref(qa.t().contiguous()))
    if mode == "dgrad":
        # the Linear's weight is Wl (K_l = N, N_l = K): out (M, N) = dy (M, K) @ Wl, Wl = q s (K x N rows)
        wl = torch.randn(K, N, device=d, generator=g) / N ** 0.5
        q, s, wd = _e4m3_rows(wl)
        ref = ops.gemm_ws(x, _frag_ref(wd.t().contiguous()).contiguous(), N, torch.bfloat16)
        got = ops.gemm_ws(x, (_frag8(q, True), s, 2), N, torch.bfloat16)
    else:
        w = torch.randn(N, K, device=d, generator=g) / K ** 0.5
        q, s, wd = _e4m3_rows(w)
        bias = torch.randn(N, device=d, generator=g) if mode != "f32" else None
        resid = torch.randn(M, N, device=d, generator=g) if mode == "resid" else None
        odt = torch.bfloat16 if mode == "bf16_bias" else torch.float32
        ref = ops.gemm_ws(x, _frag_ref(wd).contiguous(), N, odt, bias=bias, resid=resid)
        got = ops.gemm_ws(x, (_frag8(q, False), s, 1), N, odt, bias=bias, resid=resid)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), float((got.double() - ref.double()).abs().max())


@pytest.mark.parametrize("M,C", [(16384, 256), (4096, 128), (8192, 64)])
def test_gemm_ws_ln_e4m3_bitwise_vs_dequantised(M, C):
    """csu_gemm_ws_ln_e4m3 (proj + residual + norm2 on e4m3 weights) == csu_gemm_ws_ln on the
    dequantised bf16 weight, every output bit for bit."""
    from csu._lib import lib, ptr, stream_ptr
    d = dev()
    g = torch.Generator(device=d).manual_seed(M + C + 1)
    x = torch.randn(M, C, device=d, generator=g).bfloat16()
    q, s, wd = _e4m3_rows(torch.randn(C, C, device=d, generator=g) / C ** 0.5)
    bias = torch.randn(C, device=d, generator=g)
    res = torch.randn(M, C, device=d, generator=g) * 2 + 0.5
    gam = torch.randn(C, device=d, generator=g) * 0.5 + 1
    bet = torch.randn(C, device=d, generator=g) * 0.1
    outs = []
    for e4 in (False, True):
        y = torch.empty(M, C, device=d)
        h = torch.empty(M, C, device=d, dtype=torch.bfloat16)
        mean, rstd = torch.empty(M, device=d), torch.empty(M, device=d)
        if e4:
            f8 = _frag8(q, False)
            rc = lib().csu_gemm_ws_ln_e4m3(M, C, ptr(x), C, ptr(f8), ptr(s), ptr(bias), ptr(res), ptr(y), ptr(gam), ptr(bet),
                                           1e-5, ptr(h), ptr(mean), ptr(rstd), stream_ptr(d))
        else:
            wf = _frag_ref(wd).contiguous()
            rc = lib().csu_gemm_ws_ln(M, C, ptr(x), C, ptr(wf), ptr(bias), ptr(res), ptr(y), ptr(gam), ptr(bet), 1e-5,
                                      ptr(h), ptr(mean), ptr(rstd), stream_ptr(d))
        torch.cuda.synchronize()
        assert rc == 0
        outs.append((y, h, mean, rstd))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
