"""Stripe attention bf16 vs fp64 oracle: per-output relative errors (debug helper)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from oracle import cswin_ref as O
from csu import ops

d = torch.device("cuda:0")
for case in [(16, 0, 1, 32, 1, 2), (8, -1, 8, 128, 4, 2), (32, 0, 8, 128, 4, 1)]:
    reso, idx, sw, cb, heads, B = case
    g = torch.Generator().manual_seed(0)
    L = reso * reso
    qkv = torch.randn(B, L, 3 * cb, generator=g).bfloat16()
    w = torch.randn(cb, 1, 3, 3, generator=g) * 0.3
    b = torch.randn(cb, generator=g) * 0.1
    gout = torch.randn(B, L, cb, generator=g).bfloat16()
    hs, ws = O.stripe_geometry(reso, idx, sw)
    scale = (cb // heads) ** -0.5
    q64 = qkv.double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = O.lepe_attention(q64[..., :cb], q64[..., cb:2 * cb], q64[..., 2 * cb:], reso, hs, ws, heads, w64, b64, scale)
    ref.backward(gout.double())
    qd = qkv.to(d).requires_grad_(True)
    wd, bd = w.to(d).requires_grad_(True), b.to(d).requires_grad_(True)
    geom = ops.StripeGeometry(reso, cb, heads, [(hs, ws, 0)], scale)
    out = ops.stripe_attention(qd, geom, [wd], [bd])
    out.backward(gout.to(d))
    torch.cuda.synchronize()
    rel = lambda a, b: float((a.double().cpu() - b).norm() / b.norm())
    print(case, "out", rel(out, ref), "dq", rel(qd.grad[..., :cb], q64.grad[..., :cb]), "dk", rel(qd.grad[..., cb:2 * cb], q64.grad[..., cb:2 * cb]),
          "dv", rel(qd.grad[..., 2 * cb:], q64.grad[..., 2 * cb:]), "dw", rel(wd.grad, w64.grad), flush=True)
