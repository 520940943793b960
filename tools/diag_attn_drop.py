"""Per-part error of the stripe-attention gradients (dQ / dK / dV, per image) vs the oracle under
the same dropout masks, for one geometry (debugging aid).
    python tools/diag_attn_drop.py reso C heads split last B p"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]

import torch  # noqa: E402

from oracle import cswin_ref as O  # noqa: E402


def main():
    reso, C, heads, split, last, B = (int(v) for v in sys.argv[1:7])
    p = float(sys.argv[7])
    from csu import ops, rng
    d = torch.device("cuda:0")
    torch.manual_seed(0)
    L = reso * reso
    if last:
        branches, nh, cb = [(reso, reso, 0)], heads, C
    else:
        branches, nh, cb = [(reso, split, 0), (split, reso, C // 2)], heads // 2, C // 2
    scale = (cb // nh) ** -0.5
    geom = ops.StripeGeometry(reso, C, nh, branches, scale, head_dim=cb // nh)
    qkv = torch.randn(B, L, 3 * C, device=d).bfloat16()
    ws = [torch.randn(cb, 1, 3, 3, device=d) * 0.2 for _ in branches]
    bs = [torch.randn(cb, device=d) * 0.1 for _ in branches]
    snap = torch.tensor([77, 1], dtype=torch.int64, device=d)
    q = qkv.clone().requires_grad_(True)
    out = ops.stripe_attention(q, geom, ws, bs, ops.AttnDrop(snap, 40, p) if p > 0 else None)
    g = torch.randn(B, L, C, device=d)
    out.float().backward(g)
    Q = qkv.double().cpu().requires_grad_(True)
    outs = []
    for i, (hs, wsp, off) in enumerate(branches):
        def mask(shape, i=i):
            Bw, H, N, _ = shape
            npad = -(-N // 32) * 32
            m = rng.dropout_mask(snap, 40 + i, p, Bw * H * N * npad).view(Bw, H, N, npad)[..., :N]
            return m.double().cpu() / (1 - p)
        outs.append(O.lepe_attention(Q[..., off:off + cb], Q[..., C + off:C + off + cb], Q[..., 2 * C + off:2 * C + off + cb],
                                     reso, hs, wsp, nh, ws[i].double().cpu(), bs[i].double().cpu(), scale,
                                     attn_mask=mask if p > 0 else None))
    ref = torch.cat(outs, -1)
    ref.backward(g.double().cpu())

    def rel(a, b):
        return float((a.double().cpu() - b).norm() / b.norm())
    print("out", rel(out.detach(), ref.detach()))
    for b in range(B):
        for name, sl in (("dQ", slice(0, C)), ("dK", slice(C, 2 * C)), ("dV", slice(2 * C, 3 * C))):
            a, r = q.grad[b, :, sl], Q.grad[b, :, sl]
            err = (a.double().cpu() - r).abs().amax(-1)
            bad = (err > 0.05 * r.abs().max()).nonzero().flatten().tolist()
            print(f"b{b} {name} rel {rel(a, r):.4f}  rows with large error: {len(bad)} {bad[:12]}")


if __name__ == "__main__":
    main()
