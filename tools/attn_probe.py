"""Per-stage timing of the stripe-attention kernels at the 512x512 B16 shapes (HIP events)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
import torch
from csu import ops

d = torch.device("cuda")
B = int(os.environ.get("BS", "16"))
img = int(os.environ.get("IMG", "512"))
stages = [(img // 4, 64, 2, 1, False), (img // 8, 128, 4, 2, False), (img // 16, 256, 8, 8, False), (img // 32, 512, 16, 8, True)]


def bench(fn, n=10):
    """GPU time per call: n calls captured in one HIP graph, replayed (no host launch overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(); fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * n) * 1e3


for reso, C, heads, sw, last in stages:
    last = last or reso == sw
    if last:
        geom = ops.StripeGeometry(reso, C, heads, [(reso, reso, 0)], 32 ** -0.5)
        nb = 1
    else:
        geom = ops.StripeGeometry(reso, C, heads // 2, [(reso, sw, 0), (sw, reso, C // 2)], 32 ** -0.5)
        nb = 2
    L = reso * reso
    qkv = torch.randn(B, L, 3 * C, device=d, dtype=torch.bfloat16, requires_grad=True)
    cb = C // nb
    ws = [torch.randn(cb, 1, 3, 3, device=d, requires_grad=True) for _ in range(nb)]
    bs = [torch.randn(cb, device=d, requires_grad=True) for _ in range(nb)]
    out = ops.stripe_attention(qkv, geom, ws, bs)
    g = torch.randn_like(out)
    t_f = bench(lambda: ops.stripe_attention(qkv, geom, ws, bs))
    t_fb = bench(lambda: torch.autograd.grad(ops.stripe_attention(qkv, geom, ws, bs), [qkv] + ws + bs, g))
    nbytes, flops = ops._stripe_fwd_work(geom, B, 2)
    print(f"reso {reso:4d} C {C:4d} N {geom.branches[0][0] * geom.branches[0][1]:5d}: fwd {t_f:7.1f}us "
          f"({nbytes / t_f / 1e3:6.0f} GB/s, {flops / t_f / 1e6:6.1f} TF/s)  fwd+bwd {t_fb:7.1f}us  bwd~{t_fb - t_f:7.1f}us",
          flush=True)
