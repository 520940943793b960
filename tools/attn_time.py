"""Stage-3 (and stage-1/2) stripe attention fwd / bwd kernel times with HIP events (eager)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda")


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


# NOLEPE=1: LePE weights without gradients (no weight-gradient partials in the backward)
LEPE_GRAD = os.environ.get("NOLEPE", "0") != "1"
SHAPES = [(16, 32, 256, 8, 8), (16, 64, 128, 4, 2), (16, 128, 64, 2, 1), (16, 16, 512, 16, 16),
          (4, 64, 256, 8, 8), (4, 256, 64, 2, 1)]
if os.environ.get("ONLY"):
    SHAPES = [SHAPES[int(i)] for i in os.environ["ONLY"].split(",")]
for B, reso, C, heads, sw in SHAPES:
    nb = 1 if sw == reso else 2
    brs = [(reso, sw, 0), (sw, reso, C // 2)] if nb == 2 else [(reso, reso, 0)]
    geom = ops.StripeGeometry(reso, C, heads // nb, brs, 32 ** -0.5)
    qkv = torch.randn(B, reso * reso, 3 * C, device=d, dtype=torch.bfloat16, requires_grad=True)
    ws = [torch.randn(C // nb, 1, 3, 3, device=d, requires_grad=LEPE_GRAD) for _ in range(nb)]
    bs = [torch.randn(C // nb, device=d, requires_grad=LEPE_GRAD) for _ in range(nb)]
    g = torch.randn(B, reso * reso, C, device=d, dtype=torch.bfloat16)
    f = t(lambda: ops.stripe_attention(qkv, geom, ws, bs))
    def fb():
        out = ops.stripe_attention(qkv, geom, ws, bs)
        out.backward(g)
    tb = t(fb)
    print(f"B {B} reso {reso} C {C} sw {sw}: fwd {f:7.1f} us  fwd+bwd {tb:7.1f} us  bwd {tb - f:7.1f} us", flush=True)
