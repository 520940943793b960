"""Stage-3 stripe attention fwd+bwd repeated eagerly (rocprofv3 PMC passes / kernel traces)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda")
B, reso, C, heads, sw = int(os.environ.get("BS", "16")), int(os.environ.get("RESO", "32")), 256, 8, 8
geom = ops.StripeGeometry(reso, C, heads // 2, [(reso, sw, 0), (sw, reso, C // 2)], 32 ** -0.5)
qkv = torch.randn(B, reso * reso, 3 * C, device=d, dtype=torch.bfloat16, requires_grad=True)
ws = [torch.randn(C // 2, 1, 3, 3, device=d, requires_grad=True) for _ in range(2)]
bs = [torch.randn(C // 2, device=d, requires_grad=True) for _ in range(2)]
for _ in range(20):
    out = ops.stripe_attention(qkv, geom, ws, bs)
    out.backward(torch.ones_like(out))
torch.cuda.synchronize()
