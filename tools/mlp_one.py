"""A few csu_mlp_fwd / csu_mlp_bwd launches per encoder-stage shape (for rocprofv3 PMC passes)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd"))
import torch
from csu._lib import check, lib, ptr, stream_ptr

d = torch.device("cuda:0")
st = stream_ptr(d)
for C, M in [(64, 262144), (128, 65536), (256, 16384)]:
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.zeros(4 * C, device=d), torch.zeros(C, device=d)
    res, y = torch.randn(M, C, device=d), torch.empty(M, C, device=d)
    dy = torch.randn(M, C, device=d).bfloat16()
    dh, g = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16), torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    for _ in range(3):
        check(lib().csu_mlp_fwd(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), st), "f")
        check(lib().csu_mlp_bwd(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx), st), "b")
    torch.cuda.synchronize()
print("ok")
