"""Which output elements of csu_gemm_ex are wrong, per configuration (debug aid)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda")
for (M, N, K) in ((1000, 64, 64), (128, 64, 64), (64, 64, 64), (4096, 256, 256)):
    g = torch.Generator(device=d).manual_seed(0)
    a = torch.randn(M, K, device=d, generator=g).bfloat16()
    w = (torch.randn(N, K, device=d, generator=g) * 0.1).bfloat16()
    ref = a.float() @ w.float().t()
    for cfg in (1, 10, 11, 12, 13, 14, 15):
        out = ops.gemm(a, w, False, torch.float32, cfg=cfg)
        bad = (out - ref).abs() > 1e-2 * ref.abs().max()
        rows = bad.any(1).nonzero().flatten().tolist()
        cols = bad.any(0).nonzero().flatten().tolist()
        print(f"M={M} N={N} K={K} cfg={cfg}: bad {int(bad.sum())} rows {rows[:8]}..{len(rows)} cols {cols[:40]}", flush=True)
