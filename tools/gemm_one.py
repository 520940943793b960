"""Run one token-GEMM shape repeatedly (for rocprofv3 PMC passes): python gemm_one.py M K N cfg [epi]."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
M, K, N, cfg = (int(v) for v in sys.argv[1:5])
epi = sys.argv[5] if len(sys.argv) > 5 else "plain"
d = torch.device("cuda")
a = torch.randn(M, K, device=d, dtype=torch.bfloat16)
w = torch.randn(N, K, device=d, dtype=torch.bfloat16) * 0.05
b = torch.randn(N, device=d)
for _ in range(30):
    if epi == "gout":
        ops.gemm(a, w, False, torch.bfloat16, bias=b, gelu_out=True, cfg=cfg)
    else:
        ops.gemm(a, w, False, torch.bfloat16, bias=b, cfg=cfg)
torch.cuda.synchronize()
