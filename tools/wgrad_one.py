"""Run one linear-wgrad shape repeatedly (PMC passes): python wgrad_one.py M N K"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
M, N, K = (int(v) for v in sys.argv[1:4])
d = torch.device("cuda")
dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
for _ in range(30):
    ops.linear_wgrad(dy, x)
torch.cuda.synchronize()
