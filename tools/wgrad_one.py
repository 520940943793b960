"""Run one linear-wgrad shape repeatedly (PMC passes): python wgrad_one.py M N K [tn tk chunks]"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu._lib import check, lib, ptr, stream_ptr
M, N, K = (int(v) for v in sys.argv[1:4])
tn, tk, ch = (int(v) for v in (sys.argv[4:7] if len(sys.argv) > 6 else (0, 0, 0)))
d = torch.device("cuda")
dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
L = lib()
n = L.csu_linear_wgrad_tuned_workspace(M, N, K, tn, tk, ch)
ws = torch.empty(max(n, 16), dtype=torch.uint8, device=d)
out = torch.empty(N * K + N, device=d)
for _ in range(30):
    check(L.csu_linear_wgrad_tuned(M, N, K, 1, ptr(dy), ptr(x), ptr(out), ptr(ws), n, tn, tk, ch, stream_ptr(d)), "wgrad")
torch.cuda.synchronize()
