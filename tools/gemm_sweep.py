"""K / M sweeps of csu_gemm_ex (plain bf16 out) to separate per-tile fixed cost from main-loop rate."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
from gemm_probe2 import timeit
d = torch.device("cuda")
bf = torch.bfloat16
cfgs = [int(c) for c in os.environ.get("CFGS", "12,15,2").split(",")]
for M, N in ((16384, 1024), (65536, 256)):
    for K in (64, 128, 256, 512, 1024, 2048, 4096):
        a = torch.randn(M, K, device=d, dtype=bf)
        w = torch.randn(N, K, device=d, dtype=bf) * 0.05
        ts = [timeit(lambda: ops.gemm(a, w, False, bf, cfg=c)) for c in cfgs]
        tt = timeit(lambda: torch.nn.functional.linear(a, w))
        fl = 2 * M * N * K
        print(f"M={M} N={N} K={K:5d}: " + "  ".join(f"c{c} {t:7.1f}us {fl / t / 1e6:5.0f}TF" for c, t in zip(cfgs, ts))
              + f"  | hipBLASLt {tt:7.1f}us {fl / tt / 1e6:5.0f}TF", flush=True)
