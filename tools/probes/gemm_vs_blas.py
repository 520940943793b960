"""Time csu's token GEMM (ops.gemm, gemm4) against torch's hipBLASLt for the stage-2/3 token-GEMM
shapes of the 512x512 B16 step (a calibration point for the achievable rate, not a product path).
    python tools/probes/gemm_vs_blas.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
from csu import ops  # noqa: E402


def t_us(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


d = torch.device("cuda")
for M, N, K in [(16384, 768, 256), (16384, 256, 768), (16384, 256, 256), (16384, 1024, 256), (16384, 256, 1024),
                (65536, 384, 128), (65536, 128, 384), (65536, 128, 128), (4096, 2048, 512)]:
    a = torch.randn(M, K, device=d).bfloat16()
    w = torch.randn(N, K, device=d).bfloat16()
    tb = t_us(lambda: torch.nn.functional.linear(a, w))
    tc = t_us(lambda: ops.gemm(a, w, False, torch.bfloat16))
    roof = (M * K + N * K + M * N) * 2 / 8e6
    print(f"{M:6d}x{N:5d}x{K:5d}  hipBLASLt {tb:7.2f} us  csu gemm4 {tc:7.2f} us  roof {roof:6.2f} us", flush=True)
