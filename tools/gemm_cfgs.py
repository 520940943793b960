"""gemm4 tile configs (cfg 10..15) on the step's token-GEMM shapes (fwd / input-gradient), plus hipBLASLt."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda")
bf = torch.bfloat16


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


cfgs = [int(c) for c in os.environ.get("CFGS", "10,11,12,13,14,15").split(",")]
shapes = [("qkv dgrad C256", 16384, 256, 768), ("qkv fwd C256", 16384, 768, 256), ("proj C256", 16384, 256, 256),
          ("qkv dgrad C128", 65536, 128, 384), ("qkv fwd C128", 65536, 384, 128), ("qkv dgrad C64", 262144, 64, 192),
          ("qkv fwd C64", 262144, 192, 64), ("fc1 C512", 4096, 2048, 512), ("fc2 dgrad C512", 4096, 2048, 512)]
for name, M, N, K in shapes:
    a = torch.randn(M, K, device=d, dtype=bf)
    w = torch.randn(N, K, device=d, dtype=bf) * 0.05
    ts = [timeit(lambda: ops.gemm(a, w, False, bf, cfg=c)) for c in cfgs]
    tt = timeit(lambda: torch.nn.functional.linear(a, w))
    by = (M * K + N * K + M * N) * 2
    print(f"{name:16s} M={M:6d} N={N:5d} K={K:4d}: " + "  ".join(f"c{c} {t:6.1f}" for c, t in zip(cfgs, ts))
          + f"  | hipBLASLt {tt:6.1f} us  (min {by / 8e6:5.1f} us at 8 TB/s)", flush=True)
