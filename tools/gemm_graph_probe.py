"""gemm4 tile configurations on the 512x512 step's token-GEMM shapes, timed inside a HIP graph
(20 launches per replay: no host launch overhead), vs the HBM-byte minimum at 8 TB/s.
CFGS: comma list of csu_gemm_ex cfg values (10 + kG4Cfgs index)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda")
bf = torch.bfloat16
cfgs = [int(c) for c in os.environ.get("CFGS", "11,16,17").split(",")]
# (name, M, N, K, resid): fwd / input-gradient GEMMs of the 512x512 B16 step
shapes = [("qkv fwd C256", 16384, 768, 256, False), ("qkv dgrad C256", 16384, 256, 768, False),
          ("proj+res C256", 16384, 256, 256, True), ("qkv fwd C128", 65536, 384, 128, False),
          ("qkv dgrad C128", 65536, 128, 384, False), ("qkv fwd C64", 262144, 192, 64, False),
          ("qkv dgrad C64", 262144, 64, 192, False), ("fc1 C512", 4096, 2048, 512, False),
          ("fc2 dgrad C512", 4096, 512, 2048, False)]


def graph_time(fn, n=20, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (n * reps) * 1e3


for name, M, N, K, res in shapes:
    a = torch.randn(M, K, device=d, dtype=bf)
    w = torch.randn(N, K, device=d, dtype=bf) * 0.05
    r = torch.randn(M, N, device=d) if res else None
    od = torch.float32 if res else bf
    ts = [graph_time(lambda: ops.gemm(a, w, False, od, resid=r, cfg=c)) for c in cfgs]
    by = (M * K + N * K) * 2 + M * N * (8 if res else 2)
    print(f"{name:16s} M={M:6d} N={N:5d} K={K:4d}: " + "  ".join(f"c{c} {t:6.1f}" for c, t in zip(cfgs, ts))
          + f"  us  (min {by / 8e6:5.1f} us at 8 TB/s)", flush=True)
