"""Per-shape timing of every token-Linear kernel call of the 512x512 B16 bf16 step, with the
algorithmic bytes/FLOPs of each call -> achieved GB/s and TFLOP/s (graph-replayed, 20 launches)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
from gemm_probe2 import timeit

d = torch.device("cuda")
bf = torch.bfloat16
B = int(os.environ.get("B", "16"))
tot = {}


CFGS = [int(c) for c in os.environ.get("CFGS", "").split(",") if c]


def rep(tag, t, nbytes, flops, alt=()):
    tot[tag.split()[0]] = tot.get(tag.split()[0], 0) + t
    extra = "  cfgs " + " ".join(f"{c}:{v:.1f}" for c, v in alt) if alt else ""
    print(f"{tag:22s} {t:7.1f} us  {nbytes / t / 1e3:7.0f} GB/s  {flops / t / 1e6:6.0f} TF/s  ({nbytes / 1e6:.1f} MB){extra}", flush=True)


def sweep(fn):
    return [(c, timeit(lambda: fn(c))) for c in CFGS]


big = torch.empty(256 << 20, dtype=torch.uint8, device=d)
for mb in (64, 128):
    src = big[: mb << 20]
    dst = torch.empty_like(src)
    t = timeit(lambda: dst.copy_(src))
    print(f"copy {mb} MB: {t:.1f} us = {2 * src.numel() / t / 1e3:.0f} GB/s (read+write)")
for reso, C in ((128, 64), (64, 128), (32, 256), (16, 512)):
    M = B * reso * reso
    x = torch.randn(M, C, device=d, dtype=bf)
    h = torch.randn(M, 4 * C, device=d, dtype=bf)
    res = torch.randn(M, C, device=d)
    for name, N, K in (("qkv", 3 * C, C), ("proj", C, C), ("fc1", 4 * C, C), ("fc2", C, 4 * C)):
        a = x if K == C else h
        w = torch.randn(N, K, device=d, dtype=bf) * 0.05
        wt = w.t().contiguous()
        b = torch.randn(N, device=d)
        dy = torch.randn(M, N, device=d, dtype=bf)
        fl = 2 * M * N * K
        if name == "fc1":
            rep(f"fwd {name}{C} gelu_out", timeit(lambda: ops.gemm(a, w, False, bf, bias=b, gelu_out=True)), M * K * 2 + 2 * M * N * 2, fl,
                sweep(lambda c: ops.gemm(a, w, False, bf, bias=b, gelu_out=True, cfg=c)))
        elif name in ("proj", "fc2"):
            rep(f"fwd {name}{C} +res", timeit(lambda: ops.gemm(a, w, False, torch.float32, bias=b, resid=res)), M * K * 2 + M * N * 8, fl,
                sweep(lambda c: ops.gemm(a, w, False, torch.float32, bias=b, resid=res, cfg=c)))
        else:
            rep(f"fwd {name}{C}", timeit(lambda: ops.gemm(a, w, False, bf, bias=b)), M * K * 2 + M * N * 2, fl,
                sweep(lambda c: ops.gemm(a, w, False, bf, bias=b, cfg=c)))
        if name == "fc2":   # dh = (dY W2) * gelu'(h)
            rep(f"dgrad {name}{C} gaux", timeit(lambda: ops.gemm(dy, wt, False, bf, gelu_aux=h)), M * N * 2 + 2 * M * K * 2, fl,
                sweep(lambda c: ops.gemm(dy, wt, False, bf, gelu_aux=h, cfg=c)))
        else:
            rep(f"dgrad {name}{C}", timeit(lambda: ops.gemm(dy, wt, False, bf)), M * N * 2 + M * K * 2, fl,
                sweep(lambda c: ops.gemm(dy, wt, False, bf, cfg=c)))
        rep(f"wgrad {name}{C}", timeit(lambda: ops.linear_wgrad(dy, a)), M * (N + K) * 2, fl)
print("totals per kind (one block of each stage):", {k: round(v, 1) for k, v in tot.items()})
