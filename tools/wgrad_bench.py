"""Weight-gradient kernel sweep over the exact Linear shapes of one CSWin-UNet train step.

    python tools/wgrad_bench.py [--img 512] [--batch 16] [--plans auto,c1,c2,...]

Records every ops.linear_wgrad call (M, N, K) of one eager bf16 step, then times
csu_linear_wgrad_tuned per unique shape and plan with HIP events (20 back-to-back launches) and
prints us/launch, the algorithmic GB/s (M*(N+K)*2 bytes read + N*K*4 written) and the per-step total
(launches x time).  Plans: "auto" (the library's choice), "cX" = X chunks per tile-count target
(chunks = ceil(X * CUs / tiles)), "tNxK:cX" forces the tile."""
import argparse
import collections
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch

from csu import ops
from csu._lib import check, lib, ptr, stream_ptr


def record_shapes(img, batch):
    from csu.model import CSWinTransformer
    from csu.train import bce_loss
    from csu.data import ellipse_batch
    d = torch.device("cuda:0")
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=img, split_size=[1, 2, 8, 8]).to(d)
    x, t = ellipse_batch(np.random.default_rng(0), batch, img)
    x, t = x.to(d), t.to(d)
    shapes = collections.Counter()
    orig = ops.linear_wgrad

    def rec(dy2, x2, out=None, work=None):
        shapes[(dy2.shape[0], dy2.shape[1], x2.shape[1])] += 1
        return orig(dy2, x2, out, work)
    ops.linear_wgrad = rec
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        bce_loss(y, t).backward()
        torch.cuda.synchronize()
    finally:
        ops.linear_wgrad = orig
    return shapes


def time_plan(M, N, K, tn, tk, chunks, reps=20):
    d = torch.device("cuda:0")
    dy = torch.randn(M, N, device=d).bfloat16()
    x = torch.randn(M, K, device=d).bfloat16()
    L = lib()
    n = L.csu_linear_wgrad_tuned_workspace(M, N, K, tn, tk, chunks)
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=d)
    out = torch.empty(N * K + N, device=d)
    st = stream_ptr(d)

    def go():
        check(L.csu_linear_wgrad_tuned(M, N, K, 1, ptr(dy), ptr(x), ptr(out), ptr(ws), n, tn, tk, chunks, st), "wgrad")
    for _ in range(3):
        go()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def time_torch(M, N, K, reps=20):
    """hipBLASLt reference: dY^T X in bf16 (fp32 accumulation, bf16 out; no bias)."""
    d = torch.device("cuda:0")
    dy = torch.randn(M, N, device=d).bfloat16()
    x = torch.randn(M, K, device=d).bfloat16()
    for _ in range(3):
        dy.t() @ x
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dy.t() @ x
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def parse_plan(p, M, N, K, cus):
    tn = tk = 0
    if p.startswith("t"):
        t, p = p[1:].split(":")
        tn, tk = (int(v) for v in t.split("x"))
    if p == "auto":
        return tn, tk, 0
    x = float(p[1:])
    tn_ = tn or (128 if N % 128 == 0 else 64)
    tk_ = tk or (128 if K % 128 == 0 else 64)
    tiles = -(-N // tn_) * -(-K // tk_)
    chunks = max(1, min(-(-int(x * cus) // tiles), -(-M // 256)))
    return tn, tk, chunks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--plans", default="auto,c1,c2,c4")
    a = ap.parse_args()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    shapes = record_shapes(a.img, a.batch)
    plans = a.plans.split(",")
    tot = collections.Counter()
    print(f"{'M':>8} {'N':>5} {'K':>5} {'n':>3} " + " ".join(f"{p:>18}" for p in plans))
    for (M, N, K), cnt in sorted(shapes.items(), key=lambda kv: -kv[0][0] * (kv[0][1] + kv[0][2]) * kv[1]):
        nbytes = M * (N + K) * 2 + (N * K + N) * 4
        cells = []
        for p in plans:
            if p == "torch":
                us = time_torch(M, N, K)
            else:
                tn, tk, ch = parse_plan(p, M, N, K, cus)
                us = time_plan(M, N, K, tn, tk, ch)
            tot[p] += us * cnt
            cells.append(f"{us:7.1f}us {nbytes / us / 1e3:6.0f}GB/s")
        print(f"{M:8d} {N:5d} {K:5d} {cnt:3d} " + " ".join(f"{c:>18}" for c in cells), flush=True)
    print("per-step total: " + "  ".join(f"{p}={v / 1e3:.3f}ms" for p, v in tot.items()))


if __name__ == "__main__":
    main()
