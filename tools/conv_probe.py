"""Time the convolutions of the 512x512 B16 model (patch embed, Merge_Block, CARAFE encoders) through
the C ABI: forward, input gradient and weight gradient of each, with HIP events on the launch stream,
next to the roofline min(2MNK / 2.5 PF/s, bytes / 8 TB/s).
    python tools/conv_probe.py [reps] [only-substring]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]

import ctypes  # noqa: E402

import torch  # noqa: E402

from csu import ops  # noqa: E402
from csu._lib import lib  # noqa: E402

B = 16
# name, H, W, C, N, K, stride, pad (input geometry of the forward conv)
SHAPES = [
    ("patch_embed", 512, 512, 8, 64, 7, 4, 2),
    ("merge1", 128, 128, 64, 128, 3, 2, 1),
    ("merge2", 64, 64, 128, 256, 3, 2, 1),
    ("merge3", 32, 32, 256, 512, 3, 2, 1),
    ("enc16", 16, 16, 128, 36, 3, 1, 1),
    ("enc32", 32, 32, 64, 36, 3, 1, 1),
    ("enc64", 64, 64, 32, 36, 3, 1, 1),
    ("enc128x4", 128, 128, 16, 144, 3, 1, 1),
]


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    d = torch.device("cuda:0")
    L = lib()
    sp = ops.stream_ptr(d)
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    print(f"{'conv':12s} {'pass':6s} {'us':>8s} {'roof us':>8s} {'frac':>6s}  M x N x K")
    for name, H, W, C, N, K, s, p in SHAPES:
        if only and only not in name:
            continue
        g = ops._conv_geom(B, H, W, C, N, K, K, s, p)
        OH, OW = g.OH, g.OW
        x = torch.randn(B, H, W, C, device=d).to(torch.bfloat16)
        w = torch.randn(N, K, K, C, device=d).to(torch.bfloat16) * 0.05        # OHWI
        wt = w.permute(3, 1, 2, 0).contiguous()                                  # IHWO
        bias = torch.randn(N, device=d)
        y = torch.empty(B, OH, OW, N, device=d, dtype=torch.bfloat16)
        dy = torch.randn(B, OH, OW, N, device=d).to(torch.bfloat16)
        dx = torch.empty_like(x)
        nws = L.csu_conv2d_wgrad_workspace(ctypes.byref(g))
        ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=d)
        dwb = torch.empty(N * K * K * C + N, dtype=torch.float32, device=d)
        bf = ops.dtype_code(x)
        M = B * OH * OW
        flops = 2 * M * N * K * K * C
        io = (x.numel() + y.numel() + w.numel()) * 2
        runs = {
            "fwd": lambda: L.csu_conv2d_fwd(ctypes.byref(g), bf, ops.ptr(x), ops.ptr(w), ops.ptr(bias), ops.ptr(y), sp),
            "dgrad": lambda: L.csu_conv2d_dgrad(ctypes.byref(g), bf, ops.ptr(dy), ops.ptr(wt), None, ops.ptr(dx), sp),
            "wgrad": lambda: L.csu_conv2d_wgrad(ctypes.byref(g), bf, ops.ptr(x), ops.ptr(dy), ops.ptr(dwb), ops.ptr(ws),
                                                nws, sp),
        }
        for k, fn in runs.items():
            ops.check(fn(), f"{name} {k}")
            us = timed(fn, reps)
            roof = max(flops / 2.5e15, (io + (dwb.numel() * 4 if k == "wgrad" else 0)) / 8e12) * 1e6
            tot[k] += us
            print(f"{name:12s} {k:6s} {us:8.1f} {roof:8.1f} {roof / us:6.2f}  {M} x {N} x {K * K * C}", flush=True)
    print("totals us:", {k: round(v, 1) for k, v in tot.items()}, "sum", round(sum(tot.values()), 1))


if __name__ == "__main__":
    main()
