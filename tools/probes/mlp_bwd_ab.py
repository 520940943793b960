"""Isolated csu_mlp_bwd timing at C = 256 (16384 tokens: stage 3 at 512x512 B16), product library
against libcsu_hip_ab.so, and the max |difference| of their outputs.
    python tools/probes/mlp_bwd_ab.py"""
import ctypes
import os

import torch

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "cswin-simam-unet_amd",
                   "csu", "_lib")


def main():
    d = torch.device("cuda:0")
    C, M = 256, 16384
    g = torch.Generator(device=d).manual_seed(0)
    x = torch.randn(M, C, device=d, generator=g).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d, generator=g) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d, generator=g) * (4 * C) ** -0.5).bfloat16()
    b1 = torch.randn(4 * C, device=d, generator=g) * 0.1
    dy = torch.randn(M, C, device=d, generator=g).bfloat16()
    P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731

    class Drop(ctypes.Structure):   # csu_mlp_dropout with p = 0: only rows_per_sample (the chunk rotation)
        _fields_ = [("rng", ctypes.c_void_p), ("site_hidden", ctypes.c_uint32), ("site_out", ctypes.c_uint32),
                    ("p", ctypes.c_float), ("row_scale", ctypes.c_void_p), ("rows_per_sample", ctypes.c_int64)]
    dd = Drop(None, 0, 0, 0.0, None, 4096)
    st = ctypes.c_void_p(torch.cuda.current_stream(d).cuda_stream)
    outs = {}
    for name in ("libcsu_hip.so", "libcsu_hip_ab.so"):
        L = ctypes.CDLL(os.path.join(LIB, name))
        L.csu_mlp_bwd_dp.restype = ctypes.c_int
        dh = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
        gg = torch.empty_like(dh)
        dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)

        def run(m=M):
            return L.csu_mlp_bwd_dp(ctypes.c_long(m), C, P(x), P(dy), P(w1), P(b1), P(w2), P(dh), P(gg), P(dx),
                                    ctypes.byref(dd), st)
        assert run() == 0
        torch.cuda.synchronize()
        outs[name] = (dh.clone(), gg.clone(), dx.clone())
        for m in (M, 64):
            for _ in range(3):
                run(m)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(50):
                run(m)
            b.record()
            torch.cuda.synchronize()
            print(f"{name:18s} M={m:6d}: {a.elapsed_time(b) / 50 * 1e3:6.1f} us", flush=True)
    for i, n in enumerate(("dH", "g", "dX")):
        u, v = outs["libcsu_hip.so"][i].float(), outs["libcsu_hip_ab.so"][i].float()
        print(f"{n}: max |a - b| {(u - v).abs().max().item():.3e}  (max |b| {v.abs().max().item():.3e})")


if __name__ == "__main__":
    main()
