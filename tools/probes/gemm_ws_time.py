"""csu_gemm_ws vs gemm4 on the stage-2/3 shapes: hot (the same operands replayed back to back) and
cold (a 512 MB buffer written between launches, so operands come from HBM as in the train step).
    python tools/probes/gemm_ws_time.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd"), os.path.join(REPO, "tests")]
from csu import ops  # noqa: E402


def frag(w):
    R, C = w.shape
    return w.reshape(R // 32, 32, C // 16, 2, 8).permute(0, 2, 3, 1, 4).reshape(-1).contiguous()


def t_us(fn, cold, it=20):
    junk = torch.empty(128 << 20, device="cuda")
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    es = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
    for a, b in es:
        if cold:
            junk.fill_(1.0)
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in es)
    return ts[len(ts) // 2]


d = torch.device("cuda")
SHAPES = [(16384, 768, 256, "b"), (16384, 256, 768, ""), (16384, 256, 256, "rb"), (16384, 256, 256, ""),
          (65536, 384, 128, "b"), (65536, 128, 384, ""), (65536, 128, 128, "rb")]
# SHAPES=s1: the stage-1 (262144-token, C = 64) qkv / proj Linears and their input gradients
S1 = [(262144, 192, 64, "b"), (262144, 64, 192, ""), (262144, 64, 64, "rb"), (262144, 64, 64, ""), (262144, 64, 64, "bf")]
for M, N, K, mode in (S1 if os.environ.get("SHAPES") == "s1" else SHAPES):
    x = torch.randn(M, K, device=d).bfloat16()
    w = (torch.randn(N, K, device=d) / K ** 0.5).bfloat16()
    wf = frag(w)
    bias = torch.randn(N, device=d) if "b" in mode else None
    res = torch.randn(M, N, device=d) if "r" in mode else None
    odt = torch.float32 if res is not None or "f" in mode else torch.bfloat16
    f_ws = lambda: ops.gemm_ws(x, wf, N, odt, bias=bias, resid=res)  # noqa: E731
    f_g4 = lambda: ops.gemm(x, w, False, odt, bias=bias, resid=res)  # noqa: E731
    print(f"{M:6d}x{N:4d}x{K:4d}{mode:3s} ws hot {t_us(f_ws, False):6.2f} cold {t_us(f_ws, True):6.2f} | "
          f"gemm4 hot {t_us(f_g4, False):6.2f} cold {t_us(f_g4, True):6.2f} us", flush=True)
