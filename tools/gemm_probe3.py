"""Epilogue cost probe: csu_gemm_ex plain / +gelu_out / +gelu_aux / +resid vs hipBLASLt (+ torch GELU)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
from gemm_probe2 import timeit

d = torch.device("cuda")
F = torch.nn.functional
for name, M, K, N in (("fc1_256", 16384, 256, 1024), ("fc2dg_256", 16384, 256, 1024), ("fc1_64", 262144, 64, 256),
                      ("fc1_128", 65536, 128, 512), ("qkv256", 16384, 256, 768), ("fc2_256", 16384, 1024, 256)):
    x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=d, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=d)
    aux = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    res = torch.randn(M, N, device=d)
    r = [("torch", timeit(lambda: F.linear(x, w))), ("torch+gelu", timeit(lambda: F.gelu(F.linear(x, w))))]
    for c in (-1, 0, 1, 2, 3):
        r.append((f"c{c} plain", timeit(lambda: ops.gemm(x, w, False, torch.bfloat16, bias=b, cfg=c))))
        r.append((f"c{c} gout", timeit(lambda: ops.gemm(x, w, False, torch.bfloat16, bias=b, cfg=c, gelu_out=True))))
        r.append((f"c{c} gaux", timeit(lambda: ops.gemm(x, w, False, torch.bfloat16, gelu_aux=aux, cfg=c))))
        r.append((f"c{c} res", timeit(lambda: ops.gemm(x, w, False, torch.float32, bias=b, resid=res, cfg=c))))
    print(f"{name:10s} M={M} K={K} N={N}: " + "  ".join(f"{k} {v:.1f}" for k, v in r), flush=True)
