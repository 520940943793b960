"""Time csu_mlp_fwd / csu_mlp_bwd against the two-GEMM Mlp on the encoder stage shapes (batch 16)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd"))
import torch
from csu import ops
from csu._lib import check, lib, ptr, stream_ptr


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


d = torch.device("cuda:0")
st = stream_ptr(d)
for C, M in [(64, 262144), (128, 65536), (256, 16384)]:
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.zeros(4 * C, device=d), torch.zeros(C, device=d)
    res, y = torch.randn(M, C, device=d), torch.empty(M, C, device=d)
    dy = torch.randn(M, C, device=d).bfloat16()
    dh, g = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16), torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    f = t(lambda: check(lib().csu_mlp_fwd(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), st), "f"))
    bw = t(lambda: check(lib().csu_mlp_bwd(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx), st), "b"))
    w1t, w2t = w1.t().contiguous(), w2.t().contiguous()
    def unf():
        h, gg = ops.gemm(x, w1, False, torch.bfloat16, bias=b1, gelu_out=True)
        ops.gemm(gg, w2, False, torch.float32, bias=b2, resid=res)
    def unb():
        hh = ops.gemm(dy, w2t, False, torch.bfloat16, gelu_aux=dh)
        ops.gemm(hh, w1t, False, torch.bfloat16)
    uf, ub = t(unf), t(unb)
    fl = 2 * M * C * 4 * C * 2
    print(f"C={C:4d} M={M:7d}  fused fwd {f:7.1f} us ({fl / f / 1e6:6.1f} TF/s)  bwd {bw:7.1f} us ({1.5 * fl / bw / 1e6:6.1f} TF/s)"
          f"   two-GEMM fwd {uf:7.1f}  dgrad pair {ub:7.1f}", flush=True)
