"""Time the fp8 fused Mlp (csu_mlp_fp8_fwd / _bwd) against the bf16 fused Mlp on the stage shapes of
the 512x512 B16 / 1024x1024 B4 step (same token counts)."""
import ctypes
import os
import sys
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
    w1f = torch.randn(4 * C, C, device=d) * C ** -0.5
    w2f = torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5
    w1, w2 = w1f.bfloat16(), w2f.bfloat16()
    b1, b2 = torch.zeros(4 * C, device=d), torch.zeros(C, device=d)
    res, y = torch.randn(M, C, device=d), torch.empty(M, C, device=d)
    dy = torch.randn(M, C, device=d).bfloat16()
    dh, g = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16), torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
    dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
    fp8 = ops.Fp8Weights([w1f, w2f], mlp_pairs=[(w1f, w2f)])
    fp8.quantize()
    w1q, sw1, w2p, sw2, w2t, w1tp = fp8.mlp_operands(w1f, w2f)
    md = ops.MlpDrop(None, 0, 0, 0.0).c_struct()
    md.rows_per_sample = {64: 65536, 128: 16384, 256: 4096}[C]
    mdp = ctypes.byref(md)
    f = t(lambda: check(lib().csu_mlp_fwd_dp(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), mdp, st), "f"))
    bw = t(lambda: check(lib().csu_mlp_bwd_dp(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx),
                                              mdp, st), "b"))
    fd1 = t(lambda: check(lib().csu_mlp_fwd_ex(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), mdp, 1, st), "d1"))
    fd2 = t(lambda: check(lib().csu_mlp_fwd_ex(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), mdp, 2, st), "d2"))
    bd1 = t(lambda: check(lib().csu_mlp_bwd_ex(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx),
                                               mdp, 1, st), "bd1"))
    bd2 = t(lambda: check(lib().csu_mlp_bwd_ex(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx),
                                               mdp, 2, st), "bd2"))
    f8 = t(lambda: check(lib().csu_mlp_fp8_fwd(M, C, ptr(x), ptr(w1q), ptr(sw1), ptr(b1), ptr(w2p), ptr(sw2), ptr(b2),
                                               ptr(res), ptr(y), mdp, st), "f8"))
    b8 = t(lambda: check(lib().csu_mlp_fp8_bwd(M, C, ptr(x), ptr(dy), ptr(w1q), ptr(sw1), ptr(b1), ptr(w2t), ptr(sw2),
                                               ptr(w1tp), ptr(dh), ptr(g), ptr(dx), mdp, st), "b8"))
    print(f"C={C:4d} M={M:7d}  bf16 fwd {f:6.1f} us (deep ring {fd1:6.1f} / {fd2:6.1f})  bwd {bw:6.1f} us ({bd1:6.1f} / {bd2:6.1f})  "
          f"fp8 fwd {f8:6.1f} us  bwd {b8:6.1f} us", flush=True)
