"""Time csu_stripe_lepe_wgrad (LePE weight/bias gradient) per 512x512 B16 stage shape."""
import ctypes, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
from csu._lib import check, lib, ptr, stream_ptr, dtype_code

d = torch.device("cuda:0")
B = 16
for reso, C, heads, sp, last in [(128, 64, 2, 1, False), (64, 128, 4, 2, False), (32, 256, 8, 8, False), (16, 512, 16, 16, True)]:
    br = [(reso, reso, 0)] if last else [(reso, sp, 0), (sp, reso, C // 2)]
    nh = heads if last else heads // 2
    cb = C if last else C // 2
    geom = ops.StripeGeometry(reso, C, nh, br, (cb // nh) ** -0.5, head_dim=32)
    qkv = torch.randn(B, reso * reso, 3 * C, device=d).bfloat16()
    dout = torch.randn(B, reso * reso, C, device=d).bfloat16()
    ws = [torch.randn(cb, 1, 3, 3, device=d) for _ in br]
    bs = [torch.randn(cb, device=d) for _ in br]
    dws = [torch.empty_like(w) for w in ws]
    dbs = [torch.empty_like(b) for b in bs]
    a = geom.args(B, ws, bs, dws, dbs)
    n = lib().csu_stripe_attn_bwd_workspace(ctypes.byref(a))
    work = torch.empty(n, dtype=torch.uint8, device=d)
    st = stream_ptr(d)
    f = lambda: check(lib().csu_stripe_lepe_wgrad(ctypes.byref(a), dtype_code(qkv), ptr(qkv), ptr(dout), ptr(work), n, st), "l")
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    nb = B * reso * reso * C * 2 * 2
    print(f"reso {reso:4d} C {C:4d}: {us:7.1f} us  ({nb / us / 1e3:6.0f} GB/s of dout + V)", flush=True)
