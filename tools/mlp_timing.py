"""mlp_fwd per-workgroup timing (debug library built with -DMLP_TIMING, CSU_LIB_PATH): prologue
(x fragments + first weight chunk), step loop, summed per-step waits (DMA + barrier), total."""
import ctypes, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu._lib import check, lib, ptr, stream_ptr
d = torch.device("cuda:0")
st = stream_ptr(d)
L = lib()
L.csu_debug_mlp_ts.argtypes = [ctypes.c_void_p, ctypes.c_int]
for C, M in [(256, 16384), (128, 65536), (64, 262144), (256, 64)]:
    x = torch.randn(M, C, device=d).bfloat16()
    w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
    b1, b2 = torch.zeros(4 * C, device=d), torch.zeros(C, device=d)
    res, y = torch.randn(M, C, device=d), torch.empty(M, C, device=d)
    for _ in range(3):
        check(L.csu_mlp_fwd(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), st), "f")
    torch.cuda.synchronize()
    ts = np.zeros((6, 4096), dtype=np.uint64)
    assert L.csu_debug_mlp_ts(ts.ctypes.data, ts.size) == 0
    nwg = min((M + 63) // 64, 4096)
    t = ts[:6, :nwg].astype(np.int64)
    clk = np.median(t[5] / np.maximum(t[4], 1)) * 100   # shader cycles per 10-ns tick -> MHz
    us = lambda v: v * 0.01
    print(f"C={C} M={M} WGs={nwg}: span {us(t[0].max() + t[4][np.argmax(t[0])] - t[0].min()):6.2f} | entry spread {us(t[0].max() - t[0].min()):5.2f} | "
          f"prologue {us(np.median(t[1])):5.2f} | to loop end {us(np.median(t[2])):6.2f} | waits in loop {us(np.median(t[3])):6.2f} | "
          f"total {us(np.median(t[4])):6.2f} us (median per WG) | shader clock {clk:6.0f} MHz", flush=True)
