"""gemm4 per-workgroup phase timestamps (debug library built with -DG4_TIMING, CSU_LIB_PATH):
0 entry, 1 first slice landed, 2 last slice landed (tile 0), 3 MFMAs done, 4 epilogue done, 5 exit.
Prints medians of the phase durations and the spread of entry times (100 MHz real-time clock)."""
import ctypes, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu import ops
from csu._lib import lib
d = torch.device("cuda")
bf = torch.bfloat16
L = lib()
L.csu_debug_g4_ts.argtypes = [ctypes.c_void_p, ctypes.c_int]
for name, M, N, K in [("proj C256", 16384, 256, 256), ("qkv dgrad C256", 16384, 256, 768), ("qkv fwd C64", 262144, 192, 64)]:
    a = torch.randn(M, K, device=d, dtype=bf)
    w = torch.randn(N, K, device=d, dtype=bf) * 0.05
    for _ in range(5):
        ops.gemm(a, w, False, bf)
    torch.cuda.synchronize()
    ts = np.zeros((8, 4096), dtype=np.uint64)
    assert L.csu_debug_g4_ts(ts.ctypes.data, ts.size) == 0
    nwg = 512
    t = ts[:6, :nwg].astype(np.int64)
    t0 = t[0].min()
    us = lambda x: x * 0.01   # 100 MHz ticks -> us
    print(f"{name}: span {us(t[5].max() - t0):6.2f} us | entry spread {us(t[0].max() - t0):5.2f} | "
          f"first-slice wait {us(np.median(t[1] - t[0])):5.2f} | to last slice {us(np.median(t[2] - t[1])):5.2f} | "
          f"last mma {us(np.median(t[3] - t[2])):5.2f} | epilogue {us(np.median(t[4] - t[3])):5.2f} | "
          f"rest {us(np.median(t[5] - t[4])):5.2f} | exit spread {us(t[5].max() - t[5].min()):5.2f}", flush=True)
