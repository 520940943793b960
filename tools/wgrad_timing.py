"""Per-workgroup phase timeline of wgrad_tile (debug library built with WG_TIMING):
    make -C cswin-simam-unet_amd/csrc dbg && python tools/wgrad_timing.py M N K [tn tk chunks]
Stamps (100 MHz realtime clock): 0 entry, 1 prologue done (first step staged), 2 main loop done,
3 epilogue done.  Prints the spread of each phase over the workgroups (us)."""
import ctypes, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
os.environ["CSU_LIB_PATH"] = os.path.join(HERE, "..", "cswin-simam-unet_amd", "csu", "_lib", "libcsu_hip_dbg.so")
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu._lib import check, lib, ptr, stream_ptr

def run(M, N, K, tn=0, tk=0, ch=0):
    d = torch.device("cuda")
    dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    L = lib()
    n = L.csu_linear_wgrad_tuned_workspace(M, N, K, tn, tk, ch)
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=d)
    out = torch.empty(N * K + N, device=d)
    for _ in range(5):
        check(L.csu_linear_wgrad_tuned(M, N, K, 1, ptr(dy), ptr(x), ptr(out), ptr(ws), n, tn, tk, ch, stream_ptr(d)), "w")
    torch.cuda.synchronize()
    buf = np.zeros((4, 16384), dtype=np.uint64)
    fn = L.csu_debug_wgrad_ts
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    used = buf[0] != 0
    t = buf[:, used].astype(np.int64)
    t0 = t[0].min()
    t = (t - t0) / 100.0   # us
    q = lambda v: f"min {v.min():6.2f} med {np.median(v):6.2f} max {v.max():6.2f}"
    print(f"M={M} N={N} K={K} plan=({tn},{tk},{ch}): {used.sum()} WGs, span {t[3].max():.2f} us")
    print("  start    ", q(t[0]))
    print("  prologue ", q(t[1] - t[0]))
    print("  loop     ", q(t[2] - t[1]))
    print("  epilogue ", q(t[3] - t[2]))
    print("  end      ", q(t[3]))
    st = np.zeros((4, 64), dtype=np.uint64)
    f2 = L.csu_debug_wgrad_steps
    f2.argtypes = [ctypes.c_void_p]
    assert f2(st.ctypes.data) == 0
    st = st.astype(np.int64)
    nst = min(16, int((st[0] != 0).sum()))
    for i in range(nst):
        print(f"    step {i:2d}: stage {st[1][i] - st[0][i]:6d}  load+mfma {st[2][i] - st[1][i]:6d}  barrier {st[3][i] - st[2][i]:6d}"
              f"  total {st[3][i] - st[0][i]:6d} cyc")
    buf[:] = 0
    assert L.csu_debug_wgrad_steps  # noqa

args = [int(v) for v in sys.argv[1:]]
if args:
    run(*args)
else:
    for shp in [(16384, 1024, 256, 0, 0, 16), (16384, 1024, 256, 0, 0, 1), (262144, 192, 64, 0, 0, 0)]:
        run(*shp)
