"""csu_gemm_f32 vs torch (hipBLASLt) fp32 matmul on the fp32-path Linear shapes (256x256 B8)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops


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
for (M, N, K) in [(32768, 192, 64), (32768, 256, 64), (8192, 768, 256), (2048, 2048, 512), (8192, 1024, 256)]:
    x, w = torch.randn(M, K, device=d), torch.randn(N, K, device=d)
    dy = torch.randn(M, N, device=d)
    f0 = t(lambda: ops.gemm_f32(0, x, w, M, N, K))
    f1 = t(lambda: ops.gemm_f32(1, dy, w, M, K, N))
    f2 = t(lambda: ops.gemm_f32(2, dy, x, N, K, M))
    r0 = t(lambda: x @ w.t())
    r1 = t(lambda: dy @ w)
    r2 = t(lambda: dy.t() @ x)
    fl = 2 * M * N * K / 1e6
    print(f"M={M:6d} N={N:5d} K={K:4d}  csu NT {f0:7.1f}us ({fl / f0:5.1f} TF/s) NN {f1:7.1f} TN {f2:7.1f}   "
          f"torch NT {r0:7.1f} NN {r1:7.1f} TN {r2:7.1f}", flush=True)
