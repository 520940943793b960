"""csu_gemm vs torch (hipBLASLt) on the token-GEMM shapes of the 512x512 B16 step (fwd and dgrad)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda")
torch.manual_seed(0)
B = 16
shapes = []
for reso, C in ((128, 64), (64, 128), (32, 256), (16, 512)):
    M = B * reso * reso
    shapes += [(f"qkv{C}", M, C, 3 * C), (f"proj{C}", M, C, C), (f"fc1_{C}", M, C, 4 * C), (f"fc2_{C}", M, 4 * C, C)]


def timeit(fn, n=20):
    """Per-launch time of n back-to-back launches captured in one HIP graph (no host overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    g.replay()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
  for name, M, K, N in shapes:
      x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
      w = torch.randn(N, K, device=d, dtype=torch.bfloat16)
      dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
      bias = torch.randn(N, device=d)
      wt = w.t().contiguous()
      t_f = timeit(lambda: torch.nn.functional.linear(x, w))
      t_d = timeit(lambda: dy @ w)
      cf = [timeit(lambda: ops.gemm(x, w, False, torch.bfloat16, bias=bias, cfg=c)) for c in range(4)]
      cd = [timeit(lambda: ops.gemm(dy, wt, False, torch.bfloat16, cfg=c)) for c in range(4)]
      c_a = timeit(lambda: ops.gemm(x, w, False, torch.bfloat16, bias=bias))
      c_g = timeit(lambda: ops.gemm(x, w, False, torch.bfloat16, bias=bias, a_gelu=True))
      err = (ops.gemm(x, w, False, torch.float32) - (x.float() @ w.float().t())).abs().max().item()
      errd = (ops.gemm(dy, wt, False, torch.float32) - (dy.float() @ w.float())).abs().max().item()
      print(f"{name:8s} M={M:7d} K={K:5d} N={N:5d}  torch fwd {t_f:6.1f} dgrad {t_d:6.1f} | csu auto fwd {c_a:6.1f} "
            f"gelu-fwd {c_g:6.1f} | cfg fwd " + " ".join(f"{v:6.1f}" for v in cf) + " | cfg dgrad " +
            " ".join(f"{v:6.1f}" for v in cd) + f"  err {err:.2g} {errd:.2g}", flush=True)


if __name__ == "__main__":
    main()
