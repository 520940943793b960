"""Microbenchmark of the token GEMM shapes of the 512x512 B16 CSWin-UNet step (fwd / dgrad / wgrad),
torch (hipBLASLt) baseline vs split-K variants.  Prints time and achieved GB/s vs compulsory bytes."""
import sys, time, torch
d = torch.device("cuda")
torch.manual_seed(0)
B = 16
shapes = []  # (name, M, K, N)
for reso, C, depth in ((128, 64, 2), (64, 128, 4), (32, 256, 18), (16, 512, 2)):
    M = B * reso * reso
    shapes += [(f"qkv{C}", M, C, 3 * C), (f"proj{C}", M, C, C), (f"fc1_{C}", M, C, 4 * C), (f"fc2_{C}", M, 4 * C, C)]
shapes += [("carafe4_out", B * 512 * 512 // 16 * 16, 64, 64)]

def timeit(fn, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3  # us

for name, M, K, N in shapes:
    x = torch.randn(M, K, device=d, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=d, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=d, dtype=torch.bfloat16)
    fwd = timeit(lambda: torch.nn.functional.linear(x, w))
    dgr = timeit(lambda: dy @ w)
    wgr = timeit(lambda: dy.t() @ x)
    res = [f"{name:12s} M={M:8d} K={K:4d} N={N:4d}  fwd {fwd:8.1f}us ({(M*K+M*N+N*K)*2/fwd/1e3:6.0f}GB/s)",
           f"dgrad {dgr:8.1f}us ({(M*K+M*N+N*K)*2/dgr/1e3:6.0f})", f"wgrad {wgr:8.1f}us ({(M*K+M*N)*2/wgr/1e3:6.0f})"]
    for S in (8, 32, 128):
        if M % S: continue
        xs, dys = x.view(S, M // S, K), dy.view(S, M // S, N)
        t = timeit(lambda: torch.bmm(dys.transpose(1, 2), xs).float().sum(0))
        res.append(f"sk{S} {t:7.1f}")
    print("  ".join(res), flush=True)
