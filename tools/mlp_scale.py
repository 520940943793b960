"""csu_mlp_fwd / bwd time vs token count (workgroups) at fixed C, and the device's CU count."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd"))
import torch
from csu._lib import check, lib, ptr, stream_ptr

d = torch.device("cuda:0")
print("CUs", torch.cuda.get_device_properties(d).multi_processor_count)
st = stream_ptr(d)


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


for C in [int(c) for c in (sys.argv[1:] or ["256"])]:
    for M in [64, 4096, 8192, 16384, 32768, 65536]:
        x = torch.randn(M, C, device=d).bfloat16()
        w1 = (torch.randn(4 * C, C, device=d) * C ** -0.5).bfloat16()
        w2 = (torch.randn(C, 4 * C, device=d) * (4 * C) ** -0.5).bfloat16()
        b1, b2 = torch.zeros(4 * C, device=d), torch.zeros(C, device=d)
        res, y = torch.randn(M, C, device=d), torch.empty(M, C, device=d)
        dy = torch.randn(M, C, device=d).bfloat16()
        dh, g = torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16), torch.empty(M, 4 * C, device=d, dtype=torch.bfloat16)
        dx = torch.empty(M, C, device=d, dtype=torch.bfloat16)
        f = t(lambda: check(lib().csu_mlp_fwd(M, C, ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(res), ptr(y), st), "f"))
        b = t(lambda: check(lib().csu_mlp_bwd(M, C, ptr(x), ptr(dy), ptr(w1), ptr(b1), ptr(w2), ptr(dh), ptr(g), ptr(dx), st), "b"))
        print(f"C={C} M={M:6d} WGs={M // 64:5d}  fwd {f:7.1f} us  bwd {b:7.1f} us", flush=True)
