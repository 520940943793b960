"""linear_wgrad bitwise reproducibility while other kernels run concurrently on another stream."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
d = torch.device("cuda:0")
g = torch.Generator(device=d).manual_seed(0)
side = torch.cuda.Stream()
big_a = torch.randn(8192, 8192, device=d, dtype=torch.bfloat16)
for (M, N, K) in [(16384, 768, 256), (16384, 1024, 256), (16384, 256, 1024), (16384, 256, 256), (65536, 384, 128), (262144, 192, 64)]:
    dy = torch.randn(M, N, device=d, generator=g).bfloat16()
    x = torch.randn(M, K, device=d, generator=g).bfloat16()
    ref = ops.linear_wgrad(dy, x)
    ref = (ref[0].clone(), ref[1].clone())
    nbad = 0
    for it in range(20):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            w, b = ops.linear_wgrad(dy, x)
        for _ in range(3):
            big_a @ big_a          # concurrent load on the main stream
        torch.cuda.synchronize()
        if not (torch.equal(w, ref[0]) and torch.equal(b, ref[1])):
            nbad += 1
    print(f"M={M} N={N} K={K}: {nbad}/20 runs differ", flush=True)
