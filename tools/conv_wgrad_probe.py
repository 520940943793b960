"""Conv weight-gradient kernels on the plain-UNet 512x512 B16 / CSWin shapes: parity of every
csu_conv2d_wgrad_ex configuration vs torch fp32 (batch 2) and graph-timed calls (incl. the chunk
reduction) at the full batch, MFMA utilisation vs 2.5 PF/s.  CFGS: cfg list (0 = v2, 1 + k = v3 k)."""
import ctypes, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
from csu import ops
from csu._lib import lib, CSU_BF16
sys.path.insert(0, os.path.dirname(__file__))
from conv_probe import graph_time  # noqa: E402
d = torch.device("cuda")
bf = torch.bfloat16
cfgs = [int(c) for c in os.environ.get("CFGS", "0,1,2,3,4,5").split(",")]
B = int(os.environ.get("B", "16"))
# (name, H, W, C, N, k, stride, pad) of the forward conv whose weight gradient is taken
shapes = [("u1 64->64", 512, 512, 64, 64, 3, 1, 1), ("u1 128->64", 512, 512, 128, 64, 3, 1, 1),
          ("u2 64->128", 256, 256, 64, 128, 3, 1, 1), ("u2 128->128", 256, 256, 128, 128, 3, 1, 1),
          ("u3 256->256", 128, 128, 256, 256, 3, 1, 1), ("u4 512->512", 64, 64, 512, 512, 3, 1, 1),
          ("u5 1024->1024", 32, 32, 1024, 1024, 3, 1, 1), ("convT 128->64", 512, 512, 64, 128, 2, 2, 0),
          ("convT 1024->512", 64, 64, 512, 1024, 2, 2, 0), ("merge 64->128 s2", 128, 128, 64, 128, 3, 2, 1),
          ("merge 256->512 s2", 32, 32, 256, 512, 3, 2, 1), ("embed 8->64 7x7 s4", 512, 512, 8, 64, 7, 4, 2),
          ("carafe4 enc 16->144", 128, 128, 16, 144, 3, 1, 1), ("carafe enc 32->36", 64, 64, 32, 36, 3, 1, 1),
          ("merge 128->256 s2", 64, 64, 128, 256, 3, 2, 1), ("carafe enc 128->36 16x16", 16, 16, 128, 36, 3, 1, 1),
          ("carafe enc 64->36 32x32", 32, 32, 64, 36, 3, 1, 1)]
if os.environ.get("ONLY"):
    shapes = [x for x in shapes if any(k in x[0] for k in os.environ["ONLY"].split(","))]


def call(g, x, dy, out, work, cfg):
    return lib().csu_conv2d_wgrad_ex(ctypes.byref(g), CSU_BF16, x.data_ptr(), dy.data_ptr(), 0, out.data_ptr(),
                                     work.data_ptr(), work.numel(), cfg, torch.cuda.current_stream().cuda_stream)


def case(H, W, C, N, k, s, p, b):
    g = ops._conv_geom(b, H, W, C, N, k, k, s, p)
    x = torch.randn(b, H, W, C, device=d).to(bf)
    dy = torch.randn(b, g.OH, g.OW, N, device=d).to(bf)
    out = torch.empty(N * k * k * C + N, device=d)
    nws = max(lib().csu_conv2d_wgrad_workspace_ex(ctypes.byref(g), c) for c in cfgs + [-1])
    work = torch.empty(max(nws, 16), dtype=torch.uint8, device=d)
    return g, x, dy, out, work


print(f"batch {B}; cfgs {cfgs}")
for name, H, W, C, N, k, s, p in shapes:
    g, x, dy, out, work = case(H, W, C, N, k, s, p, 2)
    xt = x.permute(0, 3, 1, 2).float().requires_grad_(False)
    dyt = dy.permute(0, 3, 1, 2).float()
    dwr = torch.nn.grad.conv2d_weight(xt, (N, C, k, k), dyt, stride=s, padding=p)   # (N, C, k, k)
    ref = torch.cat([dwr.permute(0, 2, 3, 1).reshape(-1), dyt.sum((0, 2, 3))])
    errs = []
    for c in cfgs:
        out.fill_(float("nan"))
        e = call(g, x, dy, out, work, c)
        torch.cuda.synchronize()
        errs.append(f"{c}:n/a" if e else f"{c}:{float((out - ref).norm() / ref.norm()):.1e}")
    g, x, dy, out, work = case(H, W, C, N, k, s, p, B)
    flops = 2 * B * g.OH * g.OW * N * C * k * k
    times = []
    for c in cfgs:
        if call(g, x, dy, out, work, c):
            times.append(f"{c}:   -  ")
            continue
        t = graph_time(lambda: call(g, x, dy, out, work, c), n=5, reps=3)
        times.append(f"{c}:{t:7.1f}us {flops / t / 1e6 / 2500:4.0%}")
    print(f"{name:20s} {flops / 1e9:7.1f} GF | parity " + " ".join(errs) + " | " + " ".join(times), flush=True)
