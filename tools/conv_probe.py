"""Implicit-GEMM conv kernels on the plain-UNet 512x512 B16 and CSWin conv shapes: parity of every
csu_conv2d_ex configuration vs torch fp32 on the same bf16 operands (small batch), and graph-timed
launches at the full batch (MFMA utilisation vs the 2.5 PF/s dense bf16 peak).
CFGS: comma list of csu_conv2d_ex cfg values (0 = v2, 1 + k = igemm_dma config k)."""
import ctypes, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import torch
import torch.nn.functional as F
from csu import ops
from csu._lib import lib, CSU_BF16
d = torch.device("cuda")
bf = torch.bfloat16
cfgs = [int(c) for c in os.environ.get("CFGS", "0,1,2,3,4,5,6").split(",")]
B = int(os.environ.get("B", "16"))
# (name, op, H, W, C, N, k, stride, pad): op 0 forward conv, 1 input gradient (also ConvTranspose2d fwd)
shapes = [("u1 64->64", 0, 512, 512, 64, 64, 3, 1, 1), ("u1 128->64", 0, 512, 512, 128, 64, 3, 1, 1),
          ("u2 64->128", 0, 256, 256, 64, 128, 3, 1, 1), ("u2 128->128", 0, 256, 256, 128, 128, 3, 1, 1),
          ("u3 256->256", 0, 128, 128, 256, 256, 3, 1, 1), ("u4 512->512", 0, 64, 64, 512, 512, 3, 1, 1),
          ("u5 1024->1024", 0, 32, 32, 1024, 1024, 3, 1, 1),
          ("dg u1 64->64", 1, 512, 512, 64, 64, 3, 1, 1), ("dg u2 64->128", 1, 256, 256, 64, 128, 3, 1, 1),
          ("convT 128->64", 1, 512, 512, 64, 128, 2, 2, 0), ("convT 1024->512", 1, 64, 64, 512, 1024, 2, 2, 0),
          ("merge 64->128 s2", 0, 128, 128, 64, 128, 3, 2, 1), ("dg merge 64->128 s2", 1, 128, 128, 64, 128, 3, 2, 1),
          # CSWin 512x512: patch embed (3 -> 8 padded channels), CARAFE(4) encoders, merges
          ("embed 8->64 7x7 s4", 0, 512, 512, 8, 64, 7, 4, 2), ("carafe4 enc 16->144", 0, 128, 128, 16, 144, 3, 1, 1),
          ("dg carafe4 enc", 1, 128, 128, 16, 144, 3, 1, 1), ("carafe enc 32->36", 0, 64, 64, 32, 36, 3, 1, 1),
          ("dg carafe enc 32->36", 1, 64, 64, 32, 36, 3, 1, 1), ("merge 128->256 s2", 0, 64, 64, 128, 256, 3, 2, 1),
          ("dg merge 128->256 s2", 1, 64, 64, 128, 256, 3, 2, 1), ("merge 256->512 s2", 0, 32, 32, 256, 512, 3, 2, 1),
          ("dg merge 256->512 s2", 1, 32, 32, 256, 512, 3, 2, 1), ("carafe enc 128->36 16x16", 0, 16, 16, 128, 36, 3, 1, 1),
          ("dg carafe enc 128->36 16x16", 1, 16, 16, 128, 36, 3, 1, 1), ("carafe enc 64->36 32x32", 0, 32, 32, 64, 36, 3, 1, 1),
          ("dg carafe enc 64->36 32x32", 1, 32, 32, 64, 36, 3, 1, 1)]
if os.environ.get("ONLY"):
    shapes = [x for x in shapes if any(k in x[0] for k in os.environ["ONLY"].split(","))]


def graph_time(fn, n=10, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (n * reps) * 1e3


def run(op, g, src, w, bias, out, cfg):
    e = lib().csu_conv2d_ex(op, ctypes.byref(g), CSU_BF16, src.data_ptr(), w.data_ptr(),
                            bias.data_ptr() if bias is not None else None, out.data_ptr(), cfg,
                            torch.cuda.current_stream().cuda_stream)
    return e


def run_ws(op, g, src, w, bias, out, ws):
    """the plain operator with its K-split workspace (csu_conv2d_fwd_ws / _dgrad_ws)"""
    f = lib().csu_conv2d_fwd_ws if op == 0 else lib().csu_conv2d_dgrad_ws
    return f(ctypes.byref(g), CSU_BF16, src.data_ptr(), w.data_ptr(), bias.data_ptr() if bias is not None else None,
             out.data_ptr(), ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
             torch.cuda.current_stream().cuda_stream)


def case(name, op, H, W, C, N, k, s, p, b):
    g = ops._conv_geom(b, H, W, C, N, k, k, s, p)
    x = torch.randn(b, H, W, C, device=d).to(bf)
    wt = (torch.randn(N, C, k, k, device=d) / (C * k * k) ** 0.5).to(bf)
    bias = torch.randn(N, device=d) if op == 0 else None
    if op == 0:
        src, w = x, wt.permute(0, 2, 3, 1).contiguous()
        out = torch.empty(b, g.OH, g.OW, N, device=d, dtype=bf)
        ref = lambda: F.conv2d(x.permute(0, 3, 1, 2).float(), wt.float(), bias, s, p).permute(0, 2, 3, 1)
        flops = 2 * b * g.OH * g.OW * N * C * k * k
    else:
        src = torch.randn(b, g.OH, g.OW, N, device=d).to(bf)
        w = wt.permute(1, 2, 3, 0).contiguous()
        out = torch.empty(b, H, W, C, device=d, dtype=bf)
        ref = lambda: F.conv_transpose2d(src.permute(0, 3, 1, 2).float(), wt.float(), None, s, p,
                                         output_padding=(H - ((g.OH - 1) * s - 2 * p + k))).permute(0, 2, 3, 1)
        flops = 2 * b * g.OH * g.OW * N * C * k * k
    return g, src, w, bias, out, ref, flops


if __name__ == "__main__":
    print(f"batch {B}; cfgs {cfgs}")
    for sh in shapes:
        name, op = sh[0], sh[1]
        # parity at batch 2
        g, src, w, bias, out, ref, _ = case(*sh, b=2)
        r = ref()
        errs = []
        for c in cfgs:
            out.fill_(float("nan"))
            e = run(op, g, src, w, bias, out, c)
            torch.cuda.synchronize()
            if e:
                errs.append(f"{c}:n/a")
                continue
            rel = float((out.float() - r).norm() / r.norm())
            errs.append(f"{c}:{rel:.1e}")
        g, src, w, bias, out, ref, flops = case(*sh, b=B)
        times = []
        for c in cfgs:
            if run(op, g, src, w, bias, out, c):
                times.append(f"{c}:   -  ")
                continue
            t = graph_time(lambda: run(op, g, src, w, bias, out, c))
            times.append(f"{c}:{t:7.1f}us {flops / t / 1e6 / 2500:4.0%}")
        nws = lib().csu_conv2d_workspace(op, ctypes.byref(g), CSU_BF16)
        if nws:
            ws = torch.empty(nws, dtype=torch.uint8, device=d)
            t = graph_time(lambda: run_ws(op, g, src, w, bias, out, ws))
            times.append(f"ksplit:{t:7.1f}us {flops / t / 1e6 / 2500:4.0%}")
        # MIOpen (torch channels_last bf16) for reference
        try:
            xt = (src if op == 0 else src).permute(0, 3, 1, 2)
            wt_ = w.permute(0, 3, 1, 2) if op == 0 else w.permute(3, 0, 1, 2)
            if op == 0:
                fn = lambda: F.conv2d(xt, wt_, None, sh[7], sh[8])
            else:
                fn = lambda: F.conv_transpose2d(xt, wt_, None, sh[7], sh[8], output_padding=(sh[2] - ((g.OH - 1) * sh[7] - 2 * sh[8] + sh[6])))
            tm = graph_time(fn, n=5, reps=3)
            times.append(f"miopen:{tm:7.1f}us {flops / tm / 1e6 / 2500:4.0%}")
        except Exception as ex:  # noqa: BLE001
            times.append(f"miopen:err {type(ex).__name__}")
        print(f"{name:22s} {flops / 1e9:7.1f} GF | parity " + " ".join(errs) + " | " + " ".join(times), flush=True)
