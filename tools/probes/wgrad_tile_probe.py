"""Token weight gradients (dW = dY^T X, db) at steady state: the grouped register-staged tile
(csu_linear_wgrad_group + csu_wslab_reduce_batch, what the step runs) against the LDS-DMA conv
weight-gradient tiles on the same Linear as a 1x1 conv (csu_conv2d_wgrad_ex cfg 1 + k, incl. its
colsum).  Run against a lib built with -DWD_PROBE256 (cfg 5 = the 256 x 256 DMA tile).
  ROWS=16384 ITEMS=8 CFGS=4,5 python tools/probes/wgrad_tile_probe.py"""
import ctypes, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "cswin-simam-unet_amd"),
                os.path.join(os.path.dirname(__file__), "..")]
import torch
from csu import ops, _lib
from csu._lib import lib, CSU_BF16
from conv_probe import graph_time  # noqa: E402
d = torch.device("cuda")
M = int(os.environ.get("ROWS", "16384"))
G = int(os.environ.get("ITEMS", "8"))
cfgs = [int(c) for c in os.environ.get("CFGS", "4,5").split(",")]
shapes = [(768, 256), (256, 256), (1024, 256), (256, 1024), (384, 128), (512, 128), (128, 512)]
print(f"M {M}; {G} items per grouped launch (time per item); conv cfgs {cfgs} (one call per Linear)")
for N, K in shapes:
    dy = torch.randn(M, N, device=d).to(torch.bfloat16)
    x = torch.randn(M, K, device=d).to(torch.bfloat16)
    ref = torch.cat([(dy.float().t() @ x.float()).reshape(-1), dy.float().sum(0)])
    flops = 2 * M * N * K
    tn, tk, ch = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    nb = lib().csu_linear_wgrad_group_plan(M, N, K, ctypes.byref(tn), ctypes.byref(tk), ctypes.byref(ch))
    # the step groups many Linears per launch (few chunks each): G items of this shape, time / G
    slabs = [torch.empty(max(nb // 4, 4), device=d) for _ in range(G)]
    outs = [torch.empty(N * K + N, device=d) for _ in range(G)]
    out = outs[0]
    its = (_lib.WgradGroupItem * G)(*[_lib.WgradGroupItem(dy.data_ptr(), x.data_ptr(), o.data_ptr(), sl.data_ptr() if nb else None,
                                                          M, N, K) for o, sl in zip(outs, slabs)])
    wis = (_lib.WslabItem * G)(*[_lib.WslabItem(sl.data_ptr(), o.data_ptr(), N, K, tn.value, tk.value, ch.value, 0)
                                 for o, sl in zip(outs, slabs)])

    def grp():
        st = torch.cuda.current_stream().cuda_stream
        assert lib().csu_linear_wgrad_group(its, G, st) == 0
        if ch.value > 1:
            assert lib().csu_wslab_reduce_batch(wis, G, st) == 0
    out.zero_(); grp(); torch.cuda.synchronize()
    errs = [f"grp:{float((out - ref).norm() / ref.norm()):.1e}"]
    times = [f"grp {tn.value}x{tk.value}/{ch.value}:{graph_time(grp, n=5, reps=3) / G:7.1f}us"]
    g = ops._conv_geom(M // 1024, 32, 32, K, N, 1, 1, 1, 0)
    nws = max(lib().csu_conv2d_wgrad_workspace_ex(ctypes.byref(g), c) for c in cfgs)
    work = torch.empty(max(nws, 16), dtype=torch.uint8, device=d)
    for c in cfgs:
        call = lambda: lib().csu_conv2d_wgrad_ex(ctypes.byref(g), CSU_BF16, x.data_ptr(), dy.data_ptr(), 0, out.data_ptr(),
                                                work.data_ptr(), work.numel(), c, torch.cuda.current_stream().cuda_stream)
        out.zero_()
        if call():
            errs.append(f"{c}:n/a"); continue
        torch.cuda.synchronize()
        errs.append(f"{c}:{float((out - ref).norm() / ref.norm()):.1e}")
        times.append(f"cfg{c}:{graph_time(call, n=5, reps=3):7.1f}us")
    t0 = float(times[0].split(":")[1][:-2])
    print(f"N {N:5d} K {K:5d} {flops / 1e9:6.1f} GF ({flops / t0 / 1e6 / 2500:4.0%} grp) | " + " ".join(errs) + " | " + " ".join(times), flush=True)
