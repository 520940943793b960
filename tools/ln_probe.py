"""LayerNorm forward / backward at the CSWin 512x512 B16 stage shapes: graph-timed launches vs the
HBM roofline (forward: x fp32 read, y bf16 + mean / rstd written; backward: x fp32, dy bf16, dres
fp32 read, dx fp32 + dx bf16 written), the backward with and without its dgamma / dbeta reduction."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]

SHAPES = [(262144, 64), (65536, 128), (16384, 256), (4096, 512)]


def child():
    import torch
    from csu._lib import lib, CSU_BF16, CSU_F32
    d = torch.device("cuda")
    L = lib()

    def graph_time(fn, n=20, reps=5):
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

    for rows, C in SHAPES:
        x = torch.randn(rows, C, device=d)
        gam, bet = torch.randn(C, device=d), torch.randn(C, device=d)
        y = torch.empty(rows, C, device=d, dtype=torch.bfloat16)
        m, r = torch.empty(rows, device=d), torch.empty(rows, device=d)
        dy = torch.randn(rows, C, device=d).bfloat16()
        dres = torch.randn(rows, C, device=d)
        dx, dxb = torch.empty_like(x), torch.empty(rows, C, device=d, dtype=torch.bfloat16)
        dg, db = torch.empty(C, device=d), torch.empty(C, device=d)
        ws = torch.empty(L.csu_layernorm_bwd_workspace(rows, C), device=d, dtype=torch.uint8)

        def fwd():
            assert L.csu_layernorm_fwd(rows, C, 1e-5, CSU_F32, x.data_ptr(), gam.data_ptr(), bet.data_ptr(), CSU_BF16,
                                       y.data_ptr(), m.data_ptr(), r.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0

        def bwd(reduce=True):
            assert L.csu_layernorm_bwd_ex(rows, C, CSU_F32, x.data_ptr(), gam.data_ptr(), m.data_ptr(), r.data_ptr(),
                                          CSU_BF16, dy.data_ptr(), dres.data_ptr(), dx.data_ptr(), dxb.data_ptr(),
                                          dg.data_ptr() if reduce else None, db.data_ptr() if reduce else None,
                                          ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream) == 0

        fwd()
        tf = graph_time(fwd)
        tb = graph_time(lambda: bwd(False))
        tbr = graph_time(bwd)
        bf_ = rows * C * (4 + 2) + rows * 8
        bb = rows * C * (4 + 2 + 4 + 4 + 2) + rows * 8
        print(f"rows {rows:7d} C {C:4d}: fwd {tf:6.2f} us ({bf_ / tf / 1e6 / 8:.2f} of 8 TB/s)  "
              f"bwd {tb:6.2f} us ({bb / tb / 1e6 / 8:.2f})  bwd+reduce {tbr:6.2f} us", flush=True)


if __name__ == "__main__":
    child()
