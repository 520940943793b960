"""Per-workgroup phase timeline of the whole-window attention kernels (debug build with WG_TIMING:
start / K,V staged / end stamps at 100 MHz) for one stripe-attention forward + backward at a stage
of the 512x512 B16 model.
    CSU_LIB_PATH=.../libcsu_hip_dbg.so python tools/attn_wg_timeline.py [stage 1..4]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
os.environ.setdefault("CSU_LIB_PATH", os.path.join(REPO, "cswin-simam-unet_amd", "csu", "_lib", "libcsu_hip_dbg.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from csu import ops  # noqa: E402
from csu._lib import lib  # noqa: E402

STAGES = {1: (128, 64, 2, 1), 2: (64, 128, 4, 2), 3: (32, 256, 8, 8), 4: (16, 512, 16, 16),
          # 1024x1024 B4: stage 3 (512-token windows, stripe_bwd_fused_w<512, 8 waves>)
          13: (64, 256, 8, 8)}


def main():
    st = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reso, C, heads, sw = STAGES[st]
    B = 4 if st >= 10 else 16
    d = torch.device("cuda")
    nb = 1 if sw == reso else 2
    brs = [(reso, sw, 0), (sw, reso, C // 2)] if nb == 2 else [(reso, reso, 0)]
    geom = ops.StripeGeometry(reso, C, heads // nb, brs, 32 ** -0.5)
    qkv = torch.randn(B, reso * reso, 3 * C, device=d, dtype=torch.bfloat16, requires_grad=True)
    ws = [torch.randn(C // nb, 1, 3, 3, device=d, requires_grad=True) for _ in range(nb)]
    bs = [torch.randn(C // nb, device=d, requires_grad=True) for _ in range(nb)]
    g = torch.randn(B, reso * reso, C, device=d, dtype=torch.bfloat16)
    for _ in range(3):
        out = ops.stripe_attention(qkv, geom, ws, bs)
        out.backward(g)
    torch.cuda.synchronize()
    L = lib()
    fn = L.csu_debug_attn_ts
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    buf = np.zeros((3, 6, 16384), dtype=np.uint64)
    assert fn(buf.ctypes.data) == 0
    if st <= 4 and max(sw * reso, reso * reso if sw == reso else 0) <= 256 or True:
        t = buf[1, :5].astype(np.int64)
        valid = (t[0] > 0) & (t[4] > 0)
        if valid.any():   # one-pass backward (stripe_bwd_fused_w): start, staged, prologue, main loop, end
            t = t[:, valid]
            ph = np.diff(t, axis=0) / 100.0
            tot = (t[4] - t[0]) / 100.0
            print(f"stage {st} fused bwd: {t.shape[1]} workgroups, span {(t[4].max() - t[0].min()) / 100:.1f} us, "
                  f"per WG p50 {np.median(tot):.1f} us = staging {np.median(ph[0]):.1f} + prologue "
                  f"{np.median(ph[1]):.1f} + main {np.median(ph[2]):.1f} + epilogue {np.median(ph[3]):.1f}")
            s2 = buf[2, :3].astype(np.int64)[:, valid]
            if (s2 > 0).all():   # the prologue's sub-phases (stamped into the unused dkdv slots)
                sub = np.diff(np.vstack([t[1], s2, t[2]]), axis=0) / 100.0
                print(f"   prologue p50: rows {np.median(sub[0]):.1f} + weight-gradient sums {np.median(sub[1]):.1f} + "
                      f"fragments and barrier {np.median(sub[2]):.1f} + partial stores {np.median(sub[3]):.1f} us")
                buf[2] = 0
    for k, name in enumerate(("fwd", "dq", "dkdv")):
        t = buf[k, :3].astype(np.int64)
        valid = t[0] > 0
        t = t[:, valid]
        n = t.shape[1]
        if n == 0:
            continue
        t0 = t[0].min()
        start, staged, end = (t[0] - t0) / 100.0, (t[1] - t0) / 100.0, (t[2] - t0) / 100.0   # us
        stage_us, comp_us = staged - start, end - staged
        span = end.max()
        # resident workgroups over time (1 us bins)
        bins = np.arange(0, span + 1.0, 1.0)
        res = [int(((start <= b) & (end > b)).sum()) for b in bins]
        print(f"stage {st} {name}: {n} workgroups, span {span:.1f} us; start spread p50 {np.median(start):.1f} "
              f"p90 {np.percentile(start, 90):.1f} max {start.max():.1f}; staging p50 {np.median(stage_us):.1f} "
              f"p90 {np.percentile(stage_us, 90):.1f}; compute p50 {np.median(comp_us):.1f} p90 {np.percentile(comp_us, 90):.1f}")
        print("   resident WGs per us:", res[:40])


if __name__ == "__main__":
    main()
