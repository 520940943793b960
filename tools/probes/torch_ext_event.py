"""Probe: csu_event_record_ext inside torch.cuda.graph captures (global / thread_local modes)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "cswin-simam-unet_amd")]
import torch
from csu.ledger import _HipEvent
x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
for mode in ("thread_local", "global", "relaxed"):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        y = x * 2.0 + 1.0
    torch.cuda.synchronize()
    e0, e1 = _HipEvent(), _HipEvent()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            e0.record()
            y = x * 2.0 + 1.0
            e1.record()
        g.replay(); torch.cuda.synchronize()
        print(mode, "ok", "%.1f us" % (e0.elapsed_time(e1) * 1e3), flush=True)
    except Exception as ex:
        print(mode, "FAILED", repr(ex)[:300], flush=True)
