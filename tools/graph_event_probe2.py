"""Probe: timing events created with external=True, recorded inside a captured HIP graph -- do they
give per-replay kernel durations (vs the same kernels timed eagerly)?"""
import torch

d = torch.device("cuda")
x = torch.randn(8192, 8192, device=d, dtype=torch.bfloat16)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3):
        y = x @ x
torch.cuda.synchronize()
n = 6
ev = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(n + 1)]
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    ev[0].record()
    for i in range(n):
        y = x @ x if i % 2 == 0 else (x + 1.0)
        ev[i + 1].record()
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", r, ["%.1f" % (ev[i].elapsed_time(ev[i + 1]) * 1e3) for i in range(n)], "us")
# eager reference
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for op in ("mm", "add"):
    a.record()
    for _ in range(10):
        y = x @ x if op == "mm" else (x + 1.0)
    b.record()
    torch.cuda.synchronize()
    print("eager", op, "%.1f us" % (a.elapsed_time(b) * 1e3 / 10))
# graph without events: total per replay
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2, stream=s):
    for i in range(n):
        y = x @ x if i % 2 == 0 else (x + 1.0)
g2.replay(); torch.cuda.synchronize()
a.record(); g2.replay(); b.record(); torch.cuda.synchronize()
a2 = torch.cuda.Event(enable_timing=True); b2 = torch.cuda.Event(enable_timing=True)
a2.record(); g.replay(); b2.record(); torch.cuda.synchronize()
print("graph replay total: plain %.1f us, with events %.1f us" % (a.elapsed_time(b) * 1e3, a2.elapsed_time(b2) * 1e3))
