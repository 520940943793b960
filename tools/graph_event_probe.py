"""Probe: do timing events recorded inside a captured HIP graph give per-replay kernel times?"""
import torch

x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
s = torch.cuda.Stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s):
    y = x @ x
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    e0.record()
    y = x @ x
    e1.record()
for i in range(3):
    g.replay()
torch.cuda.synchronize()
print("graph event ms", e0.elapsed_time(e1))
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(); y = x @ x; b.record(); torch.cuda.synchronize()
print("eager event ms", a.elapsed_time(b))
