"""Minimal check of cross-stream fork/join edges in a captured HIP graph: a side-stream branch
forked and joined many times (as the side-stream weight gradients are) must be complete before the
main stream reads its outputs."""
import torch
d = torch.device("cuda:0")
main = torch.cuda.Stream()
side = torch.cuda.Stream()
N = 24
src = [torch.randn(4096, 4096, device=d) for _ in range(N)]
outs = [torch.empty(4096, 4096, device=d) for _ in range(N)]
acc = torch.zeros(4096, 4096, device=d)
big = torch.randn(8192, 8192, device=d)
for st in (main, side):   # hipBLASLt handles exist before the capture
    with torch.cuda.stream(st):
        torch.mm(src[0], src[0])
        torch.mm(big, big)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(main):
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=main):
        acc.zero_()
        evs = []
        for i in range(N):
            side.wait_stream(main)
            with torch.cuda.stream(side):
                torch.mm(src[i], src[i], out=outs[i])       # slow side work
            e = torch.cuda.Event()
            e.record(side)
            evs.append(e)
            torch.mm(big, big)                               # main keeps going
        for e in evs:
            main.wait_event(e)
        for i in range(N):
            acc.add_(outs[i])                                # reads the side outputs
ref = sum(torch.mm(s, s) for s in src)
bad = 0
for r in range(10):
    for o in outs:
        o.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    if not torch.allclose(acc, ref, rtol=1e-3, atol=1e-2):
        bad += 1
print(f"fork/join graph: {bad}/10 replays read incomplete side outputs")
