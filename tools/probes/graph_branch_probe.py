"""Does a replayed HIP graph run two captured branches concurrently?  A = a chain of small
(latency-bound) GEMMs on the capturing stream, B = a few large GEMMs forked onto a side stream and
joined at the end.  Prints the replay time of A alone, B alone, A then B (one stream) and A || B.
    python tools/probes/graph_branch_probe.py"""
import torch


def graph_of(fn, prio=0):
    s = torch.cuda.Stream(priority=prio)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    return g


def time_graph(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    d = torch.device("cuda")
    xa = torch.randn(16384, 256, device=d, dtype=torch.bfloat16)
    wa = torch.randn(256, 256, device=d, dtype=torch.bfloat16)
    xb = torch.randn(16384, 1024, device=d, dtype=torch.bfloat16)
    wb = torch.randn(16384, 256, device=d, dtype=torch.bfloat16)
    oa = [torch.empty(16384, 256, device=d, dtype=torch.bfloat16) for _ in range(200)]
    ob = [torch.empty(1024, 256, device=d, dtype=torch.bfloat16) for _ in range(2)]

    def A():
        y = xa
        for o in oa:
            torch.mm(y, wa, out=o)
            y = o

    def B():
        for o in ob:
            torch.mm(xb.t(), wb, out=o)   # a weight-gradient shape: (1024 x 16384) @ (16384 x 256)

    side = torch.cuda.Stream()
    side_lo = torch.cuda.Stream(priority=0)

    def AB_par():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            B()
        A()
        main.wait_stream(side)

    def AB_ser():
        A()
        B()

    lo, hi = torch.cuda.Stream.priority_range()
    print("priority range (low, high):", torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else "n/a")
    ga, gb, gs, gp = graph_of(A), graph_of(B), graph_of(AB_ser), graph_of(AB_par)
    gph = graph_of(AB_par, prio=hi)     # the chain captured on a high-priority stream, B on a default one
    for name, g in (("A alone", ga), ("B alone", gb), ("A then B", gs), ("A || B", gp), ("A||B hiA", gph),
                    ("A alone", ga), ("A || B", gp), ("A then B", gs), ("A||B hiA", gph)):
        print(f"{name:10s} {time_graph(g):9.1f} us per replay", flush=True)


if __name__ == "__main__":
    main()
