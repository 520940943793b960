"""Eager train steps on the default stream, then a GraphedTrainStep capture of the same model
(the order bench.py avoids).  Prints what happens at each stage.
    python tools/graph_after_eager.py <eager steps> <side-stream wgrad 0/1> [img] [batch]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    n_eager, side = int(sys.argv[1]), sys.argv[2] == "1"
    img = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    from csu import ops
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    ops.SIDE_WGRAD = side
    d = torch.device("cuda:0")
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=img, split_size=[1, 2, 8, 8]).to(d)
    opt = make_optimizer(m, capturable=True)
    x, t = (v.to(d) for v in ellipse_batch(np.random.default_rng(0), batch, img))
    for i in range(n_eager):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        bce_loss(y, t).backward()
        opt.step()
    torch.cuda.synchronize()
    if len(sys.argv) > 5 and sys.argv[5] == "drop":
        del y          # the caller's reference to the last eager step's graph
    print(f"eager steps done: {n_eager} (side-stream wgrad {side})", flush=True)
    stats = torch.cuda.memory_stats(d)
    print("allocator: active", stats.get("active.all.current"), "segments", stats.get("segment.all.current"), flush=True)
    gs = GraphedTrainStep(m, opt, bce_loss, x, t, torch.bfloat16, warmup=2)
    print("captured", flush=True)
    for _ in range(3):
        loss = gs(x, t)[0]
    torch.cuda.synchronize()
    print("replayed, loss", float(loss), flush=True)


if __name__ == "__main__":
    main()
