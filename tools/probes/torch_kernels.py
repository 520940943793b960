"""Which host ops launch the torch (non-csu) kernels of a train step?  Two eager steps of a bench
workload under torch.profiler; prints, per torch kernel name, the count and the launching aten ops.
    python tools/probes/torch_kernels.py [--img 256 --batch 8 --dtype fp32]"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]

import torch  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="fp32")
    a = ap.parse_args()
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss, make_optimizer
    import numpy as np
    d = torch.device("cuda")
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=a.img, split_size=[1, 2, 8, 8], simam=True).to(d)
    opt = make_optimizer(m, lr=1e-4)
    x, t = (v.to(d) for v in ellipse_batch(np.random.default_rng(0), a.batch, a.img))
    amp = a.dtype == "bf16"

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            y = m(x)
        loss = bce_loss(y, t)
        loss.backward()
        opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    ev = prof.events()
    cnt = collections.Counter()
    for e in ev:   # CPU ops (the innermost ones that launched a kernel) and their kernels
        if e.device_type.name == "CUDA":
            continue
        for k in getattr(e, "kernels", []) or []:
            if "csu" in k.name:
                continue
            cnt[(k.name[:50], e.name)] += 1
    for (k, op), n in cnt.most_common(30):
        print(f"{n:4d}  {k:50s}  <- {op}")

if __name__ == "__main__":
    main()
