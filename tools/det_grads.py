"""Bitwise run-to-run check of every gradient of one bf16 train-step backward (same weights, same
inputs, R repetitions in one process): names the parameters whose gradient is not reproducible."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu.model import CSWinTransformer
from csu.train import bce_loss
from csu.data import ellipse_batch

d = torch.device("cuda:0")
img = int(os.environ.get("IMG", "256"))
R = int(os.environ.get("R", "6"))
torch.manual_seed(0)
model = CSWinTransformer(img_size=img, depth=[1, 2, 9, 1], split_size=[1, 2, 8, 8]).to(d)
x, t = ellipse_batch(np.random.default_rng(1), 4, img)
x, t = x.to(d), t.to(d)
ref = None
bad = {}
for r in range(R):
    model.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = model(x)
    loss = bce_loss(y, t)
    loss.backward()
    torch.cuda.synchronize()
    g = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    g["__prob"] = y.detach().float().clone()
    if ref is None:
        ref = g
        continue
    for n, v in g.items():
        if not torch.equal(v, ref[n]):
            bad.setdefault(n, 0)
            bad[n] += 1
print(f"{len(bad)} tensors differ across {R} repetitions")
for n, c in sorted(bad.items(), key=lambda kv: kv[0])[:60]:
    print(f"  {n}: {c}/{R - 1}")
