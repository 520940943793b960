"""Run-to-run check of K eager train steps (fwd, bwd, FusedAdamW) from one initial state."""
import copy, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu.model import CSWinTransformer
from csu.train import bce_loss, make_optimizer
from csu.data import ellipse_batch

d = torch.device("cuda:0")
img, K = 256, int(os.environ.get("K", "4"))
torch.manual_seed(0)
m0 = CSWinTransformer(img_size=img, depth=[1, 2, 9, 1], split_size=[1, 2, 8, 8])
rng = np.random.default_rng(1)
batches = [tuple(t.to(d) for t in ellipse_batch(rng, 4, img)) for _ in range(2)]
res = []
for rep in range(3):
    m = copy.deepcopy(m0).to(d)
    opt = make_optimizer(m, capturable=os.environ.get("CAPT") == "1")
    L = []
    for i in range(K):
        x, t = batches[i % 2]
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        loss = bce_loss(y, t)
        loss.backward()
        g = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        opt.step()
        L.append(loss.item())
    res.append((L, g))
for i, (L, g) in enumerate(res[1:], 1):
    bad = [n for n in g if not torch.equal(g[n], res[0][1][n])]
    print(f"rep {i}: losses equal {L == res[0][0]}; last-step grads differing {len(bad)}: {' '.join(bad[:12])}")
