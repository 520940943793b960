"""Which parameters get a COPY of their side-stream weight gradient (AccumulateGrad clone on the
launching stream = a read before the end-of-backward join) instead of the side-stream buffer."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu import ops
from csu.model import CSWinTransformer
from csu.train import bce_loss
from csu.data import ellipse_batch

ptrs = set()
orig = ops._side_run


def spy(fn, *inputs):
    out = orig(fn, *inputs)
    for t in (out if isinstance(out, (tuple, list)) else (out,)):
        if isinstance(t, torch.Tensor):
            ptrs.add((t.untyped_storage().data_ptr(), t.untyped_storage().nbytes()))
    return out


ops._side_run = spy
d = torch.device("cuda:0")
torch.manual_seed(0)
m = CSWinTransformer(img_size=256, depth=[1, 2, 9, 1], split_size=[1, 2, 8, 8]).to(d)
x, t = ellipse_batch(np.random.default_rng(1), 4, 256)
with torch.autocast("cuda", dtype=torch.bfloat16):
    y = m(x.to(d))
bce_loss(y, t.to(d)).backward()
torch.cuda.synchronize()
inside = lambda p: any(b <= p < b + n for b, n in ptrs)
copied = [n for n, p in m.named_parameters() if p.grad is not None and not inside(p.grad.data_ptr())]
print(f"{len(ptrs)} side outputs; params whose grad is not a side buffer: {len(copied)}")
print(" ".join(c for c in copied if any(k in c for k in ("qkv", "fc1", "fc2", "proj", "down", "out", "concat", "conv"))))
