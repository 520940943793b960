"""Which aten ops launch GPU kernels in one eager bench step (torch.profiler, shapes recorded):
the PyTorch-side kernels left between the csu kernels."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from torch.profiler import profile, ProfilerActivity
from csu.model import CSWinTransformer
from csu.train import bce_loss, make_optimizer
from csu.data import ellipse_batch

d = torch.device("cuda:0")
torch.manual_seed(0)
model = CSWinTransformer(img_size=512, depth=[1, 2, 9, 1], split_size=[1, 2, 8, 8]).to(d)
opt = make_optimizer(model)
x, t = ellipse_batch(np.random.default_rng(1), 16, 512)
x, t = x.to(d), t.to(d)


def step():
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = model(x)
    loss = bce_loss(y, t)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
STACK = os.environ.get("STACK", "0") == "1"   # group by the Python call site instead of the shapes
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=STACK) as prof:
    step()
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_stack_n=6) if STACK else prof.key_averages(group_by_input_shape=True)
rows = [e for e in ka if e.key.startswith("aten::") and e.self_device_time_total > 0]
rows.sort(key=lambda e: -e.self_device_time_total)
for e in rows[:60]:
    where = " <- ".join(f.split("/")[-1] for f in e.stack[:6]) if STACK else str(e.input_shapes)[:150]
    print(f"{e.self_device_time_total:9.1f} us  n={e.count:4d}  {e.key:32s} {where}")

if os.environ.get("TREE", "0") == "1":
    # each aten op with device time, with its chain of CPU parents (autograd node names show where a
    # backward-side copy/add comes from)
    for e in prof.events():
        if not e.key.startswith("aten::") or e.device_time_total <= 0 or e.cpu_parent is None:
            continue
        if e.cpu_parent.key.startswith("aten::") and e.cpu_parent.device_time_total > 0:
            continue   # print the outermost aten op only
        chain, p = [], e.cpu_parent
        while p is not None and len(chain) < 5:
            chain.append(p.key[:60])
            p = p.cpu_parent
        print(f"{e.device_time_total:8.1f} us {e.key:22s} {str(e.input_shapes)[:70]:70s} <- {' <- '.join(chain)}")
