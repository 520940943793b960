"""Run-to-run check of the HIP-graph train step: two copies of one model, each with its own
GraphedTrainStep, K replays on the same batches -> bitwise-equal losses and parameters?"""
import copy, os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd")]
import numpy as np
import torch
from csu.model import CSWinTransformer
from csu.train import GraphedTrainStep, bce_loss, make_optimizer
from csu.data import ellipse_batch

d = torch.device("cuda:0")
# DIAG=noconv / nolinear: keep that family of weight gradients off the side stream (bisecting a
# side-stream-in-graph race)
_diag = os.environ.get("DIAG", "")
if _diag:
    from csu import ops
    _orig_ok, _in_conv = ops._side_ok, [False]
    _cb = ops._Conv2dFn.backward

    def _conv_bwd(ctx, dy):
        _in_conv[0] = True
        try:
            return _cb(ctx, dy)
        finally:
            _in_conv[0] = False
    ops._Conv2dFn.backward = staticmethod(_conv_bwd)
    ops._side_ok = lambda *a, **k: (False if (_in_conv[0] == (_diag == "noconv")) else _orig_ok(*a, **k))
img, K = int(os.environ.get("IMG", "256")), int(os.environ.get("K", "6"))
torch.manual_seed(0)
m0 = CSWinTransformer(img_size=img, depth=[1, 2, 9, 1], split_size=[1, 2, 8, 8])
rng = np.random.default_rng(1)
batches = [tuple(t.to(d) for t in ellipse_batch(rng, 4, img)) for _ in range(2)]
DP = os.environ.get("DP") == "1"   # rep 0 single-process, reps >= 1 with the captured RCCL reducer
if DP:
    import torch.distributed as dist
    from csu.dist import GradAllReduce
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29631")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=d)
res = []
for rep in range(int(os.environ.get("REPS", "3"))):
    m = copy.deepcopy(m0).to(d)
    opt = make_optimizer(m, capturable=True)
    red = GradAllReduce(m.parameters()) if DP and rep > 0 else None
    gs = GraphedTrainStep(m, opt, bce_loss, batches[0][0], batches[0][1], torch.bfloat16,
                          warmup=int(os.environ.get("WARM", "2")), reducer=red)
    losses = [float(gs(*batches[i % 2])[0].item()) for i in range(K)]
    torch.cuda.synchronize()
    res.append((losses, [p.detach().clone() for p in m.parameters()],
                {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}))
    if red is not None:
        red.remove()
    del gs, opt
for i, (l, ps, gr) in enumerate(res[1:], 1):
    nd = sum(not torch.equal(a, b) for a, b in zip(ps, res[0][1]))
    print(f"rep {i}: losses equal {l == res[0][0]}, params differing {nd}/{len(ps)}  {l[-1]!r} vs {res[0][0][-1]!r}")
    if os.environ.get("GRADS"):
        bad = [n for n, g in gr.items() if not torch.equal(g, res[0][2][n])]
        print(f"  grads differing after the last replay: {len(bad)}: " + " ".join(bad[:40]))
