"""Find which op breaks HIP-graph capture of the training step (prints a line per stage)."""
import faulthandler, os, sys
faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
import torch
import torch.nn.functional as F
d = torch.device("cuda")
torch.backends.cudnn.benchmark = True


def capture(name, fn, n_warm=2):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(n_warm):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print("capturing", name, flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    print("replaying", name, flush=True)
    g.replay()
    torch.cuda.synchronize()
    print("ok", name, flush=True)


from csu import ops
stage = sys.argv[1] if len(sys.argv) > 1 else "all"
conv = torch.nn.Conv2d(64, 128, 3, 2, 1).to(d)
x = torch.randn(4, 64, 32, 32, device=d).contiguous(memory_format=torch.channels_last).requires_grad_(True)


def f_conv():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = conv(x)
    y.float().sum().backward()


lin_w = torch.randn(256, 64, device=d, requires_grad=True)
xl = torch.randn(8, 1024, 64, device=d, requires_grad=True)


def f_lin():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.linear(xl, lin_w, None)
    y.float().sum().backward()


geom = ops.StripeGeometry(32, 64, 1, [(32, 1, 0), (1, 32, 32)], 32 ** -0.5)
qkv = torch.randn(2, 1024, 192, device=d, dtype=torch.bfloat16, requires_grad=True)
lw = [torch.randn(32, 1, 3, 3, device=d, requires_grad=True) for _ in range(2)]
lb = [torch.randn(32, device=d, requires_grad=True) for _ in range(2)]


def f_attn():
    y = ops.stripe_attention(qkv, geom, lw, lb)
    y.float().sum().backward()


ln_w = torch.ones(64, device=d, requires_grad=True)
ln_b = torch.zeros(64, device=d, requires_grad=True)


def f_ln():
    y = ops.layer_norm(xl, ln_w, ln_b, 1e-5, torch.bfloat16)
    y.float().sum().backward()


for name, fn in (("layernorm", f_ln), ("linear", f_lin), ("attn", f_attn), ("conv", f_conv)):
    if stage in ("all", name):
        capture(name, fn)

if stage in ("all", "model"):
    from csu.model import CSWinTransformer
    from csu.train import bce_loss, make_optimizer, GraphedTrainStep
    img, bs = int(os.environ.get("IMG", "128")), int(os.environ.get("BS", "2"))
    split = [1, 2, 4, 4] if img == 128 else [1, 2, 8, 8]
    m = CSWinTransformer(img_size=img, split_size=split).to(d)
    opt = make_optimizer(m, capturable=True)
    xi = torch.rand(bs, 3, img, img, device=d)
    ti = (torch.rand(bs, 1, img, img, device=d) > 0.5).float()
    print("capturing model", flush=True)
    gs = GraphedTrainStep(m, opt, bce_loss, xi, ti, torch.bfloat16, warmup=2)
    print("replaying model", flush=True)
    l, _ = gs(xi, ti)
    torch.cuda.synchronize()
    print("ok model", l.item(), flush=True)
