"""Plain-UNet BatchNorm2d + ReLU and MaxPool2d(2) kernels (csu_bn_relu_*, csu_maxpool2_*) vs
torch's own ops in float64 on the same inputs (unet:177-204: DoubleConv's BN / ReLU, Down's pool).
Tolerances: fp32 rtol 1e-4 (dx: atol 1e-5 * max|ref|); bf16 rel-L2 2e-2 (SURVEY §8c calibration)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _ref_bn(x64, w, b, rm, rv, training, relu, momentum=0.1, eps=1e-5):
    """torch BatchNorm2d (+ ReLU) in float64 on the NCHW view of an NHWC tensor."""
    xn = x64.permute(0, 3, 1, 2)
    y = F.batch_norm(xn, rm, rv, w, b, training, momentum, eps)
    if relu:
        y = F.relu(y)
    return y.permute(0, 2, 3, 1)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("shape", [(2, 16, 16, 64), (3, 5, 7, 128), (1, 2, 2, 1024), (4, 9, 11, 72)])
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_relu_train_vs_torch(shape, relu, dtype):
    from csu.unet import bn_relu_nhwc
    d = dev()
    g = torch.Generator().manual_seed(sum(shape))
    C = shape[-1]
    x = (torch.randn(shape, generator=g) * 3 + 5).to(dtype)        # far from 0: exercises the pivot shift
    dy = torch.randn(shape, generator=g).to(dtype)
    bn = nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.3)
        bn.running_mean.copy_(torch.randn(C, generator=g))
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
    ref = {k: v.double().clone() for k, v in bn.state_dict().items() if v.is_floating_point()}
    bnd = bn.to(d).train()
    xd = x.to(d).requires_grad_(True)
    y = bn_relu_nhwc(xd, bnd, relu)
    y.backward(dy.to(d))
    x64 = x.double().requires_grad_(True)
    w64 = ref["weight"].requires_grad_(True)
    b64 = ref["bias"].requires_grad_(True)
    yr = _ref_bn(x64, w64, b64, ref["running_mean"], ref["running_var"], True, relu)
    yr.backward(dy.double())
    assert y.dtype == dtype and y.shape == x.shape
    if dtype == torch.float32:
        torch.testing.assert_close(y.cpu().double(), yr.detach(), rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(xd.grad.cpu().double(), x64.grad, rtol=1e-4, atol=1e-5 * float(x64.grad.abs().max()))
        torch.testing.assert_close(bnd.weight.grad.cpu().double(), w64.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(bnd.bias.grad.cpu().double(), b64.grad, rtol=1e-4, atol=1e-4)
    else:
        assert _rel(y.cpu(), yr.detach()) < 2e-2
        assert _rel(xd.grad.cpu(), x64.grad) < 2e-2
        assert _rel(bnd.weight.grad.cpu(), w64.grad) < 2e-2
        assert _rel(bnd.bias.grad.cpu(), b64.grad) < 2e-2
    torch.testing.assert_close(bnd.running_mean.cpu().double(), ref["running_mean"], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bnd.running_var.cpu().double(), ref["running_var"], rtol=1e-4, atol=1e-5)
    assert int(bnd.num_batches_tracked) == 1


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_relu_eval_vs_torch(dtype):
    from csu.unet import bn_relu_nhwc
    d = dev()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 8, 8, 64, generator=g).to(dtype)
    dy = torch.randn(2, 8, 8, 64, generator=g).to(dtype)
    bn = nn.BatchNorm2d(64)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(64, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(64, generator=g))
        bn.running_mean.copy_(torch.randn(64, generator=g) * 0.2)
        bn.running_var.copy_(torch.rand(64, generator=g) + 0.5)
    ref = {k: v.double().clone() for k, v in bn.state_dict().items() if v.is_floating_point()}
    bnd = bn.to(d).eval()
    xd = x.to(d).requires_grad_(True)
    y = bn_relu_nhwc(xd, bnd)
    y.backward(dy.to(d))
    x64 = x.double().requires_grad_(True)
    w64 = ref["weight"].requires_grad_(True)
    b64 = ref["bias"].requires_grad_(True)
    yr = _ref_bn(x64, w64, b64, ref["running_mean"], ref["running_var"], False, True)
    yr.backward(dy.double())
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(y.cpu(), yr.detach()) < tol and _rel(xd.grad.cpu(), x64.grad) < tol
    assert _rel(bnd.weight.grad.cpu(), w64.grad) < tol and _rel(bnd.bias.grad.cpu(), b64.grad) < tol
    torch.testing.assert_close(bnd.running_mean.cpu().double(), ref["running_mean"])    # untouched in eval
    assert int(bnd.num_batches_tracked) == 0


def test_bn_relu_deterministic():
    from csu.unet import bn_relu_nhwc
    d = dev()
    g = torch.Generator().manual_seed(3)
    x = torch.randn(8, 32, 32, 128, generator=g).to(d)
    dy = torch.randn(8, 32, 32, 128, generator=g).to(d)
    outs = []
    for _ in range(2):
        bn = nn.BatchNorm2d(128).to(d)
        xd = x.clone().requires_grad_(True)
        y = bn_relu_nhwc(xd, bn)
        y.backward(dy)
        outs.append((y.detach(), xd.grad, bn.weight.grad, bn.running_var.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(2, 8, 8, 64), (3, 7, 9, 16), (1, 2, 2, 1024)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_maxpool2_vs_torch(shape, dtype):
    """Ties (small-integer inputs) pick torch's first maximum; odd H / W drop the last row/column."""
    from csu.unet import max_pool2_nhwc
    d = dev()
    g = torch.Generator().manual_seed(shape[1])
    x = torch.randint(-3, 4, shape, generator=g).to(dtype)
    dy = torch.randn(shape[0], shape[1] // 2, shape[2] // 2, shape[3], generator=g).to(dtype)
    xd = x.to(d).requires_grad_(True)
    y = max_pool2_nhwc(xd)
    y.backward(dy.to(d))
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    yr.backward(dy)
    assert torch.equal(y.cpu(), yr.detach())
    assert torch.equal(xd.grad.cpu(), xr.grad)


def test_unet_graph_step_uses_csu_bn(monkeypatch):
    """A UNet train step launches the csu BN / pool kernels (ledger names) and no torch batch_norm."""
    from csu import ledger
    from csu.unet import UNet
    d = dev()
    m = UNet(3, 1).to(d).train()
    x = torch.rand(2, 3, 32, 32, device=d)
    seen = []
    orig = ledger.launch

    def spy(name, fn, *a, **k):
        seen.append(name)
        return orig(name, fn, *a, **k)
    import csu.unet as U
    monkeypatch.setattr(U, "launch", spy)
    calls = []
    monkeypatch.setattr(torch.nn.functional, "batch_norm", lambda *a, **k: calls.append(1))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.mean().backward()
    assert seen.count("bn_relu_fwd") == 18 and seen.count("bn_relu_bwd") == 18
    assert seen.count("maxpool2_fwd") == 4 and seen.count("maxpool2_bwd") == 4
    assert not calls
