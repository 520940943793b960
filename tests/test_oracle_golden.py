"""Pin the CPU oracle against golden vectors produced by the reference itself.

The fixtures were computed by the reference in fp64 from fp32-representable inputs and stored as
fp32; the oracle recomputes in fp64, so agreement is to fp32 rounding (tolerances below)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import cswin_ref as O
from oracle import unet_ref as U
from oracle.recipe import recipe_from_contract

RTOL, ATOL = 2e-5, 2e-6


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def t64(a):
    return torch.from_numpy(np.asarray(a)).double()


def close(a, b, rtol=RTOL, atol=ATOL):
    a = a.detach().double().numpy() if torch.is_tensor(a) else np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(1.0, float(np.abs(b).max()))
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol * scale)


def test_f1_lepe_attention(golden_dir):
    z = load(golden_dir, "f1_lepe.npz")
    ncase = len([k for k in z.files if k.endswith("_meta")])
    assert ncase >= 8
    for ci in range(ncase):
        reso, idx, sw, cb, heads = (int(v) for v in z[f"c{ci}_meta"])
        qkv = t64(z[f"c{ci}_qkv"]).requires_grad_(True)
        w = t64(z[f"c{ci}_w"]).requires_grad_(True)
        b = t64(z[f"c{ci}_b"]).requires_grad_(True)
        hs, ws = O.stripe_geometry(reso, idx, sw)
        y = O.lepe_attention(qkv[0], qkv[1], qkv[2], reso, hs, ws, heads, w, b, (cb // heads) ** -0.5)
        close(y, z[f"c{ci}_out"])
        y.backward(t64(z[f"c{ci}_gout"]))
        close(qkv.grad, z[f"c{ci}_dqkv"])
        close(w.grad, z[f"c{ci}_dw"])
        close(b.grad, z[f"c{ci}_db"])


def _params(z, pre):
    return {k[len(pre) + 2:]: t64(z[k]).requires_grad_(True) for k in z.files if k.startswith(pre + "p:")}


def _check_grads(z, pre, p):
    for k, v in p.items():
        if pre + "g:" + k in z.files:
            close(v.grad, z[pre + "g:" + k])


def test_f2_block(golden_dir):
    z = load(golden_dir, "f2_block.npz")
    for pre in ("two_", "last_", "s1_"):
        dim, reso, heads, sw, last = (int(v) for v in z[pre + "meta"])
        p = _params(z, pre)
        x = t64(z[pre + "x"]).requires_grad_(True)
        y = O.cswin_block(x, {"." + k: v for k, v in p.items()}, "", reso, heads, sw, bool(last))
        close(y, z[pre + "y"])
        y.backward(t64(z[pre + "gy"]))
        close(x.grad, z[pre + "dx"])
        _check_grads(z, pre, p)


def mask_provider(z, pre, p):
    """Oracle drop provider over the masks the reference block recorded (f9_dropout.npz)."""
    def drop(name, shape):
        k = pre + "mask:" + name
        if k not in z.files:
            return None
        m = t64(z[k]) / (1 - p)
        assert tuple(m.shape) == tuple(shape), (name, m.shape, shape)
        return m
    return drop


def test_f9_dropout_block(golden_dir):
    """Train-mode CSWinBlock at the reference main() rates (drop / attn_drop / drop_path 0.3):
    the oracle under the reference's recorded masks reproduces its y, dx and every gradient."""
    z = load(golden_dir, "f9_dropout.npz")
    p_drop = float(z["p"])
    for pre in ("two_", "last_"):
        dim, reso, heads, sw, last = (int(v) for v in z[pre + "meta"])
        assert len([k for k in z.files if k.startswith(pre + "mask:")]) == (5 if last else 6)
        p = _params(z, pre)
        x = t64(z[pre + "x"]).requires_grad_(True)
        y = O.cswin_block(x, {"blk." + k: v for k, v in p.items()}, "blk", reso, heads, sw, bool(last),
                          drop=mask_provider(z, pre, p_drop))
        close(y, z[pre + "y"])
        y.backward(t64(z[pre + "gy"]))
        close(x.grad, z[pre + "dx"])
        _check_grads(z, pre, p)
        # the masks matter: without them the forward differs
        with torch.no_grad():
            y0 = O.cswin_block(x, {"blk." + k: v for k, v in p.items()}, "blk", reso, heads, sw, bool(last))
        assert float((y0 - t64(z[pre + "y"])).abs().max()) > 1e-2


def test_f3_modules(golden_dir):
    z = load(golden_dir, "f3_modules.npz")
    cases = {
        "merge_": lambda x, p: O.merge_block(x, p, ""),
        "embed_": lambda x, p: O.patch_embed(x, {"stage1_conv_embed" + k: v for k, v in p.items()}),
        "carafe_": lambda x, p: O.carafe(x, p, "", 2),
        "carafe4_": lambda x, p: O.carafe(x, p, "", 4),
        "mlp_": lambda x, p: O.mlp(x, p, ""),
    }
    for pre, fn in cases.items():
        p = _params(z, pre)
        x = t64(z[pre + "x"]).requires_grad_(True)
        y = fn(x, {"." + k: v for k, v in p.items()})
        close(y, z[pre + "y"])
        y.backward(t64(z[pre + "gy"]))
        close(x.grad, z[pre + "dx"])
        _check_grads(z, pre, p)


def test_f4_whole_model(golden_dir):
    z = load(golden_dir, "f4_model.npz")
    cfg = O.CSWinConfig(img_size=128, split_size=(1, 2, 4, 4))
    p = {k: v.double().requires_grad_(True) for k, v in O.recipe_params(cfg, seed=0).items()}
    x, t = t64(z["x"]), t64(z["t"])
    y, (x1, x2, x3) = O.cswin_forward(p, x, cfg, return_skips=True)
    close(y, z["y"], rtol=1e-4, atol=1e-6)
    close(x1, z["x1"], rtol=1e-4, atol=1e-5)
    loss = O.bce_loss(y, t)
    close(loss, z["loss"], rtol=1e-5)
    loss.backward()
    names = list(z["grad_names"])
    assert names == [k for k, _ in O.state_dict_contract(cfg)]
    gn = np.array([p[k].grad.norm().item() for k in names])
    np.testing.assert_allclose(gn, z["grad_norms"], rtol=2e-3, atol=1e-7)
    for k in z.files:
        if k.startswith("g:"):
            close(p[k[2:]].grad, z[k], rtol=1e-3, atol=1e-5)


def test_f5_metrics(golden_dir):
    z = load(golden_dir, "f5_metrics.npz")
    p, t = torch.from_numpy(z["p"]), torch.from_numpy(z["t"])
    close(O.bce_loss(p, t), z["bce"], rtol=1e-6)
    d, i = O.dice_iou(p, t)
    assert abs(d - float(z["dice"])) < 1e-6 and abs(i - float(z["iou"])) < 1e-6
    d0, i0 = O.dice_iou(torch.zeros(8), torch.zeros(8))
    assert abs(d0 - float(z["dice_empty"])) < 1e-6 and abs(i0 - float(z["iou_empty"])) < 1e-6


def test_f6_unet(golden_dir):
    z = load(golden_dir, "f6_unet.npz")
    p = recipe_from_contract(U.unet_contract(), seed=1)
    for k, v in p.items():
        if v.is_floating_point() and "running" not in k:
            v.requires_grad_(True)
    x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["t"])
    y = U.unet_forward(p, x, training=True)
    close(y, z["y_train"], rtol=1e-3, atol=1e-5)
    loss = O.bce_loss(y, t)
    close(loss, z["loss"], rtol=1e-5)
    loss.backward()
    names = list(z["grad_names"])
    gn = np.array([p[k].grad.norm().item() for k in names])
    np.testing.assert_allclose(gn, z["grad_norms"], rtol=5e-3, atol=1e-6)
    for k in z.files:
        if k.startswith("rm:"):
            close(p[k[3:]], z[k], rtol=1e-4, atol=1e-6)
    with torch.no_grad():
        ye = U.unet_forward(p, x, training=False)
    close(ye, z["y_eval"], rtol=1e-3, atol=1e-5)


def test_f7_contract(golden_dir):
    with open(os.path.join(golden_dir, "f7_contract.json")) as f:
        ref = json.load(f)
    cfgs = {"default_224": O.CSWinConfig(img_size=224),
            "cfg512": O.CSWinConfig(img_size=512, split_size=(1, 2, 8, 8)),
            "deep512": O.CSWinConfig(img_size=512, depth=(2, 4, 32, 2), split_size=(1, 2, 8, 8))}
    for name, cfg in cfgs.items():
        assert [[k, list(s)] for k, s in O.state_dict_contract(cfg)] == ref[name], name
    assert [[k, list(s)] for k, s in U.unet_contract()] == ref["unet"]


def test_known_answer_lepe_center_column():
    """SURVEY §4 KAT (i): with width-1 stripes (idx 0, sw 1) the LePE kernel gradient is non-zero
    only in the centre column (window-local zero padding, cswin:256-269)."""
    torch.manual_seed(0)
    reso, cb = 8, 32
    q, k, v = (torch.randn(1, reso * reso, cb, dtype=torch.float64) for _ in range(3))
    w = torch.randn(cb, 1, 3, 3, dtype=torch.float64, requires_grad=True)
    b = torch.zeros(cb, dtype=torch.float64, requires_grad=True)
    y = O.lepe_attention(q, k, v, reso, reso, 1, 1, w, b, cb ** -0.5)
    y.sum().backward()
    g = w.grad.abs().sum(dim=(0, 1, 2))
    assert g[0] == 0 and g[2] == 0 and g[1] > 0
