"""CPU oracle for the CSWin-UNet training path -- TEST INFRASTRUCTURE ONLY.

This module is a functional restatement (plain PyTorch, CPU, fp32/fp64) of the algorithm in
``train_cswinunet_segmentation.py`` of TrungMasterChef/CSWin-SimAM-UNet.  It is the checker the
parity tests, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` compare the
HIP path against.  Nothing in the product package (``cswin-simam-unet_amd/csu``) imports it.

Parity pin: every function here is checked against golden vectors produced by running the
reference itself (``tests/golden/make_golden.py``; fixtures ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.  SimAM has no reference implementation, so
``simam`` below is "parity unpinned" vs the reference: it follows the published SimAM formula.

Citations: ``cswin:N`` = reference ``train_cswinunet_segmentation.py`` line N.

Parameters are passed as a flat ``{state_dict_key: tensor}`` mapping using the reference's
state_dict key names (cswin:489-688), so weights interchange with reference ``.pth`` files.

Dropout (train mode, cswin:188-195/246/290/344/367-368/512): the functions take an optional mask
provider ``drop(name, shape) -> scale tensor or None`` (0 or 1/keep per element; per sample for
DropPath), so a parity test can replay exactly the masks the device drew.  Names: ``pos``
(pos_drop), ``<block>.attn<i>`` (P of branch i, (B*nWin, heads, N, N)), ``<block>.mlp.h`` /
``<block>.mlp.o`` (Mlp hidden / output), ``<block>.dp_attn`` / ``<block>.dp_mlp`` (the two
DropPath draws, shape (B,)).  Without a provider the forward is the eval / p = 0 forward.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


# --------------------------------------------------------------------------------------------
# Stripe-window layout (cswin:199-217)
# --------------------------------------------------------------------------------------------
def stripe_partition(t: torch.Tensor, reso: int, hs: int, ws: int) -> torch.Tensor:
    """(B, reso*reso, C) tokens -> (B*nWin, hs*ws, C) windows.

    Window order batch -> H-block -> W-block, tokens row-major inside a window (cswin:199-206,
    reached through ``im2cswin`` cswin:248-254)."""
    B, L, C = t.shape
    g = t.reshape(B, reso // hs, hs, reso // ws, ws, C)
    return g.permute(0, 1, 3, 2, 4, 5).reshape(-1, hs * ws, C)


def stripe_merge(w: torch.Tensor, reso: int, hs: int, ws: int) -> torch.Tensor:
    """Inverse of :func:`stripe_partition` -> (B, reso*reso, C) (cswin:209-217)."""
    nwin = (reso // hs) * (reso // ws)
    B = w.shape[0] // nwin
    C = w.shape[-1]
    g = w.reshape(B, reso // hs, reso // ws, hs, ws, C).permute(0, 1, 3, 2, 4, 5)
    return g.reshape(B, reso * reso, C)


def stripe_geometry(reso: int, idx: int, split: int) -> Tuple[int, int]:
    """(H_sp, W_sp) of a LePEAttention branch (cswin:232-240)."""
    if idx == -1:
        return reso, reso
    if idx == 0:
        return reso, split
    if idx == 1:
        return split, reso
    raise ValueError(f"ERROR MODE {idx}")


# --------------------------------------------------------------------------------------------
# LePE stripe attention (cswin:220-298)
# --------------------------------------------------------------------------------------------
def lepe_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, reso: int, hs: int, ws: int,
                   heads: int, w: torch.Tensor, b: torch.Tensor, scale: float,
                   attn_drop: float = 0.0, training: bool = False, attn_mask=None) -> torch.Tensor:
    """softmax(q*scale @ k^T) @ v + dwconv3x3(v) per stripe window, window-local zero padding.

    q, k, v: (B, L, Cb) with L == reso*reso (assert cswin:281).  w: (Cb,1,3,3), b: (Cb,).
    Returns (B, L, Cb)."""
    B, L, Cb = q.shape
    assert L == reso * reso, "flatten img_tokens has wrong size"
    hd = Cb // heads
    N = hs * ws

    def heads_first(t):  # (B', N, Cb) -> (B', heads, N, hd)   (cswin:253)
        return t.reshape(t.shape[0], N, heads, hd).permute(0, 2, 1, 3)

    qw = heads_first(stripe_partition(q, reso, hs, ws))
    kw = heads_first(stripe_partition(k, reso, hs, ws))
    vwin = stripe_partition(v, reso, hs, ws)                       # (B', N, Cb)
    # LePE: depthwise 3x3 on each window as its own image (cswin:256-269, 244)
    vimg = vwin.transpose(1, 2).reshape(-1, Cb, hs, ws)
    lepe = F.conv2d(vimg, w, b, stride=1, padding=1, groups=Cb)
    lepe = lepe.reshape(-1, heads, hd, N).permute(0, 1, 3, 2)
    vw = heads_first(vwin)
    # scores in the input dtype, softmax over keys (cswin:287-292)
    att = torch.matmul(qw * scale, kw.transpose(-2, -1))
    att = torch.softmax(att, dim=-1)
    if attn_mask is not None:                                       # attn_drop with given masks (cswin:290)
        att = att * attn_mask(att.shape)
    elif attn_drop > 0 and training:
        att = F.dropout(att, attn_drop, training=True)
    o = torch.matmul(att, vw) + lepe
    o = o.transpose(1, 2).reshape(-1, N, Cb)                       # head merge (cswin:293)
    return stripe_merge(o, reso, hs, ws)                            # cswin:296


# --------------------------------------------------------------------------------------------
# Blocks
# --------------------------------------------------------------------------------------------
def _ln(x, p, key):
    return F.layer_norm(x, (x.shape[-1],), p[key + ".weight"], p[key + ".bias"], 1e-5)


def _lin(x, p, key):
    return F.linear(x, p[key + ".weight"], p.get(key + ".bias"))


def _drop(drop, name, t):
    """t times the provider's mask of `name` (identity without a provider / mask)."""
    m = drop(name, tuple(t.shape)) if drop is not None else None
    return t if m is None else t * m


def _drop_path(drop, name, t):
    """DropPath (timm drop_path, cswin:344): per-sample scale of `name`."""
    m = drop(name, (t.shape[0],)) if drop is not None else None
    return t if m is None else t * m.reshape(-1, *([1] * (t.dim() - 1)))


# Optional fp8 form of the Mlp (None: the reference form).  The fp8 parity tests install a function
# (x, p, key, hidden_mask) -> fc2 output, or None to keep the reference form for that Mlp, that runs
# the roundings of the fp8 weight format (oracle/fp8_ref.py).
MLP_FP8 = None


def mlp(x: torch.Tensor, p: Params, key: str, drop=None) -> torch.Tensor:
    """fc1 -> exact-erf GELU -> Dropout -> fc2 -> Dropout (cswin:180-196)."""
    if MLP_FP8 is not None:
        hshape = tuple(x.shape[:-1]) + (p[key + ".fc1.weight"].shape[0],)
        m_h = drop(key + ".h", hshape) if drop is not None else None
        y = MLP_FP8(x, p, key, m_h)
        if y is not None:
            return _drop(drop, key + ".o", y)
    h = _drop(drop, key + ".h", F.gelu(_lin(x, p, key + ".fc1")))
    return _drop(drop, key + ".o", _lin(h, p, key + ".fc2"))


# Optional transform of the norm1 output before qkv (None: identity).  The fp8 parity test installs
# the e4m3 per-token quantiser of BASELINE config 5 here (the format's activation rounding).
QKV_INPUT_QUANT = None


def cswin_block(x: torch.Tensor, p: Params, key: str, reso: int, heads: int, split: int,
                last_stage: bool, qk_scale=None, drop=None) -> torch.Tensor:
    """Pre-LN CSWin block (cswin:301-370)."""
    B, L, C = x.shape
    assert L == reso * reso, "flatten img_tokens has wrong size"
    if reso == split:                                                # cswin:317-318
        last_stage = True
    y = _ln(x, p, key + ".norm1")
    if QKV_INPUT_QUANT is not None:
        y = QKV_INPUT_QUANT(y)
    qkv = _lin(y, p, key + ".qkv")                                   # (B, L, 3C): Q | K | V
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    if last_stage:
        hs, ws = stripe_geometry(reso, -1, split)
        scale = qk_scale or (C // heads) ** -0.5
        a = lepe_attention(q, k, v, reso, hs, ws, heads,
                           p[key + ".attns.0.get_v.weight"], p[key + ".attns.0.get_v.bias"], scale,
                           attn_mask=None if drop is None else (lambda shp: drop(key + ".attn0", shp)))
    else:
        h2, c2 = heads // 2, C // 2
        scale = qk_scale or (c2 // h2) ** -0.5
        outs = []
        for i, sl in enumerate((slice(0, c2), slice(c2, C))):       # cswin:360-363
            hs, ws = stripe_geometry(reso, i, split)
            outs.append(lepe_attention(q[..., sl], k[..., sl], v[..., sl], reso, hs, ws, h2,
                                       p[f"{key}.attns.{i}.get_v.weight"],
                                       p[f"{key}.attns.{i}.get_v.bias"], scale,
                                       attn_mask=None if drop is None else
                                       (lambda shp, i=i: drop(f"{key}.attn{i}", shp))))
        a = torch.cat(outs, dim=-1)
    x = x + _drop_path(drop, key + ".dp_attn", _lin(a, p, key + ".proj"))          # cswin:366-367
    return x + _drop_path(drop, key + ".dp_mlp", mlp(_ln(x, p, key + ".norm2"), p, key + ".mlp", drop))  # cswin:368


def tokens_to_nchw(x: torch.Tensor) -> torch.Tensor:
    B, L, C = x.shape
    s = int(math.isqrt(L))
    return x.transpose(1, 2).reshape(B, C, s, s)


def nchw_to_tokens(x: torch.Tensor) -> torch.Tensor:
    B, C = x.shape[:2]
    return x.reshape(B, C, -1).transpose(1, 2)


def merge_block(x: torch.Tensor, p: Params, key: str) -> torch.Tensor:
    """Conv3x3 s2 p1 (C -> C') then LayerNorm (cswin:373-388)."""
    y = F.conv2d(tokens_to_nchw(x), p[key + ".conv.weight"], p[key + ".conv.bias"], stride=2, padding=1)
    return _ln(nchw_to_tokens(y), p, key + ".norm")


def carafe(x: torch.Tensor, p: Params, key: str, up: int, ksize: int = 3) -> torch.Tensor:
    """Content-aware reassembly upsampling x``up`` (CARAFE cswin:391-437, CARAFE4 cswin:440-486).

    kernel prediction: 1x1 down -> 3x3 encoder -> per output sub-pixel softmax over the 9 taps;
    reassembly: out[c, y*s+i, x*s+j] = sum_t k[t,i,j,y,x] * xpad[c, y+ky-1, x+kx-1]; 1x1 out conv."""
    xi = tokens_to_nchw(x)
    B, C, H, W = xi.shape
    enc = F.conv2d(xi, p[key + ".down.weight"], p[key + ".down.bias"])
    enc = F.conv2d(enc, p[key + ".encoder.weight"], p[key + ".encoder.bias"], padding=ksize // 2)
    kern = enc.reshape(B, ksize * ksize, up, up, H, W).softmax(dim=1)     # (b, tap, i, j, y, x)
    nb = F.unfold(xi, ksize, padding=ksize // 2).reshape(B, C, ksize * ksize, H, W)
    o = torch.einsum("btijhw,bcthw->bchiwj", kern, nb).reshape(B, C, H * up, W * up)
    o = F.conv2d(o, p[key + ".out.weight"], p[key + ".out.bias"])
    return nchw_to_tokens(o)


def patch_embed(x: torch.Tensor, p: Params) -> torch.Tensor:
    """Conv2d(3, 64, k7, s4, p2) -> tokens -> LayerNorm (cswin:504-508)."""
    y = F.conv2d(x, p["stage1_conv_embed.0.weight"], p["stage1_conv_embed.0.bias"], stride=4, padding=2)
    return _ln(nchw_to_tokens(y), p, "stage1_conv_embed.2")


def simam(x: torch.Tensor, lam: float = 1e-4) -> torch.Tensor:
    """SimAM on tokens (B, L, C): per (b, c) over the L positions.  NOT in the reference
     -- public SimAM formula, parity unpinned vs the reference."""
    n = x.shape[1] - 1
    d = (x - x.mean(dim=1, keepdim=True)).pow(2)
    v = d.sum(dim=1, keepdim=True) / n
    e = d / (4 * (v + lam)) + 0.5
    return x * torch.sigmoid(e)


# --------------------------------------------------------------------------------------------
# Whole model (cswin:489-688)
# --------------------------------------------------------------------------------------------
class CSWinConfig:
    def __init__(self, img_size=224, in_chans=3, num_classes=1, embed_dim=64, depth=(1, 2, 9, 1),
                 split_size=(1, 2, 7, 7), num_heads=(2, 4, 8, 16), mlp_ratio=4.0, qkv_bias=True,
                 qk_scale=None, simam=False):
        self.img_size, self.in_chans, self.num_classes = img_size, in_chans, num_classes
        self.embed_dim, self.depth, self.split_size = embed_dim, list(depth), list(split_size)
        self.num_heads, self.mlp_ratio, self.qkv_bias = list(num_heads), mlp_ratio, qkv_bias
        self.qk_scale, self.simam = qk_scale, simam

    def stages(self):
        """(state_dict prefix, reso, heads, split, dim, depth, forced_last) per block stage."""
        S, e, d, sp, h = self.img_size, self.embed_dim, self.depth, self.split_size, self.num_heads
        return [("stage1", S // 4, h[0], sp[0], e, d[0], False),
                ("stage2", S // 8, h[1], sp[1], 2 * e, d[1], False),
                ("stage3", S // 16, h[2], sp[2], 4 * e, d[2], False),
                ("stage4", S // 32, h[3], sp[-1], 8 * e, d[-1], True),
                ("stage_up4", S // 32, h[3], sp[-1], 8 * e, d[-1], True),
                ("stage_up3", S // 16, h[2], sp[2], 4 * e, d[2], False),
                ("stage_up2", S // 8, h[1], sp[1], 2 * e, d[1], False),
                ("stage_up1", S // 4, h[0], sp[0], e, d[0], False)]


def state_dict_contract(cfg: CSWinConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """(key, shape) list in the reference's module registration order (cswin:493-603)."""
    e, C3 = cfg.embed_dim, cfg.in_chans
    out: List[Tuple[str, Tuple[int, ...]]] = []

    def block(prefix, dim, heads, reso, split, last):
        hid = int(dim * cfg.mlp_ratio)
        out.append((f"{prefix}.qkv.weight", (3 * dim, dim)))
        if cfg.qkv_bias:
            out.append((f"{prefix}.qkv.bias", (3 * dim,)))
        out.extend([(f"{prefix}.norm1.weight", (dim,)), (f"{prefix}.norm1.bias", (dim,)),
                    (f"{prefix}.proj.weight", (dim, dim)), (f"{prefix}.proj.bias", (dim,))])
        last = last or reso == split
        nb, cb = (1, dim) if last else (2, dim // 2)
        for i in range(nb):
            out.extend([(f"{prefix}.attns.{i}.get_v.weight", (cb, 1, 3, 3)), (f"{prefix}.attns.{i}.get_v.bias", (cb,))])
        out.extend([(f"{prefix}.mlp.fc1.weight", (hid, dim)), (f"{prefix}.mlp.fc1.bias", (hid,)),
                    (f"{prefix}.mlp.fc2.weight", (dim, hid)), (f"{prefix}.mlp.fc2.bias", (dim,)),
                    (f"{prefix}.norm2.weight", (dim,)), (f"{prefix}.norm2.bias", (dim,))])

    def stage(name, reso, heads, split, dim, depth, last):
        for i in range(depth):
            block(f"{name}.{i}", dim, heads, reso, split, last)

    def carafe_keys(prefix, dim, dim_out, up):
        out.extend([(f"{prefix}.down.weight", (dim // 4, dim, 1, 1)), (f"{prefix}.down.bias", (dim // 4,)),
                    (f"{prefix}.encoder.weight", (up * up * 9, dim // 4, 3, 3)), (f"{prefix}.encoder.bias", (up * up * 9,)),
                    (f"{prefix}.out.weight", (dim_out, dim, 1, 1)), (f"{prefix}.out.bias", (dim_out,))])

    st = cfg.stages()
    out.extend([("stage1_conv_embed.0.weight", (e, C3, 7, 7)), ("stage1_conv_embed.0.bias", (e,)),
            ("stage1_conv_embed.2.weight", (e,)), ("stage1_conv_embed.2.bias", (e,))])
    stage(*st[0])
    out.extend([("merge1.conv.weight", (2 * e, e, 3, 3)), ("merge1.conv.bias", (2 * e,)),
            ("merge1.norm.weight", (2 * e,)), ("merge1.norm.bias", (2 * e,))])
    stage(*st[1])
    out.extend([("merge2.conv.weight", (4 * e, 2 * e, 3, 3)), ("merge2.conv.bias", (4 * e,)),
            ("merge2.norm.weight", (4 * e,)), ("merge2.norm.bias", (4 * e,))])
    stage(*st[2])
    out.extend([("merge3.conv.weight", (8 * e, 4 * e, 3, 3)), ("merge3.conv.bias", (8 * e,)),
            ("merge3.norm.weight", (8 * e,)), ("merge3.norm.bias", (8 * e,))])
    stage(*st[3])
    out.extend([("norm.weight", (8 * e,)), ("norm.bias", (8 * e,))])
    stage(*st[4])
    carafe_keys("upsample4", 8 * e, 4 * e, 2)
    out.extend([("concat_linear4.weight", (256, 512)), ("concat_linear4.bias", (256,))])
    stage(*st[5])
    carafe_keys("upsample3", 4 * e, 2 * e, 2)
    out.extend([("concat_linear3.weight", (128, 256)), ("concat_linear3.bias", (128,))])
    stage(*st[6])
    carafe_keys("upsample2", 2 * e, e, 2)
    out.extend([("concat_linear2.weight", (64, 128)), ("concat_linear2.bias", (64,))])
    stage(*st[7])
    carafe_keys("upsample1", e, 64, 4)
    out.extend([("norm_up.weight", (e,)), ("norm_up.bias", (e,)), ("output.weight", (cfg.num_classes, e, 1, 1))])
    return out


def recipe_params(cfg: CSWinConfig, seed: int = 0, dtype=torch.float32) -> Params:
    """Deterministic weights for ``cfg`` (SURVEY §8c F4 recipe; see ``oracle/recipe.py``)."""
    from .recipe import recipe_from_contract
    return recipe_from_contract(state_dict_contract(cfg), seed, dtype)


def cswin_forward(p: Params, x: torch.Tensor, cfg: CSWinConfig, return_skips: bool = False, drop=None):
    """(B, 3, S, S) in [0,1] -> (B, num_classes, S, S) sigmoid probabilities (cswin:625-688).
    ``drop``: train-mode dropout mask provider (module docstring)."""
    st = cfg.stages()

    def run(name, x):
        _, reso, heads, split, dim, depth, last = next(s for s in st if s[0] == name)
        for i in range(depth):
            x = cswin_block(x, p, f"{name}.{i}", reso, heads, split, last, cfg.qk_scale, drop)
        return x

    skip = simam if cfg.simam else (lambda t: t)
    x = _drop(drop, "pos", patch_embed(x, p))                        # pos_drop (cswin:628)
    x = run("stage1", x); x1 = x; x = merge_block(x, p, "merge1")
    x = run("stage2", x); x2 = x; x = merge_block(x, p, "merge2")
    x = run("stage3", x); x3 = x; x = merge_block(x, p, "merge3")
    x = run("stage4", x)
    x = _ln(x, p, "norm")
    x = run("stage_up4", x)
    x = _lin(torch.cat([skip(x3), carafe(x, p, "upsample4", 2)], -1), p, "concat_linear4")
    x = run("stage_up3", x)
    x = _lin(torch.cat([skip(x2), carafe(x, p, "upsample3", 2)], -1), p, "concat_linear3")
    x = run("stage_up2", x)
    x = _lin(torch.cat([skip(x1), carafe(x, p, "upsample2", 2)], -1), p, "concat_linear2")
    x = run("stage_up1", x)
    x = _ln(x, p, "norm_up")
    y = carafe(x, p, "upsample1", 4)                                  # (B, 16L, 64)
    y = F.conv2d(tokens_to_nchw(y), p["output.weight"])              # cswin:674-682
    y = torch.sigmoid(y)                                              # cswin:688
    return (y, (x1, x2, x3)) if return_skips else y


# --------------------------------------------------------------------------------------------
# Loss and metrics (cswin:692-708, 936)
# --------------------------------------------------------------------------------------------
def bce_loss(prob: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """nn.BCELoss(mean) semantics: log terms clamped at -100."""
    lp = torch.clamp(torch.log(prob), min=-100.0)
    l1p = torch.clamp(torch.log1p(-prob), min=-100.0)
    return -(target * lp + (1 - target) * l1p).mean()


def dice_iou(prob: torch.Tensor, target: torch.Tensor, smooth: float = 1e-6):
    """Batch-flattened Dice and IoU of thresholded predictions (cswin:692-708, 791-794)."""
    pred = (prob > 0.5).to(torch.float64).reshape(-1)
    t = target.to(torch.float64).reshape(-1)
    inter = (pred * t).sum()
    s = pred.sum() + t.sum()
    return float((2 * inter + smooth) / (s + smooth)), float((inter + smooth) / (s - inter + smooth))


class OracleCSWin(torch.nn.Module):
    """nn.Module shell over :func:`cswin_forward` (for CPU training baselines and trajectories)."""

    def __init__(self, cfg: CSWinConfig, params: Params):
        super().__init__()
        self.cfg = cfg
        self.keys = list(params.keys())
        self.plist = torch.nn.ParameterList([torch.nn.Parameter(params[k].clone()) for k in self.keys])

    def params(self) -> Params:
        return dict(zip(self.keys, self.plist))

    def forward(self, x):
        return cswin_forward(self.params(), x, self.cfg)
