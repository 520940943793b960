"""Drop-in nn.Modules of the CSWin-(SimAM-)UNet (train_cswinunet_segmentation.py cswin:180-688).

Class names, constructor signatures, parameter registration order and therefore state_dict keys
are those of the reference, so reference ``.pth`` files load unchanged (cswin:992) and
``model.apply(model._init_weights)`` reproduces the reference initialisation (cswin:605-614).
Forward passes run the hand-written gfx950 kernels of libcsu_hip.so (``csu.ops``) on
token-major (B, L, C) = NHWC activations; the dense projections (qkv/proj/fc1/fc2/concat_linear)
run on csu's token GEMMs and the convolutions on its implicit-GEMM NHWC kernels (no vendor GEMM /
conv library on the path).

Precision policy (bf16 under ``torch.autocast('cuda', torch.bfloat16)``, the BASELINE setting):
residual stream fp32; LayerNorm emits the GEMM's input dtype directly; attention, MLP and
upsampling activations bf16; softmax/LN statistics and all reductions fp32; loss head fp32.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np
import torch
import torch.nn as nn

from . import ops, rng
from .simam import SimAM


def _compute_dtype(x: torch.Tensor) -> torch.dtype:
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


def trunc_normal_(t, std=1.0, a=-2.0, b=2.0):
    """timm.models.layers.trunc_normal_ semantics (cswin:14, 609): absolute cut-offs a, b."""
    return nn.init.trunc_normal_(t, mean=0.0, std=std, a=a, b=b)


class DropPath(nn.Module):
    """Stochastic depth (timm DropPath, cswin:344): per-sample Bernoulli(keep)/keep in training,
    drawn from the counter-based RNG (csu.rng, site ``_site``) and applied by one kernel."""

    def __init__(self, drop_prob: float = 0.0):
        super().__init__()
        self.drop_prob = drop_prob
        self._site = rng.SITE_BASE + rng.OFF_DROPPATH_ATTN

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        B = x.shape[0]
        rows = x.numel() // x.shape[-1]
        rs = ops.droppath_scale(B, self.drop_prob, self._site, x.device)
        return ops.dropout(x, 0.0, self._site, row_scale=rs, rows_per_sample=rows // B)


def _ln(x: torch.Tensor, norm: nn.LayerNorm, out_dtype=None) -> torch.Tensor:
    return ops.layer_norm(x, norm.weight, norm.bias, norm.eps, out_dtype)


def _tokens_as_nchw(x: torch.Tensor) -> torch.Tensor:
    """(B, L, C) token tensor viewed (no copy) as a channels_last NCHW tensor."""
    B, L, C = x.shape
    H = W = int(math.isqrt(L))
    return x.transpose(1, 2).reshape(B, C, H, W)


def _nchw_as_tokens(x: torch.Tensor) -> torch.Tensor:
    B, C = x.shape[:2]
    return x.reshape(B, C, -1).transpose(1, 2)


class Mlp(nn.Module):
    """fc1 -> GELU(erf) -> Dropout -> fc2 -> Dropout (cswin:180-196)."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)
        self._site_h = rng.SITE_BASE + rng.OFF_MLP_HIDDEN
        self._site_o = rng.SITE_BASE + rng.OFF_MLP_OUT

    def forward(self, x):
        if self.training and self.drop.p > 0 and x.is_cuda:
            with rng.ensure_scope(x.device) as snap:
                return self.forward_residual(x, snap=snap)
        return self.forward_residual(x)

    def forward_residual(self, x, residual=None, row_scale=None, rows_per_sample=1, snap=None):
        """[residual +] [row_scale *] Mlp(x): the dropout sites draw from `snap` (csu.rng) in
        training, and the output dropout, DropPath scale and residual add are one kernel."""
        p = self.drop.p if self.training and snap is not None else 0.0
        h = self.act(ops.linear(x, self.fc1.weight, self.fc1.bias))
        if p > 0:
            h = ops.dropout(h, p, self._site_h, snap)
        y = ops.linear(h, self.fc2.weight, self.fc2.bias)
        if p > 0 or row_scale is not None:
            return ops.dropout(y, p, self._site_o, snap, row_scale=row_scale, rows_per_sample=rows_per_sample,
                               residual=residual)
        return y if residual is None else residual + y


def img2windows(img: torch.Tensor, H_sp: int, W_sp: int) -> torch.Tensor:
    """(B, C, H, W) -> (B*nWin, H_sp*W_sp, C) (cswin:199-206).  Layout utility kept for API
    compatibility; the hot path never materialises windows (the kernels gather by index)."""
    B, C, H, W = img.shape
    t = img.reshape(B, C, H // H_sp, H_sp, W // W_sp, W_sp)
    return t.permute(0, 2, 4, 3, 5, 1).reshape(-1, H_sp * W_sp, C)


def windows2img(img_splits_hw: torch.Tensor, H_sp: int, W_sp: int, H: int, W: int) -> torch.Tensor:
    """(B*nWin, H_sp*W_sp, C) -> (B, H, W, C) (cswin:209-217)."""
    B = int(img_splits_hw.shape[0] / (H * W / H_sp / W_sp))
    t = img_splits_hw.reshape(B, H // H_sp, W // W_sp, H_sp, W_sp, -1)
    return t.permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, -1)


class LePEAttention(nn.Module):
    """Stripe-window MHSA + LePE (cswin:220-298).  forward(qkv (3, B, L, C)) -> (B, L, C)."""

    def __init__(self, dim, resolution, idx, split_size, dim_out=None, num_heads=9, attn_drop=0.0,
                 proj_drop=0.0, qk_scale=None):
        super().__init__()
        self.dim = dim
        self.dim_out = dim_out or dim
        self.resolution = resolution
        self.split_size = split_size
        self.num_heads = num_heads
        self.idx = idx
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        if idx == -1:
            H_sp, W_sp = resolution, resolution
        elif idx == 0:
            H_sp, W_sp = resolution, split_size
        elif idx == 1:
            W_sp, H_sp = resolution, split_size
        else:
            raise ValueError(f"ERROR MODE {idx}")   # the reference prints and exit(0)s (cswin:239-240)
        self.H_sp, self.W_sp = H_sp, W_sp
        self.get_v = nn.Conv2d(dim, dim, kernel_size=3, stride=1, padding=1, groups=dim)
        self.attn_drop_p = attn_drop
        self.attn_drop = nn.Dropout(attn_drop)
        self._site = rng.SITE_BASE + rng.OFF_ATTN + max(idx, 0)

    def drop_args(self, device) -> Optional[ops.AttnDrop]:
        """Attention dropout (cswin:290) of a training forward: applied to P inside the kernels."""
        if not (self.training and self.attn_drop.p > 0):
            return None
        return ops.AttnDrop(rng.snapshot(device), self._site, self.attn_drop.p)

    def forward(self, qkv):
        _, B, L, C = qkv.shape
        packed = torch.cat([qkv[0], qkv[1], qkv[2]], dim=-1)
        geom = ops.StripeGeometry(self.resolution, C, self.num_heads, [(self.H_sp, self.W_sp, 0)], self.scale)
        return ops.stripe_attention(packed, geom, [self.get_v.weight], [self.get_v.bias], self.drop_args(qkv.device))


class CSWinBlock(nn.Module):
    """Pre-LN CSWin block (cswin:301-370); both stripe branches run in one fused launch."""

    def __init__(self, dim, reso, num_heads, split_size, mlp_ratio=4.0, qkv_bias=False, qk_scale=None, drop=0.0,
                 attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU, norm_layer=nn.LayerNorm, last_stage=False):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.patches_resolution = reso
        self.split_size = split_size
        self.mlp_ratio = mlp_ratio
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.norm1 = norm_layer(dim)
        if self.patches_resolution == split_size:
            last_stage = True
        self.branch_num = 1 if last_stage else 2
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(drop)          # built but never applied, as in cswin:324/366
        if last_stage:
            self.attns = nn.ModuleList([LePEAttention(dim, resolution=reso, idx=-1, split_size=split_size,
                                                      num_heads=num_heads, dim_out=dim, qk_scale=qk_scale,
                                                      attn_drop=attn_drop, proj_drop=drop)])
        else:
            self.attns = nn.ModuleList([LePEAttention(dim // 2, resolution=reso, idx=i, split_size=split_size,
                                                      num_heads=num_heads // 2, dim_out=dim // 2, qk_scale=qk_scale,
                                                      attn_drop=attn_drop, proj_drop=drop)
                                        for i in range(self.branch_num)])
        mlp_hidden_dim = int(dim * mlp_ratio)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.mlp = Mlp(in_features=dim, hidden_features=mlp_hidden_dim, out_features=dim, act_layer=act_layer, drop=drop)
        self.norm2 = norm_layer(dim)
        a0 = self.attns[0]
        offs = [0] if last_stage else [0, dim // 2]
        self._geom = ops.StripeGeometry(reso, dim, a0.num_heads,
                                        [(a.H_sp, a.W_sp, o) for a, o in zip(self.attns, offs)], a0.scale,
                                        head_dim=a0.dim // a0.num_heads)
        self.set_drop_sites(rng.SITE_BASE)

    def set_drop_sites(self, base: int):
        """Dropout site ids of this block (csu.rng): attention branch i, Mlp hidden / output, and
        the two DropPath draws (attention and Mlp residual, cswin:367-368)."""
        self._site_base = base
        for i, a in enumerate(self.attns):
            a._site = base + rng.OFF_ATTN + i
        self.mlp._site_h = base + rng.OFF_MLP_HIDDEN
        self.mlp._site_o = base + rng.OFF_MLP_OUT
        if isinstance(self.drop_path, DropPath):
            self.drop_path._site = base + rng.OFF_DROPPATH_ATTN

    def forward(self, x):
        tr = self.training
        if tr and (self.attns[0].attn_drop.p > 0 or self.mlp.drop.p > 0
                   or (isinstance(self.drop_path, DropPath) and self.drop_path.drop_prob > 0)) and x.is_cuda:
            with rng.ensure_scope(x.device) as snap:   # every site of this block: one snapshot
                return self._forward(x, snap)
        return self._forward(x, None)

    def _forward(self, x, snap):
        H = W = self.patches_resolution
        B, L, C = x.shape
        assert L == H * W, "flatten img_tokens has wrong size"
        cd = _compute_dtype(x)
        on = snap is not None
        p_attn = self.attns[0].attn_drop.p if on else 0.0
        p_mlp = self.mlp.drop.p if on else 0.0
        p_path = self.drop_path.drop_prob if on and isinstance(self.drop_path, DropPath) else 0.0
        base = self._site_base
        # residual junctions x -> (x, LN(x)): their backward adds the two branch gradients in the
        # LayerNorm-backward kernel and hands the upstream GEMMs a bf16 copy (ops.layer_norm_fork)
        n1, n2 = self.norm1, self.norm2
        got = ops.ln_linear_fp8(x, n1, self.qkv) if cd == torch.bfloat16 else None
        if got is None and cd == torch.bfloat16:
            got = ops.ln_linear_ws(x, n1, self.qkv)   # norm1 backward inside the qkv input-gradient GEMM
        if got is not None:
            xa, qkv = got        # fp8 weight format: e4m3 norm1 output x e4m3 qkv weight on fp8 MFMA
        else:
            xa, h1 = ops.layer_norm_fork(x, n1.weight, n1.bias, n1.eps, cd)
            qkv = ops.linear(h1, self.qkv.weight, self.qkv.bias)
        ad = ops.AttnDrop(snap, base + rng.OFF_ATTN, p_attn) if p_attn > 0 else None
        att = ops.stripe_attention(qkv, self._geom, [a.get_v.weight for a in self.attns],
                                   [a.get_v.bias for a in self.attns], ad)
        # DropPath (cswin:367-368): per-sample scales of the two residual branches
        rs1 = rs2 = None
        if p_path > 0:
            rs1 = ops.droppath_scale(B, p_path, base + rng.OFF_DROPPATH_ATTN, x.device, snap)
            rs2 = ops.droppath_scale(B, p_path, base + rng.OFF_DROPPATH_MLP, x.device, snap)
        fused = ops.fused_ok(x, C, self.mlp.fc1.out_features)
        if fused and rs1 is None:
            # bf16 fused path: proj + residual in one GEMM
            # ... and norm2 in its epilogue where the weight-streaming GEMM has the shape
            x = ops.linear_residual(xa, att, self.proj.weight, self.proj.bias,
                                    ln_next=(n2.weight, n2.bias, n2.eps) if cd == torch.bfloat16 else None)
        else:
            y = ops.linear(att, self.proj.weight, self.proj.bias)
            x = ops.dropout(y, 0.0, 0, row_scale=rs1, rows_per_sample=L, residual=xa) if rs1 is not None else xa + y
        xb, h2 = ops.layer_norm_fork(x, n2.weight, n2.bias, n2.eps, cd)
        if fused:
            # fc1 -> GELU -> [dropout] -> fc2 -> [dropout, DropPath] + residual (csrc/mlp.hip)
            md = None
            if on and (p_mlp > 0 or rs2 is not None):
                md = ops.MlpDrop(snap, self.mlp._site_h, self.mlp._site_o, p_mlp, rs2, L)
            nn1 = getattr(self, "_next_norm", None)   # the next block's norm1: computed in the Mlp's epilogue
            ln_next = (nn1.weight, nn1.bias, nn1.eps) if nn1 is not None and cd == torch.bfloat16 else None
            return ops.mlp_residual(xb, h2, self.mlp.fc1, self.mlp.fc2, md, ln_next=ln_next)
        return self.mlp.forward_residual(h2, xb, rs2, L, snap)


class Merge_Block(nn.Module):
    """Conv3x3 s2 p1 (C -> C') + LayerNorm (cswin:373-388)."""

    def __init__(self, dim, dim_out, norm_layer=nn.LayerNorm):
        super().__init__()
        self.conv = nn.Conv2d(dim, dim_out, 3, 2, 1)
        self.norm = norm_layer(dim_out)

    def forward(self, x):
        B, L, C = x.shape
        H = W = int(math.isqrt(L))
        # implicit-GEMM 3x3/s2 conv straight on the NHWC token layout (csu_conv2d_fwd)
        y = ops.conv2d(x.reshape(B, H, W, C), self.conv.weight, self.conv.bias, 2, 1)
        y = y.reshape(B, -1, y.shape[-1])
        return _ln(y, self.norm, torch.float32 if y.dtype == torch.bfloat16 else y.dtype)


class CARAFE(nn.Module):
    """Content-aware reassembly upsampling (cswin:391-437).  forward((B, L, C)) -> (B, s^2 L, C_out)."""

    def __init__(self, dim, dim_out, kernel_size=3, up_factor=2):
        super().__init__()
        self.kernel_size = kernel_size
        self.up_factor = up_factor
        self.down = nn.Conv2d(dim, dim // 4, 1)
        self.encoder = nn.Conv2d(dim // 4, self.up_factor ** 2 * self.kernel_size ** 2, self.kernel_size, 1,
                                 self.kernel_size // 2)
        self.out = nn.Conv2d(dim, dim_out, 1)

    def forward(self, x):
        B, L, C = x.shape
        H = W = int(math.isqrt(L))
        s = self.up_factor
        if self.kernel_size != 3:
            raise NotImplementedError("the fused CARAFE kernel is specialised for kernel_size=3 (the reference's)")
        xc, enc = self.kernels(x)
        # fused pixel_shuffle + softmax + unfold + matmul + pixel_shuffle (cswin:410-432)
        r = ops.carafe_reassemble(xc, enc, H, W, s)                        # (B, s^2 L, C)
        return ops.linear(r, self.out.weight.reshape(self.out.weight.shape[0], C), self.out.bias)

    def kernels(self, x):
        """Kernel prediction (cswin:408-409): 1x1 down as a token GEMM, 3x3 encoder conv on the
        NHWC view.  Returns (x in the compute dtype, enc (B, H, W, 9 s^2) NHWC logits)."""
        B, L, C = x.shape
        H = W = int(math.isqrt(L))
        if self.kernel_size != 3:
            raise NotImplementedError("the fused CARAFE kernel is specialised for kernel_size=3 (the reference's)")
        cd = _compute_dtype(x)
        if x.is_cuda:
            # one bf16 copy (or x itself when already bf16) for both consumers (down conv,
            # reassembly): their two input gradients are joined in one pass (ops.grad_join) instead
            # of autograd's add (+ cast)
            xd, xc = ops.shared_cast(x, cd)
        else:
            xd = xc = x.to(cd)
        d = ops.linear(xd, self.down.weight.reshape(C // 4, C), self.down.bias)
        enc = ops.conv2d(d.reshape(B, H, W, C // 4), self.encoder.weight, self.encoder.bias, 1, self.kernel_size // 2)
        return xc, enc


def carafe_sigmoid_head(up: CARAFE, w_output: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """sigmoid(output(up(x))) for the 1-class bias-free `output` conv (cswin:674-688) in one pass.

    CARAFE reassembly -> `out` 1x1 conv -> `output` 1x1 conv is linear up to the sigmoid, so it
    collapses to u = W_out^T w_output and c = w_output . b_out (folded by csu_head_fold_fwd, its
    backward inside the head's backward) and the fused kernel ops.carafe_head.  Returns prob
    (B, 1, sH, sW) fp32."""
    B, L, C = x.shape
    H = W = int(math.isqrt(L))
    xc, enc = up.kernels(x)
    if xc.is_cuda:
        return ops.carafe_head_folded(xc, enc, up.out.weight, up.out.bias, w_output, H, W, up.up_factor)
    w_out = up.out.weight.reshape(up.out.weight.shape[0], C).float()
    w_h = w_output.reshape(-1).float()
    u = w_out.t() @ w_h
    cb = (w_h * up.out.bias.float()).sum()
    return ops.carafe_head(xc, enc, u, cb, H, W, up.up_factor)


class CARAFE4(CARAFE):
    """CARAFE with up_factor 4 (cswin:440-486)."""

    def __init__(self, dim, dim_out, kernel_size=3, up_factor=4):
        super().__init__(dim, dim_out, kernel_size, up_factor)


class CSWinTransformer(nn.Module):
    """CSWin-Transformer U-Net with CARAFE upsampling (cswin:489-688).

    Extra (not in the reference): ``simam=True`` applies the parameter-free SimAM gate to the
    skip features x1/x2/x3 before the concat_linear fusions; the default False
    is exact reference behaviour.  State_dict keys are unchanged either way."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, num_classes=1, embed_dim=64, depth=[1, 2, 9, 1],
                 split_size=[1, 2, 7, 7], num_heads=[2, 4, 8, 16], mlp_ratio=4.0, qkv_bias=True, qk_scale=None,
                 drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0, hybrid_backbone=None,
                 norm_layer=nn.LayerNorm, use_chk=False, simam=False):
        super().__init__()
        self.use_chk = use_chk
        self.num_classes = num_classes
        self.num_features = self.embed_dim = embed_dim
        self.img_size = img_size
        heads = num_heads
        self.stage1_conv_embed = nn.Sequential(nn.Conv2d(in_chans, embed_dim, 7, 4, 2), _TokensRearrange(img_size // 4),
                                               nn.LayerNorm(embed_dim))
        curr_dim = embed_dim
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, int(np.sum(depth)))]

        def blocks(dim, reso, nh, sp, dps, last=False):
            return nn.ModuleList([CSWinBlock(dim=dim, num_heads=nh, reso=reso, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                                             qk_scale=qk_scale, split_size=sp, drop=drop_rate, attn_drop=attn_drop_rate,
                                             drop_path=dp, norm_layer=norm_layer, last_stage=last) for dp in dps])

        d0, d1, d2 = int(np.sum(depth[:1])), int(np.sum(depth[:2])), int(np.sum(depth[:-1]))
        self.stage1 = blocks(curr_dim, img_size // 4, heads[0], split_size[0], dpr[:depth[0]])
        self.merge1 = Merge_Block(curr_dim, curr_dim * 2)
        curr_dim *= 2
        self.stage2 = blocks(curr_dim, img_size // 8, heads[1], split_size[1], dpr[d0:d0 + depth[1]])
        self.merge2 = Merge_Block(curr_dim, curr_dim * 2)
        curr_dim *= 2
        self.stage3 = blocks(curr_dim, img_size // 16, heads[2], split_size[2], dpr[d1:d1 + depth[2]])
        self.merge3 = Merge_Block(curr_dim, curr_dim * 2)
        curr_dim *= 2
        self.stage4 = blocks(curr_dim, img_size // 32, heads[3], split_size[-1], dpr[d2:d2 + depth[-1]], last=True)
        self.norm = norm_layer(curr_dim)
        # decoder (reuses the encoder drop-path indices, cswin:562/574/587/598)
        self.stage_up4 = blocks(curr_dim, img_size // 32, heads[3], split_size[-1], dpr[d2:d2 + depth[-1]], last=True)
        self.upsample4 = CARAFE(curr_dim, curr_dim // 2)
        curr_dim //= 2
        self.concat_linear4 = nn.Linear(512, 256)
        self.stage_up3 = blocks(curr_dim, img_size // 16, heads[2], split_size[2], dpr[d1:d1 + depth[2]])
        self.upsample3 = CARAFE(curr_dim, curr_dim // 2)
        curr_dim //= 2
        self.concat_linear3 = nn.Linear(256, 128)
        self.stage_up2 = blocks(curr_dim, img_size // 8, heads[1], split_size[1], dpr[d0:d0 + depth[1]])
        self.upsample2 = CARAFE(curr_dim, curr_dim // 2)
        curr_dim //= 2
        self.concat_linear2 = nn.Linear(128, 64)
        self.stage_up1 = blocks(curr_dim, img_size // 4, heads[0], split_size[0], dpr[:depth[0]])
        self.upsample1 = CARAFE4(curr_dim, 64)
        self.norm_up = norm_layer(embed_dim)
        self.output = nn.Conv2d(in_channels=embed_dim, out_channels=self.num_classes, kernel_size=1, bias=False)
        self.simam = SimAM() if simam else None
        self.apply(self._init_weights)
        rng.assign_sites(self)
        # the LayerNorm that consumes each block's output, when it is the next block's norm1 (or norm_up
        # after the last decoder block): the block's fused Mlp computes it in its epilogue
        # (ops.mlp_residual(ln_next=...)); a plain attribute, not a registered submodule
        for st in (self.stage1, self.stage2, self.stage3, self.stage4, self.stage_up4, self.stage_up3, self.stage_up2,
                   self.stage_up1):
            for a, b in zip(list(st)[:-1], list(st)[1:]):
                object.__setattr__(a, "_next_norm", b.norm1)
        object.__setattr__(self.stage_up1[-1], "_next_norm", self.norm_up)

    def _init_weights(self, m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, (nn.LayerNorm, nn.BatchNorm2d)):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {"pos_embed", "cls_token"}

    @torch.jit.ignore
    def no_weight_decay_keywords(self):
        return {"relative_position_bias_table"}

    @staticmethod
    def _fuse(lin: nn.Linear, x: torch.Tensor) -> torch.Tensor:
        """concat_linear (cswin:568/581/592): its output starts a decoder residual stream, kept
        fp32 like the encoder's (written fp32 by the GEMM epilogue, no conversion pass)."""
        return ops.linear(x, lin.weight, lin.bias, out_dtype=torch.float32 if x.is_cuda else None)

    def _skip(self, t):
        return self.simam(t) if self.simam is not None else t

    def _share_skip(self, x):
        """(merge input, decoder skip in bf16 or None) for an encoder stage output.  bf16 autocast
        on the device: without SimAM one shared bf16 copy feeds both the Merge_Block conv and the
        split-weight concat_linear (ops.shared_cast / ops.concat_linear); with SimAM the gate's passes
        write both the bf16 copy for the conv and the gated bf16 skip (simam_fork: no cat, no cast,
        one joined backward pass); otherwise x twice (reference form)."""
        if x.is_cuda and torch.is_autocast_enabled("cuda") \
                and torch.get_autocast_dtype("cuda") == torch.bfloat16 and x.dtype == torch.float32:
            if self.simam is not None:
                return self.simam.fork(x)
            return ops.shared_cast(x, torch.bfloat16)
        return x, None

    def _concat(self, lin, skip_fp, skip_b, up):
        if skip_b is not None and up.dtype == torch.bfloat16:
            return ops.concat_linear(skip_b, up, lin.weight, lin.bias)
        return self._fuse(lin, torch.cat([self._skip(skip_fp), up], -1))

    def forward_features(self, x):
        conv, _, ln = self.stage1_conv_embed
        B = x.shape[0]
        # patch embed Conv2d(3, 64, 7, 4, 2) as an implicit-GEMM conv on the NHWC image
        y = ops.conv2d(x.permute(0, 2, 3, 1), conv.weight, conv.bias, conv.stride[0], conv.padding[0])
        y = y.reshape(B, -1, y.shape[-1])
        x = _ln(y, ln, torch.float32 if y.dtype == torch.bfloat16 else y.dtype)
        if self.training and self.pos_drop.p > 0:
            x = ops.dropout(x, self.pos_drop.p, rng.SITE_POS_DROP)
        for blk in self.stage1:
            x = blk(x)
        self.x1 = x
        x, self._x1s = self._share_skip(x)
        x = self.merge1(x)
        for blk in self.stage2:
            x = blk(x)
        self.x2 = x
        x, self._x2s = self._share_skip(x)
        x = self.merge2(x)
        for blk in self.stage3:
            x = blk(x)
        self.x3 = x
        x, self._x3s = self._share_skip(x)
        x = self.merge3(x)
        for blk in self.stage4:
            x = blk(x)
        return _ln(x, self.norm)

    def forward_up_features(self, x):
        for blk in self.stage_up4:
            x = blk(x)
        x = self._concat(self.concat_linear4, self.x3, self._x3s, self.upsample4(x))
        for blk in self.stage_up3:
            x = blk(x)
        x = self._concat(self.concat_linear3, self.x2, self._x2s, self.upsample3(x))
        for blk in self.stage_up2:
            x = blk(x)
        x = self._concat(self.concat_linear2, self.x1, self._x1s, self.upsample2(x))
        for blk in self.stage_up1:
            x = blk(x)
        return _ln(x, self.norm_up, _compute_dtype(x))

    def up_x4(self, x):
        """CARAFE4 x4 upsampling + 1x1 output conv (cswin:674-682); returns LOGITS only when the
        fused sigmoid head cannot be used (num_classes != 1)."""
        B, new_HW, C = x.shape
        H = W = int(math.isqrt(new_HW))
        x = self.upsample1(x)                                             # (B, 16 L, 64) tokens
        w = self.output.weight.reshape(self.num_classes, -1)
        nc = self.num_classes
        n8 = (nc + 7) // 8 * 8        # csu token GEMM: output features padded to a multiple of 8
        if n8 != nc:
            w = torch.cat([w, w.new_zeros(n8 - nc, w.shape[1])], 0)
        logits = ops.linear(x, w)[..., :nc]
        return logits.transpose(1, 2).reshape(B, nc, 4 * H, 4 * W)

    def _linear_weights(self):
        """Weights the bf16 cast cache shadows: every nn.Linear and the CARAFE 1x1 convs that run
        as token Linears (down / out)."""
        for m in self.modules():
            if isinstance(m, nn.Linear):
                yield m.weight
                if m.bias is not None:
                    yield m.bias
            elif isinstance(m, CARAFE):
                yield m.down.weight
                yield m.out.weight

    def _conv_weights(self):
        """KxK conv weights whose channels-last bf16 layouts the cast cache keeps (patch embed,
        Merge_Block, CARAFE encoders)."""
        yield self.stage1_conv_embed[0].weight
        for m in self.modules():
            if isinstance(m, Merge_Block):
                yield m.conv.weight
            elif isinstance(m, CARAFE):
                yield m.encoder.weight

    def set_weight_format(self, fmt: str = "bf16"):
        """'bf16' (default) or 'fp8_e4m3' (BASELINE config 5: fp8-e4m3 Linear weights with per-row
        power-of-two scales, bf16 activations, fp32 accumulate; applies under bf16 autocast)."""
        if fmt not in ("bf16", "fp8_e4m3"):
            raise ValueError(f"weight format {fmt!r}")
        self._weight_format = fmt
        self._fp8 = None
        return self

    def forward(self, x):
        cd = _compute_dtype(x)
        if cd != torch.float32 and x.is_cuda:
            if not hasattr(self, "_cast_cache"):
                self._cast_cache = ops.CastCache()
            weights = list(self._linear_weights())
            sources = None
            if getattr(self, "_weight_format", "bf16") == "fp8_e4m3" and cd == torch.bfloat16:
                if self._fp8 is None or not self._fp8.valid_for(weights):
                    pairs = [(m.fc1.weight, m.fc2.weight) for m in self.modules() if isinstance(m, Mlp)]
                    self._fp8 = ops.Fp8Weights(weights, mlp_pairs=pairs)
                sources = self._fp8.sources()
            # bf16 shadows of every Linear weight (+ transposes) and conv layouts: AdamW-written, or one
            # cast launch; in the fp8 format the quantised weights' shadows come from the quantiser
            self._cast_cache.refresh(weights, cd, self._conv_weights(), sources=sources)
            if sources is not None:
                self._fp8.quantize(self._cast_cache)   # one launch: e4m3 + scales + exact bf16 shadows
            if sources is None or not ops.FP8_WS:
                # fragment-ordered W / W^T of the qkv / proj Linears (csu_gemm_ws); the fp8 format streams
                # the e4m3 fragments its quantiser lays out instead (ops.FP8_WS, csu_gemm_ws_e4m3)
                self._cast_cache.refresh_frag()
            ops.set_cast_cache(self._cast_cache, self._fp8 if sources is not None else None)
        try:
            return self._forward(x)
        finally:
            ops.set_cast_cache(None)

    def _dropout_on(self) -> bool:
        if not self.training:
            return False
        return any((isinstance(m, nn.Dropout) and m.p > 0) or (isinstance(m, DropPath) and m.drop_prob > 0)
                   for m in self.modules())

    def _forward(self, x):
        if x.is_cuda and self._dropout_on():
            # one RNG snapshot for every dropout site of this forward (csu.rng)
            with rng.scope(x.device):
                return self._forward_impl(x)
        return self._forward_impl(x)

    def _forward_impl(self, x):
        try:
            return self._forward_body(x)
        finally:
            self._release_skips()

    def _release_skips(self):
        """Keep the encoder skips (x1, x2, x3 as the reference exposes them, cswin:632-642) but not
        the autograd graph behind them: a module attribute holding a graph of the last forward keeps
        that step's AccumulateGrad nodes alive, and a later HIP-graph capture then runs them on the
        stream they were created on (the legacy default stream) -> the capture breaks and
        hipGraphInstantiate segfaults (tools/graph_after_eager.py)."""
        for k in ("x1", "x2", "x3"):
            t = getattr(self, k, None)
            if t is not None and t.requires_grad:
                setattr(self, k, t.detach())
        self._x1s = self._x2s = self._x3s = None

    def _forward_body(self, x):
        x = self.forward_features(x)
        x = self.forward_up_features(x)
        if self.num_classes == 1:
            B, L, C = x.shape
            H = W = int(math.isqrt(L))
            return carafe_sigmoid_head(self.upsample1, self.output.weight, x)
        return torch.sigmoid(self.up_x4(x).float())


class _TokensRearrange(nn.Module):
    """einops Rearrange('b c h w -> b (h w) c', h=w=reso) (cswin:506); no parameters."""

    def __init__(self, reso):
        super().__init__()
        self.reso = reso

    def forward(self, x):
        assert x.shape[2] == self.reso and x.shape[3] == self.reso
        return _nchw_as_tokens(x)
