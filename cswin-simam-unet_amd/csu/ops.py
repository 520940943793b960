"""Autograd wrappers over the libcsu_hip.so C ABI.  Every op here runs a hand-written gfx950
kernel; there is no CPU or eager-PyTorch fallback (CPU tensors raise ``CsuError``)."""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import check, dtype_code, lib, ptr, require_device, stream_ptr


# ---------------------------------------------------------------------------------------------
# Stripe attention + LePE (LePEAttention cswin:220-298, branches of CSWinBlock cswin:358-363)
# ---------------------------------------------------------------------------------------------
class StripeGeometry:
    """Static description of the attention branches of one CSWinBlock.

    branches: [(H_sp, W_sp, ch_off)] -- geometry per LePEAttention (cswin:232-240)."""

    def __init__(self, reso: int, C: int, heads: int, branches: Sequence[Tuple[int, int, int]], scale: float,
                 head_dim: int = 32):
        self.reso, self.C, self.heads, self.scale, self.head_dim = reso, C, heads, float(scale), head_dim
        self.branches = [tuple(int(v) for v in b) for b in branches]
        if not 1 <= len(self.branches) <= 2:
            raise ValueError("1 or 2 branches")
        for hs, ws, off in self.branches:
            if reso % hs or reso % ws:
                raise ValueError(f"resolution {reso} not divisible by stripe window {hs}x{ws} (cswin:204)")

    def args(self, B: int, ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor],
             dws: Optional[Sequence[torch.Tensor]] = None, dbs: Optional[Sequence[torch.Tensor]] = None):
        a = _lib.StripeArgs()
        a.B, a.reso, a.C, a.heads, a.head_dim = B, self.reso, self.C, self.heads, self.head_dim
        a.nbranch, a.scale = len(self.branches), self.scale
        for i, (hs, wsp, off) in enumerate(self.branches):
            br = a.br[i]
            br.H_sp, br.W_sp, br.ch_off = hs, wsp, off
            br.lepe_w, br.lepe_b = ws[i].data_ptr(), bs[i].data_ptr()
            if dws is not None:
                br.lepe_dw, br.lepe_db = dws[i].data_ptr(), dbs[i].data_ptr()
        return a


class _StripeAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, geom: StripeGeometry, *lepe):
        nb = len(geom.branches)
        ws = [w.detach().float().contiguous() for w in lepe[:nb]]
        bs = [b.detach().float().contiguous() for b in lepe[nb:]]
        require_device(qkv, *ws, *bs)
        qkv = qkv.contiguous()
        B, L, C3 = qkv.shape
        if C3 != 3 * geom.C or L != geom.reso * geom.reso:
            raise ValueError("flatten img_tokens has wrong size")  # cswin:281/356
        out = torch.empty(B, L, geom.C, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(nb, B, geom.heads, L, dtype=torch.float32, device=qkv.device)
        a = geom.args(B, ws, bs)
        check(lib().csu_stripe_attn_fwd(ctypes.byref(a), dtype_code(qkv), ptr(qkv), ptr(out), ptr(lse),
                                        stream_ptr(qkv.device)), "csu_stripe_attn_fwd")
        ctx.geom = geom
        ctx.lepe_dtypes = [t.dtype for t in lepe]
        ctx.save_for_backward(qkv, out, lse, *ws, *bs)
        return out

    @staticmethod
    def backward(ctx, dout):
        geom = ctx.geom
        nb = len(geom.branches)
        qkv, out, lse, *wb = ctx.saved_tensors
        ws, bs = wb[:nb], wb[nb:]
        dout = dout.to(qkv.dtype).contiguous()
        B = qkv.shape[0]
        dqkv = torch.empty_like(qkv)
        delta = torch.empty_like(lse)
        dws = [torch.empty_like(w) for w in ws]
        dbs = [torch.empty_like(b) for b in bs]
        a = geom.args(B, ws, bs, dws, dbs)
        L = lib()
        nbytes = L.csu_stripe_attn_bwd_workspace(ctypes.byref(a))
        work = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=qkv.device)
        check(L.csu_stripe_attn_bwd(ctypes.byref(a), dtype_code(qkv), ptr(qkv), ptr(out), ptr(dout), ptr(lse),
                                    ptr(delta), ptr(dqkv), ptr(work), nbytes, stream_ptr(qkv.device)),
              "csu_stripe_attn_bwd")
        grads = [g.to(dt) for g, dt in zip(dws + dbs, ctx.lepe_dtypes)]
        return (dqkv, None, *grads)


def stripe_attention(qkv: torch.Tensor, geom: StripeGeometry, lepe_w: Sequence[torch.Tensor],
                     lepe_b: Sequence[torch.Tensor]) -> torch.Tensor:
    """(B, L, 3C) qkv -> (B, L, C) attention output of every branch (+LePE), channels concatenated."""
    return _StripeAttnFn.apply(qkv, geom, *lepe_w, *lepe_b)


# ---------------------------------------------------------------------------------------------
# LayerNorm (nn.LayerNorm over the last dim; eps 1e-5)
# ---------------------------------------------------------------------------------------------
class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps: float, out_dtype):
        require_device(x, weight, bias)
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        w = weight.detach().float().contiguous()
        b = bias.detach().float().contiguous()
        y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        check(lib().csu_layernorm_fwd(rows, C, float(eps), dtype_code(x), ptr(x), ptr(w), ptr(b), dtype_code(y), ptr(y),
                                      ptr(mean), ptr(rstd), stream_ptr(x.device)), "csu_layernorm_fwd")
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.pdtypes = (weight.dtype, bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        C = x.shape[-1]
        rows = x.numel() // C
        dx = torch.empty_like(x)
        dg = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty(C, dtype=torch.float32, device=x.device)
        L = lib()
        nbytes = L.csu_layernorm_bwd_workspace(rows, C)
        work = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=x.device)
        check(L.csu_layernorm_bwd(rows, C, dtype_code(x), ptr(x), ptr(w), ptr(mean), ptr(rstd), dtype_code(dy), ptr(dy),
                                  ptr(dx), ptr(dg), ptr(db), ptr(work), nbytes, stream_ptr(x.device)),
              "csu_layernorm_bwd")
        return dx, dg.to(ctx.pdtypes[0]), db.to(ctx.pdtypes[1]), None, None


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5,
               out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    return _LayerNormFn.apply(x, weight, bias, eps, out_dtype or x.dtype)
