"""fp8-e4m3 pieces of BASELINE config 5 ("fp8 MFMA weights") -- TEST INFRASTRUCTURE ONLY.

The reference trains in fp32 (cswin:865-941); it has no fp8 path.  These functions restate, in
float64 on the CPU, the quantisation rules the csu fp8 kernels document (include/csu.h:
csu_quant_e4m3_batch, csu_mlp_fp8_fwd / csu_mlp_fp8_bwd), so the parity tests can run the
reference's Mlp (cswin:180-196) with exactly the roundings the device applies.  Parity of these
rules against the reference is therefore "parity unpinned": the reference has no such format;
what is pinned is that the device computes the reference Mlp on these rounded operands.

* per-row weight quantisation: s = 2^ceil(log2(amax / 448)), q = e4m3fn(w / s) round-to-nearest-even
* MX block quantisation (activations, gradients): per block of 32 consecutive channels (or hidden
  features), s = 2^e with e the smallest integer such that amax <= 448 * 2^e (0 for an all-zero
  block, clamped to [-127, 127]), q = e4m3fn(v / s) -- the OCP MX rule with e4m3 elements, which the
  kernels apply in registers in the hardware's k order (tools/probes/mx_layout_probe.hip).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

E4M3_MAX = 448.0


def _e4m3(v: torch.Tensor) -> torch.Tensor:
    """Round to the nearest e4m3fn value (RNE; |v| <= 448 by construction of the scales)."""
    return v.float().to(torch.float8_e4m3fn).to(torch.float64)


def block_exponent(amax: torch.Tensor) -> torch.Tensor:
    """e = the smallest integer with amax <= 448 * 2^e, 0 for amax == 0, clamped to [-127, 127]
    (amax = m 2^E with m in [1, 2): e = E - 8 + (m > 1.75), since 448 = 1.75 * 2^8)."""
    a = amax.double()
    m, E = torch.frexp(a)                       # a = m 2^E, m in [0.5, 1)
    e = (E - 1) - 8 + (2 * m > 1.75).to(E.dtype)
    e = torch.where(a > 0, e, torch.zeros_like(e))
    return e.clamp(-127, 127)


def mx_quant(v: torch.Tensor) -> torch.Tensor:
    """MX e4m3 rounding (dequantised, float64) with blocks of 32 consecutive values of the last dim."""
    shp = v.shape
    b = v.double().reshape(*shp[:-1], shp[-1] // 32, 32)
    s = torch.exp2(block_exponent(b.abs().amax(-1, keepdim=True)).double())
    return (_e4m3(b / s) * s).reshape(shp)


def quant_rows(w: torch.Tensor):
    """(dequantised weight, e4m3 values q, row scales s) of csu_quant_e4m3_batch."""
    w2 = w.reshape(w.shape[0], -1).double()
    amax = w2.abs().amax(1)
    s = torch.where(amax > 0, torch.exp2(torch.ceil(torch.log2(amax / E4M3_MAX))), torch.ones_like(amax))
    q = _e4m3(w2 / s[:, None])
    return (q * s[:, None]).reshape(w.shape), q.reshape(w.shape), s


class Fp8MlpFn(torch.autograd.Function):
    """fc2(Dropout(gelu(fc1(x)))) of cswin:180-196 with the fp8 fused Mlp's roundings (float64):

    forward   h = mx(x) W1^T + b1,  g = gelu(h) * m_h,  y = mx(g) W2^T + b2
    backward  (straight-through: gradients flow through every rounding unchanged, except that the
              device multiplies rounded operands in the two input-gradient products as well)
              dg = mx(dy * s2) q2,  dh = dg * gelu'(h) * m_h,  dx = mx(dh * s1) q1,
              dW1 = dh^T x,  db1 = sum dh,  dW2 = dy^T mx(g),  db2 = sum dy
    w1 = q1 * s1[:, None], w2 = q2 * s2[:, None] are the dequantised e4m3 weights (quant_rows);
    m_h the hidden dropout mask (scale 0 or 1/keep) or None.
    ``bwd_fp8`` False: the backward of csu's bf16 fused Mlp on the dequantised weights instead (what
    the product runs where that kernel is the faster one, csu.ops.FP8_MLP_BWD_C): h recomputed from
    the unrounded x, dg = dy w2, dh = dg gelu'(h) m_h, dx = dh w1, dW2 = dy^T (gelu(h) m_h)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, s1, s2, m_h, bwd_fp8=True):
        xd = x.double()
        h = mx_quant(xd) @ w1.double().t() + b1.double()
        g = F.gelu(h)
        if m_h is not None:
            g = g * m_h
        gq = mx_quant(g)
        ctx.save_for_backward(xd, h, gq, w1.double(), w2.double(), s1.double(), s2.double(), b1.double())
        ctx.m_h = m_h
        ctx.bwd_fp8 = bwd_fp8
        return gq @ w2.double().t() + b2.double()

    @staticmethod
    def backward(ctx, dy):
        xd, h, gq, w1, w2, s1, s2, b1 = ctx.saved_tensors
        dy = dy.double()
        if not ctx.bwd_fp8:
            h = xd @ w1.t() + b1
            gq = F.gelu(h) if ctx.m_h is None else F.gelu(h) * ctx.m_h
        dgelu = 0.5 * (1 + torch.erf(h / math.sqrt(2))) + h * torch.exp(-0.5 * h * h) / math.sqrt(2 * math.pi)
        if ctx.bwd_fp8:
            q1, q2 = w1 / s1[:, None], w2 / s2[:, None]
            dg = mx_quant(dy * s2) @ q2
        else:
            dg = dy @ w2
        dh = dg * dgelu
        if ctx.m_h is not None:
            dh = dh * ctx.m_h
        dx = mx_quant(dh * s1) @ q1 if ctx.bwd_fp8 else dh @ w1
        lead = dy.reshape(-1, dy.shape[-1])
        dh2 = dh.reshape(-1, dh.shape[-1])
        dw1 = dh2.t() @ xd.reshape(-1, xd.shape[-1])
        dw2 = lead.t() @ gq.reshape(-1, gq.shape[-1])
        return dx, dw1, dh2.sum(0), dw2, lead.sum(0), None, None, None, None


def fp8_mlp(x, w1, b1, w2, b2, s1, s2, m_h=None, bwd_fp8=True):
    return Fp8MlpFn.apply(x, w1, b1, w2, b2, s1, s2, m_h, bwd_fp8)
