"""SimAM: parameter-free attention gate (NOT in the reference).

Public SimAM formula on token tensors (B, L, C), statistics per (b, c) over the L positions:
``y = x * sigmoid((x - mu)^2 / (4 (var + lambda)) + 1/2)`` with the unbiased variance.  Runs
the gfx950 kernels of libcsu_hip.so (csu_simam_fwd/bwd); parity is pinned only to the float64
formula (tests), not to the reference, which has no SimAM.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ._lib import dtype_code, lib, ptr, require_device, stream_ptr
from .ledger import launch, prec_of


class _SimAMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lam: float, out_dtype):
        require_device(x)
        x = x.contiguous()
        B, L, C = x.shape
        y = torch.empty(x.shape, dtype=out_dtype or x.dtype, device=x.device)
        stats = torch.empty(B, C, 2, dtype=torch.float32, device=x.device)
        Lb = lib()
        n = Lb.csu_simam_workspace(B, L, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        # algorithmic bytes: x read twice (statistics pass, gate pass), y written once
        launch("simam_fwd", lambda: Lb.csu_simam_fwd(B, L, C, float(lam), dtype_code(x), ptr(x), dtype_code(y), ptr(y),
                                                     ptr(stats), ptr(work), n, stream_ptr(x.device)),
               12 * x.numel(), x.numel() * (2 * x.element_size() + y.element_size()), prec=prec_of(x))
        ctx.save_for_backward(x, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, stats = ctx.saved_tensors
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        dy = dy.contiguous()
        B, L, C = x.shape
        dx = torch.empty_like(x)
        Lb = lib()
        n = Lb.csu_simam_workspace(B, L, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        # x and dy read twice (partial sums, gradient pass), dx written once
        launch("simam_bwd", lambda: Lb.csu_simam_bwd(B, L, C, dtype_code(x), ptr(x), ptr(stats), dtype_code(dy), ptr(dy),
                                                     ptr(dx), ptr(work), n, stream_ptr(x.device)),
               30 * x.numel(), x.numel() * (3 * x.element_size() + 2 * dy.element_size()), prec=prec_of(x))
        return dx, None, None


class _SimAMForkFn(torch.autograd.Function):
    """(xc, y) = (bf16(x), bf16(SimAM(x))) for an fp32 encoder stage output with two consumers: the
    Merge_Block conv takes xc, the decoder's concat_linear the gated skip y (the SimAM counterpart of
    ops.shared_cast).  Forward: one statistics pass + one gate pass that also writes xc.  Backward:
    the conv's gradient g1 and the gate's dy meet in the gate-gradient pass (dx = g1 + SimAM'(dy)),
    which also writes the bf16 copy the upstream GEMM backward reads (``_csu_bf16``, ops._bf16_of)
    -- instead of autograd's cast, add and the consumer's cast (three extra passes)."""

    @staticmethod
    def forward(ctx, x, lam: float):
        require_device(x)
        x = x.contiguous()
        B, L, C = x.shape
        y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        xc = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        stats = torch.empty(B, C, 2, dtype=torch.float32, device=x.device)
        Lb = lib()
        n = Lb.csu_simam_workspace(B, L, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        launch("simam_fwd", lambda: Lb.csu_simam_fwd_fork(B, L, C, float(lam), ptr(x), ptr(y), ptr(xc), ptr(stats), ptr(work),
                                                          n, stream_ptr(x.device)),
               12 * x.numel(), x.numel() * (2 * 4 + 2 + 2), prec="f32")
        ctx.save_for_backward(x, stats)
        ctx.lam = lam
        return xc, y

    @staticmethod
    def backward(ctx, g1, dy):
        x, stats = ctx.saved_tensors
        if dy is None:
            from .ops import grad_join
            return grad_join(g1, None, torch.float32), None
        if g1 is None or g1.dtype != torch.bfloat16:
            dx = _SimAMFn.backward(ctx, dy)[0]
            return (dx if g1 is None else dx + g1.float()), None
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        dy, g1 = dy.contiguous(), g1.contiguous()
        B, L, C = x.shape
        dx = torch.empty_like(x)
        dxb = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        Lb = lib()
        n = Lb.csu_simam_workspace(B, L, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        launch("simam_bwd", lambda: Lb.csu_simam_bwd_join(B, L, C, ptr(x), ptr(stats), dtype_code(dy), ptr(dy), ptr(g1),
                                                          ptr(dx), ptr(dxb), ptr(work), n, stream_ptr(x.device)),
               30 * x.numel(), x.numel() * (3 * 4 + 2 * dy.element_size() + 2 + 4 + 2), prec="f32")
        dx._csu_bf16 = dxb
        return dx, None


def simam_fork(x: torch.Tensor, lam: float = 1e-4):
    """(bf16(x), bf16(SimAM(x))) of an fp32 (B, L, C) tensor in one forward / one backward pass each
    (see _SimAMForkFn)."""
    return _SimAMForkFn.apply(x, lam)


def simam(x: torch.Tensor, lam: float = 1e-4, out_dtype=None) -> torch.Tensor:
    """SimAM on (B, L, C) tokens (C a multiple of 4); ``out_dtype``: write the gated output in that
    dtype (e.g. bf16 for the GEMM that consumes it) from the same pass."""
    return _SimAMFn.apply(x, lam, out_dtype)


class SimAM(nn.Module):
    """Parameter-free SimAM module on token tensors (B, L, C); e_lambda as in the SimAM paper."""

    def __init__(self, e_lambda: float = 1e-4):
        super().__init__()
        self.e_lambda = e_lambda

    def forward(self, x, out_dtype=None):
        return simam(x, self.e_lambda, out_dtype)

    def fork(self, x):
        """(bf16(x), bf16(SimAM(x))) for a tensor with a second, ungated consumer (simam_fork)."""
        return simam_fork(x, self.e_lambda)
