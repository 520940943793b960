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
    def forward(ctx, x, lam: float):
        require_device(x)
        x = x.contiguous()
        B, L, C = x.shape
        y = torch.empty_like(x)
        stats = torch.empty(B, C, 2, dtype=torch.float32, device=x.device)
        Lb = lib()
        n = Lb.csu_simam_workspace(B, L, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        launch("simam_fwd", lambda: Lb.csu_simam_fwd(B, L, C, float(lam), dtype_code(x), ptr(x), ptr(y), ptr(stats),
                                                     ptr(work), n, stream_ptr(x.device)),
               8 * x.numel(), 2 * x.numel() * x.element_size(), prec=prec_of(x))
        ctx.save_for_backward(x, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, stats = ctx.saved_tensors
        dy = dy.to(x.dtype).contiguous()
        B, L, C = x.shape
        dx = torch.empty_like(x)
        Lb = lib()
        n = Lb.csu_simam_workspace(B, L, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        launch("simam_bwd", lambda: Lb.csu_simam_bwd(B, L, C, dtype_code(x), ptr(x), ptr(stats), ptr(dy), ptr(dx),
                                                     ptr(work), n, stream_ptr(x.device)),
               16 * x.numel(), 3 * x.numel() * x.element_size(), prec=prec_of(x))
        return dx, None


def simam(x: torch.Tensor, lam: float = 1e-4) -> torch.Tensor:
    """SimAM on (B, L, C) tokens."""
    return _SimAMFn.apply(x, lam)


class SimAM(nn.Module):
    """Parameter-free SimAM module on token tensors (B, L, C); e_lambda as in the SimAM paper."""

    def __init__(self, e_lambda: float = 1e-4):
        super().__init__()
        self.e_lambda = e_lambda

    def forward(self, x):
        return simam(x, self.e_lambda)
