"""Drop-in plain UNet (train_unet_segmentation.py unet:177-250) on channels-last activations.

Same classes (DoubleConv, Down, Up, UNet), constructor arguments and state_dict keys as the
reference; every op of the step runs libcsu_hip.so kernels on NHWC activations: the 3x3 / 1x1
convolutions and the ConvTranspose2d(k2, s2) upsampling on the implicit-GEMM kernels
(csu.ops.conv2d / conv_transpose2d), BatchNorm2d + ReLU fused (csu_bn_relu_fwd/bwd: batch
statistics, running-stat update, ReLU mask recomputed in the backward) and MaxPool2d(2)
(csu_maxpool2_fwd/bwd).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops
from ._lib import dtype_code, lib, ptr, require_device, stream_ptr
from .ledger import launch, prec_of


def _ws(M, C, dev):
    return torch.empty(max(int(lib().csu_bn_workspace(M, C)), 16), dtype=torch.uint8, device=dev)


class _BnReluFn(torch.autograd.Function):
    """BatchNorm2d (+ ReLU) on NHWC rows: F.batch_norm + F.relu of unet:183-187 in three csu
    launches per direction (statistics partials, fixed-order combine + running stats, apply)."""

    @staticmethod
    def forward(ctx, x, weight, bias, rmean, rvar, training: bool, momentum: float, eps: float, relu: bool):
        require_device(x)
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        y = torch.empty_like(x)
        save = torch.empty(2, C, dtype=torch.float32, device=x.device)
        w, b = weight.detach().float().contiguous(), bias.detach().float().contiguous()
        ws = _ws(M, C, x.device)
        nb = x.numel() * x.element_size()
        launch("bn_relu_fwd", lambda: lib().csu_bn_relu_fwd(M, C, dtype_code(x), ptr(x), ptr(w), ptr(b), ptr(rmean),
                                                            ptr(rvar), float(momentum), float(eps), int(training),
                                                            int(relu), ptr(save), ptr(y), ptr(ws), ws.numel(),
                                                            stream_ptr(x.device)),
               8 * x.numel(), nb * (3 if training else 2), idem=not (training and rmean is not None), prec=prec_of(x))
        ctx.save_for_backward(x, w, b, save)
        ctx.flags = (training, relu)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, save = ctx.saved_tensors
        training, relu = ctx.flags
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        dy = dy.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        dx = torch.empty_like(x)
        dg = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty(C, dtype=torch.float32, device=x.device)
        ws = _ws(M, C, x.device)
        nb = x.numel() * (2 * x.element_size() + 2 * dy.element_size())
        launch("bn_relu_bwd", lambda: lib().csu_bn_relu_bwd(M, C, dtype_code(x), ptr(x), ptr(w), ptr(b), ptr(save),
                                                            int(training), int(relu), dtype_code(dy), ptr(dy), ptr(dx),
                                                            ptr(dg), ptr(db), ptr(ws), ws.numel(), stream_ptr(x.device)),
               12 * x.numel(), nb, prec=prec_of(x))
        return dx, dg, db, None, None, None, None, None, None


def bn_relu_nhwc(x: torch.Tensor, bn: nn.BatchNorm2d, relu: bool = True) -> torch.Tensor:
    """BatchNorm2d (unet:183/186) [+ ReLU (unet:184/187)] on an NHWC tensor, nn.BatchNorm2d's
    semantics: batch statistics in training (or without running stats), running-stat update
    with ``momentum`` (None: cumulative average over num_batches_tracked), eval on running stats."""
    use_batch = bn.training or not bn.track_running_stats
    momentum = bn.momentum if bn.momentum is not None else 0.0
    if bn.training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
        if bn.momentum is None:
            momentum = 1.0 / float(bn.num_batches_tracked)
    track = bn.track_running_stats and bn.running_mean is not None
    rm = bn.running_mean if track else None
    rv = bn.running_var if track else None
    if not use_batch and rm is None:
        raise ValueError("bn_relu_nhwc: eval mode needs running statistics")
    w = bn.weight if bn.affine else torch.ones(x.shape[-1], device=x.device)
    b = bn.bias if bn.affine else torch.zeros(x.shape[-1], device=x.device)
    return _BnReluFn.apply(x, w, b, rm, rv, use_batch, momentum, bn.eps, relu)


class _MaxPool2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        require_device(x)
        x = x.contiguous()
        B, H, W, C = x.shape
        y = torch.empty(B, H // 2, W // 2, C, dtype=x.dtype, device=x.device)
        launch("maxpool2_fwd", lambda: lib().csu_maxpool2_fwd(B, H, W, C, dtype_code(x), ptr(x), ptr(y),
                                                              stream_ptr(x.device)),
               3 * y.numel(), (x.numel() + y.numel()) * x.element_size(), prec=prec_of(x))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        dy = dy.contiguous()
        B, H, W, C = x.shape
        # odd H / W: the last row / column is in no window (floor), its gradient is 0
        dx = torch.zeros_like(x) if (H % 2 or W % 2) else torch.empty_like(x)
        launch("maxpool2_bwd", lambda: lib().csu_maxpool2_bwd(B, H, W, C, dtype_code(x), ptr(x), dtype_code(dy), ptr(dy),
                                                              ptr(dx), stream_ptr(x.device)),
               3 * dy.numel(), 2 * x.numel() * x.element_size() + dy.numel() * dy.element_size(), prec=prec_of(x))
        return dx


def max_pool2_nhwc(x: torch.Tensor) -> torch.Tensor:
    """MaxPool2d(2) (unet:200) on an NHWC tensor."""
    return _MaxPool2Fn.apply(x)


class DoubleConv(nn.Module):
    """(Conv2D -> BN -> ReLU) * 2 (unet:177-191); forward takes/returns NHWC."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.double_conv = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1),
            nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True),
        )

    def forward(self, x, x_cat=None):
        """x_cat: a second input concatenated after x on channels (Up; the concatenation is never
        materialised when the two-source conv kernels take the geometry)."""
        c1, b1, _, c2, b2, _ = self.double_conv
        y = ops.conv2d(x, c1.weight, c1.bias, 1, 1) if x_cat is None else ops.conv2d_cat(x, x_cat, c1.weight, c1.bias, 1)
        x = bn_relu_nhwc(y, b1)
        return bn_relu_nhwc(ops.conv2d(x, c2.weight, c2.bias, 1, 1), b2)


class Down(nn.Module):
    """MaxPool2d(2) then DoubleConv (unet:194-204)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    def forward(self, x):
        return self.maxpool_conv[1](max_pool2_nhwc(x))


class Up(nn.Module):
    """ConvTranspose2d(C, C/2, 2, 2), cat([skip, up]) on channels, DoubleConv (unet:207-218)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x1, x2):
        x1 = ops.conv_transpose2d(x1, self.up.weight, self.up.bias, 2)
        return self.conv(x2, x1)   # conv(cat([x2, x1], channels)), unet:213-216


class UNet(nn.Module):
    """UNet(n_channels=3, n_classes=1) (unet:221-250): NCHW image in, NCHW probabilities out."""

    def __init__(self, n_channels=3, n_classes=1):
        super(UNet, self).__init__()
        self.n_channels = n_channels
        self.n_classes = n_classes
        self.inc = DoubleConv(n_channels, 64)
        self.down1 = Down(64, 128)
        self.down2 = Down(128, 256)
        self.down3 = Down(256, 512)
        self.down4 = Down(512, 1024)
        self.up1 = Up(1024, 512)
        self.up2 = Up(512, 256)
        self.up3 = Up(256, 128)
        self.up4 = Up(128, 64)
        self.outc = nn.Conv2d(64, n_classes, kernel_size=1)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        x = x.permute(0, 2, 3, 1)                      # NHWC view of the image
        x1 = self.inc(x)
        x2 = self.down1(x1)
        x3 = self.down2(x2)
        x4 = self.down3(x3)
        x5 = self.down4(x4)
        x = self.up1(x5, x4)
        x = self.up2(x, x3)
        x = self.up3(x, x2)
        x = self.up4(x, x1)
        logits = ops.conv2d(x, self.outc.weight, self.outc.bias, 1, 0)   # (B, H, W, n_classes)
        return self.sigmoid(logits.float()).permute(0, 3, 1, 2)
