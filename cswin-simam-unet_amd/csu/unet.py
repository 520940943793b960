"""Drop-in plain UNet (train_unet_segmentation.py unet:177-250) on channels-last activations.

Same classes (DoubleConv, Down, Up, UNet), constructor arguments and state_dict keys as the
reference; the 3x3 convolutions and the ConvTranspose2d(k2, s2) upsampling run the implicit-GEMM
NHWC kernels of libcsu_hip.so (csu.ops.conv2d / conv_transpose2d); BatchNorm/ReLU/MaxPool run on
the same NHWC bytes viewed as a channels_last NCHW tensor (no layout copies).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


def _bn_nhwc(x: torch.Tensor, bn: nn.BatchNorm2d) -> torch.Tensor:
    """BatchNorm2d (unet:183/186) on an NHWC tensor through its channels_last NCHW view."""
    y = F.batch_norm(x.permute(0, 3, 1, 2), bn.running_mean, bn.running_var, bn.weight, bn.bias,
                     bn.training or not bn.track_running_stats, bn.momentum if bn.momentum is not None else 0.0, bn.eps)
    if bn.training and bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    return y.permute(0, 2, 3, 1)


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

    def forward(self, x):
        c1, b1, _, c2, b2, _ = self.double_conv
        x = F.relu(_bn_nhwc(ops.conv2d(x, c1.weight, c1.bias, 1, 1), b1))
        return F.relu(_bn_nhwc(ops.conv2d(x, c2.weight, c2.bias, 1, 1), b2))


class Down(nn.Module):
    """MaxPool2d(2) then DoubleConv (unet:194-204)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    def forward(self, x):
        pooled = F.max_pool2d(x.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
        return self.maxpool_conv[1](pooled)


class Up(nn.Module):
    """ConvTranspose2d(C, C/2, 2, 2), cat([skip, up]) on channels, DoubleConv (unet:207-218)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x1, x2):
        x1 = ops.conv_transpose2d(x1, self.up.weight, self.up.bias, 2)
        x = torch.cat([x2.to(x1.dtype), x1], dim=-1)
        return self.conv(x)


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
