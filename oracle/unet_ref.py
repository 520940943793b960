"""CPU oracle for the plain-UNet stages -- TEST INFRASTRUCTURE ONLY.

Functional restatement of ``train_unet_segmentation.py`` (``unet:N`` = line N) of
TrungMasterChef/CSWin-SimAM-UNet: DoubleConv / Down / Up / UNet (unet:177-250).  Pinned against
golden vectors from the reference itself (``tests/golden/make_golden.py``, fixture F6).
Only tests, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline may use it.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


def double_conv(x: torch.Tensor, p: Params, key: str, training: bool) -> torch.Tensor:
    """(Conv3x3 p1 -> BatchNorm2d -> ReLU) x 2 (unet:177-191).  BN indices 1 and 4 of the
    Sequential; running stats updated in place when ``training`` (momentum 0.1, unbiased var)."""
    for ci, bi in ((0, 1), (3, 4)):
        c, b = f"{key}.double_conv.{ci}", f"{key}.double_conv.{bi}"
        x = F.conv2d(x, p[c + ".weight"], p[c + ".bias"], padding=1)
        x = F.batch_norm(x, p[b + ".running_mean"], p[b + ".running_var"], p[b + ".weight"],
                         p[b + ".bias"], training=training, momentum=0.1, eps=1e-5)
        x = F.relu(x)
    return x


def unet_forward(p: Params, x: torch.Tensor, training: bool = True) -> torch.Tensor:
    """UNet(n_channels, n_classes) forward -> sigmoid probabilities (unet:221-250)."""
    x1 = double_conv(x, p, "inc", training)
    xs = [x1]
    for i in range(1, 5):                                              # Down: maxpool2 + DoubleConv
        xs.append(double_conv(F.max_pool2d(xs[-1], 2), p, f"down{i}.maxpool_conv.1", training))
    y = xs[4]
    for i in range(1, 5):                                              # Up: convT k2 s2, cat([skip, up])
        up = F.conv_transpose2d(y, p[f"up{i}.up.weight"], p[f"up{i}.up.bias"], stride=2)
        y = double_conv(torch.cat([xs[4 - i], up], dim=1), p, f"up{i}.conv", training)
    y = F.conv2d(y, p["outc.weight"], p["outc.bias"])
    return torch.sigmoid(y)


def unet_contract(n_channels: int = 3, n_classes: int = 1) -> List[Tuple[str, Tuple[int, ...]]]:
    """state_dict (key, shape) list in registration order (unet:221-237)."""
    out: List[Tuple[str, Tuple[int, ...]]] = []

    def dc(key, cin, cout):
        for ci, bi, a in ((0, 1, cin), (3, 4, cout)):
            out.extend([(f"{key}.double_conv.{ci}.weight", (cout, a, 3, 3)), (f"{key}.double_conv.{ci}.bias", (cout,))])
            b = f"{key}.double_conv.{bi}"
            out.extend([(b + ".weight", (cout,)), (b + ".bias", (cout,)), (b + ".running_mean", (cout,)),
                        (b + ".running_var", (cout,)), (b + ".num_batches_tracked", ())])

    dc("inc", n_channels, 64)
    ch = [64, 128, 256, 512, 1024]
    for i in range(1, 5):
        dc(f"down{i}.maxpool_conv.1", ch[i - 1], ch[i])
    for i in range(1, 5):
        cin = ch[5 - i]
        out.extend([(f"up{i}.up.weight", (cin, cin // 2, 2, 2)), (f"up{i}.up.bias", (cin // 2,))])
        dc(f"up{i}.conv", cin, ch[4 - i])
    out.extend([("outc.weight", (n_classes, 64, 1, 1)), ("outc.bias", (n_classes,))])
    return out
