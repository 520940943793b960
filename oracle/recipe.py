"""Deterministic weight recipe shared by the golden generator and the parity tests.

Weights are regenerated from a (key, shape) contract instead of being committed:
per key i in contract order a numpy ``default_rng(seed*100003 + i)`` stream gives
  conv weight / bias      ~ U(+-1/sqrt(fan_in))        (torch Conv default bound)
  Linear weight           ~ N(0, 0.02) clipped at +-2   (timm trunc_normal_, cswin:609)
  Linear bias             = 0                           (cswin:610-611)
  LayerNorm / BatchNorm   weight 1, bias 0              (cswin:612-614)
  BN running_mean/var     0 / 1, num_batches_tracked 0
Test infrastructure only.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch


def recipe_from_contract(contract: List[Tuple[str, Tuple[int, ...]]], seed: int = 0,
                         dtype=torch.float32) -> Dict[str, torch.Tensor]:
    shapes = dict(contract)
    out: Dict[str, torch.Tensor] = {}
    for i, (key, shape) in enumerate(contract):
        mod, kind = key.rsplit(".", 1)
        wshape = shapes.get(mod + ".weight", ())
        rng = np.random.default_rng(seed * 100003 + i)
        if kind in ("running_mean",):
            a = np.zeros(shape)
        elif kind == "running_var":
            a = np.ones(shape)
        elif kind == "num_batches_tracked":
            out[key] = torch.zeros((), dtype=torch.long)
            continue
        elif len(wshape) == 4:                                   # Conv2d / ConvTranspose2d
            fan_in = wshape[1] * wshape[2] * wshape[3]
            bound = 1.0 / math.sqrt(fan_in)
            a = rng.uniform(-bound, bound, size=shape)
        elif len(wshape) == 1:                                   # LayerNorm / BatchNorm affine
            a = np.ones(shape) if kind == "weight" else np.zeros(shape)
        elif kind == "weight":                                   # Linear
            a = np.clip(rng.normal(0.0, 0.02, size=shape), -2.0, 2.0)
        else:
            a = np.zeros(shape)
        out[key] = torch.tensor(a, dtype=dtype)
    return out
