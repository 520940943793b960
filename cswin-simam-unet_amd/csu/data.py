"""Synthetic segmentation data: the reference only ships a jpg loader
(``SegmentationDataset`` cswin:91-175) over a private dataset, so benchmarks and trajectories use
this generator instead.  Output contract matches ``SegmentationDataset.__getitem__`` (cswin:130-175):
image (3, S, S) float32 in [0, 1] quantised to k/255 (cswin:168), mask (1, S, S) float32 {0, 1}.
"""
from __future__ import annotations

import numpy as np
import torch


def ellipse_sample(rng: np.random.Generator, size: int):
    """One (image, mask) pair as numpy arrays (3,S,S) / (1,S,S)."""
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32) + 0.5
    mask = np.zeros((size, size), dtype=bool)
    for _ in range(int(rng.integers(1, 4))):
        cy, cx = rng.uniform(0.2, 0.8, size=2) * size
        ay, ax = rng.uniform(0.05, 0.25, size=2) * size
        th = rng.uniform(0.0, np.pi)
        c, s = np.cos(th), np.sin(th)
        dy, dx = yy - cy, xx - cx
        u, v = c * dx + s * dy, -s * dx + c * dy
        mask |= (u / ax) ** 2 + (v / ay) ** 2 <= 1.0
    bg = rng.uniform(0.2, 0.4, size=3).astype(np.float32)
    fg = rng.uniform(0.6, 0.8, size=3).astype(np.float32)
    img = np.where(mask[None], fg[:, None, None], bg[:, None, None])
    img = img + rng.normal(0.0, 0.08, size=img.shape).astype(np.float32)
    img = np.round(np.clip(img, 0.0, 1.0) * 255.0) / 255.0
    return img.astype(np.float32), mask[None].astype(np.float32)


def ellipse_batch(rng: np.random.Generator, batch: int, size: int):
    """(images (B,3,S,S), masks (B,1,S,S)) float32 CPU tensors."""
    pairs = [ellipse_sample(rng, size) for _ in range(batch)]
    imgs = torch.from_numpy(np.stack([p[0] for p in pairs]))
    masks = torch.from_numpy(np.stack([p[1] for p in pairs]))
    return imgs, masks


class SyntheticSegmentation(torch.utils.data.Dataset):
    """Deterministic map-style dataset: sample i is drawn from ``default_rng(seed + i)``."""

    def __init__(self, n: int, size: int, seed: int = 1234):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        img, mask = ellipse_sample(np.random.default_rng(self.seed + i), self.size)
        return torch.from_numpy(img), torch.from_numpy(mask)
