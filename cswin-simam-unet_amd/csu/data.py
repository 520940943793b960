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


# ---------------------------------------------------------------------------------------------
# The reference's file dataset and augmentation (cswin:20-175) with a device augmentation path.
# ---------------------------------------------------------------------------------------------
def resize_bilinear_u8(a: np.ndarray, h: int, w: int) -> np.ndarray:
    """cv2.resize(a, (w, h)) with INTER_LINEAR on uint8 HW / HWC arrays (half-pixel centres,
    border-clamped, rounded half up to uint8) -- cv2 itself is not in this image; cv2 computes the weights in
    11-bit fixed point, so individual pixels can differ from it by 1."""
    sh, sw = a.shape[:2]

    def axis(n, m):
        s = (np.arange(m, dtype=np.float32) + 0.5) * (np.float32(n) / np.float32(m)) - 0.5
        s = np.maximum(s, 0.0)
        i0 = np.minimum(s.astype(np.int64), n - 1)
        f = (s - i0).astype(np.float32)
        i1 = np.minimum(i0 + 1, n - 1)
        return i0, i1, f

    y0, y1, fy = axis(sh, h)
    x0, x1, fx = axis(sw, w)
    af = a.astype(np.float32)
    if a.ndim == 3:
        fy, fx = fy[:, None, None], fx[None, :, None]
    else:
        fy, fx = fy[:, None], fx[None, :]
    top = af[y0][:, x0] * (1 - fx) + af[y0][:, x1] * fx
    bot = af[y1][:, x0] * (1 - fx) + af[y1][:, x1] * fx
    return np.clip(np.floor(top * (1 - fy) + bot * fy + 0.5), 0, 255).astype(np.uint8)   # half up, as cv2


class AugmentationTransform:
    """Same constructor and call as the reference's (cswin:20-87): horizontal / vertical flip with
    ``flip_prob`` each, a rotation by a random multiple of 90 degrees with ``rotate_prob``, then a
    random crop of scale ``crop_scale`` resized back -- applied identically to image and mask.
    ``draw`` consumes np.random in the reference's order, so a seeded run draws the reference's
    parameters; ``__call__`` applies them on the host (numpy uint8), ``DeviceAugment`` on the GPU."""

    def __init__(self, flip_prob=0.5, rotate_prob=0.25, crop_scale=(0.75, 1.0)):
        self.flip_prob = flip_prob
        self.rotate_prob = rotate_prob
        self.crop_scale = crop_scale

    def draw(self, h: int, w: int, rng=np.random):
        """(hflip, vflip, quarter turns clockwise, top, left, crop_h, crop_w) for an h x w image."""
        hflip = int(rng.random() < self.flip_prob)
        vflip = int(rng.random() < self.flip_prob)
        rot = 0
        if rng.random() < self.rotate_prob:
            rot = int(rng.choice([0, 90, 180, 270])) // 90
        if rot % 2:
            h, w = w, h
        cs = rng.uniform(self.crop_scale[0], self.crop_scale[1])
        nh, nw = int(h * cs), int(w * cs)
        top = rng.randint(0, h - nh + 1) if h > nh else 0
        left = rng.randint(0, w - nw + 1) if w > nw else 0
        return hflip, vflip, rot, int(top), int(left), nh, nw

    @staticmethod
    def crop(image: np.ndarray, mask: np.ndarray, params):
        """Flips, rotation and crop of ``params`` (the arrays cv2.resize receives in the reference)."""
        hflip, vflip, rot, top, left, nh, nw = params
        if hflip:
            image, mask = image[:, ::-1], mask[:, ::-1]
        if vflip:
            image, mask = image[::-1], mask[::-1]
        if rot:   # np.rot90 turns counter-clockwise: k = -rot for clockwise quarter turns
            image, mask = np.rot90(image, -rot), np.rot90(mask, -rot)
        return image[top:top + nh, left:left + nw], mask[top:top + nh, left:left + nw], image.shape[:2]

    @classmethod
    def apply(cls, image: np.ndarray, mask: np.ndarray, params):
        image, mask, (h, w) = cls.crop(image, mask, params)
        return resize_bilinear_u8(np.ascontiguousarray(image), h, w), resize_bilinear_u8(np.ascontiguousarray(mask), h, w)

    def __call__(self, image, mask):
        return self.apply(image, mask, self.draw(*image.shape[:2]))


class SegmentationDataset(torch.utils.data.Dataset):
    """The reference's dataset (cswin:91-175): ``*.jpg`` images of ``image_dir`` with same-named
    masks in ``mask_dir`` (missing / unreadable mask -> zeros, as the reference), resized to
    ``image_size`` read as cv2.resize reads it, i.e. (width, height) (cswin:160-161), optionally augmented, returned as (3, H, W) / (1, H, W) float32
    in [0, 1].  Decoding uses PIL (cv2 is not in this image).  ``device_augment=True`` returns the
    resized uint8 (H, W, 3) image and (H, W) mask instead, for ``DeviceAugment`` to augment and
    normalise a whole batch on the GPU."""

    def __init__(self, image_dir, mask_dir, image_size=(224, 224), augment=False, device_augment=False):
        import glob
        import os
        self.image_dir, self.mask_dir, self.image_size = image_dir, mask_dir, tuple(image_size)
        self.augment, self.device_augment = augment, device_augment
        self.transform = AugmentationTransform(flip_prob=0.5, rotate_prob=0.25, crop_scale=(0.75, 1.0)) if augment else None
        self.image_paths = sorted(glob.glob(os.path.join(image_dir, "*.jpg")))
        if not self.image_paths:
            raise ValueError(f"no images found in: {image_dir}")

    def __len__(self):
        return len(self.image_paths)

    def load(self, idx):
        """(image uint8 (H, W, 3) RGB, mask uint8 (H, W)) resized to image_size, not augmented."""
        import os
        from PIL import Image
        path = self.image_paths[idx]
        image = np.asarray(Image.open(path).convert("RGB"))
        mpath = os.path.join(self.mask_dir, os.path.basename(path))
        try:
            mask = np.asarray(Image.open(mpath).convert("L"))
        except (FileNotFoundError, OSError):
            mask = np.zeros(image.shape[:2], dtype=np.uint8)
        w, h = self.image_size            # cv2.resize(image, dsize=(w, h)) (cswin:160-161)
        return resize_bilinear_u8(image, h, w), resize_bilinear_u8(mask, h, w)

    def __getitem__(self, idx):
        image, mask = self.load(idx)
        if self.device_augment:
            return torch.from_numpy(np.ascontiguousarray(image)), torch.from_numpy(np.ascontiguousarray(mask))
        if self.transform is not None:
            image, mask = self.transform(image, mask)
        image = torch.from_numpy(np.ascontiguousarray(image).astype(np.float32) / 255.0).permute(2, 0, 1)
        mask = torch.from_numpy(np.ascontiguousarray(mask).astype(np.float32) / 255.0).unsqueeze(0)
        return image, mask


class DeviceAugment:
    """Batch augmentation + normalisation on the GPU (csu_augment_batch): uint8 images (B, S, S, 3)
    and masks (B, S, S) on the device -> (B, 3, S, S), (B, 1, S, S) float32 / 255.  Parameters are
    drawn per image on the host by ``transform.draw`` (None: no augmentation, normalisation only)."""

    def __init__(self, transform: "AugmentationTransform" = None):
        self.transform = transform

    def __call__(self, images: torch.Tensor, masks: torch.Tensor, params=None):
        from . import ops
        B, S = images.shape[0], images.shape[1]
        if images.shape[2] != S or images.shape[3] != 3 or tuple(masks.shape) != (B, S, S):
            raise ValueError("DeviceAugment: square uint8 images (B, S, S, 3) and masks (B, S, S)")
        if params is None:
            params = [self.transform.draw(S, S) if self.transform is not None else (0, 0, 0, 0, 0, S, S)
                      for _ in range(B)]
        return ops.augment_batch(images, masks, params)


class DeviceAugmentLoader:
    """Iterates a DataLoader over a ``SegmentationDataset(..., device_augment=True)`` and yields
    batches augmented + normalised on ``device`` (one csu_augment_batch launch per batch) in place
    of the reference's per-sample host augmentation inside the DataLoader workers; ``augment=False``
    datasets are only normalised.  Drop-in for ``train_model``'s loaders (images are already on the
    device there)."""

    def __init__(self, loader, device):
        self.loader, self.device = loader, torch.device(device)
        ds = loader.dataset
        self.aug = DeviceAugment(ds.transform if getattr(ds, "augment", False) else None)
        self.sampler = getattr(loader, "sampler", None)

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for images, masks in self.loader:
            yield self.aug(images.to(self.device, non_blocking=True), masks.to(self.device, non_blocking=True))
