"""CPU restatement of the reference's augmentation + normalisation (test infrastructure only).

Follows train_cswinunet_segmentation.py:
  AugmentationTransform.__call__  cswin:36-87  (flip p, flip p, rotate p -> choice of 4 angles,
                                                 uniform crop scale, randint top/left, resize back)
  SegmentationDataset.__getitem__ cswin:159-173 (resize, augment, /255, HWC -> CHW)
cv2 is not in this image, so cv2.flip / cv2.rotate are restated from their documented semantics
and cv2.resize(INTER_LINEAR) as the textbook bilinear resize with half-pixel centres and clamped
borders, evaluated per pixel in float64 (cv2 rounds its weights to 11-bit fixed point: results can
differ from cv2 by 1 in a few pixels -- the resize is "parity unpinned" against cv2).  The random
draw order and the flip / rotate / crop geometry are pinned by tests/golden/f10_augment.npz, made by
running the reference's own AugmentationTransform (make_golden.py f10).
"""
from __future__ import annotations

import numpy as np


def draw(h, w, rng, flip_prob=0.5, rotate_prob=0.25, crop_scale=(0.75, 1.0)):
    """The reference's np.random calls in order (cswin:48-77) -> (hflip, vflip, rot_cw, top, left, nh, nw)."""
    hflip = rng.random() < flip_prob
    vflip = rng.random() < flip_prob
    rot = 0
    if rng.random() < rotate_prob:
        rot = {0: 0, 90: 1, 180: 2, 270: 3}[int(rng.choice([0, 90, 180, 270]))]
    if rot in (1, 3):
        h, w = w, h
    cs = rng.uniform(crop_scale[0], crop_scale[1])
    nh, nw = int(h * cs), int(w * cs)
    top = rng.randint(0, h - nh + 1) if h > nh else 0
    left = rng.randint(0, w - nw + 1) if w > nw else 0
    return int(hflip), int(vflip), rot, int(top), int(left), nh, nw


def geometry(a, params):
    """cv2.flip(a, 1), cv2.flip(a, 0), cv2.rotate(...) and the crop (cswin:48-81), by explicit index maps."""
    hflip, vflip, rot, top, left, nh, nw = params
    H, W = a.shape[:2]
    if hflip:
        a = np.stack([a[:, W - 1 - x] for x in range(W)], axis=1)
    if vflip:
        a = np.stack([a[H - 1 - y] for y in range(H)], axis=0)
    if rot == 1:     # ROTATE_90_CLOCKWISE: out[y][x] = in[H-1-x][y], out is W x H
        a = np.stack([np.stack([a[H - 1 - x, y] for x in range(H)]) for y in range(W)])
    elif rot == 2:
        a = np.stack([np.stack([a[H - 1 - y, W - 1 - x] for x in range(W)]) for y in range(H)])
    elif rot == 3:   # ROTATE_90_COUNTERCLOCKWISE: out[y][x] = in[x][W-1-y]
        a = np.stack([np.stack([a[x, W - 1 - y] for x in range(H)]) for y in range(W)])
    return a[top:top + nh, left:left + nw]


def resize_linear(a, h, w):
    """cv2.resize(a, (w, h)) INTER_LINEAR semantics on uint8, per pixel in float64, rounded."""
    sh, sw = a.shape[:2]
    out = np.zeros((h, w) + a.shape[2:], dtype=np.uint8)

    def coord(o, n, m):
        s = (o + 0.5) * (n / m) - 0.5
        if s < 0:
            s = 0.0
        i = min(int(s), n - 1)
        return i, min(i + 1, n - 1), s - i

    af = a.astype(np.float64)
    for y in range(h):
        y0, y1, fy = coord(y, sh, h)
        for x in range(w):
            x0, x1, fx = coord(x, sw, w)
            v = (af[y0, x0] * (1 - fx) + af[y0, x1] * fx) * (1 - fy) + (af[y1, x0] * (1 - fx) + af[y1, x1] * fx) * fy
            out[y, x] = np.clip(np.floor(v + 0.5), 0, 255)
    return out


def augment(image, mask, params):
    """One augmented pair (cswin:36-87) -> float32 (3, H, W) and (1, H, W) in [0, 1] (cswin:167-173)."""
    ci, cm = geometry(image, params), geometry(mask, params)
    rot = params[2]
    h, w = image.shape[:2]
    if rot in (1, 3):
        h, w = w, h
    ri, rm = resize_linear(ci, h, w), resize_linear(cm, h, w)
    return (ri.astype(np.float32) / 255.0).transpose(2, 0, 1), (rm.astype(np.float32) / 255.0)[None]
