"""Data path: the reference's AugmentationTransform / SegmentationDataset
(cswin:20-175) and the device batch augmentation (csu_augment_batch).

* Draw order + flip / rotate / crop geometry: bit-exact against f10_augment.npz, produced by the
  reference's own AugmentationTransform with recording cv2 stand-ins (tests/golden/make_golden.py).
* Bilinear resize: the host resize and the HIP kernel against oracle/augment_ref.py -- exact in
  geometry; <= 1/255 per pixel and >= 99% of pixels identical after the uint8 rounding (float32 vs
  float64 weights).  cv2 itself is absent: the resize is "parity unpinned" against cv2 (which rounds
  its weights to 11-bit fixed point)."""
import os

import numpy as np
import pytest
import torch

from oracle import augment_ref as A
from csu.data import AugmentationTransform, DeviceAugment, SegmentationDataset, resize_bilinear_u8

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "f10_augment.npz")


def _cases():
    z = np.load(GOLD)
    n = len([k for k in z.files if k.endswith("_meta")])
    for i in range(n):
        p = f"c{i}_"
        h, w, seed = z[p + "meta"]
        fp, rp, c0, c1 = z[p + "probs"]
        yield int(h), int(w), int(seed), (float(fp), float(rp), (float(c0), float(c1))), z[p + "crop_img"], \
            z[p + "crop_mask"], tuple(z[p + "size"])


def _coords(h, w):
    c = np.arange(h * w, dtype=np.int32).reshape(h, w)
    return np.stack([c, c + 100000, c + 200000], axis=-1), c


def test_oracle_geometry_matches_reference():
    seen_rot = set()
    for h, w, seed, (fp, rp, cs), ci, cm, size in _cases():
        np.random.seed(seed)
        prm = A.draw(h, w, np.random, fp, rp, cs)
        seen_rot.add(prm[2])
        img, msk = _coords(h, w)
        np.testing.assert_array_equal(A.geometry(img, prm), ci)
        np.testing.assert_array_equal(A.geometry(msk, prm), cm)
        oh, ow = (w, h) if prm[2] % 2 else (h, w)
        assert size == (ow, oh)                      # cv2.resize(crop, (w, h)) of the rotated image
    assert seen_rot == {0, 1, 2, 3}


def test_transform_matches_reference_draws():
    for h, w, seed, (fp, rp, cs), ci, cm, size in _cases():
        t = AugmentationTransform(flip_prob=fp, rotate_prob=rp, crop_scale=cs)
        np.random.seed(seed)
        prm = t.draw(h, w)
        img, msk = _coords(h, w)
        a, b, (oh, ow) = t.crop(img, msk, prm)
        np.testing.assert_array_equal(a, ci)
        np.testing.assert_array_equal(b, cm)
        assert (ow, oh) == size


def test_host_resize_vs_oracle():
    rng = np.random.default_rng(0)
    for sh, sw, h, w in [(12, 12, 16, 16), (13, 9, 16, 16), (16, 16, 16, 16), (9, 14, 12, 20), (20, 20, 7, 5)]:
        a = rng.integers(0, 256, (sh, sw, 3), dtype=np.uint8)
        r, o = resize_bilinear_u8(a, h, w).astype(int), A.resize_linear(a, h, w).astype(int)
        assert np.abs(r - o).max() <= 1 and (r == o).mean() >= 0.99
    a = rng.integers(0, 256, (16, 16), dtype=np.uint8)
    np.testing.assert_array_equal(resize_bilinear_u8(a, 16, 16), a)     # same size: a copy


def test_transform_end_to_end_vs_oracle():
    rng = np.random.default_rng(1)
    t = AugmentationTransform()
    for seed in range(8):
        img = rng.integers(0, 256, (16, 16, 3), dtype=np.uint8)
        msk = (rng.random((16, 16)) > 0.5).astype(np.uint8) * 255
        np.random.seed(seed)
        prm = t.draw(16, 16)
        a, b = t.apply(img, msk, prm)
        oa, ob = A.augment(img, msk, prm)
        assert np.abs(a.transpose(2, 0, 1) / 255.0 - oa).max() <= 1 / 255 + 1e-6
        assert np.abs(b / 255.0 - ob[0]).max() <= 1 / 255 + 1e-6


def test_segmentation_dataset(tmp_path):
    from PIL import Image
    (tmp_path / "img").mkdir()
    (tmp_path / "mask").mkdir()
    rng = np.random.default_rng(2)
    for name in ("b.jpg", "a.jpg", "c.jpg"):
        Image.fromarray(rng.integers(0, 256, (40, 30, 3), dtype=np.uint8)).save(tmp_path / "img" / name)
    Image.fromarray(((rng.random((40, 30)) > 0.5) * 255).astype(np.uint8)).save(tmp_path / "mask" / "a.jpg")
    ds = SegmentationDataset(str(tmp_path / "img"), str(tmp_path / "mask"), image_size=(32, 24))
    assert len(ds) == 3 and [os.path.basename(p) for p in ds.image_paths] == ["a.jpg", "b.jpg", "c.jpg"]
    x, m = ds[0]
    # image_size is cv2's dsize = (width, height) (cswin:160-161): (32, 24) -> 24 rows x 32 columns
    assert x.shape == (3, 24, 32) and m.shape == (1, 24, 32) and x.dtype == torch.float32
    assert 0 <= x.min() and x.max() <= 1 and m.max() > 0.5
    x, m = ds[1]                                        # missing mask -> zeros (cswin:155-157)
    assert float(m.abs().max()) == 0.0
    dsa = SegmentationDataset(str(tmp_path / "img"), str(tmp_path / "mask"), image_size=(24, 24), augment=True)
    x, m = dsa[0]
    assert x.shape[0] == 3 and m.shape[0] == 1
    dsd = SegmentationDataset(str(tmp_path / "img"), str(tmp_path / "mask"), image_size=(24, 24), device_augment=True)
    u8, mu8 = dsd[0]
    assert u8.dtype == torch.uint8 and u8.shape == (24, 24, 3) and mu8.shape == (24, 24)
    with pytest.raises(ValueError):
        SegmentationDataset(str(tmp_path / "mask" / "none"), str(tmp_path / "mask"))


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _params(rng, S, n, scale=(0.75, 1.0)):
    t = AugmentationTransform(crop_scale=scale)
    return [t.draw(S, S, rng) for _ in range(n)]


@pytest.mark.gpu
def test_device_augment_vs_oracle():
    d = _dev()
    rng = np.random.RandomState(3)
    B, S = 10, 24
    img = rng.randint(0, 256, (B, S, S, 3)).astype(np.uint8)
    msk = ((rng.rand(B, S, S) > 0.5) * 255).astype(np.uint8)
    prm = _params(rng, S, B - 2) + [(1, 0, 1, 0, 0, S, S), (1, 1, 3, 2, 3, S - 5, S - 7)]
    oi, om = DeviceAugment()(torch.from_numpy(img).to(d), torch.from_numpy(msk).to(d), prm)
    torch.cuda.synchronize()
    oi, om = oi.cpu().numpy(), om.cpu().numpy()
    exact = 0
    for b in range(B):
        ri, rm = A.augment(img[b], msk[b], prm[b])
        di, dm = np.abs(oi[b] - ri).max(), np.abs(om[b] - rm).max()
        assert di <= 1 / 255 + 1e-6 and dm <= 1 / 255 + 1e-6, (b, prm[b], di, dm)
        exact += (np.abs(oi[b] - ri) < 1e-6).sum() + (np.abs(om[b] - rm) < 1e-6).sum()
        if prm[b][5] == S and prm[b][6] == S:             # no crop: a pure permutation, bit-exact
            np.testing.assert_array_equal(oi[b], ri)
            np.testing.assert_array_equal(om[b], rm)
    assert exact / (B * 4 * S * S) >= 0.99


@pytest.mark.gpu
def test_device_augment_vs_host_transform():
    """The device path draws and applies exactly what the host AugmentationTransform does."""
    d = _dev()
    rng = np.random.default_rng(4)
    B, S = 6, 32
    img = rng.integers(0, 256, (B, S, S, 3), dtype=np.uint8)
    msk = ((rng.random((B, S, S)) > 0.5) * 255).astype(np.uint8)
    t = AugmentationTransform()
    np.random.seed(7)
    prm = [t.draw(S, S) for _ in range(B)]
    np.random.seed(7)
    oi, om = DeviceAugment(t)(torch.from_numpy(img).to(d), torch.from_numpy(msk).to(d))
    oi, om = oi.cpu().numpy(), om.cpu().numpy()
    for b in range(B):
        hi, hm = t.apply(img[b], msk[b], prm[b])
        assert np.abs(oi[b] - hi.transpose(2, 0, 1) / 255.0).max() <= 1 / 255 + 1e-6
        assert np.abs(om[b, 0] - hm / 255.0).max() <= 1 / 255 + 1e-6
    with pytest.raises(ValueError):
        DeviceAugment()(torch.from_numpy(img).to(d), torch.from_numpy(msk).to(d), [(0, 0, 0, 10, 0, S, S)] * B)


@pytest.mark.gpu
def test_device_augment_loader(tmp_path):
    from PIL import Image
    from csu.data import DeviceAugmentLoader
    d = _dev()
    (tmp_path / "img").mkdir()
    (tmp_path / "mask").mkdir()
    rng = np.random.default_rng(5)
    for i in range(5):
        Image.fromarray(rng.integers(0, 256, (40, 36, 3), dtype=np.uint8)).save(tmp_path / "img" / f"{i}.jpg")
        Image.fromarray(((rng.random((40, 36)) > 0.5) * 255).astype(np.uint8)).save(tmp_path / "mask" / f"{i}.jpg")
    plain = SegmentationDataset(str(tmp_path / "img"), str(tmp_path / "mask"), image_size=(32, 32))
    dev = SegmentationDataset(str(tmp_path / "img"), str(tmp_path / "mask"), image_size=(32, 32), device_augment=True)
    ld = DeviceAugmentLoader(torch.utils.data.DataLoader(dev, batch_size=2), d)
    got = [(x.cpu(), m.cpu()) for x, m in ld]
    assert len(got) == 3 and got[0][0].shape == (2, 3, 32, 32) and got[0][1].shape == (2, 1, 32, 32)
    x0, m0 = plain[0]
    torch.testing.assert_close(got[0][0][0], x0, rtol=0, atol=0)      # no augmentation: identical normalisation
    torch.testing.assert_close(got[0][1][0], m0, rtol=0, atol=0)
    aug = SegmentationDataset(str(tmp_path / "img"), str(tmp_path / "mask"), image_size=(32, 32), augment=True,
                              device_augment=True)
    xs = [x for x, _ in DeviceAugmentLoader(torch.utils.data.DataLoader(aug, batch_size=5), d)]
    assert xs[0].shape == (5, 3, 32, 32) and float(xs[0].min()) >= 0 and float(xs[0].max()) <= 1
