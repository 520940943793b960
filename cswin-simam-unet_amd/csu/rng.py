"""Counter-based dropout RNG (Philox4x32-7, csrc/rng.hpp) for the fused dropout sites of the
CSWin-UNet: pos_drop (cswin:512/628), attention dropout on P (cswin:246/290), Mlp dropout
(cswin:188/193/195) and DropPath (cswin:344/367-368).

Each device holds a state [seed, counter] (int64 x 2 in HBM).  A training forward takes ONE
snapshot of it (``csu_rng_advance``: snap = state, counter += 1, a device-side kernel, so a
captured HIP graph draws fresh masks on every replay) and every site of that forward draws its
mask from (snapshot, site id, element index); the backward of a site regenerates the identical
mask from the saved snapshot -- no mask tensor is ever stored.

Site ids are static per module (assigned by CSWinTransformer at construction, see
``assign_sites``), so a mask is a pure function of (seed, step, site, element) and
``csu_dropout_mask`` materialises any site's mask for the parity tests.
"""
from __future__ import annotations

import contextlib
from typing import Dict, Optional

import torch

from ._lib import check, lib, ptr, stream_ptr

_STATE: Dict[torch.device, torch.Tensor] = {}
_SCOPE: list = []          # stack of (device, snapshot) of active training forwards
_LAST: Dict[torch.device, torch.Tensor] = {}

# site layout: 0 = pos_drop; CSWinBlock k (registration order) uses SITE_BASE + SITE_STRIDE * k + offset
SITE_POS_DROP = 0
SITE_BASE = 1
SITE_STRIDE = 8
OFF_ATTN = 0          # branch i -> OFF_ATTN + i (csu_stripe_args.drop_site + i)
OFF_MLP_HIDDEN = 2
OFF_MLP_OUT = 3
OFF_DROPPATH_ATTN = 4
OFF_DROPPATH_MLP = 5


def _dev(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def manual_seed(seed: int, device=None):
    """Reset the dropout stream of `device` (every device with a state when None) to (seed, 0)."""
    devs = [_dev(device)] if device is not None else list(_STATE) or [_dev("cuda")]
    for d in devs:
        _STATE[d] = torch.tensor([int(seed) & (2 ** 63 - 1), 0], dtype=torch.int64, device=d)


def state(device) -> torch.Tensor:
    """The [seed, counter] state of `device`; created from torch.initial_seed() on first use."""
    d = _dev(device)
    if d not in _STATE:
        manual_seed(torch.initial_seed(), d)
    return _STATE[d]


def advance(device) -> torch.Tensor:
    """A fresh [seed, counter] snapshot (device int64 x 2); the device counter moves by one."""
    d = _dev(device)
    st = state(d)
    snap = torch.empty(2, dtype=torch.int64, device=d)
    check(lib().csu_rng_advance(ptr(st), ptr(snap), stream_ptr(d)), "rng_advance")
    _LAST[d] = snap
    return snap


def snapshot(device) -> torch.Tensor:
    """The snapshot of the enclosing training forward (``scope``), else a fresh one per call."""
    d = _dev(device)
    for sd, snap in reversed(_SCOPE):
        if sd == d:
            return snap
    return advance(d)


def last_snapshot(device) -> Optional[torch.Tensor]:
    """The most recent snapshot taken on `device` (tests materialise its masks)."""
    return _LAST.get(_dev(device))


@contextlib.contextmanager
def scope(device):
    """One snapshot shared by every dropout site of the enclosed forward."""
    d = _dev(device)
    _SCOPE.append((d, advance(d)))
    try:
        yield _SCOPE[-1][1]
    finally:
        _SCOPE.pop()


@contextlib.contextmanager
def ensure_scope(device):
    """The enclosing forward's snapshot, or a new scope for this module's forward (a standalone
    CSWinBlock / Mlp draws all its sites from one snapshot)."""
    d = _dev(device)
    for sd, snap in reversed(_SCOPE):
        if sd == d:
            yield snap
            return
    with scope(d) as snap:
        yield snap


def dropout_mask(snap: torch.Tensor, site: int, p: float, n: int) -> torch.Tensor:
    """uint8 keep mask (n,) of `site` under `snap` -- exactly the bits every kernel draws."""
    out = torch.empty(n, dtype=torch.uint8, device=snap.device)
    check(lib().csu_dropout_mask(n, ptr(snap), site, float(p), ptr(out), stream_ptr(snap.device)), "dropout_mask")
    return out


def droppath_scale(snap: torch.Tensor, site: int, p: float, n: int) -> torch.Tensor:
    """(n,) fp32 per-sample DropPath scale keep(site, b) / (1 - p)."""
    out = torch.empty(n, dtype=torch.float32, device=snap.device)
    check(lib().csu_droppath_scale(n, ptr(snap), site, float(p), ptr(out), stream_ptr(snap.device)), "droppath_scale")
    return out


def assign_sites(model: torch.nn.Module):
    """Give every CSWinBlock of `model` (registration order) its own block of site ids."""
    from .model import CSWinBlock
    k = 0
    for m in model.modules():
        if isinstance(m, CSWinBlock):
            m.set_drop_sites(SITE_BASE + SITE_STRIDE * k)
            k += 1
