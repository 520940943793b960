"""Fused AdamW on the csu_adamw_step kernel (the optimizer of cswin:937-941).

The same pass writes the bf16 shadow copies of the updated weights that the model's cast cache
keeps for the next forward (csu.ops.shadow_spec: W, W^T, conv OHWI / IHWO), so no separate cast
launch re-reads the fp32 weights.

Drop-in for ``torch.optim.AdamW`` (same constructor arguments, param_groups, state keys
``step`` / ``exp_avg`` / ``exp_avg_sq`` and state_dict format, ReduceLROnPlateau works on it): one
kernel launch updates every parameter of a group from a device table of pointers.  The table is
rebuilt only when the set of (param, grad) buffers changes, from a pinned host buffer, so the step
can also be captured into a HIP graph (lr and the step count then live in device tensors that are
updated in place: ``capturable=True``)."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import lib, stream_ptr
from .ledger import launch

_ITEM = np.dtype([("param", "<u8"), ("grad", "<u8"), ("exp_avg", "<u8"), ("exp_avg_sq", "<u8"), ("numel", "<i8"),
                  ("chunk0", "<i8"), ("shadow", "<u8"), ("shadow_t", "<u8"), ("rows", "<i4"), ("cols", "<i4"),
                  ("taps", "<i4"), ("cols_pad", "<i4")])
_NO_SHADOW = (0, 0, 0, 0, 0, 0)


def _chunks(n, spec, chunk):
    """Chunk (workgroup) count of one item: 64 x 64 tiles for a matrix with a transposed shadow,
    else ceil(numel / chunk) (csu.h, csu_adamw_item)."""
    sh, sht, rows, cols, taps, _ = spec
    if sh and sht and taps == 0:
        return -(-rows // 64) * -(-cols // 64)
    return -(-n // chunk)


class FusedAdamW(torch.optim.Optimizer):
    _L2 = False   # FusedAdam: coupled L2 weight decay (torch.optim.Adam)

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, capturable=False):
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError("invalid AdamW hyper-parameter")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=capturable))
        self._tables = {}
        self._gstate = {}
        self._deferred = []
        self._captured = []
        # one pinned table buffer per group, reserved for a HIP-graph capture of step()
        self._pinned = {gi: torch.empty(max(1, len(g["params"])) * _ITEM.itemsize, dtype=torch.uint8, pin_memory=True)
                        for gi, g in enumerate(self.param_groups)} if torch.cuda.is_available() else {}
        # ... and its device image, allocated HERE, outside any capture: a buffer allocated inside the
        # capture comes from the graph's private pool, where it may alias memory an earlier captured
        # kernel writes on every replay -- fine for buffers the graph itself fills, fatal for one
        # filled once after the capture (finish_capture)
        self._capture_dev = {gi: torch.empty(max(1, len(g["params"])) * _ITEM.itemsize, dtype=torch.uint8,
                                             device=g["params"][0].device)
                             for gi, g in enumerate(self.param_groups) if g["params"] and g["params"][0].is_cuda}

    def prepare_capture(self):
        """Reserve the table buffers of one more capture (outside any graph pool; each captured graph
        keeps its own).  GraphedTrainStep calls it before capturing; the first capture's buffers
        come from the constructor.  A later capture re-fills the eager-side table cache only: the
        graphs captured before keep their own tables."""
        for gi, g in enumerate(self.param_groups):
            if g["params"] and g["params"][0].is_cuda and (gi not in self._pinned or gi not in self._capture_dev):
                n = max(1, len(g["params"])) * _ITEM.itemsize
                self._pinned[gi] = torch.empty(n, dtype=torch.uint8, pin_memory=True)
                self._capture_dev[gi] = torch.empty(n, dtype=torch.uint8, device=g["params"][0].device)

    def _table(self, gi, items, device):
        """Device item table for the current (param, grad) buffers, rebuilt when they change
        (e.g. every step under zero_grad(set_to_none=True) when the allocator hands out other grad
        buffers).  Eager: an asynchronous copy from a fresh pinned buffer (no host sync; the
        caching host allocator keeps it alive until the copy has run).  Under HIP-graph capture:
        the host image goes to a pinned buffer reserved for that capture (pinned memory cannot be
        allocated while capturing) and is copied ONCE after the capture (finish_capture) into a
        device buffer allocated outside the graph's memory pool and kept for the optimizer's
        lifetime -- no copy node in the replayed graph."""
        key = (gi,) + tuple(v for it in items for v in it[:4] + it[5])
        t = self._tables.get(gi)
        if t is not None and t[0] == key:
            return t
        chunk = lib().csu_adamw_chunk_elems()
        rec = np.zeros(len(items), dtype=_ITEM)
        c0 = 0
        for i, (p, g, m, v, n, spec) in enumerate(items):
            rec[i] = (p, g, m, v, n, c0) + tuple(spec)
            c0 += _chunks(n, spec, chunk)
        raw = np.frombuffer(rec.tobytes(), dtype=np.uint8)
        if torch.cuda.is_current_stream_capturing():
            host = self._pinned.get(gi)
            dev = self._capture_dev.get(gi)
            if host is None or dev is None or host.numel() < raw.size:
                raise RuntimeError("FusedAdamW: no pinned table buffer for this capture (call prepare_capture() before capturing)")
            del self._pinned[gi]                      # frozen: owned by the captured graph from now on
            del self._capture_dev[gi]
            host[:raw.size].numpy()[:] = raw
            dev = dev[:raw.size]
            # the captured kernel reads this buffer on every replay: keep it (and its host image)
            # alive for the optimizer's lifetime, whatever later eager steps put into _tables
            self._captured.append((host, dev))
            # the table is constant over replays: copied once after the capture (finish_capture)
            # instead of by a copy node on every replay
            self._deferred.append((dev, host[:raw.size]))
        else:
            host = torch.empty(raw.size, dtype=torch.uint8, pin_memory=True)
            host.numpy()[:] = raw
            dev = torch.empty(raw.size, dtype=torch.uint8, device=device)
            dev.copy_(host, non_blocking=True)
        t = (key, host, dev, len(items), c0)
        self._tables[gi] = t
        return t

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from .ops import shadow_spec, shadows_written
        for gi, group in enumerate(self.param_groups):
            items, dev, keep, shadowed = [], None, [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse or p.dtype != torch.float32 or not p.is_cuda:
                    raise RuntimeError("FusedAdamW: dense fp32 CUDA parameters only")
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                keep.append(g)          # a contiguous temporary must outlive the launch below
                if not p.is_contiguous():
                    raise RuntimeError("FusedAdamW: contiguous parameters only")
                # the bf16 copies the next forward reads (a CastCache's layouts of p), written by the
                # same pass from the updated value
                spec = shadow_spec(p)
                if spec is not None:
                    shadowed.append(p)
                items.append((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                              p.numel(), spec or _NO_SHADOW))
                dev = p.device
            if not items:
                continue
            gs = self._gstate.get(gi)
            if gs is None:
                # one device step count per group (every parameter of a group steps together);
                # resumes from a loaded state_dict's per-parameter step
                st0 = next((self.state[p]["step"] for p in group["params"] if "step" in self.state[p]
                            and self.state[p]["step"] is not None), None)
                step0 = float(st0) if st0 is not None else 0.0
                gs = self._gstate[gi] = {"step": torch.full((), step0, dtype=torch.float32, device=dev),
                                         "lr": torch.full((), group["lr"], dtype=torch.float32, device=dev)}
            gs["step"] += 1
            for p in group["params"]:
                if p.grad is not None:
                    self.state[p]["step"] = gs["step"]
            _, _, table, n, chunks = self._table(gi, items, dev)
            lr_ptr = gs["lr"].data_ptr() if group["capturable"] else None
            b1, b2 = group["betas"]
            numel = sum(it[4] for it in items)
            fn = lib().csu_adam_l2_step if self._L2 else lib().csu_adamw_step
            nsh = sum(2 * it[4] * (1 + (it[5][1] != 0)) for it in items if it[5][0])
            launch("adamw", lambda: fn(table.data_ptr(), n, chunks, lr_ptr, float(group["lr"]), float(b1),
                                                         float(b2), float(group["eps"]), float(group["weight_decay"]),
                                                         gs["step"].data_ptr(), 0.0, stream_ptr(dev)),
                   12 * numel, 28 * numel + nsh, idem=False, prec="f32")
            shadows_written(shadowed)
        return loss

    def state_dict(self):
        """torch.optim.AdamW format with a separate ``step`` tensor per parameter (the live state
        shares one device step tensor per group), so the checkpoint also loads into
        torch.optim.AdamW, whose per-parameter steps would otherwise advance once per parameter."""
        sd = super().state_dict()
        for st in sd["state"].values():
            if isinstance(st.get("step"), torch.Tensor):
                st["step"] = st["step"].detach().clone()
        return sd

    def load_state_dict(self, state_dict):
        """Load an AdamW / FusedAdamW state; the device step / lr of every group and the pointer
        tables are rebuilt from it on the next step().  Once a step has been captured into a HIP
        graph, the graph keeps reading the current state tensors (step, lr, exp_avg, exp_avg_sq):
        the loaded values are then copied INTO them, so the captured pointers stay valid."""
        if not self._captured:
            super().load_state_dict(state_dict)
            self._gstate = {}
            self._tables = {}
            return
        old = {p: dict(self.state[p]) for g in self.param_groups for p in g["params"] if self.state.get(p)}
        super().load_state_dict(state_dict)
        with torch.no_grad():
            for gi, g in enumerate(self.param_groups):
                gs = self._gstate.get(gi)
                for p in g["params"]:
                    st, o = self.state.get(p), old.get(p)
                    if not st:
                        if o is not None:
                            # the captured step keeps updating this parameter with its old moments
                            # and the group's step count: a "fresh" loaded state cannot be honoured
                            raise RuntimeError("FusedAdamW.load_state_dict after a capture: the loaded state "
                                               "has no state for a parameter the captured step updates")
                        continue
                    if o is None:
                        raise RuntimeError("FusedAdamW.load_state_dict after a capture: the loaded state has a "
                                           "parameter the captured step has no state for")
                    for k in ("exp_avg", "exp_avg_sq"):
                        o[k].copy_(st[k])
                        st[k] = o[k]
                    if gs is not None:
                        gs["step"].fill_(float(st["step"]))
                        st["step"] = gs["step"]
                if gs is not None:
                    gs["lr"].fill_(g["lr"])

    def finish_capture(self):
        """After a HIP-graph capture of step(): fill the device tables the captured kernel reads
        (their host images were frozen during the capture).  Synchronous, once per capture."""
        for dev, host in self._deferred:
            dev.copy_(host)
        self._deferred = []
        torch.cuda.synchronize()

    def sync_lr(self):
        """Copy the host lr of every group into its device tensor (capturable groups read it at
        replay time): call after a scheduler step, outside graph replay."""
        for gi, g in enumerate(self.param_groups):
            if gi in self._gstate:
                self._gstate[gi]["lr"].fill_(g["lr"])


class FusedAdam(FusedAdamW):
    """Drop-in for ``torch.optim.Adam`` (coupled L2 weight decay: g += weight_decay * param before the
    moments) on the same one-launch kernel: the plain UNet's optimizer (unet:486-490)."""
    _L2 = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, capturable=False):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=capturable)
