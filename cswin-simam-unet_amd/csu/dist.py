"""Data-parallel plumbing: one process per GPU over RCCL (torch.distributed 'nccl' on ROCm).

The reference is single-device (cswin:865); SURVEY §8e: CSWin-UNet has no BatchNorm, so averaging
per-rank gradients of equal per-rank batches equals the global-batch gradient.  Buckets are sized
for xGMI point-to-point rings: 94 MB of fp32 gradients go in 32 MB buckets (3 all-reduces per step,
the first two overlapped with the rest of backward, ``GradAllReduce``).

``GradAllReduce`` is the graph-capturable replacement bench.py uses at N > 1: the same bucketed
averaging, recorded into the train step's HIP graph (DDP is the eager fallback)."""
from __future__ import annotations

import contextlib
import weakref
import os

import torch
import torch.distributed as dist


def init_distributed(backend: str = None):
    """Initialise from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).
    Returns (rank, world, device).  Single-process when WORLD_SIZE is unset or 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if use_cuda:
            torch.cuda.set_device(local)
            dist.init_process_group(backend or "nccl", device_id=device)
        else:
            dist.init_process_group(backend or "gloo")
    return rank, world, device


def wrap_ddp(model: torch.nn.Module, device: torch.device, bucket_cap_mb: int = 64):
    """DistributedDataParallel with gradient buckets as views (no copy into the bucket) and a
    static graph (every parameter receives a gradient every step, SURVEY §4 KAT iii)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    ids = [device.index] if device.type == "cuda" else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, gradient_as_bucket_view=True,
                                                     static_graph=True, bucket_cap_mb=bucket_cap_mb)


def make_loader(dataset, batch_size: int, shuffle: bool, seed: int = 42, num_workers: int = 0, drop_last=False):
    """DataLoader whose sampler shards the dataset across ranks (each rank sees len/world samples)."""
    sampler = None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(dataset, shuffle=shuffle, seed=seed,
                                                                  drop_last=drop_last)
        shuffle = False
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, sampler=sampler,
                                       num_workers=num_workers, pin_memory=torch.cuda.is_available(),
                                       drop_last=drop_last)


class GradAllReduce:
    """Bucketed gradient averaging that can be captured into the HIP graph of a whole train step.

    ``DistributedDataParallel`` cannot sit inside ``GraphedTrainStep``'s capture, and an eager
    step costs ~3x a graph replay at 512x512 (51 vs 16 ms), so multi-GPU training would lose most
    of its per-GPU speed to host launches.  This reducer does DDP's job for a fixed parameter set:
    buckets are filled in reverse registration order (= backward order); inside a bucket the
    parameters sit in registration order, so the weight and bias of a Linear / LayerNorm and a
    block's LePE weights are adjacent, and csu's backward writes those gradients STRAIGHT into the
    bucket (ops._GRAD_DEST: AccumulateGrad steals the bucket view -- nothing to pack).  Buckets are
    cut only between modules (``named_parameters()`` input) so such groups never straddle two.
    Post-accumulate-grad hooks count each bucket's gradients; a complete bucket is all-reduced on a
    side stream while backward continues (any gradient that did not land in place -- e.g. a conv
    weight -- is copied in by one multi-tensor copy first).  Gradients csu defers to grouped launches
    (LayerNorm, token-Linear and LePE parameter gradients) are written by ``ops.flush_deferred()``
    when the bucket completes, before its launch, so every bucket but the last starts during backward
    (``last_early`` counts them).  ``finish()`` (after ``backward()``, before ``optimizer.step()``)
    launches any bucket still pending, joins the side stream and points every ``p.grad`` at its
    averaged slice, which the optimizer reads in place.  Every call is a stream operation, so the sequence is recorded into a graph on capture and
    replayed with one launch per step (RCCL collectives are capturable once the communicator exists:
    run one eager step first).

    Averaging: ``ReduceOp.AVG`` on nccl (= RCCL), SUM then a scale on gloo.  ``grad_dtype=
    torch.bfloat16`` all-reduces a bf16 copy of each bucket (half the ring bytes; the averaged values
    are cast back into the fp32 bucket).  Bucket size 32 MB: 94 MB of CSWin-UNet gradients -> 3
    all-reduces, the first two overlapped with backward, each large enough to run the xGMI rings at
    bandwidth."""

    def __init__(self, params, bucket_mb: float = 32.0, group=None, grad_dtype=torch.float32):
        items = list(params)
        named = bool(items) and isinstance(items[0], tuple)
        pairs = [(n, p) for n, p in items] if named else [(None, p) for p in items]
        pairs = [(n, p) for n, p in pairs if p.requires_grad]
        self.params = [p for _, p in pairs]
        self.last_copied = 0
        self.last_early = 0
        if not self.params:
            raise ValueError("GradAllReduce: no trainable parameters")
        if grad_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("GradAllReduce: grad_dtype float32 or bfloat16")
        self.group = group
        self.world = dist.get_world_size(group)
        self.avg = dist.get_backend(group) == "nccl"
        self.grad_dtype = grad_dtype
        dev = self.params[0].device
        cap = int(bucket_mb * (1 << 20)) // 4
        owner = lambda n: None if n is None else n.rsplit(".", 1)[0]   # noqa: E731
        self.buckets, cur, size = [], [], 0
        rev = list(reversed(pairs))
        for i, (n, p) in enumerate(rev):
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("GradAllReduce: contiguous fp32 parameters only")
            cur.append(p)
            size += p.numel()
            nxt = rev[i + 1][0] if i + 1 < len(rev) else None
            if size >= cap and (n is None or owner(nxt) != owner(n)):
                self.buckets.append(cur[::-1])       # registration order inside the bucket
                cur, size = [], 0
        if cur:
            self.buckets.append(cur[::-1])
        self.flat = [torch.zeros(sum(p.numel() for p in b), dtype=torch.float32, device=dev) for b in self.buckets]
        self.flat_lp = [f.to(grad_dtype) for f in self.flat] if grad_dtype != torch.float32 else None
        from . import ops
        self._ops = ops
        self.views = []
        for b, f in zip(self.buckets, self.flat):
            off, vs = 0, []
            for p in b:
                vs.append(f[off:off + p.numel()].view_as(p))
                ops._GRAD_DEST[id(p)] = (weakref.ref(p), f, off)
                off += p.numel()
            self.views.append(vs)
        self.where = {id(p): bi for bi, b in enumerate(self.buckets) for p in b}
        self.side = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        ops._DIST_SAFE[0] = True   # side-stream weight gradients: ordered by _launch below
        self._reset()
        self.handles = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]

    def _reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.held = []     # gradients read on the side stream: alive until finish() joined it
        self._copied = 0   # gradients of this step that did not land in their bucket view
        self._early = 0    # buckets launched from a hook (during backward) this step

    def _hook(self, p):
        bi = self.where[id(p)]
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            # the bucket's last gradient has been accumulated, but csu may still hold some of its
            # values deferred (LayerNorm dgamma / dbeta, token-Linear dW / db, LePE dW / db are
            # written by grouped launches): write everything deferred so far, then start the bucket's
            # all-reduce on the side stream while backward continues
            if self._ops.deferred_pending():
                self._ops.flush_deferred()
            self._launch(bi)
            self._early += 1

    def _launch(self, bi):
        grads = []
        for p in self.buckets[bi]:
            if p.grad is None:      # parameter without a gradient this step: contributes zeros
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        flat = self.flat[bi]
        # late gradients of this bucket (written by a deferred launch or on the csu side stream after
        # autograd received them): if AccumulateGrad copied one instead of stealing it, its .grad holds
        # the values from before the write -- repaired below, ordered after the writers, before the
        # bucket reads it (ops.take_late; the end-of-backward check would come after the all-reduce)
        late = [(p, src) for p, src in self._ops.take_late(self.buckets[bi])
                if p.grad is not None and p.grad.data_ptr() != src.data_ptr()]
        # gradients not already in place (not written into the bucket by csu's backward)
        todo = [(v, g) for v, g in zip(self.views[bi], grads) if g.data_ptr() != v.data_ptr()]
        self.held.append(grads)
        self._copied += len(todo)
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream(flat.device))
            ws = self._ops.side_stream(flat.device)
            if ws is not None:      # weight gradients still being written on the csu side stream
                self.side.wait_stream(ws)
            for g in grads:
                g.record_stream(self.side)
            ctx = torch.cuda.stream(self.side)
        else:
            ctx = contextlib.nullcontext()
        with ctx:
            for p, src in late:
                p.grad.copy_(src)
                self._ops.STATS["late_grad_fixups"] += 1
            if todo:
                torch._foreach_copy_([v for v, _ in todo], [g for _, g in todo])
            buf = flat
            if self.flat_lp is not None:
                buf = self.flat_lp[bi]
                buf.copy_(flat)
            if self.world == 1:
                # one rank: SUM == AVG, and RCCL runs no kernel for an in-place one-rank SUM (AVG's
                # pre-multiply is a 94 MB read + write per step, ~190 us at 512x512, r06v)
                dist.all_reduce(buf, group=self.group)
            elif self.avg:
                dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=self.group)
            else:
                dist.all_reduce(buf, group=self.group)
                buf.mul_(1.0 / self.world)
            if buf is not flat:
                flat.copy_(buf)
        self.launched[bi] = True

    def finish(self):
        for bi in range(len(self.buckets)):
            if not self.launched[bi]:
                self._launch(bi)
        if self.side is not None:
            torch.cuda.current_stream(self.flat[0].device).wait_stream(self.side)
        for b, vs in zip(self.buckets, self.views):
            for p, v in zip(b, vs):
                p.grad = v
        self.last_copied = self._copied   # how many gradients of the step needed the copy-in
        self.last_early = self._early     # how many buckets started during backward (overlapped)
        self._reset()

    def remove(self):
        for h in self.handles:
            h.remove()
        self.handles = []
        for b in self.buckets:
            for p in b:
                self._ops._GRAD_DEST.pop(id(p), None)


def drain_collectives(group=None):
    """Guarantee that no collective of the process group is in flight when a HIP-graph capture
    starts (GraphedTrainStep with a reducer).  The RCCL watchdog thread polls the events of the
    collectives it still tracks; one of those queries landing inside the capture window aborted the
    process now and then.  Sequence: an async barrier whose Work is waited on and
    checked complete through the public Work API, a device-wide synchronize (every stream, the
    process group's included), then the watchdog's own list is drained.  torch exposes that last
    step only as ProcessGroup._wait_for_pending_works: when a torch build lacks it the capture is
    refused (RuntimeError) instead of risking the race."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    work = dist.barrier(group=group, async_op=True)
    work.wait()
    torch.cuda.synchronize()
    if not work.is_completed():
        raise RuntimeError("drain_collectives: the barrier did not complete")
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    wait = getattr(pg, "_wait_for_pending_works", None)
    if wait is None:
        raise RuntimeError("drain_collectives: this torch build cannot drain the process group's watchdog list "
                           "(no ProcessGroup._wait_for_pending_works); refusing to capture RCCL collectives")
    wait()
    torch.cuda.synchronize()
