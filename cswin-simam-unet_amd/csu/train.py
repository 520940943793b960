"""Training-step API of the reference (train_cswinunet_segmentation.py cswin:692-841).

Same names, arguments and return values as the reference's ``dice_coefficient``, ``iou_score``,
``evaluate_model`` and ``train_model``.  Differences are performance-only: per-batch metrics are
accumulated on the device and synchronised once per epoch instead of four ``.item()`` host syncs
per step (cswin:698, 708, 797, 803), and under ``torch.distributed`` the metric sums are
all-reduced so every rank (and the LR scheduler) sees the global values.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import contextlib
import gc
import warnings

import torch
import torch.distributed as dist
import torch.nn.functional as F

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


def sync_shadows(model):
    from .ops import sync_shadows as sync
    sync(model)


def bce_loss(prob: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """nn.BCELoss() (mean; log clamped at -100) computed in fp32 (cswin:936)."""
    with torch.autocast(prob.device.type, enabled=False):   # BCE is autocast-unsafe; always fp32
        if prob.is_cuda:
            from . import ops
            return ops.bce_loss(prob.float(), target.float())
        return F.binary_cross_entropy(prob.float(), target.float())


def bce_loss_stats(prob: torch.Tensor, target: torch.Tensor):
    """bce_loss and the per-step segmentation sums (sum(pred*t), sum(pred), sum(t), pred = prob >
    0.5; cswin:789-795) of the same pass (device: one fused csu kernel)."""
    with torch.autocast(prob.device.type, enabled=False):
        if prob.is_cuda:
            from . import ops
            return ops.bce_loss_stats(prob.float(), target.float())
        p, t = prob.float(), target.float()
        pred = (p > 0.5).float()
        return F.binary_cross_entropy(p, t), torch.stack([(pred * t).sum(), pred.sum(), t.sum()]).detach()


def _dice_t(pred, target, smooth=1e-6):
    pred, target = pred.reshape(-1), target.reshape(-1)
    inter = (pred * target).sum()
    return (2.0 * inter + smooth) / (pred.sum() + target.sum() + smooth)


def _iou_t(pred, target, smooth=1e-6):
    pred, target = pred.reshape(-1), target.reshape(-1)
    inter = (pred * target).sum()
    return (inter + smooth) / (pred.sum() + target.sum() - inter + smooth)


def dice_coefficient(pred, target, smooth=1e-6) -> float:
    """Batch-flattened Dice (cswin:692-698)."""
    return _dice_t(pred, target, smooth).item()


def iou_score(pred, target, smooth=1e-6) -> float:
    """Batch-flattened IoU (cswin:701-708)."""
    return _iou_t(pred, target, smooth).item()


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _step_stats(loss, outputs, masks):
    """Per-step sums (loss, sum(p*t), sum(p), sum(t)) of thresholded predictions, on device."""
    preds = (outputs > 0.5).to(torch.float64).reshape(-1)
    t = masks.to(torch.float64).reshape(-1)
    return torch.stack([loss.detach().double(), (preds * t).sum(), preds.sum(), t.sum()])


def _epoch_means(stats: List[torch.Tensor], smooth: float = 1e-6):
    """Mean over steps of (loss, Dice, IoU) of the GLOBAL batch: the per-step sums of every rank
    are all-reduced once per epoch, so each step's Dice/IoU is the reference's batch-flattened
    value over the concatenation of all ranks' batches (cswin:692-708, 797-811)."""
    if not stats:
        return 0.0, 0.0, 0.0
    s = torch.stack(stats)
    w = _world()
    if w > 1:
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        s[:, 0] /= w
    inter, ps, ts = s[:, 1], s[:, 2], s[:, 3]
    dice = (2.0 * inter + smooth) / (ps + ts + smooth)
    iou = (inter + smooth) / (ps + ts - inter + smooth)
    return float(s[:, 0].mean()), float(dice.mean()), float(iou.mean())


def _autocast(device, amp_dtype):
    dt = torch.device(device).type if not isinstance(device, torch.device) else device.type
    return torch.autocast(dt, dtype=amp_dtype or torch.float32, enabled=amp_dtype is not None)


class _GraphCache(dict):
    """Captured graphs of one model: {key: _GraphedTrain | _GraphedEval}, kept on the model itself
    (``model._csu_graphs``) so that model and graphs form one collectable cycle -- a module-level
    WeakKeyDictionary could never drop an entry, its values hold the model.  Copies and pickles of
    the model start with an empty cache."""

    def __deepcopy__(self, memo):
        return _GraphCache()

    def __reduce__(self):
        return (_GraphCache, ())


def _graph_cache(model):
    c = model.__dict__.get("_csu_graphs")
    if c is None:
        c = _GraphCache()
        object.__setattr__(model, "_csu_graphs", c)
    return c


def _drop_stale_train_graphs(cache, optimizer, reducer):
    """A new optimizer or reducer for the model: the train graphs captured for the old ones (and the
    memory pools they hold) are released."""
    for k in [k for k in cache if k[0] == "train" and (k[-2], k[-1]) != (id(optimizer), id(reducer))]:
        del cache[k]


@contextlib.contextmanager
def _gc_paused():
    """Python's cyclic GC off for a graph capture (after one collection): a collection inside the
    capture can run the finaliser of an unrelated object that calls the HIP runtime (a graph, stream
    or event of an earlier step) -- an illegal call during a capture that aborts the process (seen as
    'Fatal Python error: Aborted' while garbage-collecting inside a backward kernel launch)."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _capture_mode():
    """HIP-graph capture mode: under a process group the RCCL watchdog polls its collectives' events
    from another thread, so the capture is thread-local and starts with nothing in flight (see
    GraphedTrainStep)."""
    if dist.is_available() and dist.is_initialized():
        from .dist import drain_collectives
        drain_collectives()
        return "thread_local"
    return "global"


def _graphable(model, optimizer, device, criterion) -> bool:
    """The whole step can be captured: csu model on a GPU (not wrapped in DDP, which cannot be
    captured -- data parallel training passes a csu.dist.GradAllReduce instead) and csu's FusedAdamW."""
    from .optim import FusedAdamW
    dev = torch.device(device)
    return (dev.type == "cuda" and isinstance(optimizer, FusedAdamW)
            and not isinstance(model, torch.nn.parallel.DistributedDataParallel)
            and all(p.is_cuda for p in model.parameters()))


class _GraphedEval:
    """evaluate_model's per-batch body (eval-mode forward, loss, thresholded sums) captured once
    for a static batch shape and replayed."""

    def __init__(self, model, criterion, x, t, amp_dtype):
        self.model, self.crit, self.dtype = model, criterion, amp_dtype
        self.x, self.t = x.clone(), t.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), torch.no_grad():
            self._body()                 # warm-up: lazily built caches / kernels outside the capture
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        mode = _capture_mode()
        self.graph = torch.cuda.CUDAGraph()
        with _gc_paused(), torch.no_grad(), torch.cuda.graph(self.graph, capture_error_mode=mode):
            self.stats = self._body()

    def _body(self):
        with torch.autocast("cuda", dtype=self.dtype or torch.float32, enabled=self.dtype is not None):
            out = self.model(self.x)
        if self.crit is bce_loss:
            loss, st = bce_loss_stats(out, self.t)
            return torch.cat([loss.detach().double().view(1), st.double()])
        return _step_stats(self.crit(out, self.t), out, self.t)

    def __call__(self, x, t):
        self.x.copy_(x, non_blocking=True)
        self.t.copy_(t, non_blocking=True)
        sync_shadows(self.model)     # the captured forward reads the optimizer-written weight shadows
        self.graph.replay()
        return self.stats.clone()


def evaluate_model(model, data_loader, criterion, device, amp_dtype=None, graph=None):
    """eval mode, no grad; mean over batches of (loss, Dice, IoU) (cswin:712-747).  ``amp_dtype``
    (not in the reference): run the forward under autocast (e.g. torch.bfloat16).  ``graph``
    (None = automatic on a GPU): batches of the first batch's shape replay one captured HIP graph
    of the forward + loss + metric sums; other shapes (a ragged last batch) run eagerly."""
    model.eval()
    use_graph = (graph is not False and torch.device(device).type == "cuda" and torch.cuda.is_available()
                 and not isinstance(model, torch.nn.parallel.DistributedDataParallel)
                 and not torch.cuda.is_current_stream_capturing())
    cache = _graph_cache(model) if use_graph else None
    stats = []
    with torch.no_grad():
        for images, masks in data_loader:
            images = images.to(device, non_blocking=True)
            masks = masks.to(device, non_blocking=True)
            if use_graph:
                key = ("eval", tuple(images.shape), tuple(masks.shape), amp_dtype, criterion)
                g = cache.get(key)
                if g is None:
                    g = cache[key] = _GraphedEval(model, criterion, images, masks, amp_dtype)
                stats.append(g(images, masks))
                continue
            with _autocast(images.device, amp_dtype):
                outputs = model(images)
            stats.append(_step_stats(criterion(outputs, masks), outputs, masks))
    return _epoch_means(stats)


def train_step(model, images, masks, criterion, optimizer, reducer=None, amp_dtype=None):
    """One reference step (cswin:779-794): zero_grad, forward, loss, backward, optimizer step.
    ``reducer``: a ``csu.dist.GradAllReduce`` averaging the gradients across ranks (instead of DDP).
    ``amp_dtype``: forward under autocast (the loss stays fp32).
    Returns the device tensor of per-step sums (loss, sum(p*t), sum(p), sum(t)) -- no host sync."""
    optimizer.zero_grad(set_to_none=True)
    with _autocast(images.device, amp_dtype):
        outputs = model(images)
    loss = criterion(outputs, masks)
    loss.backward()
    if reducer is not None:
        reducer.finish()
    optimizer.step()
    with torch.no_grad():
        return _step_stats(loss, outputs, masks)


class _GraphedTrain:
    """train_model's step on a captured graph.  The first ``warmup`` batches of a shape are real
    steps run eagerly on a side stream (the capture's warm-up: optimizer state, cast caches, RCCL
    communicators), then the step is captured and every later batch of that shape replays it --
    each batch is trained on exactly once, as in the reference loop."""

    def __init__(self, model, optimizer, criterion, amp_dtype, reducer, warmup=2):
        self.model, self.opt, self.crit, self.dtype, self.reducer = model, optimizer, criterion, amp_dtype, reducer
        self.warmup, self.done, self.gs = warmup, 0, None

    def __call__(self, images, masks):
        if self.gs is None and self.done < self.warmup:
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                st = train_step(self.model, images, masks, self.crit, self.opt, self.reducer, self.dtype)
            cur.wait_stream(side)
            self.done += 1
            return st
        if self.gs is None:
            for g in self.opt.param_groups:     # lr / step read from the device inside the graph
                g["capturable"] = True
            self.opt.sync_lr()
            self.gs = GraphedTrainStep(self.model, self.opt, self.crit, images, masks, self.dtype, warmup=0,
                                       reducer=self.reducer, metrics=self.crit is bce_loss)
        loss, out = self.gs(images, masks)
        if self.gs.stats is not None:
            return torch.cat([loss.double().view(1), self.gs.stats.double()])
        with torch.no_grad():
            return _step_stats(loss, out, self.gs.t)


def train_model(model, train_loader, test_loader, criterion, optimizer, scheduler, device, num_epochs=100,
                verbose: bool = True, checkpoint_path: Optional[str] = None,
                resume_from: Optional[str] = None, amp_dtype=None, graph=None, reducer=None) -> Dict[str, List[float]]:
    """Epoch loop with per-epoch history and ReduceLROnPlateau on the test loss (cswin:751-841).

    Beyond the reference: ``checkpoint_path`` writes a resumable checkpoint (model, optimizer,
    scheduler, epoch, history; csu.report.save_checkpoint) after every epoch, and ``resume_from``
    restores one and continues from the epoch after it (the history then covers all epochs);
    ``amp_dtype`` runs the forward passes under autocast (the reference trains in fp32).
    ``graph`` (None = automatic): on a GPU with csu's FusedAdamW (csu.train.make_optimizer) each
    batch shape's step is captured into one HIP graph after two eager steps and replayed (the
    speed bench.py reports); a batch of another shape (ragged last batch) runs eagerly.  Graphs are
    kept per model across calls.  ``reducer``: a csu.dist.GradAllReduce for data-parallel training
    (captured with the step)."""
    history = {"train_loss": [], "train_dice": [], "train_iou": [], "test_loss": [], "test_dice": [], "test_iou": [],
               "learning_rates": []}
    rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
    start = 0
    if resume_from is not None:
        from .report import load_checkpoint
        start, past = load_checkpoint(resume_from, model, optimizer, scheduler, map_location=device)
        for k in history:
            history[k] = list(past.get(k, []))
    use_graph = graph is not False and _graphable(model, optimizer, device, criterion)
    if graph and not use_graph:
        raise ValueError("train_model(graph=True) needs a csu model on a GPU and csu.optim.FusedAdamW")
    cache = _graph_cache(model) if use_graph else None
    if cache is not None:
        _drop_stale_train_graphs(cache, optimizer, reducer)
    for epoch in range(start, num_epochs):
        model.train()
        sampler = getattr(train_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        it = train_loader
        if verbose and rank0 and tqdm is not None:
            it = tqdm(train_loader, desc=f"Epoch {epoch + 1}/{num_epochs} [TRAIN]")
        stats = []
        for images, masks in it:
            images = images.to(device, non_blocking=True)
            masks = masks.to(device, non_blocking=True)
            if use_graph:
                key = ("train", tuple(images.shape), tuple(masks.shape), amp_dtype, criterion, id(optimizer),
                       id(reducer))
                g = cache.get(key)
                if g is None:
                    g = cache[key] = _GraphedTrain(model, optimizer, criterion, amp_dtype, reducer)
                stats.append(g(images, masks))
            else:
                stats.append(train_step(model, images, masks, criterion, optimizer, reducer, amp_dtype=amp_dtype))
        train_loss, train_dice, train_iou = _epoch_means(stats)
        test_loss, test_dice, test_iou = evaluate_model(model, test_loader, criterion, device, amp_dtype=amp_dtype,
                                                        graph=use_graph)
        if scheduler is not None:
            scheduler.step(test_loss)
            if hasattr(optimizer, "sync_lr"):   # FusedAdamW: the device lr a captured step reads
                optimizer.sync_lr()
        current_lr = optimizer.param_groups[0]["lr"]
        for k, v in zip(history, (train_loss, train_dice, train_iou, test_loss, test_dice, test_iou, current_lr)):
            history[k].append(v)
        if checkpoint_path is not None:
            from .report import save_checkpoint
            save_checkpoint(checkpoint_path, model, optimizer, scheduler, epoch + 1, history)
        if verbose and rank0:
            print(f'\n{"=" * 70}\nEpoch {epoch + 1}/{num_epochs}:')
            print(f"  [TRAIN] Loss: {train_loss:.4f} | Dice: {train_dice:.4f} | IoU: {train_iou:.4f}")
            print(f"  [TEST]  Loss: {test_loss:.4f} | Dice: {test_dice:.4f} | IoU: {test_iou:.4f}")
            print(f'  [LR]    Learning Rate: {current_lr:.6f}\n{"=" * 70}\n')
    return history


def make_optimizer(model, lr=1e-4, weight_decay=1e-4, capturable=False):
    """AdamW as in cswin:937-941.  On the GPU: csu.optim.FusedAdamW (one csu_adamw_step launch for
    all 463 tensors; ``capturable=True`` reads lr/step from device tensors so the step can live in a
    HIP graph); on the CPU: torch.optim.AdamW."""
    if next(model.parameters()).is_cuda:
        from .optim import FusedAdamW
        return FusedAdamW(model.parameters(), lr=lr, weight_decay=weight_decay, capturable=capturable)
    return torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=weight_decay)


class GraphedTrainStep:
    """One whole training step (zero-grad, forward, BCE, backward, AdamW) captured once into a
    HIP graph and replayed: removes every host launch (~2k kernels per 512x512 step).

    Inputs are copied into static device buffers before each replay; the optimizer must be
    built with ``capturable=True``.  Data parallel: pass a ``csu.dist.GradAllReduce`` over the
    (unwrapped) model's parameters as ``reducer``; its bucketed RCCL all-reduces, overlapped with
    backward on a side stream, are captured into the same graph (``DistributedDataParallel`` is
    not capturable)."""

    def __init__(self, model, optimizer, criterion, example_x, example_t, autocast_dtype=None, warmup=3,
                 reducer=None, metrics=False, capture=True):
        self.model, self.opt, self.crit = model, optimizer, criterion
        # metrics (criterion bce_loss): the reference loop's per-step thresholded Dice / IoU sums
        # (cswin:789-795) computed inside the graph by the loss kernel -> self.stats after a replay
        self.metrics = metrics
        self.stats = None
        self.reducer = reducer
        self.x = example_x.clone()
        self.t = example_t.clone()
        self.dtype = autocast_dtype
        # capture=False: the same sequence (warm-up steps, static input buffers, the reducer's
        # bucket hooks + finish, the optimizer) run eagerly at every call -- no streams, no graph, so
        # it runs on a CPU process group too (the world > 1 reducer order is tested that way on gloo)
        self.capture = bool(capture)
        self.graph = None
        if not self.capture:
            for _ in range(warmup):
                self._body()
            return
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with warnings.catch_warnings(record=True) as caught:
            warnings.simplefilter("always")
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    self._body()
        torch.cuda.current_stream().wait_stream(side)
        for w in caught:
            if "AccumulateGrad node's stream does not match" in str(w.message):
                # An autograd graph of an earlier step (e.g. a kept loss / output of an eager step)
                # is alive: its AccumulateGrad nodes would run on the stream they were created on
                # inside the capture, which breaks it (hipGraphInstantiate segfaults).
                raise RuntimeError(
                    "GraphedTrainStep: an autograd graph of an earlier step is still referenced (a kept "
                    "output or loss of an eager step); delete those references before capturing")
            warnings.warn_explicit(w.message, w.category, w.filename, w.lineno)
        # drain the warm-up (its RCCL work included) before capturing: nothing of it is pending
        # when the capture starts
        torch.cuda.synchronize()
        mode = "global"
        if reducer is not None:
            # The RCCL process group's watchdog thread polls the events of its collectives
            # (hipEventQuery) concurrently with this thread.  A global-mode capture makes that query
            # illegal in every thread (hipErrorStreamCaptureUnsupported -> the watchdog aborts the
            # process); a thread-local capture restricts only this thread, so the polling stays
            # legal whatever the watchdog's timing.  The barrier lines the ranks up so no rank's
            # capture overlaps another rank's warm-up collectives.  Then the watchdog's own list is
            # drained (ProcessGroup._wait_for_pending_works returns once every issued collective,
            # the barrier's included, has been retired by the watchdog): with nothing left to poll
            # it issues no event query while the capture runs (observed: a query landing inside the
            # capture window still aborted the process now and then, thread-local mode or not).
            from .dist import drain_collectives
            drain_collectives()
            mode = "thread_local"
        prep = getattr(self.opt, "prepare_capture", None)
        if prep is not None:
            prep()
        self.graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        with _gc_paused(), torch.cuda.graph(self.graph, capture_error_mode=mode):
            self.loss, self.out = self._body(zero=False)
            self.stats = self._stats
        fin = getattr(self.opt, "finish_capture", None)
        if fin is not None:
            fin()

    def _body(self, zero=True):
        if zero:
            self.opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=self.dtype or torch.float32, enabled=self.dtype is not None):
            out = self.model(self.x)
        if self.metrics:
            if self.crit is not bce_loss:
                raise ValueError("GraphedTrainStep(metrics=True) needs criterion=csu.train.bce_loss")
            loss, self._stats = bce_loss_stats(out, self.t)
        else:
            loss, self._stats = self.crit(out, self.t), None
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish()
        self.opt.step()
        return loss.detach(), out.detach()

    def __call__(self, x, t):
        self.x.copy_(x, non_blocking=True)
        self.t.copy_(t, non_blocking=True)
        if not self.capture:
            self.loss, self.out = self._body()
            self.stats = self._stats
            return self.loss, self.out
        sync_shadows(self.model)     # weights changed outside the graph since: re-cast before the replay
        self.graph.replay()
        return self.loss, self.out


def make_scheduler(optimizer, factor=0.5, patience=5, min_lr=1e-7):
    """ReduceLROnPlateau of cswin:944-951 without the ``verbose`` kwarg torch 2.10 rejects."""
    return torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=factor, patience=patience,
                                                      min_lr=min_lr)
