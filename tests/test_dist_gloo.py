"""Multi-process data-parallel logic on CPU (gloo, world size 2 and 4): DDP gradient averaging of the
sharded batch == the single-process global batch, and the all-reduced per-step metric sums give
the reference's batch-flattened Dice/IoU of the global batch."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _setup(seed=0):
    from oracle import cswin_ref as O
    from csu.data import ellipse_batch
    cfg = O.CSWinConfig(img_size=64, split_size=(1, 2, 2, 2))
    torch.manual_seed(seed)
    model = O.OracleCSWin(cfg, O.recipe_params(cfg, seed=0))
    xs, ts = ellipse_batch(np.random.default_rng(3), 4, 64)
    return model, xs, ts


def _train(model, batches, steps=2, reducer=None):
    from csu.train import bce_loss, train_step
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    stats = []
    for i in range(steps):
        x, t = batches[i % len(batches)]
        stats.append(train_step(model, x, t, bce_loss, opt, reducer=reducer))
    return stats


def _worker(rank, world, port, out_path, mode="ddp"):
    sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from csu.dist import init_distributed, wrap_ddp
    from csu.train import _epoch_means
    r, w, device = init_distributed("gloo")
    model, xs, ts = _setup()
    per = 4 // w   # the global batch of 4, equal shards
    shard = slice(per * r, per * (r + 1))
    if mode == "ddp":
        stats = _train(wrap_ddp(model, device), [(xs[shard], ts[shard])])
    else:   # the graph-capturable bucketed reducer bench.py uses at N > 1, here eager on gloo
        from csu.dist import GradAllReduce
        if mode == "reducer_named":   # buckets cut only between modules
            named = list(model.params().items())   # the reference's state_dict names (cswin:489-688)
            red = GradAllReduce(named, bucket_mb=0.05)
            owner = {id(p): n.rsplit(".", 1)[0] for n, p in named}
            where = {}
            for bi, b in enumerate(red.buckets):
                for p in b:
                    assert where.setdefault(owner[id(p)], bi) == bi, owner[id(p)]
        else:
            red = GradAllReduce(model.parameters(), bucket_mb=0.05,   # tiny buckets: several per step
                                grad_dtype=torch.bfloat16 if mode == "reducer_bf16" else torch.float32)
        assert len(red.buckets) > 2
        if mode == "graphed":
            # GraphedTrainStep(reducer=...)'s own sequence (static input buffers, backward with the
            # bucket hooks, finish(), optimizer) at world > 1 -- the capture itself needs a GPU
            from csu.train import GraphedTrainStep, _step_stats, bce_loss
            opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
            x, t = xs[shard], ts[shard]
            gs = GraphedTrainStep(model, opt, bce_loss, x, t, None, warmup=0, reducer=red, capture=False)
            stats = []
            for _ in range(2):
                loss, out = gs(x, t)
                stats.append(_step_stats(loss, out, t))
                assert red.last_early >= len(red.buckets) - 1, (red.last_early, len(red.buckets))
                assert all(p.grad.data_ptr() == v.data_ptr() for b, vs in zip(red.buckets, red.views)
                           for p, v in zip(b, vs))   # every .grad is its averaged bucket slice
        else:
            stats = _train(model, [(xs[shard], ts[shard])], reducer=red)
        assert red.last_early >= len(red.buckets) - 1, (red.last_early, len(red.buckets))
    means = _epoch_means(stats)
    if r == 0:
        torch.save({"params": [p.detach().clone() for p in model.parameters()], "means": means}, out_path)
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("mode,world", [("ddp", 2), ("reducer", 2), ("reducer_named", 2), ("reducer_bf16", 2),
                                        ("reducer", 4), ("graphed", 2)])
def test_ddp_two_ranks_equals_global_batch(tmp_path, mode, world):
    """world 4: one image per rank -- the bucketed reducer's average over more ranks than the 2-GPU case."""
    out = str(tmp_path / "ddp.pt")
    mp.spawn(_worker, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    from csu.train import _epoch_means
    torch.set_num_threads(4)
    model, xs, ts = _setup()
    stats = _train(model, [(xs, ts)])
    ref_means = _epoch_means(stats)
    init, _, _ = _setup()
    for a, b, p0 in zip(got["params"], model.parameters(), init.parameters()):
        if mode == "reducer_bf16":
            # bf16-rounded averaged gradients: Adam turns a rounding of a near-zero gradient into an
            # O(1) change of that element's tiny step, so compare the whole update per tensor
            ua, ub = (a - p0.detach()).double(), (b.detach() - p0.detach()).double()
            assert float((ua - ub).norm()) <= 2e-2 * float(ub.norm()) + 1e-9
        else:
            torch.testing.assert_close(a, b.detach(), rtol=1e-3, atol=1e-5)   # Adam step of fp32 grads summed in another order
    # loss: mean of per-rank means == global mean (equal shards); Dice/IoU from global sums
    np.testing.assert_allclose(got["means"], ref_means, rtol=1e-6, atol=1e-7)


def test_epoch_means_match_reference_formula():
    """Single process: per-step batch-flattened Dice/IoU averaged over steps (cswin:692-708, 809-811)."""
    from csu.train import _epoch_means, _step_stats
    from oracle import cswin_ref as O
    g = torch.Generator().manual_seed(0)
    stats, ref = [], []
    for _ in range(3):
        p = torch.rand(2, 1, 16, 16, generator=g)
        t = (torch.rand(2, 1, 16, 16, generator=g) > 0.5).float()
        loss = O.bce_loss(p, t)
        stats.append(_step_stats(loss, p, t))
        d, i = O.dice_iou(p, t)
        ref.append((loss.item(), d, i))
    got = _epoch_means(stats)
    np.testing.assert_allclose(got, np.mean(np.array(ref), axis=0), rtol=1e-6)


def test_grad_dest_registry_contiguity():
    """ops._grad_dest hands out a bucket slice only for parameters adjacent in registration order
    with no existing .grad (csu.dist.GradAllReduce registers them; the ops then write in place)."""
    import weakref
    sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
    from csu import ops
    a, b, c = (torch.nn.Parameter(torch.zeros(*s)) for s in ((3, 4), (3,), (5,)))
    flat = torch.zeros(20)
    ops._GRAD_DEST.update({id(a): (weakref.ref(a), flat, 0), id(b): (weakref.ref(b), flat, 12),
                           id(c): (weakref.ref(c), flat, 15)})
    try:
        d = ops._grad_dest((a, b))
        assert d is not None and d.data_ptr() == flat.data_ptr() and d.numel() == 15
        assert ops._grad_dest((b, c)).data_ptr() == flat[12:].data_ptr()
        assert ops._grad_dest((b, a)) is None            # not in bucket order
        assert ops._grad_dest((a, c)) is None            # not adjacent
        a.grad = torch.zeros(3, 4)
        assert ops._grad_dest((a, b)) is None            # gradient accumulation: no stealing
        a.grad = None
        ops._note_use(None, b)
        ops._note_use(None, b)
        assert ops._uses(b) == 2
        assert ops._grad_dest((a, b)) is None            # shared parameter: the engine sums its uses
        assert ops._grad_dest((c,)) is not None
    finally:
        ops._USES.clear()
        for p in (a, b, c):
            ops._GRAD_DEST.pop(id(p), None)


def test_stale_ids_do_not_leak_into_new_parameters():
    """_USES / _GRAD_DEST are keyed by id(p): an entry left behind by a dead parameter (a forward
    without backward, a reducer never removed) must not apply to a new object that reuses the id --
    otherwise a parameter's deferral / bucket destination would depend on the allocation history
    (the cause of the intermittent concat-Linear bias differences)."""
    import weakref
    sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
    from csu import ops
    old = torch.nn.Parameter(torch.zeros(4))
    ops._note_use(None, old)
    ops._note_use(None, old)
    flat = torch.zeros(4)
    ops._GRAD_DEST[id(old)] = (weakref.ref(old), flat, 0)
    ops._USES[id(old)][0] = weakref.ref(torch.nn.Parameter(torch.zeros(1)))   # now points elsewhere
    ops._GRAD_DEST[id(old)] = (weakref.ref(torch.nn.Parameter(torch.zeros(1))), flat, 0)
    try:
        assert ops._uses(old) == 0                      # the entry is someone else's
        assert ops._grad_dest((old,)) is None
        # calls that cannot be differentiated (no_grad / eval forwards) count nothing: the op's ctx says so
        new = torch.nn.Parameter(torch.zeros(4))
        seen = []

        class Op(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x, w):
                ops._note_use(ctx, w)
                seen.append(ops._uses(w))
                return x * 1.0

            @staticmethod
            def backward(ctx, g):
                return g, None
        with torch.no_grad():
            Op.apply(torch.ones(2), new)
        assert seen[-1] == 0
        Op.apply(torch.ones(2), new)
        assert seen[-1] == 1
        Op.apply(torch.ones(2), new)
        assert seen[-1] == 2
    finally:
        ops._USES.clear()
        ops._GRAD_DEST.pop(id(old), None)


def test_late_gradient_copied_by_autograd_is_repaired():
    """A gradient handed to autograd before its values exist (deferred / side stream) must be stolen
    by AccumulateGrad; if autograd copies it instead (an extra reference), the end-of-backward check
    copies the final values into .grad (ops._check_late) and counts it."""
    sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
    from csu import ops
    p = torch.nn.Parameter(torch.zeros(6))
    buf = torch.zeros(8)
    keep = []

    class Late(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            gw = buf[2:]
            keep.append(gw)            # a second reference: AccumulateGrad must copy it now
            ops._late((p,), (gw,))
            return g, gw

    n0 = ops.STATS["late_grad_fixups"]
    Late.apply(torch.ones(3, requires_grad=True), p).sum().backward()
    assert p.grad is not None and p.grad.data_ptr() != buf[2:].data_ptr()
    buf[2:] = torch.arange(6.0)      # the "deferred kernel" writes the values after the copy
    ops._check_late(ops._LATE_DEFER)
    assert ops.STATS["late_grad_fixups"] == n0 + 1
    assert torch.equal(p.grad, torch.arange(6.0))
    # a stolen gradient is left alone
    p.grad = None
    keep.clear()

    class Steal(Late):
        @staticmethod
        def backward(ctx, g):
            gw = buf[2:]
            ops._late((p,), (gw,))
            return g, gw
    Steal.apply(torch.ones(3, requires_grad=True), p).sum().backward()
    assert p.grad.data_ptr() == buf[2:].data_ptr()
    ops._check_late(ops._LATE_DEFER)
    assert ops.STATS["late_grad_fixups"] == n0 + 1


def _late_reducer_worker(rank, world, port, out_path):
    sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.distributed.init_process_group("gloo")
    from csu import ops
    from csu.dist import GradAllReduce
    p = torch.nn.Parameter(torch.zeros(6))
    red = GradAllReduce([p], bucket_mb=1.0)
    buf = torch.zeros(8)
    keep = []

    class Late(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            gw = buf[2:]
            keep.append(gw)            # a second reference: AccumulateGrad copies it (stale zeros)
            ops._late((p,), (gw,))
            # the "deferred kernel": runs in the flush the bucket hook triggers, AFTER the copy
            ops._WG_POST.append(lambda: buf[2:].copy_(torch.arange(6.0) * (rank + 1)))
            return g, gw

    n0 = ops.STATS["late_grad_fixups"]
    Late.apply(torch.ones(3, requires_grad=True), p).sum().backward()
    red.finish()
    torch.save({"grad": p.grad.clone(), "fixups": ops.STATS["late_grad_fixups"] - n0,
                "left": len(ops._LATE_DEFER)}, f"{out_path}.{rank}")
    torch.distributed.destroy_process_group()


def test_late_gradient_repaired_before_bucket_allreduce(tmp_path):
    """with csu.dist.GradAllReduce attached, a late gradient that AccumulateGrad copied must
    be repaired before the bucket all-reduce reads it (not after, by the end-of-backward check): the
    averaged gradient is the mean of the values the deferred launches wrote."""
    out = str(tmp_path / "late")
    mp.spawn(_late_reducer_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        got = torch.load(f"{out}.{r}", weights_only=True)
        assert got["fixups"] == 1 and got["left"] == 0
        torch.testing.assert_close(got["grad"], torch.arange(6.0) * 1.5)


def test_use_counts_reset_without_deferred_work():
    """a backward with no deferrable LayerNorm / Linear / LePE work (the plain UNet's convs)
    must still reset the forward use counts at its end, or the second step sees every weight as
    shared (_uses > 1) and loses the side-stream / in-bucket gradient paths."""
    sys.path[:0] = [REPO, os.path.join(REPO, "cswin-simam-unet_amd")]
    from csu import ops
    w = torch.nn.Parameter(torch.ones(4))
    safe = []

    class ConvLike(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, weight):
            ops._note_use(ctx, weight)
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            safe.append(ops._param_safe(w))   # what a conv backward asks (ops._side_ok)
            return g, None

    try:
        for _ in range(3):
            w.grad = None
            ConvLike.apply(torch.ones(4, requires_grad=True), w).sum().backward()
            assert ops._uses(w) == 0
        assert safe == [True, True, True]
    finally:
        ops._USES.clear()
