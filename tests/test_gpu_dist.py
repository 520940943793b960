"""Data-parallel training with the real csu model on the MI355X (the reference loop
cswin:775-811): two ranks share cuda:0 over a gloo process group (gloo all-reduces CUDA tensors;
RCCL wants one device per rank, and this box has one GPU), each runs the csu CSWinTransformer on
HIP kernels with ``GradAllReduce`` (eager: the side-stream weight gradients stay on, the reducer
orders its bucket reads after them) on its half of the batch.  The averaged gradients of every
parameter equal a single process's gradients of the whole batch (fp32 and bf16 autocast), on the
third of three backward passes (buckets and flat buffers reused).

The 8-rank RCCL run over xGMI is the driver's; the captured-reducer path is covered at world size 1
by ``test_gpu_model.py::test_dp_path_graph_captured_allreduce_matches_single_process``."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 3


def _setup(dtype):
    from oracle import cswin_ref as O
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    d = torch.device("cuda:0")
    cfg = O.CSWinConfig(img_size=64, split_size=(1, 2, 2, 2))
    m = CSWinTransformer(img_size=64, split_size=[1, 2, 2, 2]).to(d)
    m.load_state_dict(O.recipe_params(cfg, seed=0))
    xs, ts = ellipse_batch(np.random.default_rng(3), 8, 64)
    return m, xs.to(d), ts.to(d), (torch.bfloat16 if dtype == "bf16" else None)


def _grads(m, x, t, amp, reducer=None):
    """STEPS backward passes (fresh gradients each: zero_grad(set_to_none=True) as the reference loop,
    cswin:779) through the csu kernels; the gradients of the last one, averaged by ``reducer``."""
    from csu.train import _autocast, bce_loss
    for _ in range(STEPS):
        m.zero_grad(set_to_none=True)
        with _autocast(x.device, amp):
            y = m(x)
        bce_loss(y, t).backward()
        if reducer is not None:
            reducer.finish()
    torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in m.parameters()]


def worker(rank, world, port, out, dtype, mode="reducer"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo")
    from csu.dist import GradAllReduce, wrap_ddp
    m, xs, ts, amp = _setup(dtype)
    n = xs.shape[0] // world
    red, copied = None, None
    if mode == "ddp":
        # torch DDP's C++ reducer reads p.grad as soon as it is accumulated: csu must not defer any
        # parameter gradient to its end-of-backward flush (ops._deferrable refuses)
        m = wrap_ddp(m, torch.device("cuda:0"))
    elif mode == "named":
        # named parameters: buckets cut between modules, csu writes Linear / LayerNorm / LePE
        # gradients straight into the bucket views (no pack copy)
        red = GradAllReduce(m.named_parameters(), bucket_mb=0.5)
    else:
        red = GradAllReduce(m.parameters(), bucket_mb=0.5,   # several buckets, all-reduced while backward runs
                            grad_dtype=torch.bfloat16 if mode == "bf16_allreduce" else torch.float32)
    if red is not None:
        assert len(red.buckets) > 2
    params = _grads(m, xs[rank * n:(rank + 1) * n], ts[rank * n:(rank + 1) * n], amp, red)
    early = None
    if red is not None:
        copied = (red.last_copied, len(red.params))
        early = (red.last_early, len(red.buckets))
    if rank == 0:
        torch.save({"grads": [p.cpu() for p in params], "copied": copied, "early": early}, out)
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype,mode", [("fp32", "reducer"), ("bf16", "reducer"), ("bf16", "named"),
                                        ("fp32", "named"), ("bf16", "bf16_allreduce"), ("fp32", "ddp"),
                                        ("bf16", "ddp")])
def test_two_ranks_on_csu_kernels_equal_global_batch(tmp_path, dtype, mode):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "rank0.pt")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "cswin-simam-unet_amd")]))
    code = (f"import sys; sys.path[:0] = [{REPO!r}]; from tests.test_gpu_dist import worker; "
            f"worker(int(sys.argv[1]), 2, {port}, {out!r}, {dtype!r}, {mode!r})")
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    errs = []
    for p in procs:
        try:
            _, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            _, e = p.communicate()
        errs.append((p.returncode, e))
    for rc, e in errs:
        assert rc == 0, "\n".join(ln for ln in e.splitlines() if "frame #" not in ln)[-3000:]
    res = torch.load(out, weights_only=True)
    got = res["grads"]
    if mode == "named":   # in place: everything but the few conv / CARAFE / head parameters
        copied, total = res["copied"]
        assert copied < 0.25 * total, (copied, total)
    if res["early"] is not None:
        # overlap: every bucket but the last starts its all-reduce from a hook, during backward
        # (the deferred LayerNorm / Linear / LePE gradients are flushed per bucket)
        early, nbuckets = res["early"]
        assert early >= nbuckets - 1, (early, nbuckets)
    m, xs, ts, amp = _setup(dtype)
    ref = [g.cpu() for g in _grads(m, xs, ts, amp)]
    # per-sample work is identical on both sides (every csu kernel is per token / window / image, and
    # the rotated reduction orders depend on a token's position inside its image or on the N tile,
    # never on the batch); only the batch sums (weight gradients, the loss mean) add in another
    # order -> fp32 rounding
    tol = 1e-4 if dtype == "fp32" else 1e-3
    if mode == "bf16_allreduce":
        tol = 1e-2   # the averaged gradients themselves are rounded to bf16 (2^-9 relative)
    gmax = max(float(g.norm()) for g in ref)
    checked = 0
    for (name, _), a, b in zip(m.named_parameters(), got, ref):
        assert a.shape == b.shape, name
        if float(b.norm()) < 1e-6 * gmax:
            continue
        rel = float((a.double() - b.double()).norm() / b.double().norm())
        assert rel <= tol, (name, rel)
        checked += 1
    assert checked > 0.9 * len(ref), (checked, len(ref))


def shared_worker(port, out):
    """One rank (gloo, world size 1): weights shared by several op calls (LayerNorm, Linear, LePE, conv)
    with a GradAllReduce registered: each call's gradient must be summed, not written twice into the
    bucket slice (_grad_dest refuses parameters used more than once)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("gloo")
    from csu import ops
    from csu.dist import GradAllReduce
    d = torch.device("cuda:0")
    g = torch.Generator(device=d).manual_seed(5)
    C, reso = 64, 16
    geom = ops.StripeGeometry(reso, C, 1, [(reso, 2, 0), (2, reso, C // 2)], 32 ** -0.5)
    xs = [torch.randn(2, reso * reso, C, device=d, generator=g) for _ in range(2)]
    p0 = {"lnw": 1 + 0.1 * torch.randn(C, device=d, generator=g), "lnb": 0.1 * torch.randn(C, device=d, generator=g),
          "w": 0.05 * torch.randn(3 * C, C, device=d, generator=g), "b": 0.05 * torch.randn(3 * C, device=d, generator=g),
          "lw0": 0.1 * torch.randn(C // 2, 1, 3, 3, device=d, generator=g),
          "lb0": 0.1 * torch.randn(C // 2, device=d, generator=g),
          "lw1": 0.1 * torch.randn(C // 2, 1, 3, 3, device=d, generator=g),
          "lb1": 0.1 * torch.randn(C // 2, device=d, generator=g),
          "cw": 0.05 * torch.randn(C, C, 3, 3, device=d, generator=g), "cb": 0.05 * torch.randn(C, device=d, generator=g)}
    res = {}
    for use_red in (False, True):
        ps = {k: torch.nn.Parameter(v.clone()) for k, v in p0.items()}
        red = GradAllReduce(list(ps.items()), bucket_mb=0.001) if use_red else None
        for _ in range(2):
            for p in ps.values():
                p.grad = None
            loss = 0
            with torch.autocast("cuda", dtype=torch.bfloat16):
                for x in xs:    # every parameter is used by both calls
                    h = ops.layer_norm(x, ps["lnw"], ps["lnb"])
                    qkv = ops.linear(h, ps["w"], ps["b"])
                    o = ops.stripe_attention(qkv.bfloat16().contiguous(), geom, [ps["lw0"], ps["lw1"]],
                                             [ps["lb0"], ps["lb1"]])
                    # a conv weight / bias used by both calls too (conv params count uses)
                    c = ops.conv2d(o.view(2, reso, reso, C), ps["cw"], ps["cb"], 1, 1)
                    loss = loss + (o.float() ** 2).sum() + (c.float() ** 2).sum()
            loss.backward()
            if red is not None:
                red.finish()
        torch.cuda.synchronize()
        res[use_red] = {k: p.grad.detach().cpu().clone() for k, p in ps.items()}
        if red is not None:
            red.remove()
    torch.save(res, out)
    dist.destroy_process_group()


def test_reducer_with_shared_weights_sums_every_use(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "shared.pt")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "cswin-simam-unet_amd")]))
    code = (f"import sys; sys.path[:0] = [{REPO!r}]; from tests.test_gpu_dist import shared_worker; "
            f"shared_worker({port}, {out!r})")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = torch.load(out, weights_only=True)
    for k, ref in res[False].items():
        got = res[True][k]
        rel = float((got.double() - ref.double()).norm() / ref.double().norm())
        assert rel < 1e-5, (k, rel)


def train_model_worker(port, out, use_pg):
    """train_model with (use_pg) or without a process group: RCCL world size 1 + GradAllReduce
    captured in the train graph, a ragged last train batch (eager reducer step), and the eval graph
    captured right after the epoch's metric all-reduce (drained, thread-local capture)."""
    import torch.distributed as dist
    from oracle import cswin_ref as O
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss, make_optimizer, make_scheduler, train_model
    d = torch.device("cuda:0")
    red = None
    m = CSWinTransformer(img_size=64, split_size=[1, 2, 2, 2]).to(d)
    m.load_state_dict(O.recipe_params(O.CSWinConfig(img_size=64, split_size=(1, 2, 2, 2)), seed=0))
    if use_pg:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=d)
        from csu.dist import GradAllReduce
        red = GradAllReduce(m.named_parameters(), bucket_mb=0.5)
    rng = np.random.default_rng(7)
    train = [ellipse_batch(rng, 2, 64) for _ in range(4)] + [ellipse_batch(rng, 1, 64)]
    test = [ellipse_batch(rng, 2, 64), ellipse_batch(rng, 1, 64)]
    opt = make_optimizer(m, lr=1e-3)
    h = train_model(m, train, test, bce_loss, opt, make_scheduler(opt), d, num_epochs=2, verbose=False,
                    amp_dtype=torch.bfloat16, reducer=red)
    torch.save({"hist": h, "early": None if red is None else (red.last_early, len(red.buckets))}, out)
    if use_pg:
        dist.destroy_process_group()


def test_train_model_with_reducer_and_ragged_batches(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([REPO, os.path.join(REPO, "cswin-simam-unet_amd")]))
    res = {}
    for use_pg in (False, True):
        out = str(tmp_path / f"tm{int(use_pg)}.pt")
        code = (f"import sys; sys.path[:0] = [{REPO!r}]; from tests.test_gpu_dist import train_model_worker; "
                f"train_model_worker({port}, {out!r}, {use_pg!r})")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, "\n".join(ln for ln in r.stderr.splitlines() if "frame #" not in ln)[-3000:]
        res[use_pg] = torch.load(out, weights_only=True)
    early, nb = res[True]["early"]
    assert nb > 2 and early >= nb - 1, (early, nb)
    for k, a in res[False]["hist"].items():
        b = res[True]["hist"][k]
        np.testing.assert_allclose(b, a, rtol=1e-4, atol=1e-6, err_msg=k)
