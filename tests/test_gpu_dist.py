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
    if red is not None:
        copied = (red.last_copied, len(red.params))
    if rank == 0:
        torch.save({"grads": [p.cpu() for p in params], "copied": copied}, out)
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
