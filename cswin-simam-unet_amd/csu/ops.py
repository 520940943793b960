"""Autograd wrappers over the libcsu_hip.so C ABI.  Every op here runs a hand-written gfx950
kernel; there is no CPU or eager-PyTorch fallback (CPU tensors raise ``CsuError``)."""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import CSU_BF16, CSU_F32, CsuError, check, dtype_code, lib, ptr, require_device, stream_ptr
from .ledger import esize, launch as _launch, prec_of


def _stripe_fwd_work(geom, B, esize):
    """Algorithmic bytes (qkv read once, output + lse written once) and FLOPs of one launch."""
    L = geom.reso * geom.reso
    nb = len(geom.branches)
    hs, ws, _ = geom.branches[0]
    N = hs * ws
    nbytes = B * L * (3 * geom.C + geom.C) * esize + nb * B * geom.heads * L * 4
    flops = B * L * nb * geom.heads * 4 * N * geom.head_dim + 18 * B * L * geom.C
    return nbytes, flops


# ---------------------------------------------------------------------------------------------
# Stripe attention + LePE (LePEAttention cswin:220-298, branches of CSWinBlock cswin:358-363)
# ---------------------------------------------------------------------------------------------
class StripeGeometry:
    """Static description of the attention branches of one CSWinBlock.

    branches: [(H_sp, W_sp, ch_off)] -- geometry per LePEAttention (cswin:232-240)."""

    def __init__(self, reso: int, C: int, heads: int, branches: Sequence[Tuple[int, int, int]], scale: float,
                 head_dim: int = 32):
        self.reso, self.C, self.heads, self.scale, self.head_dim = reso, C, heads, float(scale), head_dim
        self.branches = [tuple(int(v) for v in b) for b in branches]
        if not 1 <= len(self.branches) <= 2:
            raise ValueError("1 or 2 branches")
        for hs, ws, off in self.branches:
            if reso % hs or reso % ws:
                raise ValueError(f"resolution {reso} not divisible by stripe window {hs}x{ws} (cswin:204)")

    def args(self, B: int, ws: Sequence[torch.Tensor], bs: Sequence[torch.Tensor],
             dws: Optional[Sequence[torch.Tensor]] = None, dbs: Optional[Sequence[torch.Tensor]] = None,
             drop: Optional["AttnDrop"] = None):
        a = _lib.StripeArgs()
        if drop is not None and drop.p > 0:
            a.drop_rng, a.drop_site, a.drop_p = drop.snap.data_ptr(), drop.site, drop.p
        a.B, a.reso, a.C, a.heads, a.head_dim = B, self.reso, self.C, self.heads, self.head_dim
        a.nbranch, a.scale = len(self.branches), self.scale
        for i, (hs, wsp, off) in enumerate(self.branches):
            br = a.br[i]
            br.H_sp, br.W_sp, br.ch_off = hs, wsp, off
            br.lepe_w, br.lepe_b = ws[i].data_ptr(), bs[i].data_ptr()
            if dws is not None:
                br.lepe_dw, br.lepe_db = dws[i].data_ptr(), dbs[i].data_ptr()
        return a


class AttnDrop:
    """Attention dropout of one stripe launch (attn_drop cswin:246/290): snapshot, first site
    (branch i uses site + i), probability."""

    def __init__(self, snap: torch.Tensor, site: int, p: float):
        self.snap, self.site, self.p = snap, int(site), float(p)


class _StripeAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, geom: StripeGeometry, drop, *lepe):
        nb = len(geom.branches)
        ws = [w.detach().float().contiguous() for w in lepe[:nb]]
        bs = [b.detach().float().contiguous() for b in lepe[nb:]]
        require_device(qkv, *ws, *bs)
        qkv = qkv.contiguous()
        B, L, C3 = qkv.shape
        if C3 != 3 * geom.C or L != geom.reso * geom.reso:
            raise ValueError("flatten img_tokens has wrong size")  # cswin:281/356
        out = torch.empty(B, L, geom.C, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(nb, B, geom.heads, L, dtype=torch.float32, device=qkv.device)
        a = geom.args(B, ws, bs, drop=drop)
        nbytes, flops = _stripe_fwd_work(geom, B, qkv.element_size())
        _launch("stripe_attn_fwd", lambda: lib().csu_stripe_attn_fwd(ctypes.byref(a), dtype_code(qkv), ptr(qkv), ptr(out),
                                                                     ptr(lse), stream_ptr(qkv.device)),
                flops, nbytes, prec=prec_of(qkv))
        ctx.geom, ctx.drop = geom, drop
        ctx.lepe_dtypes = [t.dtype for t in lepe]
        ctx.params = tuple(lepe)   # the caller's objects (saved tensors unpack into new wrappers)
        _note_use(ctx, *ctx.params)
        ctx.save_for_backward(qkv, out, lse, *ws, *bs)
        return out

    @staticmethod
    def backward(ctx, dout):
        geom = ctx.geom
        nb = len(geom.branches)
        qkv, out, lse, *wb = ctx.saved_tensors
        ws, bs = wb[:nb], wb[nb:]
        dout = dout.to(qkv.dtype).contiguous()
        B = qkv.shape[0]
        dqkv = torch.empty_like(qkv)
        delta = torch.empty_like(lse)
        L = lib()
        # one flat buffer, views handed to autograd: a deferred reduction keeps the BASE alive, so the
        # returned views stay singly referenced and AccumulateGrad steals them instead of copying
        # them before the reduction has filled them
        # registration order (get_v.weight, get_v.bias of each branch): a GradAllReduce bucket's layout
        order = [t for i in range(nb) for t in (ws[i], bs[i])]
        porder = [p for i in range(nb) for p in (ctx.params[i], ctx.params[nb + i])]
        flat = _grad_dest(porder) if all(dt == torch.float32 for dt in ctx.lepe_dtypes) else None
        if flat is None:
            flat = torch.empty(sum(t.numel() for t in order), dtype=torch.float32, device=qkv.device)
        pv, o = [], 0
        for t in order:
            pv.append(flat[o:o + t.numel()].view(t.shape))
            o += t.numel()
        dws, dbs = pv[0::2], pv[1::2]
        views = dws + dbs
        a = geom.args(B, ws, bs, dws, dbs, drop=ctx.drop)
        nbytes = L.csu_stripe_attn_bwd_workspace(ctypes.byref(a))
        work = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=qkv.device)
        e = qkv.element_size()
        fb, ff = _stripe_fwd_work(geom, B, e)
        # the LePE weight-gradient partials are reduced at the end of backward with every other
        # block's (one csu_stripe_lepe_reduce_batch launch) when nothing reads those grads earlier
        late = DEFER_WGRAD and all(t.dtype == torch.float32 for t in dws + dbs) and _deferrable(*ctx.params)
        # algorithmic: qkv + out + dout read, dqkv written, lse read; FLOPs 2x forward (dP, dV, dQ, dK)
        bw = B * geom.reso * geom.reso * (3 * geom.C * 2 + 2 * geom.C) * e + lse.numel() * 4
        _launch("stripe_attn_bwd", lambda: L.csu_stripe_attn_bwd_ex(ctypes.byref(a), dtype_code(qkv), ptr(qkv), ptr(out),
                                                                    ptr(dout), ptr(lse), ptr(delta), ptr(dqkv), ptr(work),
                                                                    nbytes, int(late), stream_ptr(qkv.device)),
                2 * ff, bw, prec=prec_of(qkv))
        if late:
            it = _lib.LepeReduceItem()
            it.part = work.data_ptr()
            for i in range(nb):
                it.dw[i], it.db[i] = dws[i].data_ptr(), dbs[i].data_ptr()
            it.nblk = L.csu_stripe_lepe_nblk(ctypes.byref(a), dtype_code(qkv))
            it.channels, it.nbranch = geom.heads * geom.head_dim, nb
            _LEPE_PENDING.append((it, work, flat))
            _queue_flush()
            _late(ctx.params, views)
        grads = [g.to(dt) for g, dt in zip(views, ctx.lepe_dtypes)]
        return (dqkv, None, None, *grads)


def stripe_attention(qkv: torch.Tensor, geom: StripeGeometry, lepe_w: Sequence[torch.Tensor],
                     lepe_b: Sequence[torch.Tensor], drop: Optional[AttnDrop] = None) -> torch.Tensor:
    """(B, L, 3C) qkv -> (B, L, C) attention output of every branch (+LePE), channels concatenated.
    ``drop``: attention dropout on the softmax probabilities inside the same kernels."""
    return _StripeAttnFn.apply(qkv, geom, drop, *lepe_w, *lepe_b)


# ---------------------------------------------------------------------------------------------
# Dropout / DropPath (nn.Dropout cswin:188/512, timm DropPath cswin:344/367-368)
# ---------------------------------------------------------------------------------------------
def _dropout_launch(x2, res2, out, rs, rps, snap, site, p):
    rows, cols = x2.shape
    n = rows * cols
    nb = n * (x2.element_size() + out.element_size() + (0 if res2 is None else 4))
    _launch("dropout", lambda: lib().csu_dropout_apply(rows, cols, dtype_code(x2), ptr(x2),
                                                      None if res2 is None else ptr(res2), dtype_code(out), ptr(out),
                                                      None if rs is None else ptr(rs), rps,
                                                      None if snap is None else ptr(snap), site, p,
                                                      stream_ptr(x2.device)), 0, nb)


class _DropoutFn(torch.autograd.Function):
    """out = res + row_scale[row / rps] * keep(site) / (1 - p) * x in one pass (csu_dropout_apply);
    backward regenerates the mask from the saved snapshot (dx = same op on dy, dres = dy)."""

    @staticmethod
    def forward(ctx, x, res, snap, site, p, rs, rps, odt):
        cols = x.shape[-1]
        x2 = x.reshape(-1, cols).contiguous()
        res2 = None if res is None else res.float().reshape(-1, cols).contiguous()
        out = torch.empty(x2.shape, dtype=torch.float32 if res is not None else (odt or x.dtype), device=x.device)
        _dropout_launch(x2, res2, out, rs, rps, snap, site, p)
        ctx.meta = (snap, site, p, rs, rps, x.dtype, x.shape, None if res is None else res.dtype)
        return out.view(*x.shape[:-1], cols)

    @staticmethod
    def backward(ctx, dy):
        snap, site, p, rs, rps, xdt, xshape, rdt = ctx.meta
        cols = dy.shape[-1]
        dy2 = dy.reshape(-1, cols).contiguous()
        dx = torch.empty(dy2.shape, dtype=xdt, device=dy.device)
        _dropout_launch(dy2, None, dx, rs, rps, snap, site, p)
        dres = None if rdt is None else dy.to(rdt)
        return dx.view(xshape), dres, None, None, None, None, None, None


def dropout(x: torch.Tensor, p: float, site: int, snap: Optional[torch.Tensor] = None,
            row_scale: Optional[torch.Tensor] = None, rows_per_sample: int = 1,
            residual: Optional[torch.Tensor] = None, out_dtype=None) -> torch.Tensor:
    """Train-mode nn.Dropout(p) of `x` drawn from site `site` of the RNG snapshot `snap` (the
    enclosing forward's when None, csu.rng), optionally times a per-sample DropPath scale
    (row_scale[row // rows_per_sample], rows = x.numel() // x.shape[-1]) and plus an fp32
    residual, all in one kernel."""
    from . import rng
    require_device(x)
    if x.shape[-1] % 8:
        raise ValueError("dropout: last dim must be a multiple of 8")
    if p > 0 and snap is None:
        snap = rng.snapshot(x.device)
    with torch.autocast("cuda", enabled=False):
        return _DropoutFn.apply(x, residual, snap, int(site), float(p), row_scale, int(rows_per_sample), out_dtype)


def droppath_scale(B: int, p: float, site: int, device, snap: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B,) fp32 DropPath per-sample scale (0 or 1 / (1 - p)) of `site`."""
    from . import rng
    if snap is None:
        snap = rng.snapshot(device)
    return rng.droppath_scale(snap, site, p, B)


# ---------------------------------------------------------------------------------------------
# LayerNorm (nn.LayerNorm over the last dim; eps 1e-5)
# ---------------------------------------------------------------------------------------------
# LayerNorm dgamma / dbeta: the backward kernel leaves per-block partials in its workspace and ONE
# batched launch (csu_layernorm_param_reduce_batch, queued as an end-of-backward callback) reduces
# every LayerNorm's partials, instead of one small reduction launch per LayerNorm (58 per 512x512
# step).  Only when nothing can read those .grad before the end of backward: no existing .grad
# (AccumulateGrad steals the tensor) and no hooks; otherwise reduced inline.
DEFER_LN = True
_LN_PENDING: list = []
_LN_QUEUED = [False]


# forward uses per parameter since the last end-of-backward flush: a parameter used more than once in
# one graph (weight tying) gets its gradient contributions summed by the autograd engine as they
# arrive, i.e. read before a deferred reduction has filled them -- such parameters are never deferred.
# Keyed by id(p) with a weak reference that must still point at p: an entry left by a dead parameter
# (a forward without backward) must not count for a new object that happens to get the same id.
# Only forwards that can be differentiated count (no_grad / eval forwards leave nothing behind).
_USES: dict = {}


def _note_use(ctx, *params):
    """Count one use of each parameter by the op whose autograd context is ``ctx`` -- only when that
    call is recorded for backward (inside Function.forward grad mode is always off and
    needs_input_grad ignores it; a recorded call's node has its next edges already: no_grad / eval
    forwards have none).  ctx None: count unconditionally."""
    if ctx is not None and not ctx.next_functions:
        return
    if len(_USES) > 65536:
        _USES.clear()
    for p in params:
        p = _leaf(p)
        if p is not None and p.requires_grad:
            e = _USES.get(id(p))
            if e is not None and e[0]() is p:
                e[1] += 1
            else:
                _USES[id(p)] = [weakref.ref(p), 1]


def _uses(p) -> int:
    e = _USES.get(id(p))
    return e[1] if e is not None and e[0]() is p else 0


# Gradients handed to autograd BEFORE their values are written (deferred to the end-of-backward
# grouped launches, or computed on the side stream): AccumulateGrad must steal them (no existing
# .grad, a singly referenced tensor).  Should it copy one instead, the copy would read the buffer
# before the kernel that fills it -- a stale or uninitialised first-step gradient.  Every such
# gradient is recorded here (parameter, data pointer, and the storage to rebuild it -- never the
# tensor itself, which would add the reference that prevents the steal); after the values are
# written the parameter's .grad is checked to BE that tensor, and repaired (copied, counted in
# STATS["late_grad_fixups"]) if autograd copied it.
_LATE_DEFER: list = []
_LATE_SIDE: list = []
STATS = {"late_grad_fixups": 0}


def _late(params, grads, side: bool = False):
    lst = _LATE_SIDE if side else _LATE_DEFER
    for p, g in zip(params, grads):
        p = _leaf(p)
        if p is not None and g is not None:
            lst.append((weakref.ref(p), g.data_ptr(), g.untyped_storage(), g.storage_offset(), tuple(g.shape),
                        tuple(g.stride()), g.dtype))


def _check_late(lst):
    items, lst[:] = list(lst), []
    for pref, dptr, st, off, shape, stride, dt in items:
        p = pref()
        if p is None or p.grad is None or p.grad.data_ptr() == dptr:
            continue
        src = torch.empty(0, dtype=dt, device=p.grad.device).set_(st, off, shape, stride)
        p.grad.copy_(src)
        STATS["late_grad_fixups"] += 1


def take_late(params):
    """Remove and return the late-gradient entries of ``params`` as (param, registered gradient)
    pairs.  csu.dist.GradAllReduce calls it when a bucket is launched: a copied late gradient must be
    repaired BEFORE the bucket reads p.grad (the end-of-backward check comes after the all-reduce)."""
    want = {id(_leaf(p)) for p in params}
    out = []
    for lst in (_LATE_DEFER, _LATE_SIDE):
        keep = []
        for e in lst:
            p = e[0]()
            if p is not None and id(p) in want:
                pref, dptr, st, off, shape, stride, dt = e
                out.append((p, torch.empty(0, dtype=dt, device=st.device).set_(st, off, shape, stride)))
            else:
                keep.append(e)
        lst[:] = keep
    return out


def _reducer_hooks_only(hooks) -> bool:
    """True when every post-accumulate-grad hook is a csu.dist.GradAllReduce bucket counter: that
    reducer postpones a bucket holding deferred gradients until after the end-of-backward flush
    (deferred_pending()), so deferral stays legal under data parallelism."""
    from .dist import GradAllReduce
    return all(getattr(h, "__func__", None) is GradAllReduce._hook for h in hooks.values())


def _deferrable(*params) -> bool:
    _queue_flush()   # the end-of-backward flush also resets the use counts
    # backward(create_graph=True): AccumulateGrad COPIES the incoming gradient (it does not take
    # ownership), so the copy would be made before the end-of-backward flush filled the buffer
    if torch.is_grad_enabled():
        return False
    # torch DDP's C++ reducer hooks the grad accumulators directly (invisible to the checks below) and
    # reads p.grad as soon as it is accumulated: defer only without a process group, or under
    # csu.dist.GradAllReduce (which postpones buckets holding deferred gradients, deferred_pending())
    if not _DIST_SAFE[0]:
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return False
    for p in params:
        p = _leaf(p)
        if p is None:
            continue
        if p.grad is not None or p._backward_hooks:
            return False
        hooks = getattr(p, "_post_accumulate_grad_hooks", None)
        if hooks and not _reducer_hooks_only(hooks):
            return False
        if _uses(p) > 1:
            return False
    return True


def deferred_pending() -> bool:
    """Parameter gradients of the running backward pass that are filled only by the end-of-backward
    flush (LayerNorm dgamma / dbeta, token-Linear dW / db, LePE dW / db)."""
    return bool(_LN_PENDING or _WG_DEFER or _WG_PENDING or _WG_POST or _LEPE_PENDING)


def _ln_param_flush():
    pend, _LN_PENDING[:] = list(_LN_PENDING), []
    if not pend:
        return
    dev = pend[0][1].device
    items = (_lib.LnParamItem * len(pend))()
    for i, (work, dgb, rows, C, nblk) in enumerate(pend):
        items[i].workspace, items[i].dgamma, items[i].dbeta = work.data_ptr(), dgb.data_ptr(), dgb.data_ptr() + C * 4
        items[i].rows, items[i].C, items[i].nblocks = rows, C, nblk
    nv = sum(2 * e[3] for e in pend)
    _launch("layernorm_bwd", lambda: lib().csu_layernorm_param_reduce_batch(items, len(pend), stream_ptr(dev)),
            0, sum(e[0].numel() for e in pend) + nv * 4)


def _queue_flush():
    """Queue the end-of-backward flush once per backward pass (outside a backward pass -- direct
    calls, tests -- the caller flushes explicitly)."""
    if not _LN_QUEUED[0] and torch._C._current_graph_task_id() != -1:
        torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward_flush)
        _LN_QUEUED[0] = True


def _end_of_backward_flush():
    """The deferred parameter gradients of this backward pass: every LayerNorm's dgamma / dbeta (one
    launch), every deferrable token-Linear weight gradient (grouped tile launches + batched slab
    sums) and every LePE weight-gradient reduction (one launch per 32 blocks)."""
    _LN_QUEUED[0] = False
    flush_deferred()
    _check_late(_LATE_DEFER)
    _USES.clear()


def flush_deferred():
    """Write every parameter gradient deferred so far in this backward pass (the grouped launches of
    the end-of-backward flush, for what is pending now).  csu.dist.GradAllReduce calls it when a
    bucket's last gradient has been accumulated, so that bucket's all-reduce can start while the rest
    of backward runs; what later ops defer goes to the next bucket's flush or the end of backward."""
    _ln_param_flush()
    _wgrad_flush()
    _lepe_flush()


_LEPE_PENDING: list = []   # (LepeReduceItem, partials workspace, flat gradient buffer)


def _lepe_flush():
    pend, _LEPE_PENDING[:] = list(_LEPE_PENDING), []
    if not pend:
        return
    dev = pend[0][1].device
    items = (_lib.LepeReduceItem * len(pend))()
    nbytes = 0
    for i, (it, work, _) in enumerate(pend):
        items[i] = it
        nbytes += it.nbranch * it.channels * 10 * (it.nblk + 1) * 4
    _launch("stripe_attn_bwd", lambda: lib().csu_stripe_lepe_reduce_batch(items, len(pend), stream_ptr(dev)), 0, nbytes)


def _ln_params(ctx, rows, C, work, dgb, nblocks=0):
    """Reduce (later, batched) or report that the caller must pass dgamma / dbeta pointers.
    ``nblocks``: partial rows in ``work`` (0: csu_layernorm_bwd_ex's for ``rows``)."""
    if not (DEFER_LN and all(dt == torch.float32 for dt in ctx.pdtypes) and _deferrable(*ctx.params)):
        return False
    _LN_PENDING.append((work, dgb, rows, C, nblocks))
    _late(ctx.params, (dgb[:C], dgb[C:]))
    _queue_flush()
    return True


# Token-Linear weight gradients (bf16) of every Linear whose dW / db nothing reads before the end of
# backward (same conditions as the LayerNorm deferral) are computed at the end of backward: ONE
# grouped tile launch per tile size for all of them (csu_linear_wgrad_group: no per-Linear
# underfilled workgroup rounds, so each Linear needs only a few token chunks) and ONE batched
# fixed-order slab sum per 40 (csu_wslab_reduce_batch).  Their dY / X operands are kept alive until
# then.  DEFER_WGRAD = False (tests): one launch (+ reduction) per Linear, inline.
DEFER_WGRAD = True
GROUP_WGRAD = True   # False (tests): deferred slab sums only
_WG_PENDING: list = []   # (WslabItem, out, workspace): reductions of tile kernels already launched
_WG_DEFER: list = []     # (dy2, x2, out): whole weight gradients deferred to the grouped launch
_WG_POST: list = []      # callables run after the deferred weight gradients are complete


def _wgrad_flush():
    defer, _WG_DEFER[:] = list(_WG_DEFER), []
    if defer:
        L = lib()
        dev = defer[0][0].device
        gitems = (_lib.WgradGroupItem * len(defer))()
        keep, flops, nbytes = [], 0, 0
        for i, (dy2, x2, out) in enumerate(defer):
            M, N = dy2.shape
            K = x2.shape[1]
            tn, tk, ch = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            nws = L.csu_linear_wgrad_group_plan(M, N, K, ctypes.byref(tn), ctypes.byref(tk), ctypes.byref(ch))
            slab = torch.empty(nws // 4, dtype=torch.float32, device=dev) if nws else None
            keep.append(slab)
            it = gitems[i]
            it.dy, it.x, it.dw_db, it.slab, it.M, it.N, it.K = dy2.data_ptr(), x2.data_ptr(), out.data_ptr(), \
                (slab.data_ptr() if slab is not None else None), M, N, K
            if ch.value > 1:
                w = _lib.WslabItem()
                w.slab, w.dst, w.N, w.K, w.tn, w.tk, w.chunks = slab.data_ptr(), out.data_ptr(), N, K, tn.value, tk.value, \
                    ch.value
                _WG_PENDING.append((w, out, slab))
            flops += 2 * M * N * K
            nbytes += M * (N + K) * 2 + (N * K + N) * 4
        _launch("linear_wgrad", lambda: L.csu_linear_wgrad_group(gitems, len(defer), stream_ptr(dev)), flops, nbytes)
    pend, _WG_PENDING[:] = list(_WG_PENDING), []
    if not pend:
        _wgrad_post()
        return
    dev = pend[0][1].device
    items = (_lib.WslabItem * len(pend))()
    nbytes = 0
    for i, (it, out, work) in enumerate(pend):
        items[i] = it
        nbytes += it.chunks * (it.N * it.K + it.N) * 4 + (it.N * it.K + it.N) * 4
    _launch("linear_wgrad", lambda: lib().csu_wslab_reduce_batch(items, len(pend), stream_ptr(dev)), 0, nbytes)
    _wgrad_post()


def _wgrad_post():
    post, _WG_POST[:] = list(_WG_POST), []
    for fn in post:
        fn()


def _wgrad_deferrable(dy2, wdt, bdt, params) -> bool:
    return (DEFER_WGRAD and dy2.dtype == torch.bfloat16 and bool(params) and wdt in (None, torch.float32)
            and bdt in (None, torch.float32) and _deferrable(*params))


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps: float, out_dtype, pre=None):
        require_device(x, weight, bias)
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        w = weight.detach().float().contiguous()
        if pre is not None:   # computed by the producing fused Mlp (csu_mlp_fwd_ln)
            y, mean, rstd = pre[3].view(x.shape), pre[4], pre[5]
        else:
            b = bias.detach().float().contiguous()
            y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
            mean = torch.empty(rows, dtype=torch.float32, device=x.device)
            rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
            _launch("layernorm_fwd", lambda: lib().csu_layernorm_fwd(rows, C, float(eps), dtype_code(x), ptr(x), ptr(w),
                                                                     ptr(b), dtype_code(y), ptr(y), ptr(mean), ptr(rstd),
                                                                     stream_ptr(x.device)),
                    8 * rows * C, rows * C * (esize(x) + esize(y)) + rows * 8, prec=prec_of(x))
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.pdtypes = (weight.dtype, bias.dtype)
        ctx.params = (weight, bias)
        _note_use(ctx, *ctx.params)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        if dy.dtype not in (torch.float32, torch.bfloat16):
            dy = dy.float()
        C = x.shape[-1]
        rows = x.numel() // C
        dx = torch.empty_like(x)
        # fp32 input (the residual stream under norm / norm_up, cswin:554/602): the bf16 copy of dx
        # the upstream Mlp / GEMM backward consumes, written by the same pass (see _bf16_of)
        dxb = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if x.dtype == torch.float32 else None
        dgb = _grad_dest(ctx.params)   # contiguous: one reduction pass
        if dgb is None:
            dgb = torch.empty(2 * C, dtype=torch.float32, device=x.device)
        dg, db = dgb[:C], dgb[C:]
        L = lib()
        nbytes = L.csu_layernorm_bwd_workspace(rows, C)
        work = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=x.device)
        late = _ln_params(ctx, rows, C, work, dgb)
        pg, pb = (None, None) if late else (ptr(dg), ptr(db))
        _launch("layernorm_bwd", lambda: L.csu_layernorm_bwd_ex(rows, C, dtype_code(x), ptr(x), ptr(w), ptr(mean), ptr(rstd),
                                                                dtype_code(dy), ptr(dy), None, ptr(dx), ptr(dxb), pg, pb,
                                                                ptr(work), nbytes, stream_ptr(x.device)),
                12 * rows * C, rows * C * (2 * esize(x) + esize(dy) + esize(dxb)) + rows * 8, prec=prec_of(x))
        if dxb is not None:
            dx._csu_bf16 = dxb
        return dx, dg.to(ctx.pdtypes[0]), db.to(ctx.pdtypes[1]), None, None, None


def _ln_pre(x, weight, bias, eps, od):
    """The LayerNorm of x already computed by the fused Mlp that produced it (``_csu_ln``), or None."""
    pre = getattr(x, "_csu_ln", None)
    if (pre is not None and pre[0] is weight and pre[1] is bias and pre[2] == float(eps) and pre[3].dtype == od
            and pre[3].numel() == x.numel() and x.is_contiguous() and pre[6] == x._version):
        return pre
    return None


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5,
               out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    od = out_dtype or x.dtype
    pre = _ln_pre(x, weight, bias, eps, od)
    if pre is not None:
        return _LayerNormFn.apply(x, weight, bias, eps, od, pre)
    return _LayerNormFn.apply(x, weight, bias, eps, od)


def _bf16_of(g: torch.Tensor) -> torch.Tensor:
    """bf16 copy of a gradient: the one a residual junction attached to it (csu_layernorm_bwd_ex
    writes it in the same pass), else a fresh cast."""
    b = getattr(g, "_csu_bf16", None)
    if b is not None and b.shape == g.shape:
        return b
    return g.reshape(g.shape).to(torch.bfloat16).contiguous()


class _LayerNormForkFn(torch.autograd.Function):
    """Residual junction x -> (x, LN(x)) of CSWinBlock (x + f(LN(x)), cswin:367-368).  Backward
    gets the residual-branch gradient and the LN-branch gradient together and writes
    dx = dres + dLN in ONE kernel (no autograd add), plus the bf16 copy of dx that the upstream
    GEMM backward consumes (attached to dx as ``_csu_bf16``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps: float, out_dtype, pre=None):
        require_device(x, weight, bias)
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        w = weight.detach().float().contiguous()
        if pre is not None:
            # computed by the producing fused Mlp's epilogue (csu_mlp_fwd_ln): no launch here
            y, mean, rstd = pre[3].view(x.shape), pre[4], pre[5]
        else:
            b = bias.detach().float().contiguous()
            y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
            mean = torch.empty(rows, dtype=torch.float32, device=x.device)
            rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
            _launch("layernorm_fwd", lambda: lib().csu_layernorm_fwd(rows, C, float(eps), dtype_code(x), ptr(x), ptr(w),
                                                                     ptr(b), dtype_code(y), ptr(y), ptr(mean), ptr(rstd),
                                                                     stream_ptr(x.device)),
                    8 * rows * C, rows * C * (esize(x) + esize(y)) + rows * 8, prec=prec_of(x))
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.pdtypes = (weight.dtype, bias.dtype)
        ctx.params = (weight, bias)
        _note_use(ctx, *ctx.params)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, dres, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dx, dg, db = _ln_fork_backward(ctx, x, w, mean, rstd, dres, dy)
        return dx, dg, db, None, None, None


def _ln_fork_backward(ctx, x, w, mean, rstd, dres, dy):
    """dx = dres + LN'(dy) in one csu_layernorm_bwd_ex pass (+ the bf16 copy of dx as
    ``_csu_bf16``), dgamma / dbeta (deferred into the batched reduction when allowed).  ctx carries
    the LN parameters (``params``, ``pdtypes``)."""
    C = x.shape[-1]
    rows = x.numel() // C
    if dy is None:
        dy = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
    dy = dy.contiguous()
    if dy.dtype not in (torch.float32, torch.bfloat16):
        dy = dy.float()
    fp32 = x.dtype == torch.float32
    dres_k = dres.float().contiguous() if (dres is not None and fp32) else None
    dx = torch.empty_like(x)
    dxb = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if fp32 else None
    L = lib()
    nbytes = L.csu_layernorm_bwd_workspace(rows, C)
    work = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=x.device)
    dgb = _grad_dest(ctx.params)
    if dgb is None:
        dgb = torch.empty(2 * C, dtype=torch.float32, device=x.device)
    late = _ln_params(ctx, rows, C, work, dgb)
    pg, pb = (None, None) if late else (ptr(dgb[:C]), ptr(dgb[C:]))
    _launch("layernorm_bwd", lambda: L.csu_layernorm_bwd_ex(rows, C, dtype_code(x), ptr(x), ptr(w), ptr(mean),
                                                            ptr(rstd), dtype_code(dy), ptr(dy), ptr(dres_k), ptr(dx),
                                                            ptr(dxb), pg, pb, ptr(work), nbytes,
                                                            stream_ptr(x.device)),
            12 * rows * C, rows * C * (2 * esize(x) + esize(dy) + esize(dres_k) + esize(dxb)) + rows * 8,
            prec=prec_of(x))
    if dres is not None and not fp32:    # non-fp32 residual stream: plain add (not on the bf16 path)
        dx = dx + dres.to(dx.dtype)
    if dxb is not None:
        dx._csu_bf16 = dxb
    return dx, dgb[:C].to(ctx.pdtypes[0]), dgb[C:].to(ctx.pdtypes[1])


def layer_norm_fork(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5,
                    out_dtype: Optional[torch.dtype] = None):
    """(x, LN(x)) for a residual junction; use the first output as the residual input.  When x is a
    fused Mlp output that already carries this LayerNorm (mlp_residual(ln_next=...)), its values are
    used instead of a LayerNorm launch."""
    od = out_dtype or x.dtype
    pre = _ln_pre(x, weight, bias, eps, od)
    if pre is not None:
        return _LayerNormForkFn.apply(x, weight, bias, eps, od, pre)
    return _LayerNormForkFn.apply(x, weight, bias, eps, od)


# ---------------------------------------------------------------------------------------------
# CARAFE reassembly (cswin:410-432 / 459-481) and the 1-class sigmoid head (cswin:680, 688)
# ---------------------------------------------------------------------------------------------
class _CarafeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, enc, H: int, W: int, s: int):
        require_device(x, enc)
        x = x.contiguous()
        enc = enc.to(x.dtype).contiguous()
        B, L, C = x.shape
        if L != H * W or tuple(enc.shape) != (B, H, W, 9 * s * s):
            raise ValueError("carafe: shape mismatch")
        out = torch.empty(B, L * s * s, C, dtype=x.dtype, device=x.device)
        wsave = torch.empty(B, H, W, 9 * s * s, dtype=torch.float32, device=x.device)
        e, T = x.element_size(), 9 * s * s
        _launch("carafe_fwd", lambda: lib().csu_carafe_fwd(B, H, W, C, s, dtype_code(x), ptr(x), ptr(enc), ptr(out),
                                                           ptr(wsave), stream_ptr(x.device)),
                B * H * W * s * s * C * 18, B * H * W * (C * e * (1 + s * s) + T * (e + 4)), prec=prec_of(x))
        ctx.save_for_backward(x, wsave)
        ctx.geo = (B, H, W, C, s)
        ctx.enc_dtype = enc.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        x, wsave = ctx.saved_tensors
        B, H, W, C, s = ctx.geo
        dout = dout.to(x.dtype).contiguous()
        dx = torch.empty_like(x)
        denc = torch.empty(B, H, W, 9 * s * s, dtype=x.dtype, device=x.device)
        e, T = x.element_size(), 9 * s * s
        _launch("carafe_bwd", lambda: lib().csu_carafe_bwd(B, H, W, C, s, dtype_code(x), ptr(x), ptr(wsave), ptr(dout),
                                                           ptr(dx), ptr(denc), stream_ptr(x.device)),
                B * H * W * s * s * C * 36, B * H * W * (C * e * (2 + s * s) + T * (4 + e)), prec=prec_of(x))
        return dx, denc, None, None, None


def carafe_reassemble(x: torch.Tensor, enc_nhwc: torch.Tensor, H: int, W: int, s: int) -> torch.Tensor:
    """x (B, H*W, C) tokens, enc_nhwc (B, H, W, 9*s*s) kernel logits -> (B, s*s*H*W, C)."""
    return _CarafeFn.apply(x, enc_nhwc, H, W, s)


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        require_device(x, w)
        x = x.contiguous()
        wf = w.detach().float().contiguous().view(-1)
        P, C = x.numel() // x.shape[-1], x.shape[-1]
        prob = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
        _launch("head_fwd", lambda: lib().csu_head_fwd(P, C, dtype_code(x), ptr(x), ptr(wf), ptr(prob), stream_ptr(x.device)),
                2 * P * C, P * (C * x.element_size() + 4), prec=prec_of(x))
        ctx.save_for_backward(x, wf, prob)
        ctx.wshape, ctx.wdtype = w.shape, w.dtype
        return prob

    @staticmethod
    def backward(ctx, dprob):
        x, wf, prob = ctx.saved_tensors
        dprob = dprob.float().contiguous()
        P, C = x.numel() // x.shape[-1], x.shape[-1]
        dx = torch.empty_like(x)
        dw = torch.empty(C, dtype=torch.float32, device=x.device)
        L = lib()
        n = L.csu_head_bwd_workspace(P, C)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        _launch("head_bwd", lambda: L.csu_head_bwd(P, C, dtype_code(x), ptr(x), ptr(wf), ptr(prob), ptr(dprob), ptr(dx),
                                                   ptr(dw), ptr(work), n, stream_ptr(x.device)),
                4 * P * C, P * (2 * C * x.element_size() + 8), prec=prec_of(x))
        return dx, dw.view(ctx.wshape).to(ctx.wdtype)


def sigmoid_head(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """sigmoid(x @ w) for a 1-class 1x1 conv without bias: x (..., C) -> (...) fp32."""
    return _HeadFn.apply(x, weight)


class _CarafeHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, enc, u, cb, H, W, s):
        require_device(x, enc, u, cb)
        x, enc = x.contiguous(), enc.to(x.dtype).contiguous()
        uf, cf = u.detach().float().contiguous(), cb.detach().float().reshape(1).contiguous()
        B, C = x.shape[0], x.shape[-1]
        if x.numel() != B * H * W * C or enc.numel() != B * H * W * 9 * s * s:
            raise ValueError("carafe_head: x must be (B, H*W, C) and enc (B, H, W, 9 s^2)")
        z = torch.empty(B * H * W, dtype=torch.float32, device=x.device)
        prob = torch.empty(B, 1, s * H, s * W, dtype=torch.float32, device=x.device)
        e, T = x.element_size(), 9 * s * s
        _launch("carafe_head_fwd", lambda: lib().csu_carafe_head_fwd(B, H, W, C, s, dtype_code(x), ptr(x), ptr(enc), ptr(uf),
                                                                     ptr(cf), ptr(z), ptr(prob), stream_ptr(x.device)),
                B * H * W * (2 * C + 2 * T), B * H * W * (C * e + T * e + 4 + s * s * 4), prec=prec_of(x))
        ctx.save_for_backward(x, enc, z, uf, prob)
        ctx.geo = (B, H, W, C, s)
        ctx.dtypes = (u.dtype, cb.dtype, cb.shape)
        return prob

    @staticmethod
    def backward(ctx, dprob):
        x, enc, z, uf, prob = ctx.saved_tensors
        B, H, W, C, s = ctx.geo
        dprob = dprob.float().contiguous()
        dx, denc = torch.empty_like(x), torch.empty_like(enc)
        du = torch.empty(C, dtype=torch.float32, device=x.device)
        dcb = torch.empty(1, dtype=torch.float32, device=x.device)
        L = lib()
        n = L.csu_carafe_head_bwd_workspace(B, H, W, C, s)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        e, T = x.element_size(), 9 * s * s
        _launch("carafe_head_bwd", lambda: L.csu_carafe_head_bwd(B, H, W, C, s, dtype_code(x), ptr(x), ptr(enc), ptr(z),
                                                                 ptr(uf), ptr(prob), ptr(dprob), ptr(dx), ptr(denc), ptr(du),
                                                                 ptr(dcb), ptr(work), n, stream_ptr(x.device)),
                B * H * W * (4 * C + 4 * T), B * H * W * (2 * C * e + 2 * T * e + 4 + s * s * 8), prec=prec_of(x))
        udt, cdt, cshape = ctx.dtypes
        return dx, denc, du.to(udt), dcb.to(cdt).reshape(cshape), None, None, None


class _CarafeHeadFoldedFn(torch.autograd.Function):
    """_CarafeHeadFn with the head-weight folding (u = w_out^T w_h, cb = w_h . b_out, cswin:674-688)
    on csu kernels too: csu_head_fold_fwd before the head, the folding's backward inside
    csu_carafe_head_bwd_fold -- no torch GEMV / reductions / casts between them; the weight
    gradients come out in the parameters' own shapes (AccumulateGrad steals them)."""

    @staticmethod
    def forward(ctx, x, enc, w_out, b_out, w_h, H, W, s):
        require_device(x, enc, w_out, b_out, w_h)
        B, C = x.shape[0], x.shape[-1]
        O = w_out.shape[0]
        wo = w_out.detach().float().reshape(O, C).contiguous()
        bo = b_out.detach().float().contiguous()
        wh = w_h.detach().float().reshape(O).contiguous()
        uf = torch.empty(C, dtype=torch.float32, device=x.device)
        cf = torch.empty(1, dtype=torch.float32, device=x.device)
        _launch("head_fold", lambda: lib().csu_head_fold_fwd(O, C, ptr(wo), ptr(bo), ptr(wh), ptr(uf), ptr(cf),
                                                             stream_ptr(x.device)),
                2 * O * C, (O * C + 2 * O + C + 1) * 4, prec="f32")
        x, enc = x.contiguous(), enc.to(x.dtype).contiguous()
        if x.numel() != B * H * W * C or enc.numel() != B * H * W * 9 * s * s:
            raise ValueError("carafe_head: x must be (B, H*W, C) and enc (B, H, W, 9 s^2)")
        z = torch.empty(B * H * W, dtype=torch.float32, device=x.device)
        prob = torch.empty(B, 1, s * H, s * W, dtype=torch.float32, device=x.device)
        e, T = x.element_size(), 9 * s * s
        _launch("carafe_head_fwd", lambda: lib().csu_carafe_head_fwd(B, H, W, C, s, dtype_code(x), ptr(x), ptr(enc), ptr(uf),
                                                                     ptr(cf), ptr(z), ptr(prob), stream_ptr(x.device)),
                B * H * W * (2 * C + 2 * T), B * H * W * (C * e + T * e + 4 + s * s * 4), prec=prec_of(x))
        ctx.save_for_backward(x, enc, z, uf, prob, wo, bo, wh)
        ctx.geo = (B, H, W, C, s)
        ctx.pshapes = ((w_out.shape, w_out.dtype), (b_out.shape, b_out.dtype), (w_h.shape, w_h.dtype))
        ctx.params = (w_out, b_out, w_h)   # for their GradAllReduce bucket slices (_grad_dest)
        _note_use(ctx, *ctx.params)
        return prob

    @staticmethod
    def backward(ctx, dprob):
        x, enc, z, uf, prob, wo, bo, wh = ctx.saved_tensors
        B, H, W, C, s = ctx.geo
        dprob = dprob.float().contiguous()
        dx, denc = torch.empty_like(x), torch.empty_like(enc)
        du = torch.empty(C, dtype=torch.float32, device=x.device)
        (sw, tw), (sb, tb), (sh, th) = ctx.pshapes
        O = wo.shape[0]
        # the folded head's weight gradients straight into their GradAllReduce bucket slices when the
        # reducer holds them ([dW_out | db_out] adjacent, dw_h on its own), else fresh buffers
        dest = _grad_dest(ctx.params[:2]) if tw == torch.float32 and tb == torch.float32 else None
        if dest is not None and dest.numel() == O * C + O:
            dwo, dbo = dest[:O * C].view(sw), dest[O * C:].view(sb)
        else:
            dwo = torch.empty(sw, dtype=torch.float32, device=x.device)
            dbo = torch.empty(sb, dtype=torch.float32, device=x.device)
        desth = _grad_dest(ctx.params[2:]) if th == torch.float32 else None
        dwh = desth.view(sh) if desth is not None and desth.numel() == O else torch.empty(sh, dtype=torch.float32,
                                                                                          device=x.device)
        fold = _lib.HeadFold()
        fold.O, fold.w_out, fold.b_out, fold.w_h = wo.shape[0], wo.data_ptr(), bo.data_ptr(), wh.data_ptr()
        fold.dw_out, fold.db_out, fold.dw_h = dwo.data_ptr(), dbo.data_ptr(), dwh.data_ptr()
        L = lib()
        n = L.csu_carafe_head_bwd_workspace(B, H, W, C, s)
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
        e, T = x.element_size(), 9 * s * s
        _launch("carafe_head_bwd", lambda: L.csu_carafe_head_bwd_fold(B, H, W, C, s, dtype_code(x), ptr(x), ptr(enc),
                                                                      ptr(z), ptr(uf), ptr(prob), ptr(dprob), ptr(dx),
                                                                      ptr(denc), ptr(du), ctypes.byref(fold), ptr(work), n,
                                                                      stream_ptr(x.device)),
                B * H * W * (4 * C + 4 * T), B * H * W * (2 * C * e + 2 * T * e + 4 + s * s * 8), prec=prec_of(x))
        return dx, denc, dwo.to(tw), dbo.to(tb), dwh.to(th), None, None, None


def carafe_head_folded(x: torch.Tensor, enc: torch.Tensor, w_out: torch.Tensor, b_out: torch.Tensor,
                       w_h: torch.Tensor, H: int, W: int, s: int) -> torch.Tensor:
    """sigmoid(output(CARAFE(x).out)) with the raw head weights: w_out (O, C[, 1, 1]) / b_out (O) of
    the CARAFE `out` conv, w_h (1, O[, 1, 1]) of the 1-class bias-free `output` conv."""
    with torch.autocast("cuda", enabled=False):
        return _CarafeHeadFoldedFn.apply(x, enc, w_out, b_out, w_h, H, W, s)


def carafe_head(x: torch.Tensor, enc: torch.Tensor, u: torch.Tensor, cb: torch.Tensor, H: int, W: int,
                s: int) -> torch.Tensor:
    """sigmoid(output(CARAFE(x).out)) for a 1-class bias-free head, fused (csu_carafe_head_*):
    x (B, H*W, C) tokens, enc (B, H, W, 9 s^2) encoder logits, u = W_out^T w_output (C),
    cb = w_output . b_out (scalar tensor) -> prob (B, 1, sH, sW) fp32."""
    return _CarafeHeadFn.apply(x, enc, u, cb, H, W, s)


# ---------------------------------------------------------------------------------------------
# Token Linear (nn.Linear on (B, L, C) tokens) with a split-K weight gradient.
# The weight gradient dW = dY^T X reduces over all B*L tokens (K up to 4M); a plain GEMM keeps
# only (N/64)*(K/64) workgroups busy for the whole token range, so it is split into S token
# chunks computed as one batched GEMM and summed in fp32 (deterministic).
# ---------------------------------------------------------------------------------------------
def colsum(x2: torch.Tensor) -> torch.Tensor:
    """Deterministic fp32 column sum of a 2-D (rows, cols) tensor on the device (csu_colsum)."""
    require_device(x2)
    x2 = x2.contiguous()
    rows, cols = x2.shape
    out = torch.empty(cols, dtype=torch.float32, device=x2.device)
    L = lib()
    n = L.csu_colsum_workspace(rows, cols, dtype_code(x2))
    work = torch.empty(max(n, 16), dtype=torch.uint8, device=x2.device)
    _launch("colsum", lambda: L.csu_colsum(rows, cols, dtype_code(x2), ptr(x2), ptr(out), ptr(work), n,
                                           stream_ptr(x2.device)),
            rows * cols, rows * cols * x2.element_size() + cols * 4, prec=prec_of(x2))
    return out


def gemm_f32(layout: int, a: torch.Tensor, b: torch.Tensor, M: int, N: int, K: int, bias=None, resid=None,
             with_asum=False, out=None, asum=None):
    """fp32 csu_gemm_f32: layout 0 C = A B^T (+bias, +resid), 1 C = A B, 2 C = A^T B; C (M, N).
    ``with_asum`` (layout 2): also return sum_k A[k][m] (the bias gradient) from the same launch.
    ``out`` / ``asum``: caller-provided contiguous result buffers (e.g. a GradAllReduce bucket)."""
    require_device(a, b)
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=a.device)
    if with_asum and asum is None:
        asum = torch.empty(M, dtype=torch.float32, device=a.device)
    L = lib()
    n = L.csu_gemm_f32_workspace(layout, M, N, K)
    work = torch.empty(max(n, 16), dtype=torch.uint8, device=a.device) if n else None
    name = ("gemm", "gemm", "linear_wgrad")[layout]
    _launch(name, lambda: L.csu_gemm_f32(layout, M, N, K, ptr(a), ptr(b), ptr(bias), ptr(resid), ptr(out), ptr(asum),
                                         ptr(work), n, stream_ptr(a.device)),
            2 * M * N * K, (M * K + N * K + M * N) * 4 + (M * N * 4 if resid is not None else 0), prec="f32")
    return (out, asum) if with_asum else out


def linear_wgrad(dy2: torch.Tensor, x2: torch.Tensor, out=None, work=None, defer: bool = False):
    """(dW (N, K), db (N)) fp32 of a token Linear: one MFMA split-K kernel + one reduction.
    ``out`` / ``work``: caller-allocated result (N*K + N fp32) and workspace buffers.  ``defer``
    (bf16): the reduction joins the end-of-backward batch (_wgrad_flush); the returned tensors are
    filled then -- only for gradients nothing reads earlier (see _wgrad_deferrable)."""
    require_device(dy2, x2)
    M, N = dy2.shape
    K = x2.shape[1]
    if dy2.dtype == torch.float32:
        # fp32: MFMA GEMM dW = dy^T x (token splits + ordered slab sum) and the column sum for db
        if out is None:
            return gemm_f32(2, dy2.contiguous(), x2.contiguous(), N, K, M, with_asum=True)
        return gemm_f32(2, dy2.contiguous(), x2.contiguous(), N, K, M, with_asum=True, out=out[:N * K].view(N, K),
                        asum=out[N * K:])
    L = lib()
    if out is None:
        out = torch.empty(N * K + N, dtype=torch.float32, device=dy2.device)
    if defer and dy2.dtype == torch.bfloat16 and N % 8 == 0 and K % 8 == 0 and GROUP_WGRAD and M < 2 ** 31:
        # the whole weight gradient joins the end-of-backward grouped launch
        _WG_DEFER.append((dy2.contiguous(), x2.contiguous(), out))
        _queue_flush()
        return out[:N * K].view(N, K), out[N * K:]
    n = L.csu_linear_wgrad_workspace(M, N, K)
    if work is None:
        work = torch.empty(max(n, 16), dtype=torch.uint8, device=dy2.device)
    if defer and dy2.dtype == torch.bfloat16 and N % 8 == 0 and K % 8 == 0:
        it = _lib.WslabItem()
        _launch("linear_wgrad", lambda: L.csu_linear_wgrad_deferred(M, N, K, ptr(dy2), ptr(x2), ptr(out), ptr(work), n,
                                                                    ctypes.byref(it), stream_ptr(dy2.device)),
                2 * M * N * K, M * (N + K) * 2 + (N * K + N) * 4)
        if it.chunks > 1:
            _WG_PENDING.append((it, out, work))   # keeps the slab workspace and the result alive
            _queue_flush()
        return out[:N * K].view(N, K), out[N * K:]
    _launch("linear_wgrad", lambda: L.csu_linear_wgrad(M, N, K, dtype_code(dy2), ptr(dy2), ptr(x2), ptr(out), ptr(work), n,
                                                       stream_ptr(dy2.device)),
            2 * M * N * K, M * (N + K) * dy2.element_size() + (N * K + N) * 4, prec=prec_of(dy2))
    return out[:N * K].view(N, K), out[N * K:]


def gemm(a2: torch.Tensor, b: torch.Tensor, b_trans: bool, out_dtype, bias=None, a_gelu=False, gelu_aux=None,
         resid=None, cfg: int = -1, gelu_out: bool = False):
    """csu_gemm_ex: out = epi(pro(a2) @ B) with B = b^T (b_trans False, b is (N, K)) or b (b_trans True, (K, N)).
    ``cfg`` forces a tile configuration of the b_trans=False kernel (-1: per-shape choice);
    ``gelu_out`` also returns gelu(out) (bf16) written by the same epilogue: (out, gelu(out))."""
    M, K = a2.shape
    N = b.shape[1] if b_trans else b.shape[0]
    out = torch.empty(M, N, dtype=out_dtype, device=a2.device)
    g = torch.empty(M, N, dtype=torch.bfloat16, device=a2.device) if gelu_out else None
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.a, d.b, d.lda, d.ldb = M, N, K, ptr(a2), ptr(b), a2.stride(0), b.stride(0)
    d.b_trans, d.a_gelu, d.bias, d.gelu_aux, d.resid = int(b_trans), int(a_gelu), ptr(bias), ptr(gelu_aux), ptr(resid)
    d.out, d.gelu_out, d.ldc, d.out_dtype, d.cfg = ptr(out), ptr(g), N, dtype_code(out), int(cfg)
    nb = (M * K * a2.element_size() + N * K * b.element_size() + M * N * out.element_size()
          + (M * N * 2 if gelu_aux is not None else 0) + (M * N * 4 if resid is not None else 0) + (M * N * 2 if gelu_out else 0))
    _launch("gemm", lambda: lib().csu_gemm_ex(ctypes.byref(d), stream_ptr(a2.device)), 2 * M * N * K, nb, prec=prec_of(a2),
            tag=f"{M}x{N}x{K}{'T' if b_trans else ''}{'g' if a_gelu else ''}{'G' if gelu_out else ''}{'r' if resid is not None else ''}"
                f"{'b' if bias is not None else ''}:{out_dtype}")
    return (out, g) if gelu_out else out


# csu_gemm_ws (weight-streaming token GEMM, csrc/gemm_ws.hip) for the shapes it is instantiated for,
# when the cast cache holds the fragment-ordered weight; gemm4 otherwise
USE_GEMM_WS = True


def gemm_ws(x2: torch.Tensor, w_frag, N: int, out_dtype, bias=None, resid=None) -> torch.Tensor:
    """out (M, N) = x2 (M, K) @ W^T (+ bias) (+ resid) with W given fragment-ordered: a bf16 tensor
    (CastCache.get_frag) or an e4m3 operand (frag8, scales, scale_mode) of the fp8 weight format
    (Fp8Weights.get_frag8, csu_gemm_ws_e4m3: half the streamed weight bytes, bitwise the same result)."""
    M, K = x2.shape
    out = torch.empty(M, N, dtype=out_dtype, device=x2.device)
    e4 = isinstance(w_frag, tuple)
    nb = M * K * 2 + N * K * (1 if e4 else 2) + M * N * out.element_size() + (M * N * 4 if resid is not None else 0)
    tag = f"{M}x{N}x{K}{'r' if resid is not None else ''}{'b' if bias is not None else ''}:{out_dtype}:ws"
    if e4:
        wq, sc, mode = w_frag
        _launch("gemm", lambda: lib().csu_gemm_ws_e4m3(M, N, K, ptr(x2), x2.stride(0), ptr(wq), ptr(sc), mode, ptr(bias),
                                                       ptr(resid), dtype_code(out), ptr(out), stream_ptr(x2.device)),
                2 * M * N * K, nb, prec="bf16", tag=tag + "8")
        return out
    _launch("gemm", lambda: lib().csu_gemm_ws(M, N, K, ptr(x2), x2.stride(0), ptr(w_frag), ptr(bias), ptr(resid),
                                              dtype_code(out), ptr(out), stream_ptr(x2.device)),
            2 * M * N * K, nb, prec="bf16", tag=tag)
    return out


# the fp8 weight format's qkv / proj Linears (and their input gradients) stream e4m3 weight fragments
# in csu_gemm_ws_e4m3 (False: the bf16 fragments of the exact dequantised weights, same results)
FP8_WS = os.environ.get("CSU_FP8_WS", "1") != "0"


def _ws_operand(weight, transposed: bool = False):
    """The weight-streaming GEMM operand of a cached 2-D weight: the e4m3 fragments (frag8, scales,
    scale_mode) in the fp8 weight format, else the bf16 fragments of the cast cache, or None."""
    if FP8_WS and _ACTIVE_FP8 is not None:
        # the fp8 format makes no bf16 fragments (CSWinTransformer.forward skips refresh_frag)
        return _ACTIVE_FP8.get_frag8(weight, transposed)
    if _ACTIVE_CACHE is None:
        return None
    return _ACTIVE_CACHE.get_frag_t(weight) if transposed else _ACTIVE_CACHE.get_frag(weight)


def _ws_ok(M, N, K, out_dtype, resid=False) -> bool:
    return USE_GEMM_WS and bool(lib().csu_gemm_ws_supported(M, N, K, int(resid), dtype_code_of(out_dtype)))


def dtype_code_of(dt) -> int:
    """csu dtype code of a torch dtype; -1 for dtypes the kernels cannot write (csu_gemm_ws_supported
    then rejects the shape and the caller takes gemm4, whose own checks raise CsuError)."""
    return CSU_F32 if dt == torch.float32 else CSU_BF16 if dt == torch.bfloat16 else -1


# ---------------------------------------------------------------------------------------------
# Weight gradients on a side stream.  dW = dY^T X of a Linear is off the backward critical path
# (nothing in the rest of backward reads it), so in eager steps it runs on a second HIP stream
# overlapped with the input-gradient chain.  Fork: the side stream waits on the launching stream;
# inputs are record_stream'ed.  Join: the launching stream waits on every side event at the end of
# backward (autograd final callback), before the optimizer or any user code can read .grad.
#
# The returned gradient is handed to autograd on the launching stream while the side kernel may
# still be writing it, so the side stream is only used when nothing reads it before the join:
# AccumulateGrad then just steals the tensor.  That holds when the parameter has no .grad yet
# (zero_grad(set_to_none=True)), no tensor hooks, and no post-accumulate hooks other than
# csu.dist.GradAllReduce's (which order their reads after side_stream()).  Gradient accumulation
# (an existing .grad: AccumulateGrad adds in place on the launching stream), DDP and user hooks run
# the weight gradient inline.  A HIP-graph capture runs it inline too: inside a graph the side
# stream measured slower (1075 vs 1090 img/s, 3 A/B pairs at 512x512) and its replays were not
# bitwise reproducible at 512x512 (tools/det_graph.py DIAG=...).
# SIDE_WGRAD = False (tests, bench ledger) disables the side stream in eager steps as well.
# ---------------------------------------------------------------------------------------------
SIDE_WGRAD = True
# diagnostics of the side-stream-in-graph nondeterminism (tools/det_graph.py): allow the side
# stream under capture / join every side launch at once
_SIDE_IN_GRAPH = False
_SIDE_JOIN_NOW = False
# convolutions of inputs with C % 8 != 0 (the 3-channel image) zero-pad the channels to 8
PAD_CHANNELS = True
_SIDE_STREAMS = {}
_SIDE_PENDING = []
_SIDE_JOIN_QUEUED = [False]
# set by csu.dist.GradAllReduce: its hooks order their reads after the side stream (side_stream()),
# so side-stream weight gradients stay on under multi-rank training with it (not with DDP)
_DIST_SAFE = [False]


def _leaf(p):
    while p is not None and getattr(p, "_base", None) is not None:
        p = p._base
    return p


# Gradient destinations registered by csu.dist.GradAllReduce: id(param) -> (flat fp32 bucket, element
# offset).  An op whose weight gradients land in one buffer (a Linear's [dW | db], a LayerNorm's
# [dgamma | dbeta], a block's LePE weights) writes them straight into the bucket when the params are
# adjacent there: AccumulateGrad steals the (fresh) view, and the reducer has nothing to pack.
_GRAD_DEST: dict = {}


def _grad_dest(params) -> Optional[torch.Tensor]:
    """One flat fp32 slice holding the gradients of ``params`` in this order (their bucket views), or
    None.  Only for parameters without a .grad (nothing to accumulate into)."""
    if not _GRAD_DEST:
        return None
    flat0, off0, n = None, 0, 0
    for p in params:
        p = _leaf(p)
        e = _GRAD_DEST.get(id(p)) if p is not None else None
        # a parameter used by several ops of this graph (shared weights): every call's backward would
        # write the same bucket memory while the engine still holds an earlier call's gradient as an
        # alias of it -- such gradients go to fresh buffers and are summed by the engine.  The entry's
        # weak reference must be p itself (an id reused by a new object is not registered).
        if e is None or e[0]() is not p or p.grad is not None or _uses(p) > 1:
            return None
        _, flat, off = e
        if flat0 is None:
            flat0, off0 = flat, off
        elif flat is not flat0 or off != off0 + n:
            return None
        n += p.numel()
    return None if flat0 is None else flat0[off0:off0 + n]


def _param_safe(p) -> bool:
    """True when no reader of p.grad can run before the end-of-backward join (see above)."""
    # the end-of-backward flush resets the forward use counts (_USES): queue it from every backward
    # that consults them, not only from deferring ones (a model with no deferrable LayerNorm / Linear /
    # LePE work -- the plain UNet -- would otherwise keep counting across steps, and from its second
    # step every conv weight would look shared and lose the side stream)
    _queue_flush()
    p = _leaf(p)
    if p is None:
        return True
    if p.grad is not None or p._backward_hooks or _uses(p) > 1:
        return False   # (shared weights: the engine would sum the side-stream gradient before the join)
    hooks = getattr(p, "_post_accumulate_grad_hooks", None)
    return not hooks or _DIST_SAFE[0]


def _side_ok(t: torch.Tensor, *dtypes, params=()) -> bool:
    if not (SIDE_WGRAD and t.is_cuda) or any(d not in (None, torch.float32) for d in dtypes):
        return False
    if torch.cuda.is_current_stream_capturing() and not _SIDE_IN_GRAPH:
        return False
    if not all(_param_safe(p) for p in params):
        return False
    dist = torch.distributed
    return _DIST_SAFE[0] or not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)


def side_stream(device) -> Optional["torch.cuda.Stream"]:
    """The side stream weight gradients of `device` are computed on (None before the first)."""
    return _SIDE_STREAMS.get(device)


def join_side_streams():
    """Make each launching stream wait for the side-stream weight gradients it forked."""
    for main, ev in _SIDE_PENDING:
        main.wait_event(ev)
    _SIDE_PENDING.clear()
    _SIDE_JOIN_QUEUED[0] = False
    _check_late(_LATE_SIDE)


def _side_run(fn, *inputs):
    dev = inputs[0].device
    main = torch.cuda.current_stream(dev)
    side = _SIDE_STREAMS.get(dev)
    if side is None:
        side = _SIDE_STREAMS[dev] = torch.cuda.Stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        out = fn()
    for t in inputs:
        t.record_stream(side)
    ev = torch.cuda.Event()
    ev.record(side)
    if _SIDE_JOIN_NOW:
        main.wait_event(ev)
        return out
    _SIDE_PENDING.append((main, ev))
    if not _SIDE_JOIN_QUEUED[0]:
        torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
        _SIDE_JOIN_QUEUED[0] = True
    return out


def wgrad_maybe_side(dy2: torch.Tensor, x2: torch.Tensor, wdt, bdt, params=()):
    """linear_wgrad on the side stream when allowed (fp32 master weights, see above), else inline."""
    dest = None
    if (dy2.dtype in (torch.bfloat16, torch.float32) and len(params) == 2 and params[1] is not None and wdt is not None
            and bdt is not None):
        dest = _grad_dest(params)                 # [dW | db] straight into a GradAllReduce bucket
    if _side_ok(dy2, wdt, bdt, params=params):
        r = _side_run(lambda: linear_wgrad(dy2, x2, out=dest), dy2, x2)
        _late(params, r, side=True)
        return r
    defer = _wgrad_deferrable(dy2, wdt, bdt, params)
    r = linear_wgrad(dy2, x2, out=dest, defer=defer)
    if defer:
        _late(params, r)
    return r


# csu_gemm_ex (fused bias / GELU / GELU' / residual token GEMM) runs every bf16 nn.Linear forward
# and input-gradient GEMM, csu_gemm_f32 every fp32 one; there is no vendor-GEMM path.
def _gemm_ok(*dims):
    return all(d % 8 == 0 for d in dims)


def _weight_t(w, wc):
    """(K, N) bf16 transpose of the (N, K) weight w: the cast cache's copy, else made here."""
    wt = _ACTIVE_CACHE.get_t(w, torch.bfloat16) if _ACTIVE_CACHE is not None else None
    return wt if wt is not None else wc.t().contiguous()


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, cd, wc, odt=None):
        xc = x if x.dtype == cd else x.to(cd)
        if wc is None:
            wc = weight.to(cd)
        K, N = xc.shape[-1], wc.shape[0]
        require_device(xc)
        ctx.fast = cd == torch.bfloat16 and _gemm_ok(K, N)
        ctx.f32 = False
        wt = None
        ctx.wtf = None
        if ctx.fast:
            x2 = xc.reshape(-1, K).contiguous()
            bf = None if bias is None else bias.detach().float().contiguous()
            wf = _ws_operand(weight)
            if wf is not None and _ws_ok(x2.shape[0], N, K, odt or cd):
                y = gemm_ws(x2, wf, N, odt or cd, bias=bf)
            else:
                y = gemm(x2, wc, False, odt or cd, bias=bf)
            y = y.view(*xc.shape[:-1], N)
            wt = _weight_t(weight, wc)
            ctx.wtf = _ws_operand(weight, True)
        elif cd == torch.float32 and K % 4 == 0 and N % 4 == 0:
            # fp32 path (no autocast, BASELINE config 2): csu fp32 MFMA GEMM, bias in its epilogue
            x2 = xc.reshape(-1, K).contiguous()
            y = gemm_f32(0, x2, wc.contiguous(), x2.shape[0], N, K,
                         bias=None if bias is None else bias.detach().contiguous()).view(*xc.shape[:-1], N)
            ctx.f32 = True
        else:
            raise CsuError(f"linear: no csu GEMM for {cd} with in/out features {K}/{N} (bf16 needs multiples "
                           f"of 8, fp32 multiples of 4)")
        ctx.save_for_backward(xc, wt if ctx.fast else wc)
        ctx.meta = (x.dtype, weight.dtype, None if bias is None else bias.dtype)
        ctx.params = (weight, bias)
        _note_use(ctx, *ctx.params)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors          # wc: (K, N) transpose on the fast path
        xdt, wdt, bdt = ctx.meta
        K, N = xc.shape[-1], dy.shape[-1]
        if dy.dtype != wc.dtype and wc.dtype == torch.bfloat16:
            dy2 = _bf16_of(dy).reshape(-1, N)   # the junction's bf16 copy when the gradient carries one
        else:
            dy2 = dy.reshape(-1, N)
            if dy2.dtype != wc.dtype:
                dy2 = dy2.to(wc.dtype)
        dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if ctx.fast:
                odt = xdt if xdt in (torch.float32, torch.bfloat16) else wc.dtype
                if ctx.wtf is not None and _ws_ok(dy2.shape[0], K, N, odt):
                    dx = gemm_ws(dy2, ctx.wtf, K, odt).view(xc.shape)
                else:
                    dx = gemm(dy2, wc, False, odt).view(xc.shape)
            else:
                dx = gemm_f32(1, dy2, wc.contiguous(), dy2.shape[0], K, N).view(xc.shape)
            if dx.dtype != xdt:
                dx = dx.to(xdt)
        vec = 16 // dy2.element_size()
        if N % vec == 0 and K % vec == 0 and dy2.dtype in (torch.float32, torch.bfloat16):
            dwf, dbf = wgrad_maybe_side(dy2, xc.reshape(-1, K), wdt if ctx.needs_input_grad[1] else None,
                                        bdt if ctx.needs_input_grad[2] else None, params=ctx.params)
            if ctx.needs_input_grad[1]:
                dw = dwf.to(wdt)
            if bdt is not None and ctx.needs_input_grad[2]:
                db = dbf.to(bdt)
            return dx, dw, db, None, None, None
        if ctx.needs_input_grad[1] or (bdt is not None and ctx.needs_input_grad[2]):
            # unreachable with the forward's width checks; no vendor-BLAS fallback
            raise CsuError(f"linear backward: no csu weight-gradient kernel for {dy2.dtype} with in/out features "
                           f"{K}/{N}")
        return dx, dw, db, None, None, None


class _SharedCastFn(torch.autograd.Function):
    """One bf16 copy of an fp32 activation handed to two consumers (the encoder skip x1/x2/x3 feeds
    both Merge_Block's conv and the decoder's concat_linear, cswin:530-545 / 568-592).  Autocast
    casts it once per consumer; here it is cast once, and the two bf16 input gradients are summed
    in fp32 as autocast's two cast nodes would."""

    @staticmethod
    def forward(ctx, x, dtype):
        ctx.xdt = x.dtype
        if x.dtype == dtype:
            # already in the compute dtype: a fork whose two gradients are summed by one csu pass
            # (the bf16 norm_up output feeding CARAFE4's down conv and the head, cswin:674-682)
            return x.view_as(x), x.view_as(x)
        if x.is_cuda and dtype == torch.bfloat16 and x.dtype == torch.float32 and x.numel() % 8 == 0:
            xc = x.contiguous()
            y = torch.empty(x.shape, dtype=dtype, device=x.device)
            n = x.numel()
            # the bare bf16 cast runs csu_grad_join's kernel: one ledger name per kernel (rocprof groups)
            _launch("grad_join", lambda: lib().csu_grad_join(n, CSU_F32, ptr(xc), 0, None, None, ptr(y),
                                                             stream_ptr(x.device)), 0, n * 6, prec="f32")
        else:
            y = x.to(dtype)
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, g1, g2):
        if g1 is None and g2 is None:
            return None, None
        return grad_join(g1, g2, ctx.xdt), None


def grad_join(g1: Optional[torch.Tensor], g2: Optional[torch.Tensor], dtype: torch.dtype) -> torch.Tensor:
    """g1 + g2 in `dtype` (either may be None).  fp32 result on the device: one csu_grad_join pass
    that also writes the bf16 copy the upstream GEMM backward consumes (attached as ``_csu_bf16``,
    see _bf16_of) -- instead of autograd's cast, add and the consumer's cast."""
    a, b = (g1, g2) if g1 is not None else (g2, None)
    if dtype == torch.bfloat16 and a.is_cuda and a.numel() % 8 == 0 and b is not None:
        # bf16 sum (fp32 add, one rounding -- as autograd's bf16 add) in one pass
        a, b = a.contiguous(), b.contiguous()
        outb = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device)
        n = a.numel()
        _launch("grad_join", lambda: lib().csu_grad_join(n, dtype_code(a), ptr(a), dtype_code(b), ptr(b), None, ptr(outb),
                                                         stream_ptr(a.device)),
                n, n * (esize(a) + esize(b) + 2), prec="bf16")
        return outb
    if dtype != torch.float32 or not a.is_cuda or a.numel() % 8:
        g = a.to(dtype)
        return g.add_(b) if b is not None else g
    a = a.contiguous()
    b = b.contiguous() if b is not None else None
    out = torch.empty(a.shape, dtype=torch.float32, device=a.device)
    outb = torch.empty(a.shape, dtype=torch.bfloat16, device=a.device)
    n = a.numel()
    _launch("grad_join", lambda: lib().csu_grad_join(n, dtype_code(a), ptr(a), dtype_code(b) if b is not None else 0,
                                                     ptr(b), ptr(out), ptr(outb), stream_ptr(a.device)),
            n, n * (esize(a) + (esize(b) if b is not None else 0) + 6), prec="f32")
    out._csu_bf16 = outb
    return out


class _BCELossFn(torch.autograd.Function):
    """nn.BCELoss() (mean) on fp32 probabilities (cswin:935): csu_bce_loss_fwd (fixed-order two-pass
    sum) and csu_bce_loss_bwd (torch's clamps), 3 launches instead of torch's 5.  with_stats: the
    same pass also returns the reference loop's per-step segmentation sums (cswin:789-795:
    sum(pred * t), sum(pred), sum(t) of pred = p > 0.5) as a non-differentiable (3,) tensor."""

    @staticmethod
    def forward(ctx, p, t, with_stats: bool = False):
        p, t = p.contiguous(), t.contiguous()
        n = p.numel()
        loss = torch.empty((), dtype=torch.float32, device=p.device)
        stats = torch.empty(3, dtype=torch.float32, device=p.device) if with_stats else None
        nws = lib().csu_bce_loss_workspace(n)
        ws = torch.empty(nws // 4, dtype=torch.float32, device=p.device)
        if with_stats:
            _launch("bce_loss", lambda: lib().csu_bce_loss_fwd_stats(n, ptr(p), ptr(t), ptr(loss), ptr(stats), ptr(ws), nws,
                                                                     stream_ptr(p.device)), 12 * n, 8 * n, prec="f32")
        else:
            _launch("bce_loss", lambda: lib().csu_bce_loss_fwd(n, ptr(p), ptr(t), ptr(loss), ptr(ws), nws,
                                                               stream_ptr(p.device)), 8 * n, 8 * n, prec="f32")
        ctx.save_for_backward(p, t)
        if with_stats:
            ctx.mark_non_differentiable(stats)
            return loss, stats
        return loss

    @staticmethod
    def backward(ctx, g, *unused):
        p, t = ctx.saved_tensors
        g = g.float().contiguous()
        dp = torch.empty_like(p)
        n = p.numel()
        _launch("bce_loss_bwd", lambda: lib().csu_bce_loss_bwd(n, ptr(p), ptr(t), ptr(g), ptr(dp), stream_ptr(p.device)),
                6 * n, 12 * n, prec="f32")
        return dp, None, None


def bce_loss(prob: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean binary cross-entropy of fp32 device probabilities (see _BCELossFn)."""
    require_device(prob, target)
    if prob.dtype != torch.float32 or target.dtype != torch.float32 or prob.shape != target.shape:
        raise ValueError("bce_loss: fp32 probabilities and targets of one shape")
    return _BCELossFn.apply(prob, target)


def bce_loss_stats(prob: torch.Tensor, target: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(bce_loss, (sum(pred * t), sum(pred), sum(t)) of pred = prob > 0.5) in one pass."""
    require_device(prob, target)
    if prob.dtype != torch.float32 or target.dtype != torch.float32 or prob.shape != target.shape:
        raise ValueError("bce_loss: fp32 probabilities and targets of one shape")
    return _BCELossFn.apply(prob, target, True)


def augment_batch(images: torch.Tensor, masks: torch.Tensor, params) -> Tuple[torch.Tensor, torch.Tensor]:
    """csu_augment_batch: uint8 (B, S, S, 3) images / (B, S, S) masks on the device, params per image
    (hflip, vflip, clockwise quarter turns, top, left, crop_h, crop_w) -> fp32 (B, 3, S, S) and
    (B, 1, S, S) in [0, 1] (cswin:20-87 + 166-173)."""
    require_device(images, masks)
    if images.dtype != torch.uint8 or masks.dtype != torch.uint8:
        raise ValueError("augment_batch: uint8 images and masks")
    B, S = images.shape[0], images.shape[1]
    p = torch.tensor([list(map(int, q)) for q in params], dtype=torch.int32)
    if tuple(p.shape) != (B, 7):
        raise ValueError("augment_batch: one 7-value parameter tuple per image")
    if ((p[:, 3] < 0) | (p[:, 4] < 0) | (p[:, 5] < 1) | (p[:, 6] < 1) | (p[:, 3] + p[:, 5] > S)
            | (p[:, 4] + p[:, 6] > S) | (p[:, 2] < 0) | (p[:, 2] > 3)).any():
        raise ValueError("augment_batch: crop outside the image or bad rotation")
    pd = p.to(images.device, non_blocking=True)
    img = images.contiguous()
    msk = masks.contiguous()
    out = torch.empty(B, 3, S, S, dtype=torch.float32, device=images.device)
    om = torch.empty(B, 1, S, S, dtype=torch.float32, device=images.device)
    _launch("augment", lambda: lib().csu_augment_batch(B, S, ptr(img), ptr(msk), ptr(pd), ptr(out), ptr(om),
                                                       stream_ptr(images.device)),
            0, B * S * S * (4 + 16), prec="f32")
    return out, om


def shared_cast(x: torch.Tensor, dtype: torch.dtype):
    """(xc, xc) -- the same `dtype` copy of x for two consumers (see _SharedCastFn)."""
    return _SharedCastFn.apply(x, dtype)


def _concat_wgrad(dy2, a2, b2, defer: bool = False, dest=None):
    """(dW (N, Ca + Cb), db) of the concat Linear.  ``defer``: both halves join the end-of-backward
    grouped launch and are joined into dW (returned now) after it (_WG_POST); ``dest``: the params'
    [dW | db] gradient-bucket slice (_grad_dest) the join writes."""
    dwa, db = linear_wgrad(dy2, a2, defer=defer)
    dwb, _ = linear_wgrad(dy2, b2, defer=defer)
    if not defer:
        return torch.cat([dwa, dwb], 1), db
    # the join holds only the base buffers: the returned views must be sole references, so that
    # AccumulateGrad steals them as .grad instead of copying them now (before the join)
    N, K = dwa.shape[0], dwa.shape[1] + dwb.shape[1]
    if dest is None:
        buf = torch.empty(N * K, dtype=torch.float32, device=dy2.device)
        _WG_POST.append(lambda: torch.cat([dwa, dwb], 1, out=buf.view(N, K)))
        return buf.view(N, K), db

    def join():
        torch.cat([dwa, dwb], 1, out=dest[:N * K].view(N, K))
        dest[N * K:].copy_(db)
    _WG_POST.append(join)
    return dest[:N * K].view(N, K), dest[N * K:]


class _ConcatLinearFn(torch.autograd.Function):
    """Linear(cat([a, b], -1)) without the cat (the decoder's concat_linear, cswin:568/581/592):
    y = a @ W[:, :Ca]^T + bias, then y += b @ W[:, Ca:]^T, two bf16 GEMMs (fp32 out, the second
    with the residual epilogue) reading the weight halves in place (ldb = Ca + Cb).  The
    reference path writes the fp32 concatenation and casts it to bf16 again (2176 -> 1408 B per
    token at C = 64); backward: two input-gradient GEMMs into the separate halves (no strided
    slices of a concatenated gradient) and two weight-gradient GEMMs."""

    @staticmethod
    def forward(ctx, a, b, weight, bias, wc):
        Ca, Cb, N = a.shape[-1], b.shape[-1], weight.shape[0]
        a2 = a.reshape(-1, Ca).contiguous()
        b2 = b.reshape(-1, Cb).contiguous()
        bf = bias.detach().float().contiguous()
        y1 = gemm(a2, wc[:, :Ca], False, torch.float32, bias=bf)
        y = gemm(b2, wc[:, Ca:], False, torch.float32, resid=y1)
        ctx.save_for_backward(a2, b2, _weight_t(weight, wc))
        ctx.meta = (a.shape, b.shape, a.dtype, b.dtype, weight.dtype, bias.dtype)
        ctx.params = (weight, bias)
        _note_use(ctx, *ctx.params)
        return y.view(*a.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        a2, b2, wt = ctx.saved_tensors     # wt: (Ca + Cb, N)
        ashape, bshape, adt, bdt_in, wdt, bdt = ctx.meta
        Ca = a2.shape[1]
        dy2 = _bf16_of(dy).reshape(-1, dy.shape[-1]).contiguous()
        da = gemm(dy2, wt[:Ca], False, adt).view(ashape) if ctx.needs_input_grad[0] else None
        db_in = gemm(dy2, wt[Ca:], False, bdt_in).view(bshape) if ctx.needs_input_grad[1] else None
        if _wgrad_deferrable(dy2, wdt, bdt, ctx.params):
            dw, dbias = _concat_wgrad(dy2, a2, b2, defer=True, dest=_grad_dest(ctx.params))
            _late(ctx.params, (dw, dbias))
        elif _side_ok(dy2, wdt, bdt, params=ctx.params):
            dw, dbias = _side_run(lambda: _concat_wgrad(dy2, a2, b2), dy2, a2, b2)
            _late(ctx.params, (dw, dbias), side=True)
        else:
            dw, dbias = _concat_wgrad(dy2, a2, b2)
        return da, db_in, dw.to(wdt), dbias.to(bdt), None


def concat_linear(a: torch.Tensor, b: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    """fp32 Linear(cat([a, b], -1)) for bf16 a, b under bf16 autocast (see _ConcatLinearFn); other
    inputs take the reference form (cat, then linear with an fp32 output)."""
    Ca, Cb, N = a.shape[-1], b.shape[-1], weight.shape[0]
    if (a.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and a.dtype == b.dtype == torch.bfloat16
            and bias is not None and _gemm_ok(Ca, Cb, N)):
        wc = _ACTIVE_CACHE.get(weight, torch.bfloat16) if _ACTIVE_CACHE is not None else None
        if wc is None:
            wc = weight.to(torch.bfloat16)
        with torch.autocast("cuda", enabled=False):
            return _ConcatLinearFn.apply(a, b, weight, bias, wc)
    return linear(torch.cat([a, b], -1), weight, bias, out_dtype=torch.float32 if a.is_cuda else None)


class _LinearResidualFn(torch.autograd.Function):
    """res + x @ W^T + b in one csu_gemm (fp32 out): proj + residual of CSWinBlock (cswin:366-367)."""

    @staticmethod
    def forward(ctx, res, x, weight, bias, wc, ln=None):
        res2 = res.float().contiguous().view(-1, res.shape[-1])
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        M, K, N = x2.shape[0], x2.shape[1], wc.shape[0]
        bf = bias.detach().float().contiguous()
        wf = _ws_operand(weight)
        if (ln is not None and wf is not None and USE_GEMM_WS and K == N
                and lib().csu_gemm_ws_ln_supported(M, N, K)):
            # + norm2 in the epilogue (csu_gemm_ws_ln), handed to the block's layer_norm_fork
            gam, bet, eps = ln
            gf, bf_ = gam.detach().float().contiguous(), bet.detach().float().contiguous()
            y = torch.empty(M, N, dtype=torch.float32, device=x2.device)
            h = torch.empty(M, N, dtype=torch.bfloat16, device=x2.device)
            mean = torch.empty(M, dtype=torch.float32, device=x2.device)
            rstd = torch.empty(M, dtype=torch.float32, device=x2.device)
            if isinstance(wf, tuple):   # e4m3 weight fragments (fp8 format)
                wq, sc, _ = wf
                _launch("gemm", lambda: lib().csu_gemm_ws_ln_e4m3(M, N, ptr(x2), K, ptr(wq), ptr(sc), ptr(bf), ptr(res2),
                                                                  ptr(y), ptr(gf), ptr(bf_), float(eps), ptr(h), ptr(mean),
                                                                  ptr(rstd), stream_ptr(x2.device)),
                        2 * M * N * K + 8 * M * N, M * K * 2 + N * K + M * N * (4 + 4 + 2) + 8 * M,
                        tag=f"{M}x{N}x{K}rbln:ws8")
            else:
                _launch("gemm", lambda: lib().csu_gemm_ws_ln(M, N, ptr(x2), K, ptr(wf), ptr(bf), ptr(res2), ptr(y), ptr(gf),
                                                             ptr(bf_), float(eps), ptr(h), ptr(mean), ptr(rstd),
                                                             stream_ptr(x2.device)),
                        2 * M * N * K + 8 * M * N, M * K * 2 + N * K * 2 + M * N * (4 + 4 + 2) + 8 * M,
                        tag=f"{M}x{N}x{K}rbln:ws")
            _LN_STASH[0] = (gam, bet, float(eps), h, mean, rstd)
        elif wf is not None and _ws_ok(M, N, K, torch.float32, resid=True):
            y = gemm_ws(x2, wf, N, torch.float32, bias=bf, resid=res2)
        else:
            y = gemm(x2, wc, False, torch.float32, bias=bf, resid=res2)
        ctx.save_for_backward(x2, _weight_t(weight, wc))
        ctx.wtf = _ws_operand(weight, True)
        ctx.meta = (res.dtype, x.shape, weight.dtype, bias.dtype)
        ctx.params = (weight, bias)
        _note_use(ctx, *ctx.params)
        return y.view(res.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, wt = ctx.saved_tensors
        rdt, xshape, wdt, bdt = ctx.meta
        dyb = _bf16_of(dy).view(-1, dy.shape[-1])
        M, N, K = dyb.shape[0], dyb.shape[1], x2.shape[1]
        if ctx.wtf is not None and _ws_ok(M, K, N, torch.bfloat16):
            dx = gemm_ws(dyb.contiguous(), ctx.wtf, K, torch.bfloat16).view(xshape)
        else:
            dx = gemm(dyb, wt, False, torch.bfloat16).view(xshape)
        dw, db = wgrad_maybe_side(dyb, x2, wdt, bdt, params=ctx.params)
        return dy.to(rdt), dx, dw.to(wdt), db.to(bdt), None, None


class MlpDrop:
    """Dropout of one Mlp + DropPath residual (Mlp.drop cswin:188/193/195, drop_path cswin:368):
    snapshot, hidden / output sites, p, and the per-sample DropPath scale (or None)."""

    def __init__(self, snap, site_h: int, site_o: int, p: float, row_scale=None, rows_per_sample: int = 1):
        self.snap, self.site_h, self.site_o, self.p = snap, int(site_h), int(site_o), float(p)
        self.row_scale, self.rps = row_scale, int(rows_per_sample)

    def c_struct(self):
        d = _lib.MlpDropout()
        d.rng = None if self.snap is None else self.snap.data_ptr()
        d.site_hidden, d.site_out, d.p = self.site_h, self.site_o, self.p
        d.row_scale = None if self.row_scale is None else self.row_scale.data_ptr()
        d.rows_per_sample = self.rps
        return d

    def out_grad(self, dy2, dt):
        """dy of the dropped, DropPath-scaled fc2 output -> gradient of fc2's output (dtype dt)."""
        dz = torch.empty(dy2.shape, dtype=dt, device=dy2.device)
        _dropout_launch(dy2, None, dz, self.row_scale, self.rps, self.snap, self.site_o, self.p)
        return dz


class _MlpResidualFn(torch.autograd.Function):
    """res + fc2(gelu(fc1(x))) (Mlp cswin:180-196 + residual cswin:368) as two csu_gemm_ex calls:
    fc1's epilogue writes the pre-activation h and gelu(h) (bf16); fc2 adds bias and the residual
    in its epilogue; backward fuses GELU' into the fc2 input-gradient epilogue.

    With ``drop`` (MlpDrop): g is dropped (hidden site) before fc2, and fc2's bf16 output goes
    through one dropout pass (output site, DropPath scale, residual); the backward applies the
    output mask to dy, and the hidden mask after the GELU' epilogue (the two commute)."""

    @staticmethod
    def forward(ctx, res, x, w1, b1, w2, b2, w1c, w2c, drop):
        C = res.shape[-1]
        res2 = res.float().contiguous().view(-1, C)
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        h, g = gemm(x2, w1c, False, torch.bfloat16, bias=b1.detach().float().contiguous(), gelu_out=True)
        if drop is None:
            y = gemm(g, w2c, False, torch.float32, bias=b2.detach().float().contiguous(), resid=res2)
        else:
            gd = torch.empty_like(g)
            _dropout_launch(g, None, gd, None, 1, drop.snap, drop.site_h, drop.p)
            g = gd
            z = gemm(g, w2c, False, torch.bfloat16, bias=b2.detach().float().contiguous())
            y = torch.empty_like(res2)
            _dropout_launch(z, res2, y, drop.row_scale, drop.rps, drop.snap, drop.site_o, drop.p)
        ctx.save_for_backward(x2, h, g, _weight_t(w1, w1c), _weight_t(w2, w2c))
        ctx.meta = (res.dtype, x.shape, w1.dtype, b1.dtype, w2.dtype, b2.dtype)
        ctx.params = (w1, b1, w2, b2)
        _note_use(ctx, *ctx.params)
        ctx.drop = drop
        return y.view(res.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, h, g, w1t, w2t = ctx.saved_tensors
        rdt, xshape, w1dt, b1dt, w2dt, b2dt = ctx.meta
        drop = ctx.drop
        if drop is None:
            dyb = _bf16_of(dy).view(-1, dy.shape[-1])
        else:
            dyb = drop.out_grad(dy.reshape(-1, dy.shape[-1]).contiguous(), torch.bfloat16)
        dh = gemm(dyb, w2t, False, torch.bfloat16, gelu_aux=h)         # (dY W2) * gelu'(h)
        if drop is not None:
            dhm = torch.empty_like(dh)
            _dropout_launch(dh, None, dhm, None, 1, drop.snap, drop.site_h, drop.p)
            dh = dhm
        dw2, db2 = wgrad_maybe_side(dyb, g, w2dt, b2dt, params=ctx.params[2:])
        dx = gemm(dh, w1t, False, torch.bfloat16).view(xshape)
        dw1, db1 = wgrad_maybe_side(dh, x2, w1dt, b1dt, params=ctx.params[:2])
        return dy.to(rdt), dx, dw1.to(w1dt), db1.to(b1dt), dw2.to(w2dt), db2.to(b2dt), None, None, None


def _weight_bf16(w):
    wc = _ACTIVE_CACHE.get(w, torch.bfloat16) if _ACTIVE_CACHE is not None else None
    return wc if wc is not None else w.detach().to(torch.bfloat16).contiguous()


def fused_ok(x: torch.Tensor, *dims) -> bool:
    """True when the bf16 fused-GEMM path applies (CUDA, autocast bf16, 16-B aligned dims)."""
    return (x.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and _gemm_ok(*dims))


FUSE_PROJ_LN = os.environ.get("CSU_FUSE_PROJ_LN", "1") != "0"   # norm2 in the proj + residual epilogue (csu_gemm_ws_ln)


def linear_residual(res, x, weight, bias, ln_next=None):
    """res + x @ W^T + b (fp32).  ``ln_next`` ((weight, bias, eps) of the LayerNorm that reads the
    result, CSWinBlock's norm2): computed in the same launch where gemm_ws has the shape and attached
    to the output for layer_norm_fork (``_csu_ln``)."""
    ln = ln_next if (FUSE_PROJ_LN and ln_next is not None and ln_next[0].dtype == torch.float32
                     and ln_next[0].numel() == weight.shape[0]) else None
    _LN_STASH[0] = None
    with torch.autocast("cuda", enabled=False):
        out = _LinearResidualFn.apply(res, x, weight, bias, _weight_bf16(weight), ln)
    if ln is not None:
        _attach_ln(out)
    return out


def _mlp_desc(drop: Optional[MlpDrop], rpi: int):
    """csu_mlp_dropout of a fused-Mlp launch: the dropout / DropPath of ``drop``, or none (p = 0);
    rows_per_sample = rows per image either way (DropPath's sample and the kernel's chunk rotation)."""
    if drop is not None:
        d = drop.c_struct()
        if drop.row_scale is None:
            d.rows_per_sample = rpi
        return d
    d = _lib.MlpDropout()
    d.p, d.rows_per_sample = 0.0, rpi
    return d


class _MlpFusedFn(torch.autograd.Function):
    """res + fc2(gelu(fc1(x))) (Mlp cswin:180-196 + residual cswin:368) in ONE csu_mlp_fwd launch
    (the 4C hidden layer never reaches HBM).  Backward: one csu_mlp_bwd launch recomputes h and
    writes dh, g = gelu(h) and dx; then the two weight gradients.  ``drop`` (MlpDrop): hidden and
    output dropout plus the DropPath scale inside the same two launches (csu_mlp_fwd_dp /
    csu_mlp_bwd_dp), the output mask applied to dy by one dropout pass first."""

    @staticmethod
    def forward(ctx, res, x, w1, b1, w2, b2, w1c, w2c, drop, ln=None):
        C = x.shape[-1]
        res2 = res.float().contiguous().view(-1, C)
        x2 = x.reshape(-1, C).contiguous()
        b1f = b1.detach().float().contiguous()
        y = torch.empty_like(res2)
        M = x2.shape[0]
        b2f = b2.detach().float().contiguous()
        rpi = x.shape[1] if x.dim() == 3 else M   # rows per image: the kernel's hidden-chunk rotation
        dd = ctypes.byref(_mlp_desc(drop, rpi))
        if ln is not None:
            # + the next block's norm1 on the output (csu_mlp_fwd_ln); handed to its layer_norm_fork
            gam, bet, eps = ln
            gf, bf_ = gam.detach().float().contiguous(), bet.detach().float().contiguous()
            h1 = torch.empty(M, C, dtype=torch.bfloat16, device=x2.device)
            mean = torch.empty(M, dtype=torch.float32, device=x2.device)
            rstd = torch.empty(M, dtype=torch.float32, device=x2.device)
            _launch("mlp_fwd", lambda: lib().csu_mlp_fwd_ln(M, C, ptr(x2), ptr(w1c), ptr(b1f), ptr(w2c), ptr(b2f), ptr(res2),
                                                            ptr(y), dd, ptr(gf), ptr(bf_), float(eps), ptr(h1), ptr(mean),
                                                            ptr(rstd), stream_ptr(x2.device)),
                    16 * M * C * C + 8 * M * C, M * C * (2 + 4 + 4 + 2) + 16 * C * C + 8 * M)
            _LN_STASH[0] = (gam, bet, float(eps), h1, mean, rstd)
        else:
            _launch("mlp_fwd", lambda: lib().csu_mlp_fwd_dp(M, C, ptr(x2), ptr(w1c), ptr(b1f), ptr(w2c), ptr(b2f), ptr(res2),
                                                            ptr(y), dd, stream_ptr(x2.device)),
                    16 * M * C * C, M * C * (2 + 4 + 4) + 16 * C * C)
        ctx.drop = drop
        ctx.rpi = rpi
        ctx.save_for_backward(x2, w1c, b1f, w2c)
        ctx.meta = (res.dtype, x.shape, w1.dtype, b1.dtype, w2.dtype, b2.dtype)
        ctx.params = (w1, b1, w2, b2)
        _note_use(ctx, *ctx.params)
        return y.view(res.shape)

    @staticmethod
    def backward(ctx, dy):
        rdt, xshape, w1dt, b1dt, w2dt, b2dt = ctx.meta
        x2, w1c, b1f, w2c = ctx.saved_tensors
        M, C = x2.shape
        drop = ctx.drop
        if drop is None:
            dyb = _bf16_of(dy).view(-1, C)
        else:
            dyb = drop.out_grad(dy.reshape(-1, C).contiguous(), torch.bfloat16)
        dh = torch.empty(M, 4 * C, dtype=torch.bfloat16, device=x2.device)
        g = torch.empty_like(dh)
        dx = torch.empty(M, C, dtype=torch.bfloat16, device=x2.device)
        dd = ctypes.byref(_mlp_desc(drop, ctx.rpi))
        _launch("mlp_bwd", lambda: lib().csu_mlp_bwd_dp(M, C, ptr(x2), ptr(dyb), ptr(w1c), ptr(b1f), ptr(w2c), ptr(dh),
                                                        ptr(g), ptr(dx), dd, stream_ptr(x2.device)),
                24 * M * C * C, M * C * (2 + 2 + 2) + M * 4 * C * (2 + 2) + 16 * C * C)
        dw2, db2 = wgrad_maybe_side(dyb, g, w2dt, b2dt, params=ctx.params[2:])
        dw1, db1 = wgrad_maybe_side(dh, x2, w1dt, b1dt, params=ctx.params[:2])
        return dy.to(rdt), dx.view(xshape), dw1.to(w1dt), db1.to(b1dt), dw2.to(w2dt), db2.to(b2dt), None, None, None, None


# the fused Mlp's LayerNorm of its output for the next block (csu_mlp_fwd_ln): (gamma, beta, eps, ln_out,
# mean, rstd), set by _MlpFusedFn.forward (or the proj GEMM's) and attached to its output by
# mlp_residual / linear_residual as ``_csu_ln`` together with the output's version counter (an in-place
# change of the output after the launch invalidates it: _ln_pre).  One slot per thread (one thread per
# device runs its own forward).
class _ThreadSlot(threading.local):
    def __init__(self):
        self.v = None

    def __getitem__(self, i):
        return self.v

    def __setitem__(self, i, v):
        self.v = v


_LN_STASH = _ThreadSlot()


def _attach_ln(out):
    st, _LN_STASH[0] = _LN_STASH[0], None
    if st is not None:
        out._csu_ln = tuple(st) + (out._version,)


# widths whose fp8 Mlp backward runs the fp8 kernel (csu_mlp_fp8_bwd); the others run the bf16 fused
# backward on the dequantised (exact) bf16 shadows of the e4m3 weights -- faster at every width since
# round 6: C = 64: 106 vs 120 us, C = 128: 64 vs 90 us per launch (profiles/r06d_step_breakdown_1024_fp8.txt),
# C = 256: the 8-wave bf16 backward (mlp_bwd8_kernel), mlp_bwd 1360 vs 1447 us/step at 1024x1024 B4
# (profiles/r08g_fp8_ab.txt).  The fp8 kernel stays a tested entry point (tests/test_gpu_fp8.py).
FP8_MLP_BWD_C = ()


class _MlpFp8Fn(torch.autograd.Function):
    """res + fc2(gelu(fc1(x))) with e4m3 weights (BASELINE config 5, "fp8 MFMA weights") in ONE
    csu_mlp_fp8_fwd launch on v_mfma_scale_f32_32x32x64_f8f6f4: x and the hidden activations are
    quantised in registers with MX block scales (per token and 32-value block), the weights' per-row
    power-of-two scales ride in the MFMA's E8M0 operands.  Backward (straight-through): one
    csu_mlp_fp8_bwd launch recomputes h exactly, runs dY W2 and dh W1 on the same fp8 MFMA (dY / dh
    quantised the same way, the weight scales folded into them) and writes dh, g_q (the forward's
    fc2 input) and dx; then the two bf16 weight gradients dW1 = dh^T x, dW2 = dY^T g_q.  For C not in
    FP8_MLP_BWD_C the backward is the bf16 fused one (_MlpFusedFn) on the dequantised weights w1c / w2c
    (oracle: fp8_ref.Fp8MlpFn with bwd_fp8=False).  That backward recomputes h and g from the
    UNQUANTISED bf16 x, so at C = 64 / 128 dW2 = dY^T g (not the forward's g_q) and dW1 uses the
    unquantised x: a different straight-through estimator from C = 256's, chosen deliberately because
    the fp8 backward kernel is slower than the bf16 one at those widths."""

    @staticmethod
    def forward(ctx, res, x, w1, b1, w2, b2, ops8, drop, w1c, w2c, ln=None):
        C = x.shape[-1]
        res2 = res.float().contiguous().view(-1, C)
        x2 = x.reshape(-1, C).contiguous()
        if x2.dtype != torch.bfloat16:
            x2 = x2.to(torch.bfloat16)
        w1q, sw1, w2p, sw2, w2t, w1tp = ops8
        b1f = b1.detach().float().contiguous()
        b2f = b2.detach().float().contiguous()
        y = torch.empty_like(res2)
        M = x2.shape[0]
        rpi = x.shape[1] if x.dim() == 3 else M
        dd = ctypes.byref(_mlp_desc(drop, rpi))
        if ln is not None:
            # + the next block's norm1 on the output (csu_mlp_fp8_fwd_ln), as _MlpFusedFn
            gam, bet, eps = ln
            gf, bf_ = gam.detach().float().contiguous(), bet.detach().float().contiguous()
            h1 = torch.empty(M, C, dtype=torch.bfloat16, device=x2.device)
            mean = torch.empty(M, dtype=torch.float32, device=x2.device)
            rstd = torch.empty(M, dtype=torch.float32, device=x2.device)
            _launch("mlp_fwd", lambda: lib().csu_mlp_fp8_fwd_ln(M, C, ptr(x2), ptr(w1q), ptr(sw1), ptr(b1f), ptr(w2p), ptr(sw2),
                                                                ptr(b2f), ptr(res2), ptr(y), dd, ptr(gf), ptr(bf_), float(eps),
                                                                ptr(h1), ptr(mean), ptr(rstd), stream_ptr(x2.device)),
                    16 * M * C * C + 8 * M * C, M * C * (2 + 4 + 4 + 2) + 8 * C * C + 8 * M, prec="fp8")
            _LN_STASH[0] = (gam, bet, float(eps), h1, mean, rstd)
        else:
            _launch("mlp_fwd", lambda: lib().csu_mlp_fp8_fwd(M, C, ptr(x2), ptr(w1q), ptr(sw1), ptr(b1f), ptr(w2p), ptr(sw2),
                                                             ptr(b2f), ptr(res2), ptr(y), dd, stream_ptr(x2.device)),
                    16 * M * C * C, M * C * (2 + 4 + 4) + 8 * C * C, prec="fp8")
        ctx.drop, ctx.rpi = drop, rpi
        ctx.save_for_backward(x2, b1f)
        ctx.ops8 = ops8
        ctx.wc = (w1c, w2c)
        ctx.meta = (res.dtype, x.shape, w1.dtype, b1.dtype, w2.dtype, b2.dtype)
        ctx.params = (w1, b1, w2, b2)
        _note_use(ctx, *ctx.params)
        return y.view(res.shape)

    @staticmethod
    def backward(ctx, dy):
        rdt, xshape, w1dt, b1dt, w2dt, b2dt = ctx.meta
        x2, b1f = ctx.saved_tensors
        w1q, sw1, w2p, sw2, w2t, w1tp = ctx.ops8
        M, C = x2.shape
        drop = ctx.drop
        if drop is None:
            dyb = _bf16_of(dy).view(-1, C)
        else:
            dyb = drop.out_grad(dy.reshape(-1, C).contiguous(), torch.bfloat16)
        dyb = dyb.contiguous()
        dh = torch.empty(M, 4 * C, dtype=torch.bfloat16, device=x2.device)
        g = torch.empty_like(dh)
        dx = torch.empty(M, C, dtype=torch.bfloat16, device=x2.device)
        dd = ctypes.byref(_mlp_desc(drop, ctx.rpi))
        if C in FP8_MLP_BWD_C:
            _launch("mlp_bwd", lambda: lib().csu_mlp_fp8_bwd(M, C, ptr(x2), ptr(dyb), ptr(w1q), ptr(sw1), ptr(b1f), ptr(w2t),
                                                             ptr(sw2), ptr(w1tp), ptr(dh), ptr(g), ptr(dx), dd,
                                                             stream_ptr(x2.device)),
                    24 * M * C * C, M * C * (2 + 2 + 2) + M * 4 * C * (2 + 2) + 12 * C * C, prec="fp8")
        else:
            w1c, w2c = ctx.wc
            _launch("mlp_bwd", lambda: lib().csu_mlp_bwd_dp(M, C, ptr(x2), ptr(dyb), ptr(w1c), ptr(b1f), ptr(w2c), ptr(dh),
                                                            ptr(g), ptr(dx), dd, stream_ptr(x2.device)),
                    24 * M * C * C, M * C * (2 + 2 + 2) + M * 4 * C * (2 + 2) + 16 * C * C)
        dw2, db2 = wgrad_maybe_side(dyb, g, w2dt, b2dt, params=ctx.params[2:])
        dw1, db1 = wgrad_maybe_side(dh, x2, w1dt, b1dt, params=ctx.params[:2])
        return (dy.to(rdt), dx.view(xshape), dw1.to(w1dt), db1.to(b1dt), dw2.to(w2dt), db2.to(b2dt), None, None, None,
                None, None)


def mlp_fp8(res, x, fc1: torch.nn.Linear, fc2: torch.nn.Linear, drop: Optional[MlpDrop] = None, ln=None):
    """The fp8 fused Mlp (_MlpFp8Fn) when the active fp8 weight format holds fc1 / fc2 as an Mlp pair
    (model.set_weight_format('fp8_e4m3') under bf16 autocast), else None.  ``ln``: (weight, bias, eps)
    of the next block's norm1, computed in the same launch (left in _LN_STASH for the caller)."""
    if _ACTIVE_FP8 is None or not x.is_cuda or fc1.out_features != 4 * x.shape[-1] or fc2.in_features != fc1.out_features:
        return None
    ops8 = _ACTIVE_FP8.mlp_operands(fc1.weight, fc2.weight)
    if ops8 is None:
        return None
    w1c = w2c = None
    if x.shape[-1] not in FP8_MLP_BWD_C:   # the bf16 backward's operands: the exact dequantised shadows
        w1c, w2c = _weight_bf16(fc1.weight), _weight_bf16(fc2.weight)
    with torch.autocast("cuda", enabled=False):
        return _MlpFp8Fn.apply(res, x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, ops8, drop, w1c, w2c, ln)


# the fused one-launch Mlp where the library has it (C in {64, 128, 256}); otherwise two gemm4 launches
FUSED_MLP = True


# the fused Mlp forward also computes the next CSWinBlock's norm1 (csu_mlp_fwd_ln), which that block's
# layer_norm_fork then uses instead of its own LayerNorm launch
FUSE_NEXT_LN = True


def mlp_residual(res, x, fc1: torch.nn.Linear, fc2: torch.nn.Linear, drop: Optional[MlpDrop] = None, ln_next=None):
    """res + DropPath(Dropout(fc2(Dropout(gelu(fc1(x)))))) on the bf16 path (``drop`` None: eval /
    no dropout).  ``ln_next`` (the next block's norm1 as (weight, bias, eps)): its LayerNorm of the
    output is computed in the same launch and attached to the output for layer_norm_fork."""
    C = x.shape[-1]
    ln = ln_next if (FUSE_NEXT_LN and ln_next is not None and ln_next[0].dtype == torch.float32
                     and ln_next[0].numel() == C) else None
    _LN_STASH[0] = None
    y = mlp_fp8(res, x, fc1, fc2, drop, ln=None if FP8_QKV else ln)   # FP8_QKV: norm1 is the e4m3 LN
    if y is not None:
        if ln is not None:
            _attach_ln(y)
        return y
    if FUSED_MLP and fc1.out_features == 4 * C and lib().csu_mlp_supported(C):
        with torch.autocast("cuda", enabled=False):
            out = _MlpFusedFn.apply(res, x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, _weight_bf16(fc1.weight),
                                    _weight_bf16(fc2.weight), drop, ln)
        if ln is not None:
            _attach_ln(out)
        return out
    with torch.autocast("cuda", enabled=False):
        return _MlpResidualFn.apply(res, x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, _weight_bf16(fc1.weight),
                                    _weight_bf16(fc2.weight), drop)


# fp32 master weight (by storage address) -> (weakref to it, its CastCache, index in the cache,
# AdamW shadow spec): csu.optim.FusedAdamW writes the bf16 shadows of these weights in its update
# pass (csu_adamw_step shadow modes), so the next forward needs no cast launch.
_SHADOW_SPECS = {}


def shadow_spec(p: torch.Tensor):
    """(shadow ptr, shadow_t ptr, rows, cols, taps, cols_pad) of the bf16 layouts a CastCache keeps of
    the fp32 weight p (csu_adamw_item shadow fields), or None."""
    e = _SHADOW_SPECS.get(p.data_ptr())
    if e is None or e[0]() is not p:
        return None
    return e[3]


def shadows_written(params):
    """FusedAdamW wrote the shadows of these weights (in its launch just enqueued): their caches
    note the weights' current versions, so the next refresh skips the cast while nothing else has
    modified them."""
    for p in params:
        e = _SHADOW_SPECS.get(p.data_ptr())
        if e is not None and e[0]() is p:
            e[1]._written[e[2]] = p._version


def sync_shadows(model):
    """Bring a model's cast cache up to date before replaying a captured graph whose forward
    relies on the optimizer-written shadows (a weight modified in place since, e.g. by
    load_state_dict, is re-cast here, outside the graph)."""
    c = getattr(model, "_cast_cache", None)
    if c is not None:
        c.ensure_fresh()


class CastCache:
    """bf16 shadow copies of fp32 master weights, plus a transposed (K, N) copy of every 2-D weight
    for the input-gradient GEMM, and the two channels-last layouts (OHWI, IHWO) of every KxK conv
    weight for the implicit-GEMM conv kernels.  Gradients still flow to the fp32 params.  Lookup is
    by storage address, so reshaped views of a cached weight (the CARAFE 1x1 convs used as token
    Linears) hit the cache too.
    Freshness: csu.optim.FusedAdamW writes every shadow in its update pass (shadow_spec), so a
    forward after an optimizer step launches nothing; ONE csu_cast_bf16_batch launch re-makes all
    of them whenever a weight's version counter moved since the last write (first forward,
    load_state_dict, any in-place change).  In the fp8 format the quantised weights' shadows come from
    the quantiser (every step); the cast batch covers the rest under the same freshness rule."""

    _REC = None

    def __init__(self):
        self.params, self.shadow, self.shadow_t, self.dtype = [], [], [], None
        self.convs, self.conv_o, self.conv_i = [], [], []
        self.index, self.cindex, self.ptrs = {}, {}, []
        self.items, self.tiles = None, 0

    @classmethod
    def _rec(cls):
        import numpy as np
        if cls._REC is None:
            cls._REC = np.dtype([("src", "<u8"), ("dst", "<u8"), ("dst_t", "<u8"), ("rows", "<i4"), ("cols", "<i4"),
                                 ("tile0", "<i8"), ("taps", "<i4"), ("pad", "<i4")])
        return cls._REC

    def _build(self, params, convs, dtype, sources=None):
        self.params, self.convs, self.dtype = params, convs, dtype
        self.sources = sources
        src = sources if sources is not None else params
        self.ptrs = [p.data_ptr() for p in params + convs]
        self.shadow = [torch.empty(p.shape, dtype=dtype, device=p.device) for p in params]
        self.shadow_t = [torch.empty(p.shape[1:].numel() if p.dim() > 1 else 0, p.shape[0], dtype=dtype, device=p.device)
                         if p.dim() > 1 else None for p in params]
        # few-channel convs (the 3-channel patch embed): OHWI zero-padded to a multiple of 8 channels,
        # the layout _Conv2dFn runs them in (pad channels zeroed here once, never written again); no
        # IHWO (their input, the image, needs no gradient)
        self.conv_cp = [_pad_channels(w.shape[1]) for w in convs]
        self.conv_o = [torch.zeros(w.shape[0], w.shape[2], w.shape[3], cp, dtype=dtype, device=w.device)
                       for w, cp in zip(convs, self.conv_cp)]
        self.conv_i = [torch.empty(w.shape[1], w.shape[2], w.shape[3], w.shape[0], dtype=dtype, device=w.device)
                       if cp == w.shape[1] else None for w, cp in zip(convs, self.conv_cp)]
        self.index = {p.data_ptr(): i for i, p in enumerate(params)}
        self.cindex = {w.data_ptr(): i for i, w in enumerate(convs)}
        self.items = None
        self._build_frag(params, dtype)
        allp = params + convs
        self._written = [None] * len(allp)
        self._cast_idx = list(range(len(allp)))
        for k in [k for k, e in _SHADOW_SPECS.items() if e[1] is self]:
            del _SHADOW_SPECS[k]
        if (dtype == torch.bfloat16 and allp and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                                                     for p in allp)):
            import numpy as np
            # a None source: that shadow is written elsewhere (the fp8 quantiser), not by the cast batch
            keep = [i for i in range(len(params)) if src[i] is not None]
            self._cast_idx = keep + [len(params) + j for j in range(len(convs))]   # what the cast batch writes
            rec = np.zeros(len(keep) + len(convs), dtype=self._rec())
            t0 = 0
            for k, i in enumerate(keep):
                p = params[i]
                rows = p.shape[0] if p.dim() > 1 else 1
                cols = p.numel() // rows
                st = self.shadow_t[i]
                rec[k] = (src[i].data_ptr(), self.shadow[i].data_ptr(), 0 if st is None else st.data_ptr(), rows, cols, t0,
                          0, 0)
                t0 += -(-rows // 64) * -(-cols // 64)
            for j, w in enumerate(convs):
                N, C, KH, KW = w.shape
                ci = self.conv_i[j]
                rec[len(keep) + j] = (w.data_ptr(), self.conv_o[j].data_ptr(), 0 if ci is None else ci.data_ptr(), N, C,
                                      t0, KH * KW, self.conv_cp[j])
                t0 += -(-(N * C * KH * KW) // 4096)
            self.tiles = t0
            self.nitems = len(rec)
            self.cast_numel = (sum(params[i].numel() for i in keep), sum(params[i].numel() for i in keep if params[i].dim() > 1))
            # no item (every source written elsewhere): an empty table, no cast launch (_cast checks nitems)
            self.items = (torch.frombuffer(bytearray(rec.tobytes()), dtype=torch.uint8).to(allp[0].device) if len(rec)
                          else torch.zeros(1, dtype=torch.uint8, device=allp[0].device))
            # FusedAdamW writes the shadows of every weight cast from itself (all of them in bf16; in
            # the fp8 format the unquantised 1-D tensors and the convs -- the quantiser writes the rest)
            if True:
                import weakref
                for i, p in enumerate(params):
                    if src[i] is not p:
                        continue
                    rows = p.shape[0] if p.dim() > 1 else 1
                    st = self.shadow_t[i]
                    _SHADOW_SPECS[p.data_ptr()] = (weakref.ref(p), self, i, (
                        self.shadow[i].data_ptr(), 0 if st is None else st.data_ptr(), rows, p.numel() // rows, 0, 0))
                for j, w in enumerate(convs):
                    ci = self.conv_i[j]
                    _SHADOW_SPECS[w.data_ptr()] = (weakref.ref(w), self, len(params) + j, (
                        self.conv_o[j].data_ptr(), 0 if ci is None else ci.data_ptr(), w.shape[0], w.shape[1],
                        w.shape[2] * w.shape[3], self.conv_cp[j]))

    def refresh(self, params, dtype, convs=(), sources=None):
        """``sources``: per param, the fp32 tensor the shadow is made from (default: the param
        itself; the fp8 weight format passes its dequantised e4m3 copies, Fp8Weights)."""
        params, convs = list(params), list(convs)
        allp = params + convs
        if (self.dtype != dtype or len(params) != len(self.params) or len(convs) != len(self.convs)
                or any(a is not b for a, b in zip(allp, self.params + self.convs))
                or any(p.data_ptr() != q for p, q in zip(allp, self.ptrs))
                or (sources is None) != (getattr(self, "sources", None) is None)
                or (sources is not None and any(a is not b for a, b in zip(sources, self.sources)))):
            self._build(params, convs, dtype, sources)
        if self.items is not None:
            if not self._fresh():
                self._cast()
            return
        src = self.sources if getattr(self, "sources", None) is not None else self.params
        with torch.no_grad():
            pairs = [(sh, p) for sh, p in zip(self.shadow, src) if p is not None]
            if pairs:
                torch._foreach_copy_([a for a, _ in pairs], [p.detach() for _, p in pairs])
            for st, p in zip(self.shadow_t, src):
                if st is not None and p is not None:
                    st.copy_(p.detach().reshape(p.shape[0], -1).t())
            for w, o, i in zip(self.convs, self.conv_o, self.conv_i):
                o[..., :w.shape[1]].copy_(w.detach().permute(0, 2, 3, 1))
                if i is not None:
                    i.copy_(w.detach().permute(1, 2, 3, 0))

    def _fresh(self) -> bool:
        """Every shadow the cast batch writes is current (the fp8 quantiser's own are not its concern)."""
        allp = self.params + self.convs
        idx = getattr(self, "_cast_idx", None) or range(len(allp))
        return all(self._written[i] is not None and self._written[i] == allp[i]._version for i in idx)

    # Fragment-ordered copies of the bf16 shadows W / W^T that the weight-streaming GEMM reads
    # (csu_gemm_ws: the qkv / proj Linears and their input gradients at C = 128 / 256), made from the
    # finished natural-layout shadows by ONE csu_frag_layout_batch launch per forward (refresh_frag,
    # after AdamW / the cast batch / the fp8 quantiser wrote them).
    def _build_frag(self, params, dtype):
        import numpy as np
        self.frag_w, self.frag_t = [None] * len(params), [None] * len(params)
        self.frag_items, self.frag_n, self.frag_chunks = None, 0, 0
        if not USE_GEMM_WS or dtype != torch.bfloat16 or not params or not all(p.is_cuda for p in params):
            return
        L = lib()
        recs = []
        for i, p in enumerate(params):
            if p.dim() != 2:
                continue
            N, K = p.shape
            if L.csu_gemm_ws_supported(1024, N, K, 0, CSU_BF16):
                self.frag_w[i] = torch.empty(N * K, dtype=dtype, device=p.device)
                recs.append((self.shadow[i], self.frag_w[i], N, K))
            if L.csu_gemm_ws_supported(1024, K, N, 0, CSU_BF16) and self.shadow_t[i] is not None:
                self.frag_t[i] = torch.empty(N * K, dtype=dtype, device=p.device)
                recs.append((self.shadow_t[i], self.frag_t[i], K, N))
        if not recs:
            return
        rec = np.zeros(len(recs), dtype=[("src", "<u8"), ("dst", "<u8"), ("rows", "<i4"), ("cols", "<i4"), ("chunk0", "<i8")])
        c0 = 0
        for k, (src, dst, rows, cols) in enumerate(recs):
            rec[k] = (src.data_ptr(), dst.data_ptr(), rows, cols, c0)
            c0 += rows * cols // 8
        self.frag_n, self.frag_chunks = len(recs), c0
        self.frag_items = torch.frombuffer(bytearray(rec.tobytes()), dtype=torch.uint8).to(params[0].device)

    def refresh_frag(self):
        """Re-make the fragment-ordered shadows from the current natural ones (one launch)."""
        if self.frag_items is None:
            return
        n = self.frag_chunks * 16
        _launch("frag_layout", lambda: lib().csu_frag_layout_batch(ptr(self.frag_items), self.frag_n, self.frag_chunks,
                                                                    stream_ptr(self.frag_items.device)), 0, 2 * n)

    def get_frag(self, p):
        """Fragment-ordered bf16 W of a cached 2-D (N, K) weight (csu_gemm_ws operand), or None."""
        i = self.index.get(p.data_ptr())
        if i is None or p.dim() != 2 or self.frag_w[i] is None or self.params[i].shape != p.shape:
            return None
        return self.frag_w[i]

    def get_frag_t(self, p):
        """Fragment-ordered bf16 W^T (K, N) of a cached 2-D (N, K) weight, or None."""
        i = self.index.get(p.data_ptr())
        if i is None or p.dim() != 2 or self.frag_t[i] is None or self.params[i].shape != p.shape:
            return None
        return self.frag_t[i]

    def _cast(self):
        allp = self.params + self.convs
        n = self.cast_numel[0] + sum(w.numel() for w in self.convs)
        nt = self.cast_numel[1] + sum(w.numel() for w in self.convs)
        if self.nitems and self.tiles:
            _launch("cast_bf16_batch", lambda: lib().csu_cast_bf16_batch(ptr(self.items), self.nitems, self.tiles,
                                                                         stream_ptr(allp[0].device)),
                    0, n * 6 + nt * 2)
        for i in getattr(self, "_cast_idx", None) or range(len(allp)):
            self._written[i] = allp[i]._version

    def ensure_fresh(self):
        """Re-cast now if a weight changed since its shadows were last written (see class doc)."""
        if self.items is not None and not self._fresh():
            self._cast()

    def get(self, p, dtype):
        i = self.index.get(p.data_ptr())
        if i is None or self.dtype != dtype or self.params[i].numel() != p.numel():
            return None
        return self.shadow[i].view(p.shape)

    def get_t(self, p, dtype):
        """(K, N) bf16 transpose of a 2-D (N, K) view of a cached weight, or None."""
        i = self.index.get(p.data_ptr())
        if i is None or self.dtype != dtype or p.dim() != 2 or self.shadow_t[i] is None:
            return None
        st = self.shadow_t[i]
        return st if tuple(st.shape) == (p.shape[1], p.shape[0]) else None

    def get_conv(self, w, dtype):
        """(OHWI, IHWO) bf16 layouts of a cached conv weight, or None.  Few-channel weights: OHWI
        channel-padded to _pad_channels(C), IHWO None."""
        j = self.cindex.get(w.data_ptr())
        if j is None or self.dtype != dtype or tuple(self.convs[j].shape) != tuple(w.shape):
            return None
        return self.conv_o[j], self.conv_i[j]


class Fp8Weights:
    """fp8-e4m3 weights (BASELINE config 5): the listed fp32 master weights quantised per output
    row to e4m3 with power-of-two scales (csu_quant_e4m3_batch, one launch per step); ``deq`` are
    the dequantised fp32 copies (exact in bf16) that the cast cache turns into the kernels' bf16
    shadows, ``q`` / ``scales`` the e4m3 bytes and row scales.  Gradients flow to the fp32 masters
    (straight-through).  1-D tensors (biases, LN) are not quantised."""

    def __init__(self, params, mlp_pairs=()):
        import numpy as np
        self.params = list(params)
        self.deq, self.q, self.scales = [], [], []
        rec = np.zeros(0, dtype=[("src", "<u8"), ("dst", "<u8"), ("dq", "<u8"), ("sc", "<u8"), ("row0", "<i8"),
                                 ("rows", "<i4"), ("cols", "<i4")])
        recs, row0 = [], 0
        for p in self.params:
            if p.dim() < 2:
                self.deq.append(p)
                self.q.append(None)
                self.scales.append(None)
                continue
            rows = p.shape[0]
            cols = p.numel() // rows
            d = torch.empty_like(p)
            q = torch.empty(p.shape, dtype=torch.uint8, device=p.device)
            sc = torch.empty(rows, dtype=torch.float32, device=p.device)
            self.deq.append(d)
            self.q.append(q)
            self.scales.append(sc)
            recs.append((p.data_ptr(), d.data_ptr(), q.data_ptr(), sc.data_ptr(), row0, rows, cols))
            row0 += rows
        rec = np.array(recs, dtype=rec.dtype)
        self.count, self.rows = len(recs), row0
        self.items = torch.frombuffer(bytearray(rec.tobytes()), dtype=torch.uint8).to(self.params[0].device)
        self.ptrs = [p.data_ptr() for p in self.params]
        self.index = {p.data_ptr(): i for i, p in enumerate(self.params) if p.dim() >= 2}
        # operand layouts of the fp8 fused Mlp (csu_mlp_fp8_fwd / _bwd), rebuilt from the e4m3 bytes
        # after every quantisation by one csu_e4m3_layout_batch launch: W2 with permuted columns,
        # W2^T, W1^T with permuted columns
        self.mlp = {}
        self.lay_of = {}   # weight ptr -> (q_perm, q_t, q_tp) written by the shadow quantiser
        lay, w0 = [], 0
        for w1, w2 in mlp_pairs:
            i1, i2 = self.index.get(w1.data_ptr()), self.index.get(w2.data_ptr())
            if i1 is None or i2 is None:
                continue
            q1, q2 = self.q[i1], self.q[i2]
            N4, C = q1.shape
            # the fp8 kernels hard-code 4C hidden features (mlp_ratio 4, cswin:337)
            if N4 != 4 * C or tuple(q2.shape) != (C, N4) or not lib().csu_mlp_fp8_supported(C):
                continue
            w2p = torch.empty_like(q2)
            w2t = torch.empty(N4, C, dtype=torch.uint8, device=q2.device)
            w1tp = torch.empty(C, N4, dtype=torch.uint8, device=q1.device)
            for src, dst, rows, cols, mode in ((q2, w2p, C, N4, 2), (q2, w2t, C, N4, 1), (q1, w1tp, N4, C, 3)):
                lay.append((src.data_ptr(), dst.data_ptr(), w0, rows, cols, mode, 0))
                w0 += rows * cols // 4
            self.mlp[w1.data_ptr()] = (w2.data_ptr(), q1, self.scales[i1], w2p, self.scales[i2], w2t, w1tp)
            self.lay_of[w1.data_ptr()] = (0, 0, w1tp.data_ptr())
            self.lay_of[w2.data_ptr()] = (w2p.data_ptr(), w2t.data_ptr(), 0)
        self.lay_count, self.lay_words = len(lay), w0
        # e4m3 fragment-ordered W and W^T of the weights the weight-streaming GEMM runs (the qkv / proj
        # Linears, csu_gemm_ws_e4m3), rebuilt from the e4m3 bytes after every quantisation (one launch)
        self.frag8 = {}
        f8, b0 = [], 0
        L = lib()
        for i, (p, q) in enumerate(zip(self.params, self.q)):
            if q is None or p.dim() != 2:
                continue
            N, K = q.shape
            if N % 32 or K % 32:
                continue
            fw = ft = None
            if L.csu_gemm_ws_supported(1024, N, K, 0, CSU_BF16):
                fw = torch.empty(N * K, dtype=torch.uint8, device=q.device)
                f8.append((q.data_ptr(), fw.data_ptr(), N, K, 0, 0, b0))
                b0 += N * K // 64
            if L.csu_gemm_ws_supported(1024, K, N, 0, CSU_BF16):
                ft = torch.empty(N * K, dtype=torch.uint8, device=q.device)
                f8.append((q.data_ptr(), ft.data_ptr(), N, K, 1, 0, b0))
                b0 += N * K // 64
            if fw is not None or ft is not None:
                self.frag8[p.data_ptr()] = (fw, ft, self.scales[i], tuple(p.shape))
        self.frag8_count, self.frag8_blocks = len(f8), b0
        if f8:
            dt8 = np.dtype([("src", "<u8"), ("dst", "<u8"), ("N", "<i4"), ("K", "<i4"), ("transpose", "<i4"),
                            ("pad", "<i4"), ("block0", "<i8")])
            self.frag8_items = torch.frombuffer(bytearray(np.array(f8, dtype=dt8).tobytes()),
                                                dtype=torch.uint8).to(self.params[0].device)
        if lay:
            lt = np.dtype([("src", "<u8"), ("dst", "<u8"), ("w0", "<i8"), ("rows", "<i4"), ("cols", "<i4"),
                           ("mode", "<i4"), ("pad", "<i4")])
            self.lay_items = torch.frombuffer(bytearray(np.array(lay, dtype=lt).tobytes()),
                                              dtype=torch.uint8).to(self.params[0].device)

    def get_frag8(self, w, transposed: bool = False):
        """(e4m3 fragments, row scales, csu_gemm_ws_e4m3 scale_mode) of W (mode 1) or W^T (mode 2) of
        a quantised weight, or None."""
        e = self.frag8.get(w.data_ptr())
        if e is None or e[3] != tuple(w.shape):
            return None
        f = e[1] if transposed else e[0]
        return None if f is None else (f, e[2], 2 if transposed else 1)

    def mlp_operands(self, w1, w2):
        """(w1q, sw1, w2p, sw2, w2t, w1tp) of the fused fp8 Mlp over fc1 / fc2 weights, or None."""
        e = self.mlp.get(w1.data_ptr())
        if e is None or e[0] != w2.data_ptr():
            return None
        return e[1:]

    def lookup(self, w):
        """(e4m3 bytes, row scales) of a quantised weight, or None."""
        i = self.index.get(w.data_ptr())
        if i is None or self.params[i].shape != w.shape:
            return None
        return self.q[i], self.scales[i]

    def valid_for(self, params) -> bool:
        params = list(params)
        return len(params) == len(self.params) and all(a is b and a.data_ptr() == q
                                                       for a, b, q in zip(params, self.params, self.ptrs))

    def sources(self):
        """Per listed param, the fp32 tensor a CastCache should cast its bf16 shadow from: None for the
        quantised weights (quantize(cache) writes their shadows itself), the param for 1-D tensors."""
        return [None if q is not None else p for p, q in zip(self.params, self.q)]

    def _shadow_items(self, cache):
        """Item table of csu_quant_e4m3_shadow_batch into ``cache``'s shadows (rebuilt when they move)."""
        import numpy as np
        key = (id(cache), tuple(cache.shadow[cache.index[p.data_ptr()]].data_ptr() for p, q in zip(self.params, self.q)
                                if q is not None))
        if getattr(self, "_skey", None) == key:
            return self._sitems, self._sblocks, self._scount
        recs, b0 = [], 0
        for p, q, sc in zip(self.params, self.q, self.scales):
            if q is None:
                continue
            i = cache.index[p.data_ptr()]
            st = cache.shadow_t[i]
            rows = p.shape[0]
            cols = p.numel() // rows
            if cols % 16:
                raise ValueError("Fp8Weights: weight columns must be a multiple of 16")
            lay = self.lay_of.get(p.data_ptr(), (0, 0, 0))
            if any(lay) and (rows % 64 or cols % 64):
                raise ValueError("Fp8Weights: fp8 Mlp layouts need rows % 64 == 0 and cols % 64 == 0")
            recs.append((p.data_ptr(), q.data_ptr(), sc.data_ptr(), cache.shadow[i].data_ptr(),
                         0 if st is None else st.data_ptr()) + lay + (b0, rows, cols))
            b0 += -(-rows // 64)
        dt = np.dtype([("src", "<u8"), ("q", "<u8"), ("sc", "<u8"), ("sh", "<u8"), ("st", "<u8"), ("qp", "<u8"),
                       ("qt", "<u8"), ("qtp", "<u8"), ("b0", "<i8"), ("rows", "<i4"), ("cols", "<i4")])
        self._sitems = torch.frombuffer(bytearray(np.array(recs, dtype=dt).tobytes()), dtype=torch.uint8).to(
            self.params[0].device)
        self._sblocks, self._scount, self._skey = b0, len(recs), key
        return self._sitems, self._sblocks, self._scount

    def quantize(self, cache: Optional["CastCache"] = None):
        """One launch: e4m3 bytes + row scales of every listed weight, and either the dequantised fp32
        copies (``deq``, returned; then the fp8 Mlp operand layouts by csu_e4m3_layout_batch) or -- with
        ``cache`` -- the bf16 shadows W and W^T straight in the cache and the fp8 Mlp operand layouts from
        the same pass (csu_quant_e4m3_shadow_batch)."""
        dev = self.params[0].device
        nq = sum(p.numel() for p, q in zip(self.params, self.q) if q is not None)
        if cache is None:
            _launch("quant_e4m3", lambda: lib().csu_quant_e4m3_batch(ptr(self.items), self.count, self.rows,
                                                                     stream_ptr(dev)), 0, nq * 9)
        else:
            items, blocks, count = self._shadow_items(cache)
            _launch("quant_e4m3", lambda: lib().csu_quant_e4m3_shadow_batch(ptr(items), count, blocks, stream_ptr(dev)),
                    0, nq * (4 + 1 + 2 + 2) + self.lay_words * 4)
            self._layout_frag8(dev)
            return self.deq
        if self.lay_count:
            _launch("quant_e4m3", lambda: lib().csu_e4m3_layout_batch(ptr(self.lay_items), self.lay_count, self.lay_words,
                                                                     stream_ptr(dev)), 0, self.lay_words * 8)
        self._layout_frag8(dev)
        return self.deq

    def _layout_frag8(self, dev):
        if self.frag8_count and FP8_WS:
            n = self.frag8_blocks * 64
            _launch("quant_e4m3", lambda: lib().csu_frag8_layout_batch(ptr(self.frag8_items), self.frag8_count,
                                                                      self.frag8_blocks, stream_ptr(dev)), 0, 2 * n)


_ACTIVE_CACHE: Optional[CastCache] = None
_ACTIVE_FP8: Optional[Fp8Weights] = None


def set_cast_cache(cache: Optional[CastCache], fp8: Optional[Fp8Weights] = None):
    global _ACTIVE_CACHE, _ACTIVE_FP8
    _ACTIVE_CACHE = cache
    _ACTIVE_FP8 = fp8


def fp8_gemm(aq: torch.Tensor, sa: torch.Tensor, wq: torch.Tensor, sw: torch.Tensor,
             bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16 (M, N) = (aq * sa[:, None]) @ (wq * sw[:, None])^T + bias on e4m3 MFMA (csu_fp8_gemm):
    aq (M, K) / wq (N, K) uint8 e4m3fn bytes, sa / sw fp32 row scales."""
    require_device(aq, wq)
    M, K = aq.shape
    N = wq.shape[0]
    if wq.shape[1] != K or sa.numel() != M or sw.numel() != N or aq.dtype != torch.uint8 or wq.dtype != torch.uint8:
        raise ValueError("fp8_gemm: shape / dtype mismatch")
    aq, wq, sa, sw = aq.contiguous(), wq.contiguous(), sa.float().contiguous(), sw.float().contiguous()
    b = None if bias is None else bias.detach().float().contiguous()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=aq.device)
    _launch("fp8_gemm", lambda: lib().csu_fp8_gemm(M, N, K, ptr(aq), ptr(sa), ptr(wq), ptr(sw), ptr(b), ptr(out),
                                                   stream_ptr(aq.device)),
            2 * M * N * K, M * K + N * K + M * N * 2 + (M + N) * 4, prec="fp8")
    return out


def dequant_e4m3_rows(q: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """bf16 q * scale[:, None] of e4m3fn bytes (exact: power-of-two scales)."""
    require_device(q)
    rows, cols = q.shape
    out = torch.empty(rows, cols, dtype=torch.bfloat16, device=q.device)
    _launch("dequant_e4m3", lambda: lib().csu_dequant_e4m3_rows(rows, cols, ptr(q), ptr(scale), ptr(out),
                                                                stream_ptr(q.device)),
            0, rows * cols * 3 + rows * 4, prec="fp8")
    return out


def layer_norm_fp8(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float = 1e-5, dq: bool = False):
    """(e4m3 bytes, row scales, mean, rstd[, bf16 dequantised copy]) of LN(x) (csu_layernorm_fwd_fp8_dq),
    no autograd."""
    require_device(x, weight, bias)
    x = x.contiguous()
    C = x.shape[-1]
    rows = x.numel() // C
    w = weight.detach().float().contiguous()
    b = bias.detach().float().contiguous()
    q = torch.empty(rows, C, dtype=torch.uint8, device=x.device)
    s = torch.empty(rows, dtype=torch.float32, device=x.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    ydq = torch.empty(rows, C, dtype=torch.bfloat16, device=x.device) if dq else None
    _launch("layernorm_fwd_fp8", lambda: lib().csu_layernorm_fwd_fp8_dq(rows, C, float(eps), dtype_code(x), ptr(x),
                                                                        ptr(w), ptr(b), ptr(q), ptr(s), ptr(ydq),
                                                                        ptr(mean), ptr(rstd), stream_ptr(x.device)),
            10 * rows * C, rows * C * (esize(x) + 1 + (2 if dq else 0)) + rows * 12, prec=prec_of(x))
    return (q, s, mean, rstd, ydq) if dq else (q, s, mean, rstd)


class _LnLinearFp8Fn(torch.autograd.Function):
    """Residual junction + LayerNorm + Linear with e4m3 operands (BASELINE config 5, "fp8 MFMA
    weights"): x -> (x, LN(x) W^T + b) for CSWinBlock's norm1 -> qkv (cswin:357 -> cswin:337).
    The LayerNorm writes its output as e4m3 with one power-of-two scale per token
    (csu_layernorm_fwd_fp8: the kernel holds the whole token row, so the amax costs nothing) and
    csu_fp8_gemm multiplies it with the e4m3 weight rows on v_mfma_scale_f32_32x32x64_f8f6f4.
    Backward (straight-through for both quantisations): dh = dY W_q (bf16 GEMM on the dequantised
    e4m3 weights, the cast cache's transpose), dW / db from dY and the dequantised e4m3 activation
    the forward multiplied, and the norm1 backward fused with the residual gradient as in
    _LayerNormForkFn."""

    @staticmethod
    def forward(ctx, x, gamma, beta, weight, bias, eps: float, wq, ws, wt):
        x = x.contiguous()
        C = x.shape[-1]
        hq, hs, mean, rstd, hdq = layer_norm_fp8(x, gamma, beta, eps, dq=True)
        y = fp8_gemm(hq, hs, wq, ws, bias).view(*x.shape[:-1], wq.shape[0])
        ctx.save_for_backward(x, gamma.detach().float().contiguous(), mean, rstd, hdq, wt)
        ctx.params = (gamma, beta)
        ctx.pdtypes = (gamma.dtype, beta.dtype)
        ctx.lin = (weight, bias)
        ctx.lmeta = (weight.dtype, None if bias is None else bias.dtype, C)
        _note_use(ctx, gamma, beta, weight, bias)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, dres, dy):
        x, g, mean, rstd, h, wt = ctx.saved_tensors     # h: the dequantised e4m3 LN output (bf16, exact)
        wdt, bdt, C = ctx.lmeta
        dh = dw = db = None
        if dy is not None:
            N = dy.shape[-1]
            dy2 = _bf16_of(dy).reshape(-1, N).contiguous()
            dh = gemm(dy2, wt, False, torch.bfloat16).view(x.shape)
            need_w, need_b = ctx.needs_input_grad[3], bdt is not None and ctx.needs_input_grad[4]
            if need_w or need_b:
                dwf, dbf = wgrad_maybe_side(dy2, h, wdt if need_w else None, bdt if need_b else None, params=ctx.lin)
                dw = dwf.to(wdt) if need_w else None
                db = dbf.to(bdt) if need_b else None
        dx, dg, dbeta = _ln_fork_backward(ctx, x, g, mean, rstd, dres, dh)
        return dx, dg, dbeta, dw, db, None, None, None, None


class _LnLinearWsFn(torch.autograd.Function):
    """Residual junction + LayerNorm + Linear on the weight-streaming GEMM (bf16): x -> (x, LN(x) W^T
    + b) for CSWinBlock's norm1 -> qkv (cswin:357 -> cswin:337) at C = 128 / 256.  Forward: the
    LayerNorm (or the values the producing fused Mlp already computed, _ln_pre) and csu_gemm_ws.
    Backward: ONE csu_gemm_ws_lnbwd launch computes dh = dY W and runs the norm1 backward on it in
    its epilogue (dx = dres + LN'(dh), its bf16 copy and the dgamma / dbeta block partials) -- dh
    never reaches HBM and the LayerNorm-backward launch is gone; dW / db of the Linear as _LinearFn."""

    @staticmethod
    def forward(ctx, x, gamma, beta, weight, bias, eps: float, wf, wtf, pre):
        x = x.contiguous()
        C = x.shape[-1]
        rows = x.numel() // C
        g = gamma.detach().float().contiguous()
        if pre is not None:
            h1, mean, rstd = pre[3].view(x.shape), pre[4], pre[5]
        else:
            b = beta.detach().float().contiguous()
            h1 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
            mean = torch.empty(rows, dtype=torch.float32, device=x.device)
            rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
            _launch("layernorm_fwd", lambda: lib().csu_layernorm_fwd(rows, C, float(eps), dtype_code(x), ptr(x), ptr(g),
                                                                     ptr(b), CSU_BF16, ptr(h1), ptr(mean), ptr(rstd),
                                                                     stream_ptr(x.device)),
                    8 * rows * C, rows * C * (4 + 2) + rows * 8, prec="f32")
        N = weight.shape[0]
        h2 = h1.view(rows, C)
        y = gemm_ws(h2, wf, N, torch.bfloat16, bias=None if bias is None else bias.detach().float().contiguous())
        ctx.save_for_backward(x, g, mean, rstd, h2, wtf)
        ctx.params = (gamma, beta)
        ctx.pdtypes = (gamma.dtype, beta.dtype)
        ctx.lin = (weight, bias)
        ctx.lmeta = (weight.dtype, None if bias is None else bias.dtype)
        _note_use(ctx, gamma, beta, weight, bias)
        return x.view_as(x), y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dres, dy):
        x, g, mean, rstd, h, wtf = ctx.saved_tensors
        wdt, bdt = ctx.lmeta
        C = x.shape[-1]
        rows = x.numel() // C
        if dy is None:    # no gradient through the Linear: the plain fork backward
            dx, dg, dbeta = _ln_fork_backward(ctx, x, g, mean, rstd, dres, None)
            return dx, dg, dbeta, None, None, None, None, None, None
        N = dy.shape[-1]
        dy2 = _bf16_of(dy).reshape(-1, N).contiguous()
        dres_k = dres.float().contiguous() if dres is not None else None
        dx = torch.empty_like(x)
        dxb = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        nblk = rows // 64
        work = torch.empty(nblk * 2 * C, dtype=torch.float32, device=x.device)
        _launch("gemm", lambda: lib().csu_gemm_ws_lnbwd(rows, C, N, ptr(dy2), ptr(wtf), ptr(x), ptr(g), ptr(mean), ptr(rstd),
                                                       ptr(dres_k), ptr(dx), ptr(dxb), ptr(work), stream_ptr(x.device)),
                2 * rows * N * C + 12 * rows * C,
                rows * N * 2 + N * C * 2 + rows * C * (4 + (4 if dres_k is not None else 0) + 4 + 2) + rows * 8,
                prec="bf16", tag=f"{rows}x{C}x{N}:lnbwd:ws")
        dgb = _grad_dest(ctx.params)
        if dgb is None:
            dgb = torch.empty(2 * C, dtype=torch.float32, device=x.device)
        if not _ln_params(ctx, rows, C, work, dgb, nblocks=nblk):
            it = (_lib.LnParamItem * 1)()
            it[0].workspace, it[0].dgamma, it[0].dbeta = work.data_ptr(), dgb.data_ptr(), dgb.data_ptr() + C * 4
            it[0].rows, it[0].C, it[0].nblocks = rows, C, nblk
            _launch("layernorm_bwd", lambda: lib().csu_layernorm_param_reduce_batch(it, 1, stream_ptr(x.device)),
                    0, work.numel() * 4 + 2 * C * 4)
        dw = db = None
        need_w, need_b = ctx.needs_input_grad[3], bdt is not None and ctx.needs_input_grad[4]
        if need_w or need_b:
            dwf, dbf = wgrad_maybe_side(dy2, h, wdt if need_w else None, bdt if need_b else None, params=ctx.lin)
            dw = dwf.to(wdt) if need_w else None
            db = dbf.to(bdt) if need_b else None
        dx._csu_bf16 = dxb
        return dx, dgb[:C].to(ctx.pdtypes[0]), dgb[C:].to(ctx.pdtypes[1]), dw, db, None, None, None, None


# the norm1 -> qkv pair on csu_gemm_ws with the LayerNorm backward in the input-gradient GEMM
FUSE_LN_QKV = False   # measured: the epilogue phase costs what the LayerNorm launch saved


def ln_linear_ws(x: torch.Tensor, ln: torch.nn.LayerNorm, lin: torch.nn.Linear):
    """(x, lin(ln(x))) through _LnLinearWsFn (bf16 autocast, fp32 residual stream x, shapes with the
    weight-streaming GEMM and its LayerNorm-backward epilogue instantiated), else None."""
    if not (FUSE_LN_QKV and USE_GEMM_WS and x.is_cuda and x.dtype == torch.float32 and _ACTIVE_CACHE is not None
            and (_ACTIVE_FP8 is None or not FP8_WS)):
        return None
    N, K = lin.weight.shape
    if x.shape[-1] != K or ln.weight.numel() != K or ln.weight.dtype != torch.float32:
        return None
    wf, wtf = _ACTIVE_CACHE.get_frag(lin.weight), _ACTIVE_CACHE.get_frag_t(lin.weight)
    M = x.numel() // K
    if wf is None or wtf is None or not _ws_ok(M, N, K, torch.bfloat16) or not lib().csu_gemm_ws_lnbwd_supported(M, K, N):
        return None
    pre = _ln_pre(x, ln.weight, ln.bias, ln.eps, torch.bfloat16)
    with torch.autocast("cuda", enabled=False):
        return _LnLinearWsFn.apply(x, ln.weight, ln.bias, lin.weight, lin.bias, ln.eps, wf, wtf, pre)


# qkv in the fp8 weight format.  False: the bf16 weight-streaming GEMM on the EXACT dequantised e4m3
# weight (the cast cache's shadow), norm1 in bf16 (fused into the previous block's Mlp epilogue where
# it can be); True: e4m3 norm1 output x e4m3 weight on the fp8 MFMA (_LnLinearFp8Fn).  Measured at
# 1024x1024 B4: fp8 qkv 422 us/step + its e4m3 LayerNorms 303 against ~320 (gemm_ws) + a share of 138
# for bf16 (profiles/r07zd_*): the fp8 qkv made the fp8 format slower than bf16 (340.1 vs 345.8 img/s).
FP8_QKV = os.environ.get("CSU_FP8_QKV", "0") != "0"


def ln_linear_fp8(x: torch.Tensor, ln: torch.nn.LayerNorm, lin: torch.nn.Linear):
    """(x, lin(ln(x))) through _LnLinearFp8Fn when the fp8 weight format holds lin's weight (bf16
    autocast forward of a model in set_weight_format('fp8_e4m3')) and FP8_QKV, else None."""
    if _ACTIVE_FP8 is None or not x.is_cuda or not FP8_QKV:
        return None
    got = _ACTIVE_FP8.lookup(lin.weight)
    N, K = lin.weight.shape
    if got is None or N % 64 or K % 64 or K > 512:
        return None
    wc = _ACTIVE_CACHE.get(lin.weight, torch.bfloat16) if _ACTIVE_CACHE is not None else None
    if wc is None:
        return None
    wt = _weight_t(lin.weight, wc)      # (K, N) bf16 of the dequantised e4m3 weight: the dX GEMM's operand
    with torch.autocast("cuda", enabled=False):
        return _LnLinearFp8Fn.apply(x, ln.weight, ln.bias, lin.weight, lin.bias, ln.eps, got[0], got[1], wt)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
           out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """nn.Linear on tokens in the autocast compute dtype (bf16 under autocast) with split-K dW.
    ``out_dtype`` (bf16 path only): write the output in that dtype from the fp32 accumulator, e.g.
    fp32 for a Linear that starts a residual stream.

    Contract (no vendor-BLAS fallback): device tensors; bf16 in / out features multiples of 8, fp32
    multiples of 4 -- anything else raises ``CsuError`` (callers with narrower layers zero-pad them,
    as the model's 1-class head does)."""
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        cd = torch.get_autocast_dtype("cuda")
    else:
        cd = torch.promote_types(x.dtype, weight.dtype)
    wc = _ACTIVE_CACHE.get(weight, cd) if _ACTIVE_CACHE is not None else None
    with torch.autocast("cuda", enabled=False):
        return _LinearFn.apply(x, weight, bias, cd, wc, out_dtype)


# ---------------------------------------------------------------------------------------------
# Implicit-GEMM NHWC convolutions (patch embed cswin:505, Merge_Block cswin:376, CARAFE encoder
# cswin:397/446, UNet DoubleConv / ConvTranspose2d unet:182-211)
# ---------------------------------------------------------------------------------------------
def _conv_geom(B, H, W, C, N, KH, KW, stride, pad):
    g = _lib.ConvGeom()
    g.B, g.H, g.W, g.C, g.N, g.KH, g.KW, g.stride, g.pad = B, H, W, C, N, KH, KW, stride, pad
    g.OH, g.OW = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    return g


def _conv_wgrad(g, x, dy, dt, c_real=None, out=None):
    """fp32 (dW, db) of the forward conv with geometry g: dW in torch's (N, c_real, KH, KW) layout,
    written so by the kernel's final reduction (input channels >= c_real, the zero padding of a
    few-channel input, dropped); c_real defaults to g.C.  out: a flat fp32 [dW | db] destination
    (a GradAllReduce bucket slice, _grad_dest) instead of a fresh buffer."""
    L = lib()
    cr = g.C if c_real is None else c_real
    if out is None:
        out = torch.empty(g.N * g.KH * g.KW * cr + g.N, dtype=torch.float32, device=x.device)
    n = L.csu_conv2d_wgrad_workspace(ctypes.byref(g))
    work = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
    _launch("conv_wgrad", lambda: L.csu_conv2d_wgrad_oihw(ctypes.byref(g), dt, ptr(x), ptr(dy), cr, ptr(out), ptr(work),
                                                          n, stream_ptr(x.device)),
            2 * g.B * g.OH * g.OW * g.N * g.KH * g.KW * g.C,
            (g.B * g.H * g.W * g.C + g.B * g.OH * g.OW * g.N) * x.element_size() + out.numel() * 4, prec=prec_of(x))
    k = g.N * g.KH * g.KW * cr
    return out[:k].view(g.N, cr, g.KH, g.KW), out[k:]


def _pad_channels(C: int) -> int:
    """Channel count a conv input is run with: few-channel inputs zero-padded to a multiple of 8."""
    return (C + 7) // 8 * 8 if (C % 8 and PAD_CHANNELS) else C


def _conv_ws(op: int, g, t: torch.Tensor):
    """(workspace tensor or None, bytes) of csu_conv2d_fwd_ws / _dgrad_ws for geometry g: the K-split
    partials of few-tile convolutions (csu_conv2d_workspace; 0 bytes: no split)."""
    n = lib().csu_conv2d_workspace(op, ctypes.byref(g), dtype_code(t))
    if not n:
        return None, 0
    return torch.empty(n, dtype=torch.uint8, device=t.device), n


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride: int, pad: int, cd):
        require_device(x, weight)
        B, H, W, C = x.shape
        N, Cw, KH, KW = weight.shape
        if Cw != C:
            raise ValueError(f"conv2d: input has {C} channels, weight expects {Cw}")
        cp = _pad_channels(C)
        if cp != C:
            # few-channel input (the 3-channel image of the patch embed): zero channels up to a
            # multiple of 8 in the image and the weight -- 16-B vector gathers in the conv kernels
            # instead of per-element ones; the padded taps add exact zeros
            xn = x.permute(0, 3, 1, 2)
            if cd == torch.bfloat16 and x.dtype == torch.float32 and xn.is_contiguous():
                # the NCHW fp32 image -> padded bf16 NHWC in one pass
                xc = torch.empty(B, H, W, cp, dtype=cd, device=x.device)
                _launch("pack_nhwc", lambda: lib().csu_pack_nhwc_bf16(B, C, H, W, cp, ptr(xn), ptr(xc), stream_ptr(x.device)),
                        0, x.numel() * 4 + xc.numel() * 2, prec="f32")
            else:
                xc = torch.zeros(B, H, W, cp, dtype=cd, device=x.device)
                xc[..., :C] = x
            cached = _ACTIVE_CACHE.get_conv(weight, cd) if _ACTIVE_CACHE is not None else None
            if cached is not None and cached[0].shape[-1] == cp:
                w_ohwi = cached[0]
            else:
                w_ohwi = torch.nn.functional.pad(weight.detach().permute(0, 2, 3, 1).to(cd), (0, cp - C)).contiguous()
            cached = None
        else:
            xc = (x if x.dtype == cd else x.to(cd)).contiguous()
            cached = _ACTIVE_CACHE.get_conv(weight, cd) if _ACTIVE_CACHE is not None else None
            w_ohwi = cached[0] if cached else weight.detach().permute(0, 2, 3, 1).to(cd).contiguous()
        g = _conv_geom(B, H, W, cp, N, KH, KW, stride, pad)
        y = torch.empty(B, g.OH, g.OW, N, dtype=cd, device=x.device)
        bf = None if bias is None else bias.detach().float().contiguous()
        ws, nws = _conv_ws(0, g, xc)
        _launch("conv_fwd", lambda: lib().csu_conv2d_fwd_ws(ctypes.byref(g), dtype_code(xc), ptr(xc), ptr(w_ohwi), ptr(bf),
                                                            ptr(y), ptr(ws), nws, stream_ptr(x.device)),
                2 * y.numel() * KH * KW * cp, (xc.numel() + w_ohwi.numel() + y.numel()) * xc.element_size(), prec=prec_of(xc))
        ctx.save_for_backward(xc, weight)
        ctx.w_ihwo = cached[1] if cached else None   # refreshed only by the next forward's cast
        ctx.bias = bias
        _note_use(ctx, weight, bias)
        ctx.conf = (stride, pad, cd, x.dtype, bias is not None, None if bias is None else bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, weight = ctx.saved_tensors
        stride, pad, cd, xdt, has_b, bdt = ctx.conf
        B, H, W, cp = xc.shape                 # cp: channels incl. the zero padding
        N, C, KH, KW = weight.shape
        g = _conv_geom(B, H, W, cp, N, KH, KW, stride, pad)
        dy = dy.to(cd).contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            if cp != C:
                w_ihwo = torch.nn.functional.pad(weight.detach().permute(1, 2, 3, 0).to(cd), (0, 0, 0, 0, 0, 0, 0, cp - C))
                w_ihwo = w_ihwo.contiguous()
            else:
                w_ihwo = ctx.w_ihwo if ctx.w_ihwo is not None else weight.detach().permute(1, 2, 3, 0).to(cd).contiguous()
            dx = torch.empty(B, H, W, cp, dtype=cd, device=dy.device)
            ws, nws = _conv_ws(1, g, dy)
            _launch("conv_dgrad", lambda: lib().csu_conv2d_dgrad_ws(ctypes.byref(g), dtype_code(dy), ptr(dy), ptr(w_ihwo),
                                                                    None, ptr(dx), ptr(ws), nws, stream_ptr(dy.device)),
                    2 * dy.numel() * KH * KW * cp, (dy.numel() + w_ihwo.numel() + dx.numel()) * dy.element_size(),
                    prec=prec_of(dy))
            if cp != C:
                dx = dx[..., :C]
            if dx.dtype != xdt:
                dx = dx.to(xdt)

        dest = None
        if has_b and weight.dtype == torch.float32 and bdt == torch.float32:
            dest = _grad_dest((weight, ctx.bias))   # [dW | db] straight into a GradAllReduce bucket
            if dest is not None and dest.numel() != N * KH * KW * C + N:
                dest = None

        def wg():   # (dW (N, C, KH, KW) contiguous, db), OIHW and unpadded by the kernel
            return _conv_wgrad(g, xc, dy, dtype_code(dy), C, out=dest)
        if _side_ok(dy, weight.dtype, bdt if has_b else None, params=(weight, ctx.bias)):
            # on the side stream, like the token-Linear weight gradients; the returned grad is
            # contiguous fp32, so autograd steals it without a kernel on this stream
            dw, db = _side_run(wg, xc, dy)
            _late((weight, ctx.bias), (dw, db if has_b else None), side=True)
            return dx, dw, (db if has_b else None), None, None, None
        dw, db = wg()
        return dx, dw.to(weight.dtype), (db.to(bdt) if has_b else None), None, None, None


def conv2d(x_nhwc: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int = 1,
           pad: int = 0) -> torch.Tensor:
    """nn.Conv2d on a channels-last (B, H, W, C) tensor -> (B, OH, OW, N); torch weight (N, C, KH, KW)."""
    if x_nhwc.is_cuda and torch.is_autocast_enabled("cuda"):
        cd = torch.get_autocast_dtype("cuda")
    else:
        cd = torch.promote_types(x_nhwc.dtype, weight.dtype)
    with torch.autocast("cuda", enabled=False):
        return _Conv2dFn.apply(x_nhwc, weight, bias, stride, pad, cd)


class _CatConv2dFn(torch.autograd.Function):
    """conv2d(cat([xa, xb], channels)) without the concatenated tensor (UNet Up, unet:213-216):
    the gathers read input channels [0, Ca) from xa and [Ca, C) from xb, the input gradient is
    written as (dxa, dxb), the weight gradient reads both (csu_conv2d_*_split)."""

    @staticmethod
    def forward(ctx, xa, xb, weight, bias, pad: int, cd):
        require_device(xa, xb, weight)
        xa, xb = xa.to(cd).contiguous(), xb.to(cd).contiguous()
        B, H, W, Ca = xa.shape
        N, C, KH, KW = weight.shape
        g = _conv_geom(B, H, W, C, N, KH, KW, 1, pad)
        cached = _ACTIVE_CACHE.get_conv(weight, cd) if _ACTIVE_CACHE is not None else None
        w_ohwi = cached[0] if cached else weight.detach().permute(0, 2, 3, 1).to(cd).contiguous()
        y = torch.empty(B, g.OH, g.OW, N, dtype=cd, device=xa.device)
        bf = None if bias is None else bias.detach().float().contiguous()
        _launch("conv_fwd", lambda: lib().csu_conv2d_fwd_split(ctypes.byref(g), dtype_code(xa), ptr(xa), ptr(xb), Ca, ptr(w_ohwi),
                                                               ptr(bf), ptr(y), stream_ptr(xa.device)),
                2 * y.numel() * KH * KW * C, (xa.numel() + xb.numel() + w_ohwi.numel() + y.numel()) * 2, prec=prec_of(xa))
        ctx.save_for_backward(xa, xb, weight)
        ctx.w_ihwo = cached[1] if cached else None
        ctx.bias = bias
        _note_use(ctx, weight, bias)
        ctx.conf = (pad, cd, bias is not None, None if bias is None else bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xa, xb, weight = ctx.saved_tensors
        pad, cd, has_b, bdt = ctx.conf
        B, H, W, Ca = xa.shape
        N, C, KH, KW = weight.shape
        g = _conv_geom(B, H, W, C, N, KH, KW, 1, pad)
        dy = dy.to(cd).contiguous()
        dxa = dxb = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            w_ihwo = ctx.w_ihwo if ctx.w_ihwo is not None else weight.detach().permute(1, 2, 3, 0).to(cd).contiguous()
            dxa = torch.empty_like(xa)
            dxb = torch.empty_like(xb)
            _launch("conv_dgrad", lambda: lib().csu_conv2d_dgrad_split(ctypes.byref(g), dtype_code(dy), ptr(dy), ptr(w_ihwo),
                                                                       ptr(dxa), ptr(dxb), Ca, stream_ptr(dy.device)),
                    2 * dy.numel() * KH * KW * C, (dy.numel() + w_ihwo.numel() + dxa.numel() + dxb.numel()) * 2, prec=prec_of(dy))

        def wg():
            L = lib()
            out = torch.empty(N * KH * KW * C + N, dtype=torch.float32, device=dy.device)
            n = L.csu_conv2d_wgrad_workspace(ctypes.byref(g))
            work = torch.empty(max(n, 16), dtype=torch.uint8, device=dy.device)
            _launch("conv_wgrad", lambda: L.csu_conv2d_wgrad_split_oihw(ctypes.byref(g), dtype_code(dy), ptr(xa), ptr(xb), Ca,
                                                                        ptr(dy), ptr(out), ptr(work), n, stream_ptr(dy.device)),
                    2 * dy.numel() * KH * KW * C, (xa.numel() + xb.numel() + dy.numel()) * 2 + out.numel() * 4, prec=prec_of(dy))
            k = N * KH * KW * C
            return out[:k].view(N, C, KH, KW), out[k:]
        if _side_ok(dy, weight.dtype, bdt if has_b else None, params=(weight, ctx.bias)):
            dw, db = _side_run(wg, xa, xb, dy)
            _late((weight, ctx.bias), (dw, db if has_b else None), side=True)
            return dxa, dxb, dw, (db if has_b else None), None, None
        dw, db = wg()
        return dxa, dxb, dw.to(weight.dtype), (db.to(bdt) if has_b else None), None, None


def conv2d_cat(xa: torch.Tensor, xb: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
               pad: int = 1) -> torch.Tensor:
    """conv2d(torch.cat([xa, xb], -1), weight, bias, 1, pad) on channels-last tensors; the
    concatenation is never materialised when csu_conv2d_split_ok accepts the geometry (bf16),
    otherwise it is (and conv2d runs on it)."""
    if xa.is_cuda and torch.is_autocast_enabled("cuda"):
        cd = torch.get_autocast_dtype("cuda")
    else:
        cd = torch.promote_types(torch.promote_types(xa.dtype, xb.dtype), weight.dtype)
    B, H, W, Ca = xa.shape
    N, C, KH, KW = weight.shape
    if Ca + xb.shape[-1] != C:
        raise ValueError(f"conv2d_cat: {Ca} + {xb.shape[-1]} input channels, weight expects {C}")
    g = _conv_geom(B, H, W, C, N, KH, KW, 1, pad)
    if cd == torch.bfloat16 and xa.is_cuda and lib().csu_conv2d_split_ok(ctypes.byref(g), Ca):
        with torch.autocast("cuda", enabled=False):
            return _CatConv2dFn.apply(xa, xb, weight, bias, pad, cd)
    return conv2d(torch.cat([xa.to(cd), xb.to(cd)], dim=-1), weight, bias, 1, pad)


class _ConvTranspose2dFn(torch.autograd.Function):
    """ConvTranspose2d(k, stride=k, pad 0) = the input-gradient operator of the matching conv."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride: int, cd):
        require_device(x, weight)
        xc = (x if x.dtype == cd else x.to(cd)).contiguous()
        B, H, W, N = xc.shape                       # N = in channels of the transposed conv
        Nw, C, KH, KW = weight.shape                # torch ConvTranspose2d weight (in, out, kh, kw)
        OH, OW = (H - 1) * stride + KH, (W - 1) * stride + KW
        g = _conv_geom(B, OH, OW, C, N, KH, KW, stride, 0)
        w_ihwo = weight.detach().permute(1, 2, 3, 0).to(cd).contiguous()
        y = torch.empty(B, OH, OW, C, dtype=cd, device=x.device)
        bf = None if bias is None else bias.detach().float().contiguous()
        _launch("convT_fwd", lambda: lib().csu_conv2d_dgrad(ctypes.byref(g), dtype_code(xc), ptr(xc), ptr(w_ihwo), ptr(bf),
                                                            ptr(y), stream_ptr(x.device)),
                2 * xc.numel() * KH * KW * C, (xc.numel() + w_ihwo.numel() + y.numel()) * xc.element_size(), prec=prec_of(xc))
        ctx.save_for_backward(xc, weight)
        ctx.conf = (stride, cd, x.dtype, bias is not None, None if bias is None else bias.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, weight = ctx.saved_tensors
        stride, cd, xdt, has_b, bdt = ctx.conf
        B, H, W, N = xc.shape
        _, C, KH, KW = weight.shape
        dy = dy.to(cd).contiguous()
        g = _conv_geom(B, dy.shape[1], dy.shape[2], C, N, KH, KW, stride, 0)
        dx = None
        if ctx.needs_input_grad[0]:
            w_ohwi = weight.detach().permute(0, 2, 3, 1).to(cd).contiguous()
            dx = torch.empty(B, H, W, N, dtype=cd, device=dy.device)
            _launch("convT_dgrad", lambda: lib().csu_conv2d_fwd(ctypes.byref(g), dtype_code(dy), ptr(dy), ptr(w_ohwi), None,
                                                                ptr(dx), stream_ptr(dy.device)),
                    2 * dx.numel() * KH * KW * C, (dy.numel() + w_ohwi.numel() + dx.numel()) * dy.element_size(),
                    prec=prec_of(dy))
            if dx.dtype != xdt:
                dx = dx.to(xdt)
        dw, _ = _conv_wgrad(g, dy, xc, dtype_code(dy))   # roles swapped: "input" = dy, "output grad" = x
        db = colsum(dy.view(-1, C)).to(bdt) if has_b else None
        return dx, dw.to(weight.dtype), db, None, None


def conv_transpose2d(x_nhwc: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                     stride: int) -> torch.Tensor:
    """nn.ConvTranspose2d(k, stride) with padding 0 on channels-last tensors."""
    if x_nhwc.is_cuda and torch.is_autocast_enabled("cuda"):
        cd = torch.get_autocast_dtype("cuda")
    else:
        cd = torch.promote_types(x_nhwc.dtype, weight.dtype)
    with torch.autocast("cuda", enabled=False):
        return _ConvTranspose2dFn.apply(x_nhwc, weight, bias, stride, cd)
