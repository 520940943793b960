"""Training-level parity on the MI355X (north_star: "Dice/IoU parity at fixed seed, Dice within
1e-3 of the reference").

* F8 / F11 trajectories: the csu CSWinTransformer trained through csu.train.train_model (graph-
  captured steps) on the reference's own batch stream (recipe weights, default_rng(1234) batches,
  AdamW 1e-4 / wd 1e-4; eval every 20 steps on a default_rng(99) batch) vs the reference's own run
  (tests/golden/f8_trajectory.json: 128x128 B8 split [1,2,4,4], 400 steps; f11_trajectory_512.json:
  the headline geometry 512x512 B4 split [1,2,8,8]; made by tests/golden/make_golden.py =
  cswin:775-811 / 692-747).  The reference was also run under bf16 autocast (the *_bf16.json files).
  Its OWN fp32-vs-bf16 spread does not settle at 4e-4 (SURVEY §8c's 120-step estimate): the eval
  Dice moves by ~1e-3 between checkpoints at lr 1e-4, any change of rounding shifts that walk, and
  the reference's bf16 run sits up to 8.9e-4 (128x128) / 4.5e-3 (512x512) away from its fp32 run at
  single checkpoints.  Gates (north_star "Dice within 1e-3"; IoU = Dice / (2 - Dice) for these
  batch-flattened metrics, so its tolerance is 2e-3):
    - converged window = eval steps from the first one after which the reference's own fp32/bf16
      spread stays within those tolerances;
    - csu fp32: EVERY checkpoint of the window within 1e-3 / 2e-3 of the reference fp32 run (the
      measured distance is ~3e-8: the same trajectory);
    - csu bf16: the window's MEAN Dice / IoU within 1e-3 / 2e-3 of the reference fp32 run's, every
      single checkpoint within 5e-3 (the reference's own worst bf16 checkpoint distance), and the
      per-epoch mean train loss within max(5 %, 1.5 x the reference's own fp32/bf16 spread of that
      epoch) in the window (the reference's bf16 run is up to 7.8 % off its fp32 run per epoch at
      512x512 late in training, where the loss is ~5e-3; fp32: 2 % everywhere);
    - csu bf16 vs the reference's OWN bf16 run (like for like): the window MEAN within 1e-3 / 2e-3,
      every checkpoint within the bf16 checkpoint tolerance above (5e-3 / 1e-2).  A tighter
      per-checkpoint gate does not hold for two bf16 runs with different rounding points: on F8 the
      measured distances are 6e-6 .. 1.7e-3 except one checkpoint of 3.4e-3 (step 160, while the Dice
      still climbs ~1.5e-3 per checkpoint; profiles/r06_dice_parity_f8_trajectory_bf16.json).
  Every eval point's values and deltas are written to $CSU_PARITY_LOG (default gpurun_out/) as
  dice_parity_<fixture>_<precision>.json (committed copies: profiles/r03_dice_parity_*.json).
* FusedAdamW checkpoints: save -> load -> continue equals the uninterrupted run; the state_dict
  loads into torch.optim.AdamW; a load after a capture keeps the captured step valid.
* HIP-graph replays are bitwise reproducible across two independent captures.
* Deep config (depth [2,4,32,2]) vs the oracle."""
import copy
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import cswin_ref as O

DICE_TOL = 1e-3    # north_star: "Dice within 1e-3 of the reference"
IOU_TOL = 2e-3     # the same tolerance carried to IoU = Dice / (2 - Dice) (dIoU/dDice ~ 1.9 at Dice ~ 0.98)


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


class _Stream:
    """The fixture's batch stream, drawn lazily: epoch e yields batches [n*e, n*e + n) of
    default_rng(train_rng) (the reference's order)."""

    def __init__(self, seed, batch, size, per_epoch):
        self.rng, self.batch, self.size, self.per_epoch = np.random.default_rng(seed), batch, size, per_epoch

    def __iter__(self):
        from csu.data import ellipse_batch
        return iter([ellipse_batch(self.rng, self.batch, self.size) for _ in range(self.per_epoch)])


def gate_step(ref, refb):
    """First eval step from which the reference's own fp32-vs-bf16 |dDice| and |dIoU| stay within
    DICE_TOL / IOU_TOL."""
    ok = [abs(a - b) <= DICE_TOL and abs(c - e) <= IOU_TOL
          for a, b, c, e in zip(ref["eval_dice"], refb["eval_dice"], ref["eval_iou"], refb["eval_iou"])]
    i = len(ok)
    while i > 0 and ok[i - 1]:
        i -= 1
    return ref["eval_step"][i] if i < len(ok) else None


def _traj_run(golden_dir, fixture, amp_dtype):
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss, make_optimizer, train_model
    d = dev()
    ref = json.load(open(os.path.join(golden_dir, fixture + ".json")))
    refb = json.load(open(os.path.join(golden_dir, fixture + "_bf16.json")))
    c = ref["config"]
    every = c.get("eval_every", 20)
    cfg = O.CSWinConfig(img_size=c["img_size"], split_size=tuple(c["split_size"]))
    m = CSWinTransformer(img_size=c["img_size"], split_size=list(c["split_size"])).to(d)
    m.load_state_dict(O.recipe_params(cfg, seed=c["seed_weights"]))
    test = [ellipse_batch(np.random.default_rng(c["eval_rng"]), c.get("eval_n", 16), c["img_size"])]
    opt = make_optimizer(m, lr=c["lr"], weight_decay=c["weight_decay"])
    h = train_model(m, _Stream(c["train_rng"], c["batch"], c["img_size"], every), test, bce_loss, opt, None, d,
                    num_epochs=c["steps"] // every, verbose=False, amp_dtype=amp_dtype)
    return ref, refb, h


def _check_trajectory(golden_dir, fixture, amp):
    ref, refb, h = _traj_run(golden_dir, fixture, amp)
    steps = ref["eval_step"]
    every = ref["config"].get("eval_every", 20)
    assert len(h["test_dice"]) == len(steps)
    g = gate_step(ref, refb)
    assert g is not None and sum(s >= g for s in steps) >= 3, \
        f"{fixture}: the reference's own fp32/bf16 spread never settles within the tolerance for 3 eval points"
    ltol = 0.02 if amp is None else 0.05
    point_tol = (DICE_TOL, IOU_TOL) if amp is None else (5e-3, 1e-2)
    rows, bad = [], []
    for i, s in enumerate(steps):
        dd = abs(h["test_dice"][i] - ref["eval_dice"][i])
        di = abs(h["test_iou"][i] - ref["eval_iou"][i])
        mean_ref = float(np.mean(ref["loss"][every * i:every * i + every]))
        own = abs(float(np.mean(refb["loss"][every * i:every * i + every])) - mean_ref) / mean_ref
        ltol_i = ltol if amp is None else max(ltol, 1.5 * own)
        rows.append({"step": s, "gated": s >= g, "csu_dice": h["test_dice"][i], "ref_dice": ref["eval_dice"][i],
                     "ref_bf16_dice": refb["eval_dice"][i], "ref_bf16_iou": refb["eval_iou"][i], "abs_d_dice": dd,
                     "abs_d_dice_vs_ref_bf16": abs(h["test_dice"][i] - refb["eval_dice"][i]),
                     "abs_d_iou_vs_ref_bf16": abs(h["test_iou"][i] - refb["eval_iou"][i]),
                     "ref_own_spread_dice": abs(ref["eval_dice"][i] - refb["eval_dice"][i]),
                     "ref_own_spread_iou": abs(ref["eval_iou"][i] - refb["eval_iou"][i]),
                     "csu_iou": h["test_iou"][i],
                     "ref_iou": ref["eval_iou"][i], "abs_d_iou": di, "csu_eval_loss": h["test_loss"][i],
                     "ref_eval_loss": ref["eval_loss"][i], "csu_train_loss": h["train_loss"][i],
                     "ref_train_loss": mean_ref, "ref_own_rel_spread_train_loss": own, "train_loss_rel_tol": ltol_i})
        if s >= g and (dd > point_tol[0] or di > point_tol[1]):
            bad.append(f"step {s}: |dDice| {dd:.2e} |dIoU| {di:.2e}")
        if (amp is None or s >= g) and abs(h["train_loss"][i] - mean_ref) > ltol_i * mean_ref:
            bad.append(f"epoch {i}: train loss {h['train_loss'][i]:.5f} vs {mean_ref:.5f}")
    gated = [r for r in rows if r["gated"]]
    mean = lambda k: float(np.mean([r[k] for r in gated]))   # noqa: E731
    win = {"csu_dice": mean("csu_dice"), "ref_dice": mean("ref_dice"), "ref_bf16_dice": mean("ref_bf16_dice"),
           "csu_iou": mean("csu_iou"), "ref_iou": mean("ref_iou")}
    win["abs_d_dice"] = abs(win["csu_dice"] - win["ref_dice"])
    win["abs_d_iou"] = abs(win["csu_iou"] - win["ref_iou"])
    win["ref_own_abs_d_dice"] = abs(win["ref_bf16_dice"] - win["ref_dice"])
    if win["abs_d_dice"] > DICE_TOL or win["abs_d_iou"] > IOU_TOL:
        bad.append(f"window mean: |dDice| {win['abs_d_dice']:.2e} |dIoU| {win['abs_d_iou']:.2e}")
    like = None
    if amp is not None:
        # like for like: csu bf16 vs the reference's OWN bf16-autocast run of the same trajectory --
        # the window mean at the north_star tolerance, every converged checkpoint at the bf16 checkpoint
        # tolerance (two bf16 runs with different rounding points; the reference's own fp32 / bf16 pair
        # differs by up to 4.5e-3 at single checkpoints)
        like = {"csu_dice": win["csu_dice"], "ref_bf16_dice": win["ref_bf16_dice"],
                "csu_iou": win["csu_iou"], "ref_bf16_iou": mean("ref_bf16_iou")}
        like["abs_d_dice"] = abs(like["csu_dice"] - like["ref_bf16_dice"])
        like["abs_d_iou"] = abs(like["csu_iou"] - like["ref_bf16_iou"])
        like["max_checkpoint_abs_d_dice"] = max(r["abs_d_dice_vs_ref_bf16"] for r in gated)
        like["max_checkpoint_abs_d_iou"] = max(r["abs_d_iou_vs_ref_bf16"] for r in gated)
        like["checkpoint_tolerance"] = point_tol
        if like["abs_d_dice"] > DICE_TOL or like["abs_d_iou"] > IOU_TOL:
            bad.append(f"vs reference bf16, window mean: |dDice| {like['abs_d_dice']:.2e} |dIoU| {like['abs_d_iou']:.2e}")
        if like["max_checkpoint_abs_d_dice"] > point_tol[0] or like["max_checkpoint_abs_d_iou"] > point_tol[1]:
            bad.append(f"vs reference bf16, checkpoint: |dDice| {like['max_checkpoint_abs_d_dice']:.2e} "
                       f"|dIoU| {like['max_checkpoint_abs_d_iou']:.2e}")
    prec = "fp32" if amp is None else "bf16"
    log = {"fixture": fixture, "precision": prec, "config": ref["config"], "gate_from_step": g, "dice_tolerance": DICE_TOL,
           "iou_tolerance": IOU_TOL, "checkpoint_tolerance": point_tol, "window_mean": win,
           "max_gated_abs_d_dice": max(r["abs_d_dice"] for r in gated),
           "max_gated_abs_d_iou": max(r["abs_d_iou"] for r in gated), "vs_reference_bf16": like, "rows": rows}
    out = os.environ.get("CSU_PARITY_LOG", "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"dice_parity_{fixture}_{prec}.json"), "w") as f:
        json.dump(log, f, indent=1)
    print(f"{fixture} {prec}: gate from step {g}, window mean |dDice| {win['abs_d_dice']:.2e} |dIoU| "
          f"{win['abs_d_iou']:.2e}, max checkpoint |dDice| {log['max_gated_abs_d_dice']:.2e}")
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("amp", [None, torch.bfloat16], ids=["fp32", "bf16"])
def test_f8_dice_iou_trajectory(golden_dir, amp):
    _check_trajectory(golden_dir, "f8_trajectory", amp)


def test_f11_dice_iou_trajectory_512_bf16(golden_dir):
    """The headline configuration's geometry and precision: 512x512 split [1,2,8,8], bf16."""
    _check_trajectory(golden_dir, "f11_trajectory_512", torch.bfloat16)


def test_fused_adamw_checkpoint_resume_and_torch_interop(tmp_path):
    """FusedAdamW save -> load -> continue == uninterrupted (bitwise); its state_dict drives
    torch.optim.AdamW to the same parameters (fp32 tolerance; per-parameter step tensors)."""
    from csu.optim import FusedAdamW
    from csu.report import load_checkpoint, save_checkpoint
    d = dev()
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.GELU(), torch.nn.Linear(128, 8)).to(d)
    xs = [torch.randn(32, 64, device=d) for _ in range(6)]

    def step(m, o, x):
        o.zero_grad(set_to_none=True)
        m(x).square().mean().backward()
        o.step()
    a = copy.deepcopy(net)
    oa = FusedAdamW(a.parameters(), lr=1e-3, weight_decay=1e-2)
    for x in xs:
        step(a, oa, x)
    b = copy.deepcopy(net)
    ob = FusedAdamW(b.parameters(), lr=1e-3, weight_decay=1e-2)
    for x in xs[:3]:
        step(b, ob, x)
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, b, ob, None, 3)
    c = copy.deepcopy(net)
    oc = FusedAdamW(c.parameters(), lr=1e-3, weight_decay=1e-2)
    ep, _ = load_checkpoint(path, c, oc, None, map_location=d)
    assert ep == 3
    for x in xs[3:]:
        step(c, oc, x)
    for pa, pc in zip(a.parameters(), c.parameters()):
        assert torch.equal(pa, pc)
    # the same checkpoint continues in torch.optim.AdamW
    t = copy.deepcopy(net)
    ot = torch.optim.AdamW(t.parameters(), lr=1e-3, weight_decay=1e-2)
    load_checkpoint(path, t, ot, None, map_location=d)
    steps = {float(s["step"]) for s in ot.state_dict()["state"].values()}
    assert steps == {3.0}
    for x in xs[3:]:
        step(t, ot, x)
    assert {float(s["step"]) for s in ot.state_dict()["state"].values()} == {6.0}
    for pa, pt in zip(a.parameters(), t.parameters()):
        torch.testing.assert_close(pt, pa, rtol=1e-5, atol=1e-6)


def test_optimizer_load_after_capture_keeps_graph_valid():
    """FusedAdamW.load_state_dict after a HIP-graph capture copies the loaded moments / step / lr
    into the tensors the captured step reads: rewinding model + optimizer to an earlier checkpoint
    and replaying the same batches reproduces the original replays bitwise."""
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    d = dev()
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4]).to(d)
    opt = make_optimizer(m, capturable=True)
    rng = np.random.default_rng(4)
    b = [tuple(v.to(d) for v in ellipse_batch(rng, 2, 128)) for _ in range(4)]
    gs = GraphedTrainStep(m, opt, bce_loss, b[0][0], b[0][1], torch.bfloat16, warmup=1)
    gs(*b[0])
    gs(*b[1])
    sd_m = copy.deepcopy(m.state_dict())
    sd_o = copy.deepcopy(opt.state_dict())
    la = [float(gs(*b[i])[0].item()) for i in (2, 3)]
    pa = [p.detach().clone() for p in m.parameters()]
    m.load_state_dict(sd_m)
    opt.load_state_dict(sd_o)
    lb = [float(gs(*b[i])[0].item()) for i in (2, 3)]
    torch.cuda.synchronize()
    assert la == lb
    assert all(torch.equal(x, y) for x, y in zip(pa, m.parameters()))
    # a loaded state missing a parameter the captured step updates cannot be honoured: refused
    bad = copy.deepcopy(sd_o)
    bad["state"].pop(next(iter(bad["state"])))
    with pytest.raises(RuntimeError, match="no state for a parameter"):
        opt.load_state_dict(bad)


def test_train_model_graphed_equals_eager():
    """train_model's captured path (graph=None on a GPU: two eager steps, then one replayed graph per
    batch shape, incl. a ragged last batch run eagerly; eval replayed too) == graph=False."""
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import bce_loss, make_optimizer, train_model
    d = dev()
    torch.manual_seed(0)
    m0 = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4])
    rng = np.random.default_rng(8)
    train = [ellipse_batch(rng, 4, 128) for _ in range(5)] + [ellipse_batch(rng, 2, 128)]
    test = [ellipse_batch(rng, 4, 128), ellipse_batch(rng, 3, 128)]
    hs, ps = [], []
    for graph in (None, False):
        m = copy.deepcopy(m0).to(d)
        opt = make_optimizer(m)
        hs.append(train_model(m, train, test, bce_loss, opt, None, d, num_epochs=2, verbose=False, graph=graph))
        ps.append([p.detach().clone() for p in m.parameters()])
    for k in hs[0]:
        np.testing.assert_allclose(hs[0][k], hs[1][k], rtol=1e-5, atol=1e-6, err_msg=k)
    for a, b in zip(*ps):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("side_in_graph", [False, True])
def test_graph_replays_bitwise_reproducible(side_in_graph, monkeypatch):
    """Two independent captures of the whole bf16 train step (GraphedTrainStep) replayed on the
    same batches give bitwise-equal losses and parameters (tools/det_graph.py as a test).
    side_in_graph: the weight gradients on the second stream INSIDE the captured graph (round-1
    drift of ~1e-6 in this mode no longer reproduces -- DESIGN.md §6)."""
    from csu import ops
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    monkeypatch.setattr(ops, "_SIDE_IN_GRAPH", side_in_graph)
    d = dev()
    torch.manual_seed(0)
    m0 = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4])
    rng = np.random.default_rng(1)
    batches = [tuple(t.to(d) for t in ellipse_batch(rng, 4, 128)) for _ in range(2)]
    res = []
    for _ in range(2):
        m = copy.deepcopy(m0).to(d)
        opt = make_optimizer(m, capturable=True)
        gs = GraphedTrainStep(m, opt, bce_loss, batches[0][0], batches[0][1], torch.bfloat16, warmup=2)
        losses = [float(gs(*batches[i % 2])[0].item()) for i in range(5)]
        torch.cuda.synchronize()
        res.append((losses, [p.detach().clone() for p in m.parameters()]))
        del gs, opt
    assert res[0][0] == res[1][0]
    names = [n for n, _ in m0.named_parameters()]
    diff = [(n, float((a - b).abs().max())) for n, a, b in zip(names, res[0][1], res[1][1]) if not torch.equal(a, b)]
    assert not diff, diff


def test_late_gradients_are_stolen_not_copied():
    """Every gradient csu hands to autograd before writing it (deferred LayerNorm / Linear / concat
    Linear / LePE parameter gradients) is taken over by AccumulateGrad as the parameter's .grad in the
    eager steps and in the capture -- no copy made before the values exist (ops._check_late would
    repair one and count it; DESIGN.md §6: the round-4 concat-Linear bias nondeterminism)."""
    from csu import ops
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    d = dev()
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4]).to(d)
    x, t = (v.to(d) for v in ellipse_batch(np.random.default_rng(1), 4, 128))
    n0 = ops.STATS["late_grad_fixups"]
    ops._LATE_DEFER.clear()
    seen = []
    real = ops._late
    ops_late = lambda params, grads, side=False: (seen.append(len(params)), real(params, grads, side))  # noqa: E731
    import unittest.mock as um
    with um.patch.object(ops, "_late", ops_late):
        gs = GraphedTrainStep(m, make_optimizer(m, capturable=True), bce_loss, x, t, torch.bfloat16, warmup=2)
        gs(x, t)
    torch.cuda.synchronize()
    assert sum(seen) > 100                       # the deferred gradients were registered
    assert ops.STATS["late_grad_fixups"] == n0, ops.STATS
    assert not ops._LATE_DEFER


FULL_CONFIGS = [
    # (img, batch, depth, split, simam, fmt) -- BASELINE configs[2..4] at their full per-GPU sizes
    (512, 16, [1, 2, 9, 1], [1, 2, 8, 8], False, None),
    (512, 16, [1, 2, 9, 1], [1, 2, 8, 8], True, None),
    (512, 16, [2, 4, 32, 2], [1, 2, 8, 8], False, None),
    (1024, 4, [1, 2, 9, 1], [1, 2, 8, 8], False, None),
    (1024, 4, [1, 2, 9, 1], [1, 2, 8, 8], False, "fp8_e4m3"),
    (1024, 4, [1, 2, 9, 1], [1, 2, 8, 8], True, "fp8_e4m3"),     # configs[4] as named: +SimAM, fp8
]


@pytest.mark.parametrize("img,batch,depth,split,simam,fmt", FULL_CONFIGS)
def test_full_size_config_graphed_steps(img, batch, depth, split, simam, fmt):
    """One captured train step of every BASELINE GPU config at its full size (the bench shapes):
    finite loss, finite and non-zero gradient norm of every parameter, and the loss falls over 3
    replays on one batch."""
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    d = dev()
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=img, depth=depth, split_size=split, simam=simam).to(d)
    if fmt:
        m.set_weight_format(fmt)
    x, t = (v.to(d) for v in ellipse_batch(np.random.default_rng(3), batch, img))
    opt = make_optimizer(m, lr=1e-4, capturable=True)
    gs = GraphedTrainStep(m, opt, bce_loss, x, t, torch.bfloat16, warmup=1)
    losses = []
    for _ in range(3):
        loss, _ = gs(x, t)
        losses.append(float(loss.item()))
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)), losses
    assert losses[2] < losses[0], losses
    norms = {n: float(p.grad.float().norm()) for n, p in m.named_parameters()}
    bad = {n: v for n, v in norms.items() if not (np.isfinite(v) and v > 0)}
    assert not bad, bad
    del gs, opt, m
    torch.cuda.empty_cache()


def test_graphed_step_metrics_in_graph():
    """GraphedTrainStep(metrics=True): the per-step segmentation sums (cswin:789-795) computed by the
    fused loss kernel inside the graph equal torch's on the step's output (pred = p > 0.5)."""
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    d = dev()
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4]).to(d)
    rng = np.random.default_rng(2)
    x, t = (v.to(d) for v in ellipse_batch(rng, 4, 128))
    gs = GraphedTrainStep(m, make_optimizer(m, capturable=True), bce_loss, x, t, torch.bfloat16, warmup=2, metrics=True)
    loss, out = gs(x, t)
    torch.cuda.synchronize()
    pred = (out > 0.5).double()
    ref = torch.stack([(pred * t).sum(), pred.sum(), t.double().sum()])
    torch.testing.assert_close(gs.stats.double(), ref, rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(loss, bce_loss(out, t).detach(), rtol=1e-6, atol=1e-7)


def test_deep_config_vs_oracle():
    """Deep CSWin (BASELINE config 4 depths [2,4,32,2]) at 128x128, split [1,2,4,4], fp32:
    probabilities, loss and every gradient norm vs the fp64 oracle on the same recipe weights."""
    from csu.model import CSWinTransformer
    from csu.train import bce_loss
    from csu.data import ellipse_batch
    d = dev()
    depth = [2, 4, 32, 2]
    cfg = O.CSWinConfig(img_size=128, depth=depth, split_size=(1, 2, 4, 4))
    p = O.recipe_params(cfg, seed=0)
    m = CSWinTransformer(img_size=128, depth=depth, split_size=[1, 2, 4, 4]).to(d)
    m.load_state_dict(p)
    x, t = ellipse_batch(np.random.default_rng(5), 1, 128)
    y = m(x.to(d))
    loss = bce_loss(y, t.to(d))
    loss.backward()
    pref = {k: v.double().requires_grad_(True) for k, v in p.items()}
    yr = O.cswin_forward(pref, x.double(), cfg)
    lr = O.bce_loss(yr, t.double())
    lr.backward()
    torch.testing.assert_close(y.detach().double().cpu(), yr.detach(), rtol=1e-4, atol=1e-4)
    assert abs(loss.item() - lr.item()) < 1e-5 * lr.item() + 1e-6
    gn = np.array([q.grad.double().norm().item() for _, q in m.named_parameters()])
    gr = np.array([pref[k].grad.norm().item() for k, _ in m.named_parameters()])
    big = gr >= 1e-6 * gr.max()
    np.testing.assert_allclose(gn[big], gr[big], rtol=2e-3)


def test_capture_after_eager_steps():
    """Eager default-stream steps, then a HIP-graph capture of the same model (the order that used
    to segfault in hipGraphInstantiate): works once no earlier autograd graph is referenced (the
    model releases its skip tensors' graph after each forward), and a still-referenced output of an
    eager step is reported as an error before the capture instead of a crash."""
    from csu.data import ellipse_batch
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    d = dev()
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=128, split_size=[1, 2, 4, 4]).to(d)
    opt = make_optimizer(m, capturable=True)
    x, t = (v.to(d) for v in ellipse_batch(np.random.default_rng(0), 2, 128))

    def eager():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        bce_loss(y, t).backward()
        opt.step()
        return y
    kept = eager()
    assert m.x1 is not None and not m.x1.requires_grad        # skips kept, their graph released
    with pytest.raises(RuntimeError, match="still referenced"):
        GraphedTrainStep(m, opt, bce_loss, x, t, torch.bfloat16, warmup=1)
    del kept
    eager()
    gs = GraphedTrainStep(m, opt, bce_loss, x, t, torch.bfloat16, warmup=1)
    losses = [float(gs(x, t)[0].item()) for _ in range(3)]
    assert all(np.isfinite(losses)) and losses[2] < losses[0]
    # eager steps with the same optimizer AFTER the capture (bench.py's roofline leg) rebuild its
    # eager pointer table; the captured step keeps reading its own (kept-alive) table
    eager()
    eager()
    more = [float(gs(x, t)[0].item()) for _ in range(2)]
    assert all(np.isfinite(more)) and more[1] < losses[0]


def test_deep_config_bf16_vs_oracle():
    """Deep CSWin (BASELINE config 4: depths [2,4,32,2]) in its own precision, bf16 autocast, at 256x256
    split [1,2,8,8] (the headline's stripe geometry, stage 4 whole-window) vs the fp64 oracle on the
    same recipe weights: probabilities 1e-2 abs, loss 1e-2 rel, gradient norms >= 1e-3 of the largest
    5e-2 rel (the bf16 calibration of test_gpu_model.py), median per-tensor rel-L2 <= 2e-2."""
    from csu.model import CSWinTransformer
    from csu.train import bce_loss
    from csu.data import ellipse_batch
    d = dev()
    depth = [2, 4, 32, 2]
    cfg = O.CSWinConfig(img_size=256, depth=depth, split_size=(1, 2, 8, 8))
    p = O.recipe_params(cfg, seed=0)
    m = CSWinTransformer(img_size=256, depth=depth, split_size=[1, 2, 8, 8]).to(d)
    m.load_state_dict(p)
    x, t = ellipse_batch(np.random.default_rng(6), 1, 256)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x.to(d))
    loss = bce_loss(y, t.to(d))
    loss.backward()
    pref = {k: v.double().requires_grad_(True) for k, v in p.items()}
    yr = O.cswin_forward(pref, x.double(), cfg)
    lr = O.bce_loss(yr, t.double())
    lr.backward()
    assert float((y.detach().double().cpu() - yr.detach()).abs().max()) < 1e-2
    assert abs(loss.item() - lr.item()) < 1e-2 * lr.item()
    names = [k for k, _ in m.named_parameters()]
    gn = np.array([q.grad.double().norm().item() for _, q in m.named_parameters()])
    gr = np.array([pref[k].grad.norm().item() for k in names])
    rel = np.array([(q.grad.double().cpu() - pref[k].grad).norm().item() / max(pref[k].grad.norm().item(), 1e-30)
                    for k, q in m.named_parameters()])
    big = gr >= 1e-3 * gr.max()
    np.testing.assert_allclose(gn[big], gr[big], rtol=5e-2)
    assert np.median(rel[big]) < 2e-2, np.median(rel[big])
