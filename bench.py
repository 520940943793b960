"""Benchmark: CSWin-UNet training throughput (images/sec) at 512x512 bf16, batch 16 per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1 is launched by the driver with torch.distributed.run (one process per GPU, RCCL).
One step = forward + BCE (with the reference loop's per-step thresholded Dice / IoU sums, cswin:789-795,
fused into the loss kernel) + backward (+ bucketed RCCL gradient all-reduce, captured in the same HIP
graph, csu.dist.GradAllReduce) + fused AdamW on a batch of
synthetic 512x512 images already resident in HBM.  Prints ONE JSON line (rank 0).

roofline: every csu kernel launch of 2 eager steps of the same workload is timed live with HIP
events on its launch stream (csu.ledger: idempotent launches re-run back-to-back between the events;
HIP events cannot be recorded inside the graph replays of the timed region) and carries its
algorithmic FLOPs and bytes (each input read once, each output written once).  Per kernel:
t_roof = max(FLOPs / P_mfma, bytes / 8 TB/s); the reported object is the kernel with the most time
per step (achieved GB/s or TFLOP/s vs its peak), plus "step_frac" = sum of t_roof over every launch of
a step / ms_per_step of the timed graph replays, and the per-kernel list.  traffic = HBM bytes per
launch of that kernel from the committed rocprofv3 PMC summary for this workload
(profiles/pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950 correction), or null.
cpu_baseline: the CPU oracle (a restatement of the reference, parity-pinned to it) timed on this
host for a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "cswin-simam-unet_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402



def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                    help="fp8: e4m3 Linear weights (per-row power-of-two scales), fp32 accumulate (BASELINE config 5); "
                         "by default only the fused Mlp (C = 64 / 128 / 256 forward, C = 256 backward) runs e4m3 x e4m3 "
                         "MFMA (activations MX-quantised per 32-value block in registers); qkv, proj, concat_linear "
                         "and the C = 512 Mlp run bf16 on the exact dequantised e4m3 weights (CSU_FP8_QKV=1: qkv on "
                         "the fp8 MFMA too)")
    ap.add_argument("--model", default="cswin", choices=["cswin", "unet"],
                    help="unet: the plain UNet of train_unet_segmentation.py (BASELINE config 1's model; Adam, "
                         "use --img 128 --batch 8)")
    ap.add_argument("--depth", default="1,2,9,1")
    ap.add_argument("--split", default="1,2,8,8")
    ap.add_argument("--simam", action=argparse.BooleanOptionalAction, default=True,
                    help="SimAM gate on the skip features: the CSWin-SimAM-UNet of BASELINE configs[2] (default); "
                         "--no-simam: the reference's own architecture (train_cswinunet_segmentation.py has no SimAM)")
    ap.add_argument("--no-ref-arch", action="store_true",
                    help="skip the second timed run of the reference architecture (no SimAM) that a SimAM bench "
                         "line carries as 'reference_architecture' (N = 1 only)")
    ap.add_argument("--dropout", type=float, default=0.0,
                    help="drop_rate = attn_drop_rate = drop_path_rate (the reference main() trains at 0.3, cswin:930-932)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="capture the whole step in a HIP graph (N > 1: with the bucketed all-reduce; off: eager DDP)")
    ap.add_argument("--bucket-mb", type=float, default=32.0, help="gradient all-reduce bucket size (N > 1)")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce precision (N > 1): bf16 halves the ring bytes")
    ap.add_argument("--api", default="step", choices=["step", "train_model"],
                    help="train_model: time the drop-in csu.train.train_model (cswin:751-841) over --steps batches "
                         "(one epoch; its own graph capture after two eager steps) instead of GraphedTrainStep")
    ap.add_argument("--traffic-key", action="store_true", help="print this workload's PMC traffic key and exit")
    ap.add_argument("--side-wgrad", action="store_true",
                    help="eager steps (--graph off) compute weight gradients on the side stream (the eager "
                         "product default); without it eager steps launch exactly the kernels the captured step "
                         "replays (grouped end-of-backward weight gradients on the launch stream) -- the PMC passes "
                         "of tools/pmc_head.sh then describe the timed graph's kernels")
    ap.add_argument("--dp-force", action="store_true",
                    help="run the data-parallel path (RCCL process group + captured all-reduce) even at N = 1")
    return ap.parse_args()


def synthetic_batches(n, batch, img, device, seed):
    from csu.data import ellipse_batch
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        x, t = ellipse_batch(rng, batch, img)
        out.append((x.to(device), t.to(device)))
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    """CPU threads of the baseline: this GPU's CPU share -- OMP_NUM_THREADS (16 per GPU on the MI355X
    boxes), capped by the affinity mask.  The affinity mask lists the whole host (many times the
    share); timing on all of it would measure other jobs' cores, not this GPU's host share."""
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(share, aff))


def _cores_note(threads):
    return (f"{threads} threads = the per-GPU CPU share (OMP_NUM_THREADS); affinity mask "
            f"{len(os.sched_getaffinity(0))} cpus (the whole host)")


def cpu_baseline_unet(args, dtype):
    """Plain-UNet oracle (oracle/unet_ref.py, parity-pinned to the reference by F6) fwd+BCE+bwd+Adam
    on the same per-GPU batch: 1 warm-up + 2 timed steps."""
    from oracle import unet_ref as U
    from oracle.recipe import recipe_from_contract
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    p = recipe_from_contract(U.unet_contract(), seed=0)
    params = {k: v.requires_grad_(True) for k, v in p.items() if "running" not in k and "num_batches" not in k}
    opt = torch.optim.Adam(params.values(), lr=1e-3, weight_decay=1e-4)
    from csu.data import ellipse_batch
    b = args.batch
    x, t = ellipse_batch(np.random.default_rng(7), b, args.img)

    def step():
        opt.zero_grad()
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
            y = U.unet_forward(p, x, training=True)
        loss = torch.nn.functional.binary_cross_entropy(y.float(), t)
        loss.backward()
        opt.step()

    step()
    t0 = time.perf_counter()
    for _ in range(2):
        step()
    el = time.perf_counter() - t0
    return {"value": round(2 * b / el, 4), "unit": "images/sec", "cores": threads, "kind": "port", "cpu": _cpu_model(),
            "cores_note": _cores_note(threads),
            "sample": f"2 train steps x batch {b} at {args.img}x{args.img} "
                      f"({'bf16 autocast' if dtype == torch.bfloat16 else 'fp32'}) after 1 warm-up step, "
                      f"oracle/unet_ref.py, {el:.1f}s, {threads} threads"}


def cpu_baseline(args, dtype):
    """Oracle (CPU restatement of the reference) fwd+BCE+bwd+AdamW on the same per-GPU batch:
    1 warm-up + 2 timed steps (~10-30 s).  Threads: the process's CPU affinity, capped at 16 -- the
    GPU box's CPU share per GPU (more threads than the share only contend)."""
    from oracle import cswin_ref as O
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    cfg = O.CSWinConfig(img_size=args.img, depth=[int(v) for v in args.depth.split(",")],
                        split_size=[int(v) for v in args.split.split(",")], simam=args.simam)
    m = O.OracleCSWin(cfg, O.recipe_params(cfg, seed=0))
    pd = args.dropout
    if pd > 0:   # Bernoulli masks at every site (the reference's train-mode dropout cost)
        m.forward = lambda x: O.cswin_forward(m.params(), x, cfg, drop=lambda name, shape:
                                              (torch.rand(shape) >= pd).float() / (1 - pd))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    from csu.data import ellipse_batch
    b = args.batch
    x, t = ellipse_batch(np.random.default_rng(7), b, args.img)

    def step():
        opt.zero_grad()
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
            y = m(x)
        loss = O.bce_loss(y.float(), t)
        loss.backward()
        opt.step()

    step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while n < 2:
        step()
        n += 1
    el = time.perf_counter() - t0
    return {"value": round(n * b / el, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "cpu": _cpu_model(), "cores_note": _cores_note(threads),
            "sample": f"{n} train steps x batch {b} at {args.img}x{args.img} "
                      f"({'bf16 autocast' if dtype == torch.bfloat16 else 'fp32'}) after 1 warm-up step, "
                      f"oracle/cswin_ref.py, {el:.1f}s, {threads} threads"}


def main():
    faulthandler.enable()
    args = parse()
    if args.traffic_key:
        print(workload_key(args))
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn_workers(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and not (args.gpus == 1 and "WORLD_SIZE" in os.environ):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dp = world > 1 or args.dp_force
    if dp:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.backends.cudnn.benchmark = True
    dtype = torch.float32 if args.dtype == "fp32" else torch.bfloat16

    from csu import ops
    from csu.model import CSWinTransformer
    from csu.train import bce_loss, bce_loss_stats, make_optimizer

    depth = [int(v) for v in args.depth.split(",")]
    split = [int(v) for v in args.split.split(",")]
    torch.manual_seed(0)
    pd = args.dropout
    if args.model == "unet":
        from csu.unet import UNet
        model = UNet(3, 1).to(device)
    else:
        model = CSWinTransformer(img_size=args.img, depth=depth, split_size=split, simam=args.simam,
                                 drop_rate=pd, attn_drop_rate=pd, drop_path_rate=pd).to(device)
    if args.dtype == "fp8":
        model.set_weight_format("fp8_e4m3")
    nparams = sum(p.numel() for p in model.parameters())
    use_graph = args.graph in ("on", "auto")
    reducer = None
    if dp and use_graph:
        # graph-captured bucketed all-reduce (DDP cannot be captured; eager steps cost ~3x)
        from csu.dist import GradAllReduce
        reducer = GradAllReduce(model.named_parameters(), bucket_mb=args.bucket_mb,
                                grad_dtype=torch.bfloat16 if args.grad_dtype == "bf16" else torch.float32)
    elif dp:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local], gradient_as_bucket_view=True,
                                                          static_graph=True, bucket_cap_mb=64)
    if args.model == "unet":   # optim.Adam(lr 1e-3, weight_decay 1e-4), unet:415-420 / 486-490
        from csu.optim import FusedAdam
        opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=1e-4, capturable=use_graph)
    else:
        opt = make_optimizer(model, capturable=use_graph)
    batches = synthetic_batches(2, args.batch, args.img, device, seed=1234 + rank)
    amp = torch.bfloat16 if dtype == torch.bfloat16 else None

    def eager_step(i):
        x, t = batches[i % len(batches)]
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp is not None):
            y = model(x)
        loss, _ = bce_loss_stats(y, t)   # + the reference loop's per-step Dice / IoU sums (cswin:789-795)
        loss.backward()
        if reducer is not None:
            reducer.finish()
        opt.step()
        return loss

    if not use_graph and not args.side_wgrad:
        ops.SIDE_WGRAD = False   # the captured step never uses the side stream (ops._side_ok)
    if args.api == "train_model":
        return _bench_train_model(args, model, batches, reducer, amp, nparams, world, rank, dp, device)
    step = eager_step
    if use_graph:
        # capture first (its eager warm-up runs on a side stream).  Eager steps may precede the
        # capture as long as nothing keeps their autograd graph alive (GraphedTrainStep raises
        # otherwise; the cause of the former hipGraphInstantiate segfault)
        from csu.train import GraphedTrainStep
        gstep = GraphedTrainStep(model, opt, bce_loss, batches[0][0], batches[0][1], amp, warmup=args.warmup,
                                 reducer=reducer, metrics=True)

        def step(i):
            x, t = batches[i % len(batches)]
            return gstep(x, t)[0]
    else:
        for i in range(args.warmup):
            eager_step(i)
    # roofline leg.  With the graph (any N): AFTER the timed region, rank 0 captures the same step
    # twice more WITHOUT the all-reduce (no collective, so no other rank takes part): once plain,
    # whose replays give the unbracketed step time, and once with an external HIP event-record node
    # around every csu launch (csu_event_record_ext), replayed 3 times -> each kernel's time inside the
    # replayed step; the per-launch bracket cost is calibrated against the plain replays.  Eager
    # bench: every launch of 2 eager steps, timed with HIP events on its launch stream.
    ledger = None
    graph_ledger = use_graph and not args.no_roofline
    if not args.no_roofline and not graph_ledger:
        from csu.ledger import KernelLedger
        ledger = KernelLedger(repeat=4)
        side, ops.SIDE_WGRAD = ops.SIDE_WGRAD, False   # serialized, like the single-stream graph replay
        try:
            with ledger:
                for i in range(2):
                    eager_step(i)
        finally:
            ops.SIDE_WGRAD = side
    for i in range(2):
        step(i)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=device)
    if dp:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    images = args.batch * world * args.steps
    lsteps = 2
    ledger_step_ms = None
    if graph_ledger and rank == 0:
        # the timed graph is not replayed again: these captures re-fill the optimizer's pointer table
        from csu.ledger import KernelLedger
        from csu.train import GraphedTrainStep
        if reducer is not None:
            reducer.remove()              # no all-reduce in the ledger captures
        plain = GraphedTrainStep(model, opt, bce_loss, batches[0][0], batches[0][1], amp, warmup=1, metrics=True)
        for i in range(2):
            plain(*batches[i % len(batches)])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(3):
            plain(*batches[i % len(batches)])
        torch.cuda.synchronize()
        ledger_step_ms = (time.perf_counter() - t1) / 3 * 1e3
        del plain
        ledger = KernelLedger(graph=True)
        with ledger:
            lstep = GraphedTrainStep(model, opt, bce_loss, batches[0][0], batches[0][1], amp, warmup=1,
                                     metrics=True)
        for i in range(3):
            lstep(*batches[i % len(batches)])
            ledger.collect()
        lsteps = 1
    elif graph_ledger:
        ledger = None
    roof = None
    if ledger is not None and os.environ.get("CSU_LEDGER_DUMP"):
        with open(os.environ["CSU_LEDGER_DUMP"], "w") as f:
            json.dump(ledger.launches(), f)
    if ledger is not None:
        roof = _roofline(ledger.summary(steps=lsteps), ledger_step_ms or el / args.steps * 1e3, args, graph=graph_ledger)
        if graph_ledger:
            roof["step_frac"] = round(roof["step_t_roof_ms"] / (el / args.steps * 1e3), 4)   # vs the TIMED step
            roof["ledger_step_ms"] = round(ledger_step_ms, 3)
        roof["ledger"] = "graph replays (external HIP event nodes)" if graph_ledger else "eager steps (HIP events)"
    ref_arch = None
    if (args.model == "cswin" and args.simam and world == 1 and not dp and use_graph and not args.no_ref_arch):
        ref_arch = _time_ref_arch(args, device, amp, batches, depth, split, pd)
    cpu = None
    if rank == 0 and world == 1 and (args.cpu_baseline == "on" or (args.cpu_baseline == "auto")):
        try:
            cpu = (cpu_baseline_unet if args.model == "unet" else cpu_baseline)(args, dtype)
        except Exception as e:  # baseline is informational; never hide the GPU number
            cpu = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        rec = {"metric": _metric(args), "value": round(images / el, 3),
               "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": _dtype_label(args), "data": "synthetic (ellipse masks, SURVEY §8d), random-init weights",
               "config": {"workload": (f"plain UNet train step {args.img}x{args.img}, Adam" if args.model == "unet" else
                                       f"CSWin-UNet train step {args.img}x{args.img} depth {depth} split {split}"
                                       f"{' +SimAM' if args.simam else ''}"
                                       f"{f', dropout/attn_drop/drop_path {pd}' if pd > 0 else ''}, AdamW"),
                          "model": "UNet" if args.model == "unet" else "CSWinTransformer", "params": nparams, "global_batch": args.batch * world,
                          "per_gpu_batch": args.batch, "img": args.img, "parallelism": f"dp{world}",
                          "dropout": pd, "workload_key": workload_key(args)},
               "roofline": roof, "cpu_baseline": cpu, "final_loss": round(float(loss.item()), 5),
               "hip_graph": use_graph,
               "grad_allreduce": None if not dp else ("graph-captured buckets" if reducer is not None else "DDP eager")}
        if ref_arch is not None:
            rec["reference_architecture"] = ref_arch
        if reducer is not None:   # of the captured step: buckets, how many started during backward, copy-ins
            rec["grad_buckets"] = {"buckets": len(reducer.buckets), "started_in_backward": reducer.last_early,
                                   "grads_copied_in": reducer.last_copied, "bucket_mb": args.bucket_mb,
                                   "grad_dtype": args.grad_dtype}
        print(json.dumps(rec), flush=True)
    if dp:
        dist.destroy_process_group()


def _time_ref_arch(args, device, amp, batches, depth, split, pd):
    """The same step (graph-captured, same batches, warm-up and step count) on the reference's own
    architecture -- CSWinTransformer without SimAM, the model train_cswinunet_segmentation.py trains
    and the Dice parity is pinned on -- timed right after the headline SimAM line."""
    from csu.model import CSWinTransformer
    from csu.train import GraphedTrainStep, bce_loss, make_optimizer
    torch.manual_seed(0)
    m = CSWinTransformer(img_size=args.img, depth=depth, split_size=split, simam=False, drop_rate=pd,
                         attn_drop_rate=pd, drop_path_rate=pd).to(device)
    if args.dtype == "fp8":
        m.set_weight_format("fp8_e4m3")
    opt = make_optimizer(m, capturable=True)
    gs = GraphedTrainStep(m, opt, bce_loss, batches[0][0], batches[0][1], amp, warmup=args.warmup, metrics=True)
    for i in range(2):
        gs(*batches[i % len(batches)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        gs(*batches[i % len(batches)])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = {"value": round(args.batch * args.steps / el, 3), "unit": "images/sec", "ms_per_step": round(el / args.steps * 1e3, 3),
           "steps": args.steps, "warmup": args.warmup,
           "workload": f"CSWin-UNet train step {args.img}x{args.img} depth {depth} split {split} without SimAM "
                       f"(the reference architecture, cswin:489-688), AdamW, same batches"}
    del gs, opt, m
    torch.cuda.empty_cache()
    return out


def _bench_train_model(args, model, batches, reducer, amp, nparams, world, rank, dp, device):
    """The reference-API path: csu.train.train_model over `steps` device-resident batches (one epoch,
    an empty test loader), after a warm-up call whose epoch covers the eager warm-up steps and the
    capture -- the graph is kept per model across calls."""
    from csu.train import bce_loss, make_optimizer, train_model
    opt = make_optimizer(model)
    warm = [batches[i % len(batches)] for i in range(max(3, args.warmup + 3))]
    train_model(model, warm, [], bce_loss, opt, None, device, num_epochs=1, verbose=False, amp_dtype=amp,
                reducer=reducer)
    loader = [batches[i % len(batches)] for i in range(args.steps)]
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    h = train_model(model, loader, [], bce_loss, opt, None, device, num_epochs=1, verbose=False, amp_dtype=amp,
                    reducer=reducer)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=device)
    if dp:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    if rank == 0:
        rec = {"metric": _metric(args), "value": round(args.batch * world * args.steps / el, 3), "unit": "images/sec",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
               "data": "synthetic (ellipse masks, SURVEY §8d), random-init weights",
               "config": {"workload": f"csu.train.train_model epoch of {args.steps} steps at {args.img}x{args.img} "
                                      f"(drop-in API, cswin:751-841), AdamW",
                          "model": "CSWinTransformer", "params": nparams, "global_batch": args.batch * world,
                          "per_gpu_batch": args.batch, "img": args.img, "parallelism": f"dp{world}"},
               "api": "train_model", "roofline": None, "cpu_baseline": None,
               "train_loss": round(h["train_loss"][-1], 5)}
        print(json.dumps(rec), flush=True)
    if dp:
        dist.destroy_process_group()


def _dtype_label(args):
    """The arithmetic the step runs in.  fp8: which GEMMs run e4m3 x e4m3 MFMA at this HEAD's defaults."""
    if args.dtype != "fp8":
        return args.dtype
    from csu import ops
    bwd = "/".join(str(c) for c in ops.FP8_MLP_BWD_C)
    scope = "fused Mlp fwd (C 64/128/256)" + (f" + bwd (C {bwd})" if bwd else "") + (" + qkv" if ops.FP8_QKV else "")
    ws = "; qkv / proj weights streamed as e4m3 (widened to bf16 in registers)" if ops.FP8_WS else ""
    return f"fp8-e4m3 x e4m3 MFMA ({scope}){ws}; bf16 MFMA on the dequantised e4m3 weights elsewhere"


def _metric(args):
    """BASELINE.json's metric string for its headline workload (512x512 bf16, default depth); the
    same form naming the resolution / precision otherwise."""
    if args.model == "unet":
        return f"images/sec at {args.img}x{args.img} {args.dtype} (plain UNet train step)"
    if (args.img, args.dtype, args.depth, args.split, args.dropout, args.simam) == (512, "bf16", "1,2,9,1", "1,2,8,8", 0.0,
                                                                                  True):
        try:
            with open(os.path.join(REPO, "BASELINE.json")) as f:
                return json.load(f)["metric"]
        except Exception:
            pass
    extra = "".join([", SimAM" if args.simam else ", reference architecture (no SimAM)",
                     f", dropout {args.dropout}" if args.dropout > 0 else ""])
    return f"images/sec at {args.img}x{args.img} {args.dtype} (CSWin-UNet train step{extra})"


def _debracket(kernels, ms_per_step):
    """Graph ledger: every launch is timed between two external event nodes, and such a bracket adds
    a roughly constant cost per launch (its dispatch and completion; ~15 % on a 14-us token GEMM,
    DESIGN.md §4).  The replayed step itself has no idle gaps (rocprof kernel-busy = 99.6 % of the
    wall step, profiles/r02ar_groups_512.md), so the per-launch bracket cost is calibrated on the
    real kernels of this very step: b = (sum of bracketed times - ms_per_step) / launches per step,
    and b is subtracted from every launch (each kept at >= 1/2 of its bracketed time).  Fractions
    then follow the kernels' own durations (rocprofv3) instead of reading ~15 % low."""
    total = sum(k["us_per_step"] for k in kernels)
    launches = sum(k["launches_per_step"] for k in kernels)
    b = max(0.0, (total - ms_per_step * 1e3) / max(launches, 1e-9))
    out = []
    for k in kernels:
        k = dict(k)
        avg = max(k["avg_us"] - b, 0.5 * k["avg_us"])
        scale = k["avg_us"] / avg if avg > 0 else 1.0
        k["bracketed_avg_us"] = k["avg_us"]
        k["avg_us"] = round(avg, 3)
        k["us_per_step"] = round(avg * k["launches_per_step"], 3)
        for f in ("achieved_GBs", "achieved_TFLOPs"):
            if k.get(f) is not None:
                k[f] = round(k[f] * scale, 3)
        if k.get("frac") is not None:
            k["frac"] = round(k["frac"] * scale, 4)
        out.append(k)
    out.sort(key=lambda k: -k["us_per_step"])
    return out, b


def _roofline(kernels, ms_per_step, args, graph=False):
    """Dominant kernel (most time per step) vs its roofline, the step fraction and the table."""
    bracket = None
    if graph:
        kernels, bracket = _debracket(kernels, ms_per_step)
    top = kernels[0]
    if top["bound"] == "hbm":
        achieved, peak, unit = top["achieved_GBs"], 8000.0, "GB/s"
    else:
        from csu.ledger import PEAK_TFLOPS
        achieved, peak, unit = top["achieved_TFLOPs"], PEAK_TFLOPS[top["precision"]], "TFLOP/s"
    t_roof_step = sum(k["t_roof_us"] * k["launches_per_step"] for k in kernels) / 1e3
    return {"kernel": top["kernel"], "bound": top["bound"], "achieved": achieved, "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": _pmc_traffic(top["kernel"], args),
            "avg_us": top["avg_us"], "launches_per_step": top["launches_per_step"],
            "bytes_per_launch": top["bytes_per_launch"], "flops_per_launch": top["flops_per_launch"],
            "step_frac": round(t_roof_step / ms_per_step, 4), "step_t_roof_ms": round(t_roof_step, 3),
            "kernel_ms_per_step": round(sum(k["us_per_step"] for k in kernels) / 1e3, 3),
            "bracket_us_per_launch": None if bracket is None else round(bracket, 3),
            "kernels": kernels}


def workload_key(args) -> str:
    """The workload a PMC traffic figure belongs to: model, depth / split / SimAM (CSWin), the --dtype
    argument, image size, per-GPU batch and dropout.  Lines of another workload never share a key."""
    if args.model == "unet":
        k = f"unet|{args.dtype}|{args.img}|{args.batch}"
    else:
        k = (f"cswin|d{args.depth}|s{args.split}|{'simam' if args.simam else 'nosimam'}|{args.dtype}|{args.img}|"
             f"{args.batch}")
    return k + (f"|drop{args.dropout}" if args.dropout > 0 else "")


def _pmc_traffic(kernel, args):
    """HBM bytes per launch of `kernel` for THIS workload from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json: {"<kernel>|<workload_key>": bytes}, tools/pmc_traffic.py), else None
    (never another workload's counter)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get(f"{kernel}|{workload_key(args)}")
    except Exception:
        return None


def _spawn_workers(args) -> int:
    """--gpus N > 1 without a torch.distributed launcher: start N ranks with torch.distributed.run as
    a CHILD process (nothing here has touched the GPU yet) and return its exit code.  Refuses when
    the node has fewer than N GPUs: a multi-GPU request never silently reports a 1-GPU number."""
    import socket
    import subprocess
    n = torch.cuda.device_count()      # does not initialise the GPU on this image
    if n < args.gpus:
        print(f"bench.py: --gpus {args.gpus} requested but only {n} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


if __name__ == "__main__":
    sys.exit(main() or 0)
