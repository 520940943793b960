"""Group a rocprofv3 kernel trace (graph-replayed bench steps) by csu C-ABI call, the same names as
the csu.ledger per-kernel list in bench.py's roofline, and compare with a bench JSON:
    python tools/prof_groups.py <kernel_trace.csv> <steps> [bench.json]
Steps are delimited by the AdamW kernel (one per step); the last <steps> steps are used."""
import collections
import csv
import json
import sys

# kernel-name fragment -> ledger name (first match wins)
GROUPS = [("head_fold_bwd", "carafe_head_bwd"), ("head_fold_fwd", "head_fold"), ("gemm_ws_kernel", "gemm"), ("frag_layout", "frag_layout"), ("lepe_wgrad", "stripe_attn_bwd"), ("wgrad_tile", "linear_wgrad"), ("wgrad_group", "linear_wgrad"), ("lepe_reduce", "stripe_attn_bwd"), ("wslab_reduce", "linear_wgrad"), ("wgrad_f32", "linear_wgrad"),
          ("stripe_fwd", "stripe_attn_fwd"), ("stripe_bwd", "stripe_attn_bwd"), ("lepe_wgrad", "stripe_attn_bwd"),
          ("stripe_delta", "stripe_attn_bwd"),
          ("gemm4_kernel", "gemm"), ("gemm3_kernel", "gemm"), ("gemm_kernel", "gemm"),
          ("ln_fwd", "layernorm_fwd"), ("ln_bwd", "layernorm_bwd"), ("ln_param_reduce", "layernorm_bwd"),
          ("mlp_fwd_kernel", "mlp_fwd"), ("mlp_bwd_kernel", "mlp_bwd"), ("mlp_fwd8_kernel", "mlp_fwd"), ("mlp_bwd8_kernel", "mlp_bwd"), ("mlp_bwd64_persist", "mlp_bwd"), ("mlp_bwd_deep", "mlp_bwd"), ("mlp_fwd_deep", "mlp_fwd"), ("mlp_fp8_fwd", "mlp_fwd"), ("mlp_fp8_bwd", "mlp_bwd"),
          ("conv_wgrad", "conv_wgrad"), ("conv3_wgrad_halo", "conv_wgrad"), ("igemm_bf16", "conv_fwd+conv_dgrad"),
          ("igemm_dma", "conv_fwd+conv_dgrad"), ("conv3_halo64", "conv_fwd+conv_dgrad"), ("conv3_c16", "conv_fwd+conv_dgrad"), ("conv3_c16d", "conv_fwd+conv_dgrad"), ("conv_split_reduce", "conv_fwd+conv_dgrad"), ("conv_gemm", "conv_fwd+conv_dgrad"),
          ("bn_stats", "bn_relu_fwd"), ("bn_apply", "bn_relu_fwd"), ("bn_grad", "bn_relu_bwd"), ("maxpool2_fwd", "maxpool2_fwd"),
          ("maxpool2_bwd", "maxpool2_bwd"),
          ("carafe_head_fwd", "carafe_head_fwd"), ("carafe_head_bwd", "carafe_head_bwd"),
          ("carafe_fwd", "carafe_fwd"), ("carafe_bwd", "carafe_bwd"),
          ("adamw_kernel", "adamw"), ("cast_batch", "cast_bf16_batch"), ("colsum", "colsum"),
          ("simam_stats", "simam_fwd"), ("simam_apply", "simam_fwd"), ("simam_bwd", "simam_bwd"),
          ("head_fwd", "head_fwd"), ("head_bwd", "head_bwd"), ("gemm_f32", "gemm"), ("slab_sum", "gemm"),
          ("dropout_apply", "dropout"), ("quant_e4m3", "quant_e4m3"), ("grad_join", "grad_join"),
          ("pack_nhwc", "pack_nhwc"), ("bce_partial", "bce_loss"), ("bce_final", "bce_loss"),
          ("bce_backward", "bce_loss_bwd"), ("head_z", "carafe_head_fwd"), ("rng_advance", "dropout")]


def group(name):
    for frag, g in GROUPS:
        if frag in name:
            return g
    return "torch:" + name.split("<")[0].replace("void ", "")[:60]


def main():
    path, nsteps = sys.argv[1], int(sys.argv[2])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adamw_kernel" in r["Kernel_Name"]]
    a, b = ends[-1 - nsteps], ends[-1]
    t, n = collections.defaultdict(float), collections.Counter()
    prev = None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if a < s <= b:
            g = group(r["Kernel_Name"])
            # the fixed-order slab reduction inside a conv / Linear weight-gradient call (csu_colsum's
            # kernels launched by csu_conv2d_wgrad_oihw) belongs to that call: a colsum kernel right
            # after a weight-gradient kernel is charged to it (ops.colsum's own launches stay "colsum")
            # (and the head's bias / encoder-bias sums launched by csu_carafe_head_bwd)
            if g == "colsum" and prev in ("conv_wgrad", "linear_wgrad", "carafe_head_bwd"):
                g = prev
            prev = g
            t[g] += (int(r["End_Timestamp"]) - s) / 1e3
            n[g] += 1
    ledger = {}
    if len(sys.argv) > 3:
        rec = json.loads([l for l in open(sys.argv[3]).read().splitlines() if l.startswith("{")][-1])
        for k in rec["roofline"]["kernels"]:
            ledger[k["kernel"]] = k
        ledger["conv_fwd+conv_dgrad"] = {"us_per_step": sum(ledger.get(x, {}).get("us_per_step", 0)
                                                            for x in ("conv_fwd", "conv_dgrad")),
                                         "launches_per_step": sum(ledger.get(x, {}).get("launches_per_step", 0)
                                                                  for x in ("conv_fwd", "conv_dgrad"))}
    tot = sum(t.values()) / nsteps
    print(f"kernel time {tot / 1e3:.3f} ms/step over the last {nsteps} graph-replayed steps "
          f"(wall {(b - a) / nsteps / 1e6:.3f} ms/step)")
    print(f"| ABI call | rocprof us/step | kernels/step | ledger us/step | ledger launches/step | ratio |")
    print("|---|---|---|---|---|---|")
    for g, v in sorted(t.items(), key=lambda kv: -kv[1]):
        us = v / nsteps
        L = ledger.get(g)
        lus = f"{L['us_per_step']:.1f}" if L else "-"
        ll = f"{L['launches_per_step']}" if L else "-"
        ratio = f"{L['us_per_step'] / us:.3f}" if L and us > 0 else "-"
        print(f"| {g} | {us:.1f} | {n[g] / nsteps:.0f} | {lus} | {ll} | {ratio} |")


if __name__ == "__main__":
    main()
