"""PMC table at HEAD: per C-ABI call and per kernel, MFMA utilisation and HBM
traffic from three rocprofv3 counter passes (tools/pmc_table.sh layout: p1 = SQ_INSTS_MFMA
SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, p2 = FETCH_SIZE, p3 = WRITE_SIZE, eager bench steps),
set against the ledger's ALGORITHMIC bytes of the same call from a bench JSON:

    python tools/pmc_groups.py <pass dir> <bench.json> [top] [--traffic <pmc_traffic.json>]

``--traffic``: also merge, per C-ABI call, the PMC HBM bytes per LEDGER launch (per-step bytes /
the bench ledger's launches per step) into that JSON under "<call>|<img>|<batch>|<dtype>" -- the
``roofline.traffic`` bench.py reports for its dominant kernel.

* steps = AdamW dispatches after the first one (the warm-up step is dropped);
* MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs);
* HBM bytes = 2 x FETCH_SIZE (gfx950 counts wide coalesced reads at half) + WRITE_SIZE, KiB units
  (MI355X_MICROARCH.md, HBM section); traffic ratio = HBM bytes / algorithmic bytes per step."""
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_table import load, short            # noqa: E402
from prof_groups import group                 # noqa: E402


def per_step(passdir, counters):
    per, dur, names = load(passdir, counters)
    ids = sorted(names, key=int)
    adam = [i for i in ids if "adamw_kernel" in names[i]]
    first = int(adam[0]) if adam else -1
    steps = max(1, len(adam) - 1)
    return per, dur, names, first, steps


def main():
    argv = list(sys.argv[1:])
    tj = None
    if "--traffic" in argv:
        i = argv.index("--traffic")
        tj = argv[i + 1]
        del argv[i:i + 2]
    d, bj = argv[0], argv[1]
    top = int(argv[2]) if len(argv) > 2 else 12
    rec = json.loads([l for l in open(bj).read().splitlines() if l.startswith("{")][-1])
    ledger = {k["kernel"]: k for k in rec["roofline"]["kernels"]}
    for a, b in (("conv_fwd", "conv_dgrad"),):
        if a in ledger or b in ledger:
            ledger[a + "+" + b] = {"bytes": sum(ledger.get(x, {}).get("bytes_per_launch", 0) *
                                                ledger.get(x, {}).get("launches_per_step", 0) for x in (a, b))}
    G = collections.defaultdict(lambda: collections.defaultdict(float))
    K = collections.defaultdict(lambda: collections.defaultdict(float))
    passes = (("p1", {"SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"}), ("p2", {"FETCH_SIZE"}),
              ("p3", {"WRITE_SIZE"}))
    nsteps, kgroup = {}, {}
    for tag, cs in passes:
        per, dur, names, first, steps = per_step(os.path.join(d, tag), cs)
        nsteps[tag] = steps
        prev = None
        for did in sorted(per, key=int):
            c = per[did]
            if int(did) <= first:
                continue
            nm = names[did]
            gk = group(nm)
            # a colsum right after a weight-gradient kernel is that call's slab reduction (prof_groups.py)
            if gk == "colsum" and prev in ("conv_wgrad", "linear_wgrad"):
                gk = prev
            prev = gk
            for tab, key in ((G, gk), (K, short(nm))):
                a = tab[key]
                for k, v in c.items():
                    a[k] += v / steps
                a["t_" + tag] += dur.get(did, 0.0) / steps * 1e6
                a["n_" + tag] += 1.0 / steps
            kgroup[short(nm)] = gk

    def row(a):
        util = a["SQ_VALU_MFMA_BUSY_CYCLES"] / (a["GRBM_GUI_ACTIVE"] / 8 * 1024) if a["GRBM_GUI_ACTIVE"] else 0.0
        hbm = a["FETCH_SIZE"] * 2048 + a["WRITE_SIZE"] * 1024
        t = a["t_p1"]
        return util, hbm, t

    cfg = rec["config"].get("workload", "")
    print(f"# PMC table: {cfg} (batch {rec['config'].get('per_gpu_batch')}, {rec['dtype']})\n")
    print(f"Counter passes: eager steps of `bench.py --graph off` (no side stream: the kernels the captured step "
          f"replays, checked by tools/kernel_match.py), {nsteps.get('p1')} steps after the warm-up step; "
          f"algorithmic bytes: the bench ledger (`{os.path.basename(bj)}`).\n")
    print("## Per C-ABI call (per step)\n")
    print("| ABI call | us/step (p1) | launches | MFMA util | MFMA TFLOP/s | HBM MB (PMC) | algorithmic MB | traffic ratio | HBM GB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    rows = sorted(G.items(), key=lambda kv: -kv[1]["t_p1"])
    for g, a in rows[:top + 8]:
        util, hbm, t = row(a)
        L = ledger.get(g)
        alg = (L.get("bytes") if L and "bytes" in L else
               (L["bytes_per_launch"] * L["launches_per_step"] if L else None))
        tf = a["SQ_VALU_MFMA_BUSY_CYCLES"] * 1024 / (t * 1e-6) / 1e12 if t else 0.0
        ratio = f"{hbm / alg:.2f}" if alg else "-"
        algs = f"{alg / 1e6:.1f}" if alg else "-"
        print(f"| {g} | {t:.1f} | {a['n_p1']:.0f} | {util * 100:.1f} % | {tf:.0f} | {hbm / 1e6:.1f} | {algs} | {ratio} | "
              f"{hbm / (t * 1e-6) / 1e9 if t else 0:.0f} |")
    if tj:
        c = rec["config"]
        if "workload_key" not in c:
            raise SystemExit("bench JSON without config.workload_key (bench.py before round 5): traffic not merged")
        suffix = "|" + c["workload_key"]
        db = json.load(open(tj)) if os.path.exists(tj) else {}
        for g, a in G.items():
            L = ledger.get(g)
            if L and L.get("launches_per_step"):
                db[g + suffix] = int(row(a)[1] / L["launches_per_step"])
        db["_note"] = ("HBM bytes per ledger launch from rocprofv3 PMC passes (2 x FETCH_SIZE + WRITE_SIZE), "
                       "tools/pmc_groups.py --traffic over profiles/r03k_pmc_*; key <call>|<bench.py workload_key>")
        db.pop("_detail", None)
        with open(tj, "w") as f:
            json.dump(db, f, indent=1, sort_keys=True)
    print("\n## Per kernel (top by time; traffic ratio of the kernel's ABI call above)\n")
    print("| kernel | ABI call | us/step | launches | MFMA util | MFMA TFLOP/s | HBM MB (PMC) | HBM GB/s |")
    print("|---|---|---|---|---|---|---|---|")
    for k, a in sorted(K.items(), key=lambda kv: -kv[1]["t_p1"])[:top]:
        util, hbm, t = row(a)
        tf = a["SQ_VALU_MFMA_BUSY_CYCLES"] * 1024 / (t * 1e-6) / 1e12 if t else 0.0
        print(f"| `{k}` | {kgroup[k]} | {t:.1f} | {a['n_p1']:.0f} | {util * 100:.1f} % | {tf:.0f} | {hbm / 1e6:.1f} | "
              f"{hbm / (t * 1e-6) / 1e9 if t else 0:.0f} |")


if __name__ == "__main__":
    main()
