"""Are the PMC passes' eager steps the kernels the timed graph replays?  Per-step kernel counts of an
eager counter pass (tools/pmc_head.sh p1, `bench.py --graph off`) against a kernel trace of the
graph-replayed bench steps of the same workload (`bench.py --no-roofline`, last <steps> steps):

    python tools/kernel_match.py <graph kernel_trace.csv> <steps> <pmc pass dir>

Steps are AdamW-delimited in both (the eager pass drops its first, warm-up, step).  Prints every
kernel whose per-step launch count differs and exits 1 if any does (torch's own copy / cat kernels
of the capture bookkeeping are listed but do not fail the check)."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_table import load, short            # noqa: E402


def graph_counts(path, nsteps):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [int(r["End_Timestamp"]) for r in rows if "adamw_kernel" in r["Kernel_Name"]]
    a, b = ends[-1 - nsteps], ends[-1]
    n = collections.Counter()
    for r in rows:
        if a < int(r["Start_Timestamp"]) <= b:
            n[short(r["Kernel_Name"])] += 1.0 / nsteps
    return n


def eager_counts(d):
    per, dur, names = load(d, {"SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
    ids = sorted(names, key=int)
    adam = [i for i in ids if "adamw_kernel" in names[i]]
    first, last = int(adam[0]), int(adam[-1])
    steps = len(adam) - 1
    n = collections.Counter()
    for i in ids:
        if first < int(i) <= last:
            n[short(names[i])] += 1.0 / steps
    return n, steps


def main():
    g = graph_counts(sys.argv[1], int(sys.argv[2]))
    e, steps = eager_counts(sys.argv[3])
    bad, soft = [], []
    for k in sorted(set(g) | set(e)):
        if abs(g[k] - e[k]) > 1e-6:
            (soft if ("at::native" in k or "rocclr" in k or "torch" in k) else bad).append((k, g[k], e[k]))
    print(f"graph replay: {sum(g.values()):.1f} kernels/step ({len(g)} distinct); eager PMC pass: "
          f"{sum(e.values()):.1f} kernels/step over {steps} steps ({len(e)} distinct)")
    for k, a, b in bad:
        print(f"  DIFF {k}: graph {a:.2f} / eager {b:.2f} per step")
    for k, a, b in soft:
        print(f"  (torch bookkeeping) {k}: graph {a:.2f} / eager {b:.2f} per step")
    print("kernel sets match" if not bad else f"{len(bad)} csu kernels differ")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
