"""Per-kernel table from tools/pmc_table.sh's three rocprofv3 passes: launches, average duration,
MFMA utilisation, achieved MFMA TFLOP/s and HBM GB/s.

    python tools/pmc_table.py <dir with p1/ p2/ p3/>
MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (busy cycles are
summed over every SIMD, GRBM_GUI_ACTIVE over the 8 XCDs: MI355X_MICROARCH.md); MFMA FLOPs =
busy cycles x 1024 (32x32x16 bf16: 32768 FLOP per 32 cycles; 16x16x32: 16384 per 16).
HBM bytes = FETCH_SIZE x 2 (gfx950 half-count of wide reads) + WRITE_SIZE, KB x 1024; durations
from the kernel trace of the same pass (counter collection serialises dispatches)."""
import collections
import csv
import glob
import re
import sys


def load(d, counter_names):
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names, ccdur = {}, {}
    for f in cc:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] in counter_names:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
                ccdur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            names.setdefault(r["Dispatch_Id"], r["Kernel_Name"])
    for k, v in ccdur.items():
        dur.setdefault(k, v)
    return per, dur, names


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    n = n.replace("csu::(anonymous namespace)::", "").replace("csu::", "")
    if n.startswith("_ZN"):   # _ZN3csu12_GLOBAL__N_1<len><name>[I<template args>E]...
        m = re.search(r"_GLOBAL__N_1(\d+)", n) or re.search(r"_ZN3csu(\d+)", n)
        if m:
            ln = int(m.group(1))
            rest = n[m.end():]
            name, rest = rest[:ln], rest[ln:]
            targs = re.match(r"I((?:Li-?\d+E|Lb[01]E|DF16b|f)+)E", rest)
            if targs:
                vals = re.findall(r"Li(-?\d+)E|Lb([01])E|(DF16b)|(f)", targs.group(1))
                name += "<" + ",".join(a or b or ("bf16" if c else "f32") for a, b, c, dd in vals) + ">"
            n = name
    return n[:48]


def main():
    d = sys.argv[1]
    p1, d1, n1 = load(d + "/p1", {"SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"})
    p2, d2, n2 = load(d + "/p2", {"FETCH_SIZE"})
    p3, d3, n3 = load(d + "/p3", {"WRITE_SIZE"})
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for did, cs in p1.items():
        k = short(n1[did])
        a = agg[k]
        a["n"] += 1
        a["t1"] += d1.get(did, 0.0)
        a["busy"] += cs["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["grbm"] += cs["GRBM_GUI_ACTIVE"]
    for pp, dd, nn, key in ((p2, d2, n2, "FETCH_SIZE"), (p3, d3, n3, "WRITE_SIZE")):
        for did, cs in pp.items():
            a = agg[short(nn[did])]
            a[key] += cs[key]
            a["t_" + key] += dd.get(did, 0.0)
            a["n_" + key] += 1
    rows = []
    for k, a in agg.items():
        if not a["n"] or not a["t1"]:
            continue
        util = a["busy"] / (a["grbm"] / 8 * 1024) if a["grbm"] else 0.0
        tf = a["busy"] * 1024 / a["t1"] / 1e12
        hb = 0.0
        if a["n_FETCH_SIZE"] and a["n_WRITE_SIZE"]:
            rd = a["FETCH_SIZE"] / a["n_FETCH_SIZE"] * 2048
            wr = a["WRITE_SIZE"] / a["n_WRITE_SIZE"] * 1024
            t = (a["t_FETCH_SIZE"] / a["n_FETCH_SIZE"] + a["t_WRITE_SIZE"] / a["n_WRITE_SIZE"]) / 2
            hb = (rd + wr) / t / 1e9 if t else 0.0
        rows.append((a["t1"], k, int(a["n"]), a["t1"] / a["n"] * 1e6, util, tf, hb))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print("| kernel | launches | avg us | share | MFMA util | MFMA TFLOP/s | HBM GB/s (PMC) | HBM frac of 8 TB/s |")
    print("|---|---|---|---|---|---|---|---|")
    for t, k, n, us, util, tf, hb in rows[:40]:
        print(f"| `{k}` | {n} | {us:.1f} | {t / tot * 100:.1f} % | {util * 100:.1f} % | {tf:.0f} | {hb:.0f} | {hb / 8000 * 100:.1f} % |")


if __name__ == "__main__":
    main()
