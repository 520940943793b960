"""Per-shape (grid) durations of kernels matching substrings in a rocprofv3 kernel-trace CSV.
    python tools/kstat.py <kernel_trace.csv> <substr> [<substr> ...]   (last 1/7 of the trace)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows = rows[-len(rows) // 7:]
for pat in sys.argv[2:]:
    seen = {}
    for r in rows:
        n = r["Kernel_Name"]
        if pat in n:
            k = (n[:48], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
            seen.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(pat, round(sum(sum(v) for v in seen.values()) / 2e3, 1), "us per step (2 steps in the window)")
    for k, v in sorted(seen.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print("  ", k, len(v), "launches, avg", round(sum(v) / len(v) / 1e3, 1), "us")
