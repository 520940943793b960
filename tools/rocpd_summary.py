"""Turn a rocprofv3 rocpd database (<dir>/<name>_results.db) into the CSVs the --output-format csv
run writes: <out>_kernel_stats.csv (per-kernel Calls/Total/Average/Min/Max ns, %) and
<out>_kernel_trace.csv (Kernel_Name, Start/End_Timestamp; input of tools/prof_summary.py)."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count,"
                     " accum_vgpr_count, sgpr_count, scratch_size from kernels order by start").fetchall()
    with open(out + "_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                    "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], r[3] * r[4] * r[5], r[6], r[7], r[8], r[9], r[10], r[11]])
    agg = {}
    for r in rows:
        d = r[2] - r[1]
        a = agg.setdefault(r[0], [0, 0, 1 << 62, 0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(a[1] for a in agg.values())
    with open(out + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, a in sorted(agg.items(), key=lambda x: -x[1][1]):
            w.writerow([name, a[0], a[1], round(a[1] / a[0], 1), round(100 * a[1] / tot, 4), a[2], a[3]])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
