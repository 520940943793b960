"""HBM bytes per launch of one kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <kernel substring> <out.json>
Counters are kilobytes per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores."""
import csv
import json
import sys


def per_launch(path, kernel, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fpath, wpath, kernel, out = sys.argv[1:5]
    f = per_launch(fpath, kernel, "FETCH_SIZE")
    w = per_launch(wpath, kernel, "WRITE_SIZE")
    fetch = sum(f) / len(f) * 1024 * 2
    write = sum(w) / len(w) * 1024
    rec = {"kernel": kernel, "launches_fetch": len(f), "launches_write": len(w),
           "fetch_bytes_per_launch_corrected": int(fetch), "write_bytes_per_launch": int(write),
           "hbm_bytes_per_launch": int(fetch + write),
           "note": "FETCH_SIZE KB x1024 x2 (gfx950 half-count of wide streaming reads) + WRITE_SIZE KB x1024"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
