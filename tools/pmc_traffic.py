"""HBM bytes per C-ABI call of a kernel group from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <key> \
        <call-marker kernel substring> <kernel substring>[,<kernel substring>...] <profiles/pmc_traffic.json>
Counters are kilobytes per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE
is exact for 16-B-per-lane stores.  Bytes of every dispatch of the group are summed and divided by
the number of calls (dispatches of the marker kernel, one per call); the result is merged into the
JSON under <key> = "<ledger kernel name>|<img>|<batch>|<dtype>" (read by bench.py).
Markers may list several kernels ("a,b": a call dispatches exactly one of them).  A marker
"step:<kernel>" names a kernel dispatched once per train step (adamw_kernel) for groups whose calls
dispatch varying kernels (the grouped weight gradients): calls = steps x the ledger's launches per
step, read from the bench JSON given as the 7th argument (roofline.kernels)."""
import csv
import json
import os
import sys


def totals(path, frags, marker, counter):
    vals, calls = 0.0, set()
    markers = marker.split(",")
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if any(f in name for f in frags):
            vals += float(r["Counter_Value"])
        if any(m in name for m in markers):
            calls.add(r["Dispatch_Id"])
    return vals, len(calls)


def main():
    fpath, wpath, key, marker, frags, out = sys.argv[1:7]
    frags = frags.split(",")
    per_step = marker.startswith("step:")
    marker = marker[5:] if per_step else marker
    f, nf = totals(fpath, frags, marker, "FETCH_SIZE")
    w, nw = totals(wpath, frags, marker, "WRITE_SIZE")
    if per_step:
        name = key.split("|")[0]
        lps = [k["launches_per_step"] for k in json.load(open(sys.argv[7]))["roofline"]["kernels"] if k["kernel"] == name][0]
        nf, nw = nf * lps, nw * lps
    fetch = f / nf * 1024 * 2
    write = w / nw * 1024
    rec = {"calls_fetch_pass": nf, "calls_write_pass": nw, "kernels": frags,
           "fetch_bytes_per_call_corrected": int(fetch), "write_bytes_per_call": int(write),
           "hbm_bytes_per_call": int(fetch + write)}
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = int(fetch + write)
    db.setdefault("_detail", {})[key] = rec
    db["_note"] = ("HBM bytes per C-ABI call: FETCH_SIZE KB x1024 x2 (gfx950 half-count of wide streaming reads) + "
                   "WRITE_SIZE KB x1024, summed over the call's kernels (tools/pmc_traffic.py)")
    json.dump(db, open(out, "w"), indent=1, sort_keys=True)
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
