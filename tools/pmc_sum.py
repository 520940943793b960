"""Average rocprofv3 PMC counters per dispatch over the counter_collection CSVs under a directory
(skipping the first `skip` dispatches, default 5): python tools/pmc_sum.py <dir> [kernel-substring] [skip]."""
import collections, csv, glob, sys
pat = sys.argv[2] if len(sys.argv) > 2 else ""
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 5
vals = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for i, (d, cs) in enumerate(sorted(per.items())):
        if i >= skip:
            for k, v in cs.items():
                vals[k].append(v)
for k, v in vals.items():
    print(f"{k:32s} {sum(v) / len(v):16.1f}")
