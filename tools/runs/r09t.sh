# FETCH_SIZE of the conv weight-gradient kernels, XCD-aware order (a, libcsu_hip.so) vs hardware order (b)
set -e
R=$(pwd); O=$R/gpurun_out/r09t; mkdir -p $O; export TMPDIR=/tmp
L=$R/cswin-simam-unet_amd/csu/_lib
for v in a b; do
  if [ $v = a ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  cd /tmp
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$v -o p -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline off --graph off --no-roofline --no-ref-arch > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  cd $R
  echo "pass $v done"
done
python3 - <<'PY'
import csv, glob, collections
for v in "ab":
    f = glob.glob(f"gpurun_out/r09t/{v}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: [0.0, 0])
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if any(s in k for s in ("conv_wgrad", "conv3_wgrad", "colsum")) and row["Counter_Name"] == "FETCH_SIZE":
            agg[k[:80]][0] += float(row["Counter_Value"]); agg[k[:80]][1] += 1
    print(v, "total", round(sum(x[0] for x in agg.values()) / 1024, 1), "MB (all launches of the run)")
    for k, (s, n) in sorted(agg.items(), key=lambda x: -x[1][0]):
        print(f"   {s/1024:9.1f} MB n={n:3d} {k}")
PY
