# per-shape gemm times in the step (graph ledger dump), G4_SMALLM a (libcsu_hip.so) vs b (libcsu_hip_ab.so)
O=gpurun_out/r09x; mkdir -p $O; L=$PWD/cswin-simam-unet_amd/csu/_lib
for i in 1 2; do for v in a b; do
  if [ $v = a ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  CSU_LEDGER_DUMP=$O/l_${v}_$i.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > $O/bench_${v}_$i.json 2> $O/bench.err || exit 1
  python tools/bench_summary.py $O/bench_${v}_$i.json | grep images
done; done
python - <<'PY'
import json, collections
for v in "ab":
    agg = collections.defaultdict(list)
    for i in (1, 2):
        d = json.load(open(f"gpurun_out/r09x/l_{v}_{i}.json"))
        tot = collections.defaultdict(float)
        for e in d:
            if e["kernel"] == "gemm" and str(e["tag"]).startswith("4096x"): tot[e["tag"]] += e["us"]
        for k, x in tot.items(): agg[k].append(round(x, 1))
    print(v, "M=4096 total", [round(sum(x[i] for x in agg.values()), 1) for i in range(2)])
    for k, x in sorted(agg.items(), key=lambda t: -t[1][0]): print("   ", k, x)
PY
