# fp32 GEMM: forward / input-gradient splits at least 128 deep (b, -DF32_MINK01=128) vs 256 (a, product)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "f32 or fp32" > gpurun_out/r0zk_tests.log 2>&1 || { tail -30 gpurun_out/r0zk_tests.log; exit 1; }
tail -2 gpurun_out/r0zk_tests.log
O=gpurun_out/r0zk; mkdir -p $O; L=$PWD/cswin-simam-unet_amd/csu/_lib
CSU_LIB_PATH=$L/libcsu_hip_ab.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm_f32" > $O/tests_ab.log 2>&1 || { tail -30 $O/tests_ab.log; exit 1; }
tail -1 $O/tests_ab.log
for i in 1 2; do for v in a b; do
  if [ $v = a ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  CSU_LEDGER_DUMP=$O/l_${v}_$i.json timeout -k 10 300 python -u bench.py --img 256 --batch 8 --dtype fp32 --steps 10 --warmup 2 --cpu-baseline off --no-ref-arch > $O/f32_${v}_$i.json 2> $O/f32.err || exit 1
  python tools/bench_summary.py $O/f32_${v}_$i.json | grep images
done; done
python - <<'PY'
import json, collections
for v in "ab":
    d = json.load(open(f"gpurun_out/r0zk/l_{v}_1.json"))
    tot = collections.defaultdict(lambda: [0.0, 0, 0])
    for e in d:
        if e["kernel"] != "gemm": continue
        k = e["tag"]
        tot[k][0] += e["us"]; tot[k][1] += 1; tot[k][2] += e["flops"]
    print(v, "gemm total", round(sum(x[0] for x in tot.values())))
    for k, (us, n, fl) in sorted(tot.items(), key=lambda x: -x[1][0])[:25]:
        print(f"   {us:8.1f} us n={n:3d} {fl/us/1e6 if us else 0:7.1f} TF/s  {k}")
PY
