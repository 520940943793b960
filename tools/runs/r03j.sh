# fp8 MFMA path + optimizer-written weight shadows: tests, then 1024x1024 B4 bench lines (bf16 / fp8)
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_kernels.py tests/test_gpu_train.py -v -x --timeout 300 --timeout-method thread -k "fp8 or adam or cast or graph or resume or f8_" > gpurun_out/r03j/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r03j/tests.log | tail -40; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --dtype fp8 --steps 6 --warmup 2 --cpu-baseline off > gpurun_out/r03j/bench_fp8.json 2> gpurun_out/r03j/bench_fp8.err || exit $?
timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --dtype bf16 --steps 6 --warmup 2 --cpu-baseline off > gpurun_out/r03j/bench_bf16.json 2> gpurun_out/r03j/bench_bf16.err || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/r03j/bench_512.json 2> gpurun_out/r03j/bench_512.err || exit $?
python - <<'PY'
import json
for k in ("fp8", "bf16", "512"):
    d = json.load(open(f"gpurun_out/r03j/bench_{k}.json"))
    r = d["roofline"]
    print(k, d["value"], d["ms_per_step"], r["kernel"], r["frac"])
    for x in r["kernels"][:14]:
        print("   %-22s %8.1f us/step %6.1f launches %s" % (x["kernel"], x["us_per_step"], x["launches_per_step"], x.get("precision")))
PY
