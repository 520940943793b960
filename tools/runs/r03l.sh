# UNet BatchNorm apply fix: UNet GPU tests + UNet bench; train_model API bench vs GraphedTrainStep (512 B16)
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "unet or bn or batchnorm or maxpool" > gpurun_out/r03l/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r03l/tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model unet --steps 6 --warmup 2 --cpu-baseline off > gpurun_out/r03l/bench_unet.json 2> gpurun_out/r03l/bench_unet.err || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/r03l/bench_step.json 2> gpurun_out/r03l/bench_step.err || exit $?
timeout -k 10 300 python -u bench.py --api train_model --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/r03l/bench_train_model.json 2> gpurun_out/r03l/bench_train_model.err || exit $?
python - <<'PY'
import json
for k in ("unet", "step", "train_model"):
    d = json.load(open(f"gpurun_out/r03l/bench_{k}.json"))
    r = d.get("roofline") or {}
    print(k, d["value"], d["ms_per_step"], r.get("kernel"), r.get("frac"), d["config"].get("api"))
    for x in (r.get("kernels") or [])[:8]:
        print("   %-22s %8.1f us/step %6.1f launches frac %.3f" % (x["kernel"], x["us_per_step"], x["launches_per_step"], x["frac"]))
PY
