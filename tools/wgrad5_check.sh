# wgrad5 configs: parity tests, per-shape timing (linear_probe wgrad rows), bench
set -e
for c in 0 1 2; do
  CSU_WGRAD5=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or fused_mlp or mlp_fused" > gpurun_out/w5_t$c.log 2>&1 || { tail -30 gpurun_out/w5_t$c.log; exit 1; }
  echo "cfg $c: $(tail -1 gpurun_out/w5_t$c.log)"
done
for c in -1 0 1 2; do
  echo "== cfg $c"; CSU_WGRAD5=$c timeout -k 10 200 python -u tools/linear_probe.py 2>&1 | grep -E "wgrad|totals"
done
for c in -1 0 1 2; do
  v=$(CSU_WGRAD5=$c timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "bench cfg $c -> $v img/s"
done
