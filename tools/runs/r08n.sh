# early grouped weight gradients on the side branch of the captured step: train / dist / graph tests,
# then interleaved benches over the threshold (0 = the serial step)
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dist.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r08n_tests.log 2>&1 || { tail -30 gpurun_out/r08n_tests.log; exit 1; }
tail -3 gpurun_out/r08n_tests.log
O=gpurun_out/r08n; mkdir -p $O
for i in 1 2; do for g in 0 60 30 120; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch --early-wgrad $g > $O/bench_${g}_$i.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "
import json;r=json.loads(open('$O/bench_${g}_$i.json').read().splitlines()[-1])
print('early $g', r['value'], r['ms_per_step'], r['roofline'].get('overlap_ms_per_step'), r['roofline']['frac'])"
done; done
