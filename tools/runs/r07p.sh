# fused attention backward prologue (single-pass staging): attention tests, per-WG timeline, bench
O=gpurun_out/r07p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stripe or attention or lepe or Stripe or gemm_ws or frag_layout or ln_linear_ws" > $O/t1.log 2>&1
rc=$?; echo "attn tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for s in 3 1 2; do timeout -k 10 120 python -u tools/attn_wg_timeline.py $s >> $O/timeline.txt 2>&1 || exit 1; done
grep -v amdgpu.ids $O/timeline.txt | grep "fused bwd"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench.json 2> $O/bench.err || exit 1
python tools/bench_summary.py $O/bench.json | grep images
python -c "
import json;r=json.loads(open('$O/bench.json').read().splitlines()[-1])
for k in r['roofline']['kernels']:
    if 'stripe' in k['kernel']: print(k['kernel'],k['us_per_step'],k['launches_per_step'])"
