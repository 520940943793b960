# SimAM skip fork (fused cast / joined backward): SimAM + model tests, bench
O=gpurun_out/r07w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "simam or SimAM or full_size or reproducible" > $O/t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench_$i.json 2> $O/bench.err || exit 1
python tools/bench_summary.py $O/bench_$i.json | grep images
python -c "
import json;r=json.loads(open('$O/bench_$i.json').read().splitlines()[-1]); print('ref arch', r['reference_architecture']['value'], 'traffic', r['roofline']['traffic'])
print([(k['kernel'],round(k['us_per_step'])) for k in r['roofline']['kernels'] if k['kernel'].startswith(('simam','grad_join','torch'))])"
done
