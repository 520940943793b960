# SimAM kernels: tests + bench with / without SimAM
O=gpurun_out/r07m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "simam or SimAM" > $O/t1.log 2>&1
rc=$?; echo "simam tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --simam --steps 20 --warmup 3 --cpu-baseline off > $O/bench_simam.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench.json 2>> $O/bench.err || exit 1
python tools/bench_summary.py $O/bench_simam.json $O/bench.json | grep images
python -c "
import json;r=json.loads(open('$O/bench_simam.json').read().splitlines()[-1])
for k in r['roofline']['kernels']:
    if 'simam' in k['kernel']: print(k['kernel'],k['us_per_step'],k['launches_per_step'], k.get('frac'))"
