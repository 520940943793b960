# the data-parallel path (GradAllReduce captured in the step graph) at N = 1 vs dp1, same box
O=gpurun_out/${1:-dpcheck}; mkdir -p $O
for m in dp1 dpforce; do
  F=""; [ $m = dpforce ] && F="--dp-force"
  timeout -k 10 400 python -u bench.py $F --steps 10 --warmup 3 --cpu-baseline off --no-ref-arch > $O/$m.json 2> $O/$m.err || { tail -20 $O/$m.err; exit 1; }
  python tools/bench_summary.py $O/$m.json | grep images
  python -c "
import json;r=json.loads(open('$O/$m.json').read().splitlines()[-1]); print('   ', r['config']['parallelism'], r.get('grad_allreduce'))"
done
