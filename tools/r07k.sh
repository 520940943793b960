# gemm_ws tile rotation: kernel tests + bench with the ledger dump
O=gpurun_out/r07k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "gemm_ws" > $O/t1.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
CSU_LEDGER_DUMP=$O/launches.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; python -c "
import json,collections;r=json.loads(open('$O/bench.json').read().splitlines()[-1]);print(r['value'],r['ms_per_step'],r['roofline']['step_frac'])
d=json.load(open('$O/launches.json')); agg=collections.defaultdict(list)
for l in d:
    if l['tag'].endswith(':ws'): agg[l['tag']].append(l['us'])
for k,v in agg.items(): print(k, len(v), round(sum(v)/len(v),2))"
