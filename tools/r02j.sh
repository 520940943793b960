set -e
mkdir -p gpurun_out/r02j
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or linear or side_stream" > gpurun_out/r02j/pytest.log 2>&1 || { tail -40 gpurun_out/r02j/pytest.log; exit 1; }
tail -2 gpurun_out/r02j/pytest.log
timeout -k 10 400 python -u tools/wgrad_bench.py --plans auto,c1,t64x64:c1,t64x64:c0.5 > gpurun_out/r02j/wgrad_bench.txt 2>&1 || { tail -30 gpurun_out/r02j/wgrad_bench.txt; exit 1; }
cat gpurun_out/r02j/wgrad_bench.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r02j/bench.json 2> gpurun_out/r02j/bench.err || { tail -30 gpurun_out/r02j/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r02j/bench.json').read())
r=d['roofline']; ks=r.pop('kernels')
print(json.dumps({k:v for k,v in d.items() if k!='roofline'}))
print(json.dumps(r))
for k in ks: print(k)
"
