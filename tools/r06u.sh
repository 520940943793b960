# round-4: conv weight gradients straight into the reducer bucket -- DP tests, then dp1 vs --dp-force pairs
set -o pipefail
O=gpurun_out/${T:-r06u}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_model.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dist or dp or reducer or conv or head or carafe" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
v() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'], d.get('grad_buckets'))" $1; }
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --cpu-baseline off --no-roofline > $O/dp1_$i.json 2> $O/dp1_$i.err || { echo A_FAIL; tail -20 $O/dp1_$i.err; exit 1; }
  timeout -k 10 200 python bench.py --dp-force --cpu-baseline off --no-roofline > $O/dpf_$i.json 2> $O/dpf_$i.err || { echo B_FAIL; tail -20 $O/dpf_$i.err; exit 1; }
  echo "pair $i: dp1 $(v $O/dp1_$i.json) | dp-force $(v $O/dpf_$i.json)"
done
echo ALL_OK
