# round-4: the data-parallel path at N = 1 (--dp-force: process group + bucketed all-reduce captured in the
# step's graph, overlapping backward) against the plain dp1 line, interleaved; one run through torch.distributed.run
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
v() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'], d.get('grad_allreduce'))" $1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --cpu-baseline off --no-roofline > $O/dp1_$i.json 2> $O/dp1_$i.err || { echo A_FAIL; tail -20 $O/dp1_$i.err; exit 1; }
  timeout -k 10 200 python bench.py --dp-force --cpu-baseline off --no-roofline > $O/dpf_$i.json 2> $O/dpf_$i.err || { echo B_FAIL; tail -20 $O/dpf_$i.err; exit 1; }
  timeout -k 10 200 python bench.py --dp-force --grad-dtype bf16 --cpu-baseline off --no-roofline > $O/dpfb_$i.json 2> $O/dpfb_$i.err || { echo C_FAIL; tail -20 $O/dpfb_$i.err; exit 1; }
  echo "pair $i: dp1 $(v $O/dp1_$i.json) | dp-force fp32 $(v $O/dpf_$i.json) | dp-force bf16 $(v $O/dpfb_$i.json)"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --dp-force --cpu-baseline off > $O/torchrun.json 2> $O/torchrun.err || { echo RUN_FAIL; tail -20 $O/torchrun.err; exit 1; }
echo "torchrun dp-force: $(v $O/torchrun.json)"
echo ALL_OK
