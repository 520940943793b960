# round 6: fp8 model tests with the bf16 8-wave Mlp backward; conv weight-gradient configurations on the
# CSWin shapes (tools/conv_wgrad_probe.py); fp8 vs bf16 at 1024x1024 B4 in interleaved runs
mkdir -p gpurun_out/r08h
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r08h/t.log 2>&1 || { tail -40 gpurun_out/r08h/t.log; exit 1; }
tail -2 gpurun_out/r08h/t.log
CFGS=-1,0,1,2,3,4,5 ONLY="merge,embed,carafe" timeout -k 10 300 python -u tools/conv_wgrad_probe.py > gpurun_out/r08h/conv_wgrad_probe.txt 2>&1 || { tail -20 gpurun_out/r08h/conv_wgrad_probe.txt; exit 1; }
cat gpurun_out/r08h/conv_wgrad_probe.txt
for i in 1 2; do
  for v in fp8 bf16; do
    timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --dtype $v --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > gpurun_out/r08h/${v}_$i.json 2> gpurun_out/r08h/bench.err || { tail -20 gpurun_out/r08h/bench.err; exit 1; }
    python tools/bench_summary.py gpurun_out/r08h/${v}_$i.json > gpurun_out/r08h/${v}_$i.txt; head -1 gpurun_out/r08h/${v}_$i.txt
  done
done
