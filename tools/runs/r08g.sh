# round 6: e4m3 weight streaming in gemm_ws (fp8 format qkv / proj and input gradients) -- kernel tests
# (bitwise vs the bf16 kernel on the dequantised weight), the fp8 model tests, then 1024x1024 B4 fp8
# benches with CSU_FP8_WS=1 / 0 interleaved and one bf16 line
mkdir -p gpurun_out/r08g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "e4m3 or fp8 or gemm_ws or frag" > gpurun_out/r08g/t.log 2>&1 || { tail -40 gpurun_out/r08g/t.log; exit 1; }
tail -2 gpurun_out/r08g/t.log
for i in 1 2; do
  for v in 1 0; do
    CSU_FP8_WS=$v timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --dtype fp8 --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > gpurun_out/r08g/fp8_ws${v}_$i.json 2> gpurun_out/r08g/bench.err || { tail -20 gpurun_out/r08g/bench.err; exit 1; }
    python tools/bench_summary.py gpurun_out/r08g/fp8_ws${v}_$i.json | head -1
  done
done
timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > gpurun_out/r08g/bf16.json 2> gpurun_out/r08g/bench.err || { tail -20 gpurun_out/r08g/bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r08g/bf16.json | head -1
