# fp32 path: the bias column sums folded into the split-K slab sum launch (a) vs two launches (b, HEAD before)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "f32 or fp32 or wgrad" > gpurun_out/r09g_tests.log 2>&1 || { tail -30 gpurun_out/r09g_tests.log; exit 1; }
tail -2 gpurun_out/r09g_tests.log
O=gpurun_out/r09g; mkdir -p $O; L=$PWD/cswin-simam-unet_amd/csu/_lib
for i in 1 2; do for v in a b; do
  if [ $v = a ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  timeout -k 10 400 python -u bench.py --img 256 --batch 8 --dtype fp32 --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > $O/f32_${v}_$i.json 2> $O/f32.err || exit 1
  python tools/bench_summary.py $O/f32_${v}_$i.json | head -3
done; done
