# conv forward / dgrad kernels (igemm_bf16, conv_gemm) and weight gradients in XCD order (CW_XCD 1,
# libcsu_hip.so) vs hardware order (libcsu_hip_ab.so): 512 B16 bf16 and the 256 B8 fp32 line
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "conv or wgrad or carafe or embed or merge or model" > gpurun_out/r09u_tests.log 2>&1 || { tail -30 gpurun_out/r09u_tests.log; exit 1; }
tail -2 gpurun_out/r09u_tests.log
bash tools/ab_lib.sh r09u conv_fwd+conv_dgrad || exit 1
O=gpurun_out/r09u; L=$PWD/cswin-simam-unet_amd/csu/_lib
for i in 1 2; do for v in a b; do
  if [ $v = a ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  timeout -k 10 300 python -u bench.py --img 256 --batch 8 --dtype fp32 --steps 10 --warmup 2 --cpu-baseline off --no-ref-arch > $O/f32_${v}_$i.json 2> $O/f32.err || exit 1
  python tools/bench_summary.py $O/f32_${v}_$i.json | grep images
  python -c "
import json;r=json.loads(open('$O/f32_${v}_$i.json').read().splitlines()[-1])
print('   ', [(k['kernel'],round(k['us_per_step'])) for k in r['roofline']['kernels'] if k['kernel'].startswith('conv')])"
done; done
