# A/B of libcsu_hip.so (a) vs libcsu_hip_ab.so (b) at 1024x1024 B4 bf16 (BASELINE configs[4] shape), interleaved pairs
#   bash tools/ab_1024.sh <tag> [kernel group to print]
O=gpurun_out/$1; mkdir -p $O; G=${2:-stripe_attn_fwd}
L=$PWD/cswin-simam-unet_amd/csu/_lib
for i in 1 2; do for v in a b; do
  if [ $v = a ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  timeout -k 10 400 python -u bench.py --img 1024 --batch 4 --steps 10 --warmup 3 --cpu-baseline off --no-ref-arch > $O/b1024_${v}_$i.json 2> $O/b1024.err || exit 1
  python tools/bench_summary.py $O/b1024_${v}_$i.json | grep images
  python -c "
import json;r=json.loads(open('$O/b1024_${v}_$i.json').read().splitlines()[-1])
print('   ', [(k['kernel'],round(k['us_per_step'])) for k in r['roofline']['kernels'] if k['kernel']=='$G'])"
done; done
