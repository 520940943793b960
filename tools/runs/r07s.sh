# A/B: stripe_attn.hip compiled with / without SLP vectorisation (libcsu_hip_noslp.so): isolated
# attention times, then the step (interleaved bench pairs)
O=gpurun_out/r07s; mkdir -p $O
L=cswin-simam-unet_amd/csu/_lib
for v in base noslp; do
  if [ $v = base ]; then export CSU_LIB_PATH=$PWD/$L/libcsu_hip.so; else export CSU_LIB_PATH=$PWD/$L/libcsu_hip_noslp.so; fi
  echo "== $v" >> $O/attn.txt
  timeout -k 10 200 python -u tools/attn_time.py >> $O/attn.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/attn.txt
for i in 1 2; do for v in base noslp; do
  if [ $v = base ]; then export CSU_LIB_PATH=$PWD/$L/libcsu_hip.so; else export CSU_LIB_PATH=$PWD/$L/libcsu_hip_noslp.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > $O/bench_${v}_$i.json 2> $O/bench.err || exit 1
  python tools/bench_summary.py $O/bench_${v}_$i.json | grep images
done; done
