# grouped weight gradients: 256 x 256 tiles (libcsu_hip.so) vs 256 x 128 (libcsu_hip_ab.so, WG_SQ256=0)
O=gpurun_out/r07v; mkdir -p $O
L=$PWD/cswin-simam-unet_amd/csu/_lib
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wgrad or reproducible" > $O/t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in sq ab; do
  if [ $v = sq ]; then export CSU_LIB_PATH=$L/libcsu_hip.so; else export CSU_LIB_PATH=$L/libcsu_hip_ab.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > $O/bench_${v}_$i.json 2> $O/bench.err || exit 1
  python tools/bench_summary.py $O/bench_${v}_$i.json | grep images
  python -c "
import json;r=json.loads(open('$O/bench_${v}_$i.json').read().splitlines()[-1])
print([ (k['kernel'],round(k['us_per_step'])) for k in r['roofline']['kernels'] if k['kernel']=='linear_wgrad'])"
done; done
