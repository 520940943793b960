# norm2 in the proj + residual epilogue (csu_gemm_ws_ln): tests, then A/B pairs (CSU_FUSE_PROJ_LN=0 / 1)
O=gpurun_out/r07za; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm_ws or linear_residual or block or model or reproducible or full_size or dice" > $O/t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 1 0; do
  CSU_FUSE_PROJ_LN=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > $O/bench_${v}_$i.json 2> $O/bench.err || exit 1
  python tools/bench_summary.py $O/bench_${v}_$i.json | grep images
  python -c "
import json;r=json.loads(open('$O/bench_${v}_$i.json').read().splitlines()[-1])
print('   ', [(k['kernel'],round(k['us_per_step']),k['launches_per_step']) for k in r['roofline']['kernels'] if k['kernel'] in ('gemm','layernorm_fwd')])"
done; done
