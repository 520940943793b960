# fp8 Mlp forward with the next norm1 in its epilogue: fp8 tests, then 1024 B4 fp8 vs bf16
O=gpurun_out/r07zf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fp8 or full_size" > $O/t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --dtype fp8 --steps 10 --warmup 3 --cpu-baseline off --no-ref-arch > $O/fp8_$i.json 2> $O/bench.err || exit 1
  python tools/bench_summary.py $O/fp8_$i.json | grep images
  timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --steps 10 --warmup 3 --cpu-baseline off --no-ref-arch > $O/bf16_$i.json 2> $O/bench.err || exit 1
  python tools/bench_summary.py $O/bf16_$i.json | grep images
done
