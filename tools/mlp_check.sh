#!/bin/bash
# Fused-Mlp check: its parity tests, then bench with the fused / two-GEMM Mlp.
set -e
OUT=gpurun_out/mlp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "mlp" > $OUT/pytest.log 2>&1 \
  || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for f in 1 0; do
  CSU_FUSED_MLP=$f timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/bench_$f.json 2> $OUT/bench_$f.err \
    || { tail -30 $OUT/bench_$f.err; exit 1; }
  echo "fused=$f $(python -c "import json;d=json.load(open('$OUT/bench_$f.json'));print(d['value'], d['ms_per_step'])")"
done
