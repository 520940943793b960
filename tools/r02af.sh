#!/bin/bash
# attention: window rows by reciprocal multiply, [tap][channel] LePE weights in LDS
set -e
O=gpurun_out/r02af; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropout.py tests/test_gpu_model.py -k "stripe or attn or lepe or block or whole_model or dropout" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --cpu-baseline off > $O/bench_1024.json 2> $O/bench_1024.err || { tail -30 $O/bench_1024.err; exit 1; }
python tools/bench_summary.py $O/bench.json $O/bench_1024.json | grep -E "json|stripe"
