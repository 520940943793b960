#!/bin/bash
# loss kernel with the per-step segmentation sums inside the graph; bench step includes them
set -e
O=gpurun_out/r02ai; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py tests/test_gpu_model.py -k "metrics or bce or graphed or f8 or whole_model or dp_path" -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json | head -3
