#!/bin/bash
# LayerNorm backward with branch-free buffer loads/stores: tests + bench A/B vs previous numbers
set -e
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "layer or ln or block or whole_model or graphed" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
python tools/bench_summary.py $O/bench.json | head -8; python -c "import json;d=json.load(open('$O/bench2.json'));print('bench2',d['value'],d['ms_per_step'])"
