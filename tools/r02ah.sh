#!/bin/bash
# data-parallel path (captured bucketed all-reduce) with the end-of-backward deferrals kept
set -e
O=gpurun_out/r02ah; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py -k "dp_path or graphed or bitwise or capture" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --dp-force --cpu-baseline off --no-roofline > $O/bench_dpforce.json 2> $O/bench_dpforce.err || { tail -30 $O/bench_dpforce.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench_dpforce.json $O/bench.json | grep json
