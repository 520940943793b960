set -e
mkdir -p gpurun_out/r02b
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or side_stream or linear" > gpurun_out/r02b/pytest.log 2>&1 || { tail -40 gpurun_out/r02b/pytest.log; exit 1; }
tail -3 gpurun_out/r02b/pytest.log
timeout -k 10 400 python -u tools/wgrad_bench.py --plans auto,c0.5,c1,c2,c4 > gpurun_out/r02b/wgrad_bench.txt 2>&1 || { tail -30 gpurun_out/r02b/wgrad_bench.txt; exit 1; }
cat gpurun_out/r02b/wgrad_bench.txt
timeout -k 10 300 python -u bench.py --cpu-baseline off > gpurun_out/r02b/bench.json 2> gpurun_out/r02b/bench.err || { tail -30 gpurun_out/r02b/bench.err; exit 1; }
cat gpurun_out/r02b/bench.json
