set -e
mkdir -p gpurun_out/r02e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or side_stream or linear" > gpurun_out/r02e/pytest.log 2>&1 || { tail -40 gpurun_out/r02e/pytest.log; exit 1; }
tail -2 gpurun_out/r02e/pytest.log
timeout -k 10 400 python -u tools/wgrad_bench.py --plans auto,c1,c2,c3,t64x64:c2 > gpurun_out/r02e/wgrad_bench.txt 2>&1 || { tail -30 gpurun_out/r02e/wgrad_bench.txt; exit 1; }
cat gpurun_out/r02e/wgrad_bench.txt
