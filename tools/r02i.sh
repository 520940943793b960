set -e
mkdir -p gpurun_out/r02i
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or linear or side_stream" > gpurun_out/r02i/pytest.log 2>&1 || { tail -40 gpurun_out/r02i/pytest.log; exit 1; }
tail -2 gpurun_out/r02i/pytest.log
timeout -k 10 400 python -u tools/wgrad_bench.py --plans auto,c0.5,t64x64:c1 > gpurun_out/r02i/wgrad_bench.txt 2>&1 || { tail -30 gpurun_out/r02i/wgrad_bench.txt; exit 1; }
cat gpurun_out/r02i/wgrad_bench.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/r02i/pytest_train.log 2>&1 || true
tail -60 gpurun_out/r02i/pytest_train.log
