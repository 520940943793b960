set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r06b/fp8.log 2>&1 || { echo FP8_FAIL; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b/tests.log 2>&1 || { echo SUITE_FAIL; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r06b/bench.json 2> gpurun_out/r06b/bench.err
