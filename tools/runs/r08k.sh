# ledger events without the system-scope fence (timing-only events): groups table ratios; the
# configs[4] +SimAM fp8 full-size row
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread -k "full_size" > gpurun_out/r08k_tests.log 2>&1 || { tail -30 gpurun_out/r08k_tests.log; exit 1; }
tail -3 gpurun_out/r08k_tests.log
bash tools/gpu_check.sh r08k notests
