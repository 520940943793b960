mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "stripe or two_branch or bce" > gpurun_out/r03b_kern.log 2>&1
rc=$?; tail -5 gpurun_out/r03b_kern.log; echo "kern rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_dropout.py tests/test_gpu_model.py > gpurun_out/r03b_model.log 2>&1
rc=$?; tail -5 gpurun_out/r03b_model.log; echo "model rc=$rc"
