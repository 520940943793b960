# fused attention backward v2: parity (attention kernels + dropout) then per-stage timing / phases
set -e
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_dropout.py -k "stripe or two_branch or attention or block or model" > gpurun_out/r03h_tests.log 2>&1 || { tail -30 gpurun_out/r03h_tests.log; exit 1; }
tail -1 gpurun_out/r03h_tests.log
bash tools/r03g.sh
