# gemm_ws 32-token panels (WS_HALF) for the 16384-token stage: gemm tests, then interleaved A/B of the
# product library (32-token panels) against libcsu_hip_ab.so (built with -DWS_HALF=0)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm_ws or e4m3 or linear or block or model or fp8" > gpurun_out/r08j_tests.log 2>&1 || { tail -30 gpurun_out/r08j_tests.log; exit 1; }
tail -3 gpurun_out/r08j_tests.log
bash tools/ab_lib.sh r08j gemm
