# gemm_ws with the weight loads two units ahead (WS_PF 2) vs one (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm_ws or e4m3 or linear or model" > gpurun_out/r09d_tests.log 2>&1 || { tail -30 gpurun_out/r09d_tests.log; exit 1; }
tail -2 gpurun_out/r09d_tests.log
bash tools/ab_lib.sh r09d gemm
