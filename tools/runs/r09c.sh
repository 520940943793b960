# grouped 256 x 128 token weight gradients with loads three steps ahead (WG_D256 3) vs two (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wgrad or model or graph" > gpurun_out/r09c_tests.log 2>&1 || { tail -30 gpurun_out/r09c_tests.log; exit 1; }
tail -2 gpurun_out/r09c_tests.log
bash tools/ab_lib.sh r09c linear_wgrad
