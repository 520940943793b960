# LayerNorm backward with 8 row groups in flight per wave iteration (LN_LU 8) vs 4 (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "layernorm or ln_ or layer_norm or model" > gpurun_out/r08z_tests.log 2>&1 || { tail -30 gpurun_out/r08z_tests.log; exit 1; }
tail -2 gpurun_out/r08z_tests.log
bash tools/ab_lib.sh r08z layernorm_bwd
