# s_setprio 1 for waves 4-7 (mlp_fwd8 / mlp_bwd8 / stripe_bwd_fused_w 8-wave) + the mlp_fwd8 stagger
# (waves 4-7 GEMM2 first) vs neither (libcsu_hip_ab.so: -DCSU_PRIO_HALF=0 -DMLP_FWD8_STAGGER=0)
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mlp or attn or stripe" > gpurun_out/r08u_tests.log 2>&1 || { tail -30 gpurun_out/r08u_tests.log; exit 1; }
tail -2 gpurun_out/r08u_tests.log
bash tools/ab_lib.sh r08u mlp_fwd || exit 1
bash tools/ab_1024.sh r08u stripe_attn_bwd
