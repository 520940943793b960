# attention forward: the step's K rows and V^T fragments read before the S MFMAs (ATT_FWD_VFIRST 1) vs
# the compiler's placement (V^T reads right before each PV MFMA; libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attn or stripe or lepe or model or dropout" > gpurun_out/r09o_tests.log 2>&1 || { tail -30 gpurun_out/r09o_tests.log; exit 1; }
tail -2 gpurun_out/r09o_tests.log
bash tools/ab_lib.sh r09o stripe_attn_fwd || exit 1
bash tools/ab_1024.sh r09o stripe_attn_fwd
