# attention forward: the LePE epilogue with zero-row taps (ATT_FWD_ZROW 1) vs
# a branch per out-of-window tap (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attn or stripe or lepe or model or dropout" > gpurun_out/r09p_tests.log 2>&1 || { tail -30 gpurun_out/r09p_tests.log; exit 1; }
tail -2 gpurun_out/r09p_tests.log
bash tools/ab_lib.sh r09p stripe_attn_fwd || exit 1
bash tools/ab_1024.sh r09p stripe_attn_fwd
