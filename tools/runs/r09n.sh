# attention backward (4-wave, whole windows): the dQ quadrant's key-tile loop branch-free (ATT_DQ_FULL 1)
# vs one branch + full LDS wait per key tile (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attn or stripe or lepe or model or dropout" > gpurun_out/r09n_tests.log 2>&1 || { tail -30 gpurun_out/r09n_tests.log; exit 1; }
tail -2 gpurun_out/r09n_tests.log
bash tools/ab_lib.sh r09n stripe_attn_bwd || exit 1
bash tools/ab_1024.sh r09n stripe_attn_bwd
