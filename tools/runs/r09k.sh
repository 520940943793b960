# attention backward prologue: the LePE weights held in registers across the row loop (ATT_WREG 1) vs
# re-read per row (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attn or stripe or lepe or model" > gpurun_out/r09k_tests.log 2>&1 || { tail -30 gpurun_out/r09k_tests.log; exit 1; }
tail -2 gpurun_out/r09k_tests.log
bash tools/ab_lib.sh r09k stripe_attn_bwd || exit 1
bash tools/ab_1024.sh r09k stripe_attn_bwd
