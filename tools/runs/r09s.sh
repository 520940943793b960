# conv weight gradients with XCD-aware workgroup order (CW_XCD 1: the tiles of one token chunk on one
# XCD, sharing its L2) vs hardware order (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "conv or wgrad or carafe or embed or merge or model" > gpurun_out/r09s_tests.log 2>&1 || { tail -30 gpurun_out/r09s_tests.log; exit 1; }
tail -2 gpurun_out/r09s_tests.log
bash tools/ab_lib.sh r09s conv_wgrad || exit 1
bash tools/ab_1024.sh r09s conv_wgrad
