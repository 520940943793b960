# gemm4: the 64 x 64 tile (3-stage ring, 2 workgroups per CU) for shapes whose 128 x 64 tiles do not fill
# 2 x CUs workgroups (the 4096-token stage; G4_SMALLM 1) vs 128 x 64 everywhere (libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm or linear or model" > gpurun_out/r09w_tests.log 2>&1 || { tail -30 gpurun_out/r09w_tests.log; exit 1; }
tail -2 gpurun_out/r09w_tests.log
bash tools/ab_lib.sh r09w gemm || exit 1
bash tools/ab_1024.sh r09w gemm
