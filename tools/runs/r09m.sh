# 8-wave Mlp kernels: every fragment read of a GEMM phase issued before its MFMAs (MLP8_LDS_FIRST 1) vs
# the compiler's interleaving (libcsu_hip_ab.so); isolated timing + bench pairs
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mlp" > gpurun_out/r09m_tests.log 2>&1 || { tail -30 gpurun_out/r09m_tests.log; exit 1; }
tail -2 gpurun_out/r09m_tests.log
timeout -k 10 120 python -u tools/probes/mlp_bwd_ab.py > gpurun_out/r09m_mlp_bwd_ab.txt 2>&1 || { cat gpurun_out/r09m_mlp_bwd_ab.txt; exit 1; }
cat gpurun_out/r09m_mlp_bwd_ab.txt
bash tools/ab_lib.sh r09m mlp_bwd
