set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or fused_mlp or linear" > gpurun_out/t_gemm.log 2>&1 || { tail -40 gpurun_out/t_gemm.log; exit 1; }
tail -3 gpurun_out/t_gemm.log
CFGS=${CFGS:-10,11,12,13,14,15} timeout -k 10 300 python -u tools/linear_probe.py > gpurun_out/linear_probe2.txt 2>&1
cat gpurun_out/linear_probe2.txt
