# mlp_bwd8p_kernel with the weight DMA two chunks ahead: Mlp tests, isolated timing against
# mlp_bwd8_kernel (libcsu_hip_ab.so), interleaved bench pairs
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mlp" > gpurun_out/r08s_tests.log 2>&1 || { tail -30 gpurun_out/r08s_tests.log; exit 1; }
tail -2 gpurun_out/r08s_tests.log
timeout -k 10 120 python -u tools/probes/mlp_bwd_ab.py > gpurun_out/r08s_mlp_bwd_ab.txt 2>&1 || { cat gpurun_out/r08s_mlp_bwd_ab.txt; exit 1; }
cat gpurun_out/r08s_mlp_bwd_ab.txt
bash tools/ab_lib.sh r08s mlp_bwd
