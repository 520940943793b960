# pipelined + staggered Mlp backward at C = 256 (mlp_bwd8p_kernel): Mlp / model / train tests, the
# isolated timing against mlp_bwd8_kernel (libcsu_hip_ab.so: -DMLP_BWD8P=0), interleaved bench pairs;
# then the attention per-workgroup timelines (debug build) at 1024 stage 3 and 512 stage 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mlp or model or graph or full_size" > gpurun_out/r08r_tests.log 2>&1 || { tail -30 gpurun_out/r08r_tests.log; exit 1; }
tail -3 gpurun_out/r08r_tests.log
timeout -k 10 120 python -u tools/probes/mlp_bwd_ab.py > gpurun_out/r08r_mlp_bwd_ab.txt 2>&1 || { cat gpurun_out/r08r_mlp_bwd_ab.txt; exit 1; }
cat gpurun_out/r08r_mlp_bwd_ab.txt
bash tools/ab_lib.sh r08r mlp_bwd || exit 1
timeout -k 10 120 python -u tools/attn_wg_timeline.py 13 > gpurun_out/r08r_tl13.txt 2>&1 && timeout -k 10 120 python -u tools/attn_wg_timeline.py 3 > gpurun_out/r08r_tl3.txt 2>&1
cat gpurun_out/r08r_tl13.txt gpurun_out/r08r_tl3.txt
