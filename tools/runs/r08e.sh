# round 6: the 8-wave C = 256 Mlp backward -- Mlp tests, the ablation probe (old / 8-wave kernels),
# then interleaved bench pairs: libcsu_hip.so (8-wave backward) vs libcsu_hip_ab.so (4-wave backward)
mkdir -p gpurun_out/r08e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mlp or Mlp or reproduc" > gpurun_out/r08e/t_mlp.log 2>&1 || { tail -30 gpurun_out/r08e/t_mlp.log; exit 1; }
tail -2 gpurun_out/r08e/t_mlp.log
timeout -k 10 180 python -u tools/probes/mlp_ablate.py run > gpurun_out/r08e/mlp_ablate.txt 2>&1 || { tail -20 gpurun_out/r08e/mlp_ablate.txt; exit 1; }
cat gpurun_out/r08e/mlp_ablate.txt
bash tools/ab_lib.sh r08e mlp_bwd
