# round 6: 8-wave C = 256 Mlp forward with 32-hidden chunks (4-stage ring) -- Mlp tests, ablation
# probe, then interleaved bench pairs libcsu_hip.so (HC 32) vs libcsu_hip_ab.so (HC 64)
mkdir -p gpurun_out/r08f
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mlp or Mlp or reproduc" > gpurun_out/r08f/t_mlp.log 2>&1 || { tail -30 gpurun_out/r08f/t_mlp.log; exit 1; }
tail -2 gpurun_out/r08f/t_mlp.log
timeout -k 10 180 python -u tools/probes/mlp_ablate.py run > gpurun_out/r08f/mlp_ablate.txt 2>&1 || { tail -20 gpurun_out/r08f/mlp_ablate.txt; exit 1; }
cat gpurun_out/r08f/mlp_ablate.txt
bash tools/ab_lib.sh r08f mlp_fwd
