# round 6: the 8-wave C = 256 Mlp forward -- Mlp tests, the isolated timing against the 4-wave
# kernel (tools/probes/mlp_ablate.py base build = the previous product), then the evidence suite
mkdir -p gpurun_out/r08d
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mlp or Mlp" > gpurun_out/r08d/t_mlp.log 2>&1 || { tail -30 gpurun_out/r08d/t_mlp.log; exit 1; }
tail -2 gpurun_out/r08d/t_mlp.log
timeout -k 10 120 python -u tools/mlp_probe.py > gpurun_out/r08d/mlp_probe.txt 2>&1 || { tail -20 gpurun_out/r08d/mlp_probe.txt; exit 1; }
cat gpurun_out/r08d/mlp_probe.txt
bash tools/gpu_check.sh r08d tests || exit 1
T=r08d_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r08d_pmc.log 2>&1 || { tail -20 gpurun_out/r08d_pmc.log; exit 1; }
echo pmc done
