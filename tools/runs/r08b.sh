# round 6: fused-Mlp C = 256 ablation (tools/probes/mlp_ablate.py), then GPU suite + smoke + bench +
# rocprof groups (timed replays only) and the PMC passes of the SimAM headline on the graph's kernels
mkdir -p gpurun_out/r08b
timeout -k 10 120 python -u tools/probes/mlp_ablate.py run > gpurun_out/r08b/mlp_ablate.txt 2>&1 || { tail -20 gpurun_out/r08b/mlp_ablate.txt; exit 1; }
cat gpurun_out/r08b/mlp_ablate.txt
bash tools/gpu_check.sh r08b tests || exit 1
T=r08b_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r08b_pmc.log 2>&1 || { tail -20 gpurun_out/r08b_pmc.log; exit 1; }
echo pmc done
