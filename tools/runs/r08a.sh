# round 6 first run: GPU suite + smoke + bench + rocprof groups (timed replays only), then the PMC passes
# of the SimAM headline on the graph's kernels (kernel_match)
bash tools/gpu_check.sh r08a tests || exit 1
T=r08a_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r08a_pmc.log 2>&1 || { tail -20 gpurun_out/r08a_pmc.log; exit 1; }
echo pmc done
