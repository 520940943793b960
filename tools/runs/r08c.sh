# round 6: GPU suite + smoke + bench + rocprof groups (timed replays only) and the PMC passes of the
# SimAM headline on the graph's kernels
bash tools/gpu_check.sh r08c tests || exit 1
T=r08c_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r08c_pmc.log 2>&1 || { tail -20 gpurun_out/r08c_pmc.log; exit 1; }
echo pmc done
