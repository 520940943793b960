# round 6 closing HEAD, part 2: PMC passes over the graph's kernels (SimAM headline, reference architecture,
# 1024x1024 B4) and every other BASELINE config
T=r08y_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch|c512n:--img 512 --batch 16 --no-simam --no-ref-arch|c1024s:--img 1024 --batch 4 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r08y_pmc.log 2>&1 || { tail -20 gpurun_out/r08y_pmc.log; exit 1; }
echo pmc done
bash tools/configs_bench.sh r08y_cfg
