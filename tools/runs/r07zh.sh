# final evidence at HEAD: full GPU suite + smoke + bench + rocprof (gpu_check.sh), then PMC traffic passes
bash tools/gpu_check.sh r07zh tests || exit 1
T=r07zh_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch|c512n:--img 512 --batch 16 --no-simam --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r07zh_pmc.log 2>&1 || { tail -20 gpurun_out/r07zh_pmc.log; exit 1; }
echo pmc done
