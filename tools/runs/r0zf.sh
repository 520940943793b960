# PMC passes over the 256x256 B8 fp32 line's graph kernels after the fp32 GEMM tile changes
T=r0zf_pmc CFGS="c256f32:--img 256 --batch 8 --dtype fp32 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r0zf_pmc.log 2>&1 || { tail -20 gpurun_out/r0zf_pmc.log; exit 1; }
echo pmc done
