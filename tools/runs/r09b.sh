# PMC traffic keys for the 256x256 fp32 +SimAM line and the plain UNet 512 B16
T=r09b_pmc CFGS="c256f32:--img 256 --batch 8 --dtype fp32 --no-ref-arch|unet:--model unet --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r09b_pmc.log 2>&1 || { tail -20 gpurun_out/r09b_pmc.log; exit 1; }
grep -h "kernel sets\|^| gemm\|^| conv" gpurun_out/r09b_pmc.log | head
