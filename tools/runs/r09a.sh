# PMC traffic keys for the BASELINE config lines that had none: 1024x1024 B4 fp8 +SimAM (configs[4] as named)
# and the deep [2,4,32,2] model (reference architecture)
T=r09a_pmc CFGS="c1024f8:--img 1024 --batch 4 --dtype fp8 --no-ref-arch|cdeep:--depth 2,4,32,2 --no-simam --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r09a_pmc.log 2>&1 || { tail -20 gpurun_out/r09a_pmc.log; exit 1; }
grep -h "kernel sets\|^| gemm\|^| linear_wgrad" gpurun_out/r09a_pmc.log | head
