# PMC passes over the graph's kernels at HEAD (after the conv weight-gradient XCD order): SimAM headline
# and 1024x1024 B4 -- new conv_wgrad traffic figures for profiles/pmc_traffic.json
T=r09v_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch|c1024s:--img 1024 --batch 4 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r09v_pmc.log 2>&1 || { tail -20 gpurun_out/r09v_pmc.log; exit 1; }
echo pmc done
