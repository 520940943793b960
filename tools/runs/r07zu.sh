# PMC tables at the closing HEAD (MFMA busy, HBM bytes per C-ABI call): the SimAM headline, the
# reference architecture, and 1024x1024 B4 bf16 +SimAM (its bench line's traffic key)
T=r07zu_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch|c512n:--img 512 --batch 16 --no-simam --no-ref-arch|c1024s:--img 1024 --batch 4 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r07zu_pmc.log 2>&1 || { tail -20 gpurun_out/r07zu_pmc.log; exit 1; }
echo pmc done
