# PMC traffic at HEAD for the headline (SimAM) and reference-architecture workloads
T=r07u CFGS="c512s:--img 512 --batch 16 --no-ref-arch|c512n:--img 512 --batch 16 --no-simam --no-ref-arch" bash tools/pmc_head.sh
