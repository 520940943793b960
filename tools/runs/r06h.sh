# round-4 PMC evidence at HEAD, part 1: 512 B16 and 1024 B4 bf16 (tools/pmc_head.sh)
T=r06h CFGS="c512:--img 512 --batch 16|c1024:--img 1024 --batch 4" bash tools/pmc_head.sh
