# round-4 PMC evidence at HEAD, part 2: 1024 B4 fp8 and the plain UNet (tools/pmc_head.sh)
T=r06h CFGS="c1024fp8:--img 1024 --batch 4 --dtype fp8|unet:--model unet" bash tools/pmc_head.sh
