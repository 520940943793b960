# round-4: CARAFE backward rewrite + 8-wave weight-gradient tile checks, 512 bench, then PMC evidence at
# HEAD part 2: 1024 B4 fp8 and the plain UNet
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropout.py -x -q -k "carafe or wgrad" --timeout 120 --timeout-method thread > $O/kern.log 2>&1 || { echo KERN_FAIL; tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
CSU_LEDGER_DUMP=$O/launches_512.json timeout -k 10 300 python bench.py --cpu-baseline off > $O/b512.json 2> $O/b512.err || { echo B512_FAIL; tail -20 $O/b512.err; exit 1; }
cut -c1-200 $O/b512.json
T=r06h CFGS="c1024fp8:--img 1024 --batch 4 --dtype fp8|unet:--model unet" bash tools/pmc_head.sh
