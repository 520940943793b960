# round-4: CARAFE backward rewrite check, then PMC evidence at HEAD part 2: 1024 B4 fp8 and the plain UNet
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropout.py -x -q -k "carafe" --timeout 120 --timeout-method thread > $O/carafe.log 2>&1 || { echo CARAFE_FAIL; tail -30 $O/carafe.log; exit 1; }
CSU_LEDGER_DUMP=$O/launches_512.json timeout -k 10 300 python bench.py --cpu-baseline off > $O/b512.json 2> $O/b512.err || { echo B512_FAIL; tail -20 $O/b512.err; exit 1; }
T=r06h CFGS="c1024fp8:--img 1024 --batch 4 --dtype fp8|unet:--model unet" bash tools/pmc_head.sh
