# round-4: conv tile / split choice check, gemm4 configurations on the step's token-GEMM shapes, benches
set -o pipefail
R=$(pwd); O=gpurun_out/r06g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv" --timeout 120 --timeout-method thread > $O/conv.log 2>&1 || { echo CONV_FAIL; tail -30 $O/conv.log; exit 1; }
ONLY=merge,carafe CFGS=-1,0 timeout -k 10 300 python -u tools/conv_probe.py > $O/conv_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/conv_probe.txt; exit 1; }
CFGS=10,11,12,13,14,15,16,17,18,19 timeout -k 10 300 python -u tools/gemm_graph_probe.py > $O/gemm_probe.txt 2>&1 || { echo GPROBE_FAIL; tail -20 $O/gemm_probe.txt; exit 1; }
CSU_LEDGER_DUMP=$O/launches_512.json timeout -k 10 300 python bench.py --cpu-baseline off > $O/b512.json 2> $O/b512.err || { echo B512_FAIL; tail -20 $O/b512.err; exit 1; }
timeout -k 10 300 python bench.py --model unet --cpu-baseline off > $O/unet.json 2> $O/unet.err || { echo UNET_FAIL; tail -20 $O/unet.err; exit 1; }
echo ALL_OK
