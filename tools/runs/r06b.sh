# round-4 validation: fp8 Mlp + attention tests first, then the whole GPU suite, then bench lines
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -v --timeout 120 --timeout-method thread > $O/fp8.log 2>&1 || { echo FP8_FAIL; tail -30 $O/fp8.log; exit 1; }
timeout -k 10 120 python -u tools/mlp8_probe.py > $O/mlp8_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/mlp8_probe.txt; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "stripe_attention or conv_c16 or conv2d_nhwc or deep_ring" --timeout 120 --timeout-method thread > $O/attn.log 2>&1 || { echo ATTN_FAIL; tail -30 $O/attn.log; exit 1; }
timeout -k 10 300 python bench.py --img 1024 --batch 4 --cpu-baseline off > $O/b1024_bf16.json 2> $O/b1024_bf16.err || { echo B1024_FAIL; tail -20 $O/b1024_bf16.err; exit 1; }
timeout -k 10 300 python bench.py --img 1024 --batch 4 --dtype fp8 --cpu-baseline off > $O/b1024_fp8.json 2> $O/b1024_fp8.err || { echo B1024F_FAIL; tail -20 $O/b1024_fp8.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline off > $O/b512.json 2> $O/b512.err || { echo B512_FAIL; tail -20 $O/b512.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo SUITE_FAIL; tail -30 $O/tests.log; exit 1; }
echo ALL_OK
