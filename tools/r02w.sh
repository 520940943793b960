#!/bin/bash
# UNet on csu kernels: BN/ReLU/MaxPool + Adam tests, plain-UNet bench lines (BASELINE config 1 model).
set -e
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_kernels.py tests/test_gpu_model.py -k "unet or bn or maxpool or adam" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --model unet --img 128 --batch 8 --dtype fp32 > $O/bench_unet_fp32.json 2> $O/bench_unet_fp32.err || { tail -30 $O/bench_unet_fp32.err; exit 1; }
timeout -k 10 300 python -u bench.py --model unet --img 128 --batch 8 --dtype bf16 --cpu-baseline off > $O/bench_unet_bf16.json 2> $O/bench_unet_bf16.err || { tail -30 $O/bench_unet_bf16.err; exit 1; }
python tools/bench_summary.py $O/bench_unet_fp32.json $O/bench_unet_bf16.json
