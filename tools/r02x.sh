#!/bin/bash
# conv weight gradients written OIHW by the kernel; BN rows in flight; torch glue census
set -e
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_kernels.py tests/test_gpu_model.py -k "unet or bn or maxpool or conv or carafe or whole_model or graphed" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TREE=1 timeout -k 10 200 python -u tools/torch_ops_profile.py > $O/torch_ops_tree.txt 2>&1 || { tail -20 $O/torch_ops_tree.txt; exit 1; }
timeout -k 10 300 python -u bench.py --model unet --img 128 --batch 8 --dtype bf16 --cpu-baseline off > $O/bench_unet_bf16.json 2> $O/bench_unet_bf16.err || { tail -30 $O/bench_unet_bf16.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench_unet_bf16.json $O/bench.json
