#!/bin/bash
# The other BASELINE configs on one GPU (bench.py's defaults = config 3 at N = 1):
#   cfg2: 256x256 fp32 batch 8 (numerics-parity config), cfg4: deep depth [2,4,32,2] 512 bf16 batch 16,
#   cfg5: 1024x1024 bf16 batch 4 (fp8 weights not implemented: bf16 weights).
set -e
mkdir -p gpurun_out/cfgs
timeout -k 10 300 python -u bench.py --img 256 --batch 8 --dtype fp32 --cpu-baseline off > gpurun_out/cfgs/cfg2.json 2> gpurun_out/cfgs/cfg2.err || { tail -20 gpurun_out/cfgs/cfg2.err; exit 1; }
cut -c1-400 gpurun_out/cfgs/cfg2.json
timeout -k 10 300 python -u bench.py --depth 2,4,32,2 --cpu-baseline off > gpurun_out/cfgs/cfg4.json 2> gpurun_out/cfgs/cfg4.err || { tail -20 gpurun_out/cfgs/cfg4.err; exit 1; }
cut -c1-400 gpurun_out/cfgs/cfg4.json
timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --cpu-baseline off > gpurun_out/cfgs/cfg5.json 2> gpurun_out/cfgs/cfg5.err || { tail -20 gpurun_out/cfgs/cfg5.err; exit 1; }
cut -c1-400 gpurun_out/cfgs/cfg5.json
