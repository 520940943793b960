#!/bin/bash
# The other BASELINE configs on one GPU at HEAD (bench.py's default line is configs[2]):
#   cfg1 256x256 fp32 B8 (+SimAM), cfg3 deep [2,4,32,2] 512 bf16 B16 (reference architecture),
#   cfg4 1024x1024 B4 (+SimAM) with fp8-e4m3 weights and in bf16, and the plain UNet 512 B16.
#   bash tools/configs_bench.sh <tag>
O=gpurun_out/${1:-cfgs}; mkdir -p $O
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 420 python -u bench.py "$@" --no-ref-arch > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python tools/bench_summary.py $O/$n.json | grep images
}
run cfg1_256_fp32 --img 256 --batch 8 --dtype fp32
run cfg3_deep --depth 2,4,32,2 --no-simam
run cfg4_1024_fp8 --img 1024 --batch 4 --dtype fp8
run cfg4_1024_bf16 --img 1024 --batch 4
run unet_512 --model unet
