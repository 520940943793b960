#!/bin/bash
# Every BASELINE config (and the drop-in variants) benched at one HEAD on one MI355X:
#   cfg1 plain UNet 128x128 B8 (fp32 and bf16; the reference runs it on CPU), cfg2 256x256 fp32 B8,
#   cfg3 512x512 bf16 B16 (bench.py default) + SimAM, + the reference main() dropout rates,
#   cfg4 deep [2,4,32,2] 512 bf16 B16, cfg5 1024x1024 B4 bf16 and fp8-e4m3 weights.
set -e
T=${T:-r02ak}; O=gpurun_out/$T; mkdir -p $O
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python tools/bench_summary.py $O/$n.json
}
run unet_fp32 --model unet --img 128 --batch 8 --dtype fp32
run unet_bf16 --model unet --img 128 --batch 8 --dtype bf16
run cfg2_fp32_256 --img 256 --batch 8 --dtype fp32
run cfg3_512 --img 512 --batch 16
run cfg3_simam512 --img 512 --batch 16 --simam
run cfg3_dropout512 --img 512 --batch 16 --dropout 0.3
run cfg4_deep512 --depth 2,4,32,2
run cfg5_bf16_1024 --img 1024 --batch 4
run cfg5_fp8_1024 --img 1024 --batch 4 --dtype fp8
