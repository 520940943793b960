#!/bin/bash
# halo conv weight gradient in the UNet step: UNet / conv GPU tests, UNet 512 B16 bench, CSWin bench
set -e
O=gpurun_out/r03u; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "unet or conv or merge or carafe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --model unet --steps 6 --warmup 2 --cpu-baseline off > $O/bench_unet.json 2> $O/bench_unet.err || { tail -20 $O/bench_unet.err; exit 1; }
python tools/bench_summary.py $O/bench_unet.json | head -12
R=$(pwd); cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o unet -- \
  python3 $R/bench.py --model unet --steps 3 --warmup 1 --cpu-baseline off --no-roofline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { tail -20 $R/$O/prof.err; exit 1; }
cd $R
KT=$(find $O/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 3 40 > $O/step_breakdown_unet.txt && head -40 $O/step_breakdown_unet.txt
