#!/bin/bash
# conv v3 picks in the whole step: UNet / conv GPU tests, UNet 512 B16 bench, CSWin 512 B16 bench,
# token-GEMM tile probe after the K-slice rotation
set -e
O=gpurun_out/r03s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "unet or conv or merge or carafe or model" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --model unet --steps 6 --warmup 2 --cpu-baseline off > $O/bench_unet.json 2> $O/bench_unet.err || { tail -20 $O/bench_unet.err; exit 1; }
python tools/bench_summary.py $O/bench_unet.json | head -10
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json | head -14
CFGS=11,16,18,19 timeout -k 10 300 python -u tools/gemm_graph_probe.py > $O/gemm_probe.txt 2>&1 || { tail -20 $O/gemm_probe.txt; exit 1; }
cat $O/gemm_probe.txt
