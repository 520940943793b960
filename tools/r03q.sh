#!/bin/bash
# A/B of the rotated reduction-slice order (default build) vs natural order (ab/libcsu_norot.so):
# parity tests of the touched kernels, conv probe, interleaved 512 B16 benches.
set -e
O=gpurun_out/r03q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mlp or gemm or linear or conv or unet or block or model" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CFGS=0,3,7,8,9 timeout -k 10 300 python -u tools/conv_probe.py > $O/conv_probe.txt 2>&1 || { tail -20 $O/conv_probe.txt; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off > $O/bench_rot$i.json 2> $O/bench_rot$i.err || { tail -20 $O/bench_rot$i.err; exit 1; }
  CSU_LIB_PATH=$PWD/ab/libcsu_norot.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline off > $O/bench_norot$i.json 2> $O/bench_norot$i.err || { tail -20 $O/bench_norot$i.err; exit 1; }
done
for f in $O/bench_*.json; do python tools/bench_summary.py $f | head -8; done
cat $O/conv_probe.txt
