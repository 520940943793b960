#!/bin/bash
# Headline bench (512 B16, no CPU baseline) + rocprofv3 kernel trace of the 512 CSWin step.  T=<tag>.
set -e
T=${T:-quick}; O=gpurun_out/$T; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json | head -3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_cswin -o $T -- \
  python3 $R/bench.py --model cswin --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench_cswin.json 2> $R/$O/prof_cswin.err || { tail -30 $R/$O/prof_cswin.err; exit 1; }
cd $R
KT=$(find $O/prof_cswin -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 5 60 > $O/step_breakdown_cswin.txt
python tools/prof_groups.py "$KT" 5 $O/bench.json > $O/groups_cswin.md || true
head -3 $O/step_breakdown_cswin.txt
