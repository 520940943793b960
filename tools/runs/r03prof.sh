#!/bin/bash
# Round-3 HEAD profile: bench 512 B16 (roofline + cpu baseline) and 1024 B4, rocprofv3 kernel trace +
# stats of both, grouped per C-ABI call.  T=<tag> names the output dir gpurun_out/<tag>.
set -e
T=${T:-r03d}; O=gpurun_out/$T; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json | head -5
[ -n "$SKIP_1024" ] || timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --cpu-baseline off > $O/bench_1024.json 2> $O/bench_1024.err || { tail -30 $O/bench_1024.err; exit 1; }
for cfg in "512 16" "1024 4"; do
  set -- $cfg
  [ -n "$SKIP_1024" ] && [ $1 = 1024 ] && continue
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof$1 -o $T -- \
    python3 $R/bench.py --img $1 --batch $2 --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench$1.json 2> $R/$O/prof$1.err || { tail -30 $R/$O/prof$1.err; exit 1; }
  cd $R
  KT=$(find $O/prof$1 -name '*kernel_trace.csv' -print -quit)
  ST=$(find $O/prof$1 -name '*kernel_stats.csv' -print -quit)
  cp "$ST" $O/kernel_stats_$1.csv
  python tools/prof_summary.py "$KT" 4 60 > $O/step_breakdown_$1.txt
  BJ=$O/bench.json; [ $1 = 1024 ] && BJ=$O/bench_1024.json
  python tools/prof_groups.py "$KT" 4 $BJ > $O/groups_$1.md
  head -12 $O/groups_$1.md
done
