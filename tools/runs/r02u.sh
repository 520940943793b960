#!/bin/bash
# HEAD profile: gpu tests, the 512 B16 bench, PMC HBM traffic of the dominant kernels at 512 (token
# weight gradient) and 1024 B4 (attention backward), a rocprofv3 kernel trace + stats at 512 and 1024.
set -e
T=${T:-r02u}; O=gpurun_out/$T; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 $O/pytest.log
timeout -k 10 400 bash tools/pmc_roofline.sh "linear_wgrad|512|16|bf16" wgrad_tile "wgrad_tile|wslab_reduce" wgrad_tile,wslab_reduce
timeout -k 10 400 bash tools/pmc_roofline.sh "stripe_attn_bwd|1024|4|bf16" stripe_bwd_dq "stripe_bwd|lepe_wgrad" stripe_bwd,lepe_wgrad --img 1024 --batch 4
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --img 1024 --batch 4 --cpu-baseline off > $O/bench_1024.json 2> $O/bench_1024.err || { tail -30 $O/bench_1024.err; exit 1; }
for cfg in "512 16" "1024 4"; do
  set -- $cfg
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof$1 -o $T -- \
    python3 $R/bench.py --img $1 --batch $2 --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench$1.json 2> $R/$O/prof$1.err || { tail -30 $R/$O/prof$1.err; exit 1; }
  cd $R
  KT=$(find $O/prof$1 -name '*kernel_trace.csv' -print -quit)
  ST=$(find $O/prof$1 -name '*kernel_stats.csv' -print -quit)
  cp "$ST" $O/kernel_stats_$1.csv
  python tools/prof_summary.py "$KT" 4 60 > $O/step_breakdown_$1.txt
done
python tools/prof_groups.py "$(find $O/prof512 -name '*kernel_trace.csv' -print -quit)" 4 $O/bench.json > $O/groups_512.md
python tools/prof_groups.py "$(find $O/prof1024 -name '*kernel_trace.csv' -print -quit)" 4 $O/bench_1024.json > $O/groups_1024.md
head -8 $O/groups_512.md; head -8 $O/groups_1024.md
python tools/bench_summary.py $O/bench.json $O/bench_1024.json
