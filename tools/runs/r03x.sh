#!/bin/bash
# Round-3 HEAD validation: full GPU suite + smoke, headline bench (512 B16, roofline + CPU baseline),
# every BASELINE config line (256 fp32, SimAM 512, deep 512, 1024 bf16 / fp8, plain UNet), rocprofv3
# kernel traces of the 512 step and the UNet step.  T=<tag>.
set -e
T=${T:-r03x}; O=gpurun_out/$T; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json | head -3
run() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" --cpu-baseline off > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }; python tools/bench_summary.py $O/bench_$n.json | head -1; }
run unet --model unet --steps 6 --warmup 2
run 1024_bf16 --img 1024 --batch 4
run 1024_fp8 --img 1024 --batch 4 --dtype fp8
run simam --simam
run deep --depth 2,4,32,2
run fp32_256 --img 256 --batch 8 --dtype fp32
for cfg in "512 cswin" "512 unet"; do
  set -- $cfg
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$2 -o $T -- \
    python3 $R/bench.py --model $2 --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench_$2.json 2> $R/$O/prof_$2.err || { tail -30 $R/$O/prof_$2.err; exit 1; }
  cd $R
  KT=$(find $O/prof_$2 -name '*kernel_trace.csv' -print -quit)
  ST=$(find $O/prof_$2 -name '*kernel_stats.csv' -print -quit)
  cp "$ST" $O/kernel_stats_$2.csv
  python tools/prof_summary.py "$KT" 5 60 > $O/step_breakdown_$2.txt
  BJ=$O/bench.json; [ $2 = unet ] && BJ=$O/bench_unet.json
  python tools/prof_groups.py "$KT" 5 $BJ > $O/groups_$2.md || true
  head -3 $O/step_breakdown_$2.txt
done
