# SimAM step: bench line + rocprofv3 kernel trace breakdown (512 B16 --simam)
O=gpurun_out/r07j; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --simam --cpu-baseline off > $O/bench.json 2> $O/bench.err || exit 1
python tools/bench_summary.py $O/bench.json | head -3
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o simam -- \
  python3 $R/bench.py --simam --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench.json 2> $R/$O/prof.err || exit 1
cd $R
KT=$(find $O/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 5 80 > $O/step_breakdown_simam.txt
grep -i "simam\|total\|busy" $O/step_breakdown_simam.txt
