# round-4: rocprofv3 kernel trace of the --dp-force step (N = 1) -- what the data-parallel path adds over dp1
set -o pipefail
O=gpurun_out/${T:-r06v}; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o dpf -- \
  python3 $R/bench.py --dp-force --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/bench.json 2> $R/$O/prof.err || { tail -30 $R/$O/prof.err; exit 1; }
cd $R
KT=$(find $O/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 5 70 > $O/step_breakdown_dpf.txt
head -45 $O/step_breakdown_dpf.txt
echo ALL_OK
