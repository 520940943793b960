# rocprofv3 kernel trace of the 1024x1024 B4 bf16 +SimAM step at the closing HEAD (after the 8-wave
# attention forward / 1024-token-window backward)
set -e
R=$(pwd); O=$R/gpurun_out/r07zz; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c1024 -- \
  python3 $R/bench.py --img 1024 --batch 4 --steps 5 --warmup 2 --cpu-baseline off --no-ref-arch > $O/prof_bench.json 2> $O/prof.err \
  || { tail -30 $O/prof.err; exit 1; }
cd $R
KT=$(find $O/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 2 60 > $O/step_breakdown.txt && head -30 $O/step_breakdown.txt
