# round-4 final HEAD: rocprofv3 kernel traces of the 1024 B4 bf16 and fp8 steps, grouped per C-ABI call
set -o pipefail
R=$(pwd); O=gpurun_out/r06s; mkdir -p $O; export TMPDIR=/tmp
for cfg in "c1024:--img 1024 --batch 4" "c1024fp8:--img 1024 --batch 4 --dtype fp8"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python -u bench.py $args --cpu-baseline off > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$tag -o $tag -- \
    python3 $R/bench.py $args --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench_$tag.json 2> $R/$O/prof_$tag.err || { tail -30 $R/$O/prof_$tag.err; exit 1; }
  cd $R
  KT=$(find $O/prof_$tag -name '*kernel_trace.csv' -print -quit)
  python tools/prof_summary.py "$KT" 5 60 > $O/step_breakdown_$tag.txt
  python tools/prof_groups.py "$KT" 5 $O/bench_$tag.json > $O/groups_$tag.md || true
  head -4 $O/step_breakdown_$tag.txt
done
echo ALL_OK
