# round-4: remaining GPU tests (train / unet / Mlp), 512 bench, kernel traces of the 1024 bf16 and fp8 steps
set -o pipefail
R=$(pwd); O=gpurun_out/r06c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_unet.py tests/test_gpu_dropout.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "mlp" --timeout 120 --timeout-method thread > $O/mlp.log 2>&1 || { echo MLP_FAIL; tail -30 $O/mlp.log; exit 1; }
timeout -k 10 300 python bench.py --cpu-baseline off > $O/b512.json 2> $O/b512.err || { echo B512_FAIL; tail -20 $O/b512.err; exit 1; }
for cfg in "bf16:--img 1024 --batch 4" "fp8:--img 1024 --batch 4 --dtype fp8"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py $args --cpu-baseline off > $O/bench_1024_$tag.json 2> $O/bench_1024_$tag.err || { echo BENCH_FAIL; tail -20 $O/bench_1024_$tag.err; exit 1; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$tag -o p -- \
    python3 $R/bench.py $args --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench_$tag.json 2> $R/$O/prof_$tag.err || { echo PROF_FAIL; tail -30 $R/$O/prof_$tag.err; exit 1; }
  cd $R
  KT=$(find $O/prof_$tag -name '*kernel_trace.csv' -print -quit)
  ST=$(find $O/prof_$tag -name '*kernel_stats.csv' -print -quit)
  cp "$ST" $O/kernel_stats_1024_$tag.csv
  python tools/prof_summary.py "$KT" 4 60 > $O/step_breakdown_1024_$tag.txt
  python tools/prof_groups.py "$KT" 4 $O/bench_1024_$tag.json > $O/groups_1024_$tag.md || true
  rm -rf $O/prof_$tag
done
echo ALL_OK
