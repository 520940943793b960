# round-4 evidence: fp8 tests, then every per-config bench line with its cpu_baseline
set -o pipefail
R=$(pwd); O=gpurun_out/r06e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 120 --timeout-method thread > $O/fp8.log 2>&1 || { echo FP8_FAIL; tail -30 $O/fp8.log; exit 1; }
for cfg in "c512:" "c1024:--img 1024 --batch 4" "c1024fp8:--img 1024 --batch 4 --dtype fp8" "simam512:--simam" \
           "simam1024:--simam --img 1024 --batch 4" "deep:--depth 2,4,32,2" "fp32_256:--img 256 --batch 8 --dtype fp32" \
           "unet:--model unet"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python -u bench.py $args > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo BENCH_FAIL $tag; tail -20 $O/bench_$tag.err; exit 1; }
  echo "$tag $(cut -c1-160 $O/bench_$tag.json)"
done
echo ALL_OK
