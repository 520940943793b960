# round-4: fp8 quantiser with the Mlp layouts, 8-wave attention backward for 512-token windows
set -o pipefail
R=$(pwd); O=gpurun_out/r06d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 120 --timeout-method thread > $O/fp8.log 2>&1 || { echo FP8_FAIL; tail -30 $O/fp8.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropout.py -x -q -k "stripe_attention" --timeout 120 --timeout-method thread > $O/attn.log 2>&1 || { echo ATTN_FAIL; tail -30 $O/attn.log; exit 1; }
timeout -k 10 300 python bench.py --img 1024 --batch 4 --cpu-baseline off > $O/bench_1024_bf16.json 2> $O/bench_1024_bf16.err || { echo B_FAIL; tail -20 $O/bench_1024_bf16.err; exit 1; }
timeout -k 10 300 python bench.py --img 1024 --batch 4 --dtype fp8 --cpu-baseline off > $O/bench_1024_fp8.json 2> $O/bench_1024_fp8.err || { echo B_FAIL; tail -20 $O/bench_1024_fp8.err; exit 1; }
CSU_LEDGER_DUMP=$O/launches_512.json timeout -k 10 300 python bench.py --cpu-baseline off > $O/b512.json 2> $O/b512.err || { echo B512_FAIL; tail -20 $O/b512.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o p -- \
  python3 $R/bench.py --img 1024 --batch 4 --dtype fp8 --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo PROF_FAIL; tail -30 $R/$O/prof.err; exit 1; }
cd $R
KT=$(find $O/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 4 60 > $O/step_breakdown_1024_fp8.txt
rm -rf $O/prof
echo ALL_OK
