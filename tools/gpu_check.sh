#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# The rocprof run skips the roofline leg (--no-roofline): its last 5 AdamW-delimited steps are then the
# 5 timed graph replays themselves (with the leg, the ledger captures' eager warm-up steps -- side-stream
# wgrad_tile kernels -- fell inside the window and skewed the groups table).
#   gpurun --timeout 1100 -- bash tools/gpu_check.sh <tag> [tests|notests]
# Every GPU step has its own time limit; the first failure ends the script.
set -e
TAG=${1:-run}
MODE=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
    || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o $TAG -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-ref-arch --no-roofline ${BENCH_ARGS:-} > $R/$OUT/prof_bench.json 2> $R/$OUT/prof.err \
  || { tail -30 $R/$OUT/prof.err; exit 1; }
cd $R
KT=$(find $OUT/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_summary.py "$KT" 2 60 > $OUT/step_breakdown.txt && head -40 $OUT/step_breakdown.txt
python tools/prof_groups.py "$KT" 5 $OUT/bench.json > $OUT/groups.md && head -30 $OUT/groups.md
