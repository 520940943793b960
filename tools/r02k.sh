set -e
T=r02k; O=gpurun_out/$T; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 400 bash tools/pmc_roofline.sh "linear_wgrad|512|16|bf16" wgrad_tile "wgrad_tile|wslab_reduce" wgrad_tile,wslab_reduce
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o $T -- \
  python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { tail -30 $R/$O/prof.err; exit 1; }
cd $R
KT=$(find $O/prof -name '*kernel_trace.csv' -print -quit)
python tools/prof_groups.py "$KT" 4 $O/bench.json > $O/groups.md
python tools/prof_summary.py "$KT" 4 60 > $O/step_breakdown.txt
cat $O/groups.md; head -5 $O/step_breakdown.txt
python -c "import json; d=json.loads(open('$O/bench.json').read()); r=d['roofline']; r.pop('kernels'); print(d['value'], json.dumps(r))"
