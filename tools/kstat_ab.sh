#!/bin/bash
# Per-kernel totals of the default bench under two env settings: bash tools/kstat_ab.sh <regex> "A=1" "A=0"
set -e
R=$GRAFT_REPO_ROOT; RX=$1; shift
cd /tmp; export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kab$i -o k -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-baseline off --no-roofline > /dev/null 2>&1
  echo "== $e"
  f=$(find $R/gpurun_out/kab$i -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,re,sys
for r in csv.DictReader(open('$f')):
    if re.search('$RX', r['Name']): print('%8.1f us avg %6s calls  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))"
done
