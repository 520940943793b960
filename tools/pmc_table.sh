#!/bin/bash
# Per-kernel MFMA utilisation + HBM traffic of the default bench workload (SURVEY §8d "MFMA
# utilisation from rocprofv3 counters per kernel, with HBM GB/s from the same run").
#   gpurun -- bash tools/pmc_table.sh <tag>      -> gpurun_out/pmct_<tag>/{p1,p2,p3}, table.md
# Three counter passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), each its own run with
# --kernel-trace only, over eager steps (--graph off: per-dispatch counters).
set -e
R=$GRAFT_REPO_ROOT; T=${1:-run}
O=$R/gpurun_out/pmct_$T; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline off --graph off --no-roofline"
i=0
for C in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/p$i -o p$i -- $CMD > $O/p$i.log 2>&1
  echo "pass $i ($C) done"
done
cd $R
python3 tools/pmc_table.py $O > $O/table.md
cat $O/table.md
