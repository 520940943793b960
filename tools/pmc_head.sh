# PMC table at HEAD (MFMA busy, FETCH/WRITE vs algorithmic bytes): T=<tag>; CFGS = "tag:bench args|tag:bench args" (default the plain UNet and 512 B16)
# Per workload: the bench line (its graph ledger = the algorithmic bytes), a kernel trace of the timed
# graph replays (p0), three counter passes over eager steps (p1-p3: `--graph off`, which launch the
# captured step's kernels -- no side stream), and tools/kernel_match.py checking that the eager passes
# ran exactly the kernels the graph replays.
set -e
R=$(pwd); O=$R/gpurun_out/${T:-r04d}; mkdir -p $O; export TMPDIR=/tmp
IFS='|' read -ra LIST <<< "${CFGS:-unet:--model unet|c512:--img 512 --batch 16}"
for cfg in "${LIST[@]}"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python -u bench.py $args --steps 6 --warmup 2 --cpu-baseline off > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag/p0 -o p0 -- python3 $R/bench.py $args --steps 5 --warmup 2 --cpu-baseline off --no-roofline > $O/$tag.p0.log 2>&1 || { tail -20 $O/$tag.p0.log; exit 1; }
  cd $R
  i=0
  for C in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    cd /tmp
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/$tag/p$i -o p$i -- python3 $R/bench.py $args --steps 2 --warmup 1 --cpu-baseline off --graph off --no-roofline > $O/$tag.p$i.log 2>&1 || { tail -20 $O/$tag.p$i.log; exit 1; }
    cd $R
    echo "$tag pass $i done"
  done
  KT=$(find $O/$tag/p0 -name '*kernel_trace.csv' -print -quit)
  python tools/kernel_match.py "$KT" 5 $O/$tag/p1 > $O/match_$tag.txt || true
  cat $O/match_$tag.txt
  python tools/prof_groups.py "$KT" 5 $O/bench_$tag.json > $O/groups_$tag.md
  [ -f $O/pmc_traffic.json ] || cp profiles/pmc_traffic.json $O/pmc_traffic.json
  python tools/pmc_groups.py $O/$tag $O/bench_$tag.json 12 --traffic $O/pmc_traffic.json > $O/pmc_$tag.md
  head -30 $O/pmc_$tag.md
done
