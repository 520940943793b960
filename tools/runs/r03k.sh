# PMC table at HEAD (MFMA busy, FETCH/WRITE vs algorithmic bytes) for 512 B16, 1024 B4 and the plain UNet
set -e
R=$(pwd); O=$R/gpurun_out/r03k; mkdir -p $O; export TMPDIR=/tmp
for cfg in "c512:--img 512 --batch 16" "c1024:--img 1024 --batch 4" "unet:--model unet"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python -u bench.py $args --steps 6 --warmup 2 --cpu-baseline off > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  i=0
  for C in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    cd /tmp
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/$tag/p$i -o p$i -- python3 $R/bench.py $args --steps 2 --warmup 1 --cpu-baseline off --graph off --no-roofline > $O/$tag.p$i.log 2>&1 || { tail -20 $O/$tag.p$i.log; exit 1; }
    cd $R
    echo "$tag pass $i done"
  done
  python tools/pmc_groups.py $O/$tag $O/bench_$tag.json 12 > $O/pmc_$tag.md
  head -30 $O/pmc_$tag.md
done
