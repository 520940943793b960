set -e
O=gpurun_out/r05f; mkdir -p $O; R=$(pwd); export TMPDIR=/tmp
for nl in 0 1; do
  cd /tmp
  NOLEPE=$nl ONLY=0,1,2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p$nl -o p -- python3 $R/tools/attn_time.py > $R/$O/attn_$nl.txt 2>&1
  cd $R
  ST=$(find $O/p$nl -name '*kernel_stats.csv' -print -quit); cp $ST $O/stats_$nl.csv
done
