# attention backward: reduce-scatter of the LePE weight-gradient partials -- attention tests, timeline
# (debug build), then the DP-path check (tools/dp_check.sh)
O=gpurun_out/r07zj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "stripe or attention or lepe or Stripe or reproducible" > $O/t1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
for s in 3 1; do timeout -k 10 120 python -u tools/attn_wg_timeline.py $s 2>&1 | grep -v amdgpu.ids | grep -A1 "fused bwd" >> $O/timeline.txt || exit 1; done
cat $O/timeline.txt
bash tools/dp_check.sh r07zj_dp
