# HBM traffic of the bench's roofline kernel (stripe_fwd_w): two rocprofv3 PMC passes over a short
# eager bench run, then tools/pmc_traffic.py -> profiles/pmc_stripe_fwd.json (read by bench.py).
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcroof; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex stripe_fwd_w --output-format csv -d $O/$C -o $C -- \
    python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline off --graph off --no-roofline > $O/$C.log 2>&1
done
cd $R
python3 tools/pmc_traffic.py $(find $O/FETCH_SIZE -name '*counter_collection.csv') $(find $O/WRITE_SIZE -name '*counter_collection.csv') stripe_fwd_w $O/pmc_stripe_fwd.json
cat $O/pmc_stripe_fwd.json
