# HBM traffic per call of the bench's roofline kernel group: two rocprofv3 PMC passes (FETCH_SIZE,
# WRITE_SIZE, each its own run) over a short eager bench run, then tools/pmc_traffic.py ->
# profiles/pmc_traffic.json (read by bench.py).
#   bash tools/pmc_roofline.sh <kernel> <marker> <kernel-regex> <comma fragments> [bench args...]
set -e
R=$GRAFT_REPO_ROOT; KERN=$1; MARK=$2; RX=$3; FR=$4; shift 4
O=$R/gpurun_out/pmcroof; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d $O/$C -o $C -- \
    python3 $R/bench.py --steps 2 --warmup 1 --cpu-baseline off --graph off --no-roofline "$@" > $O/$C.log 2>&1
done
cd $R
KEY="$KERN|$(python3 bench.py --traffic-key "$@")"
python3 tools/pmc_traffic.py $(find $O/FETCH_SIZE -name '*counter_collection.csv') $(find $O/WRITE_SIZE -name '*counter_collection.csv') \
  "$KEY" "$MARK" "$FR" profiles/pmc_traffic.json $BENCH_JSON
cp profiles/pmc_traffic.json gpurun_out/pmcroof/
