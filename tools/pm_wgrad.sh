set -e
bash tools/pmc_any.sh wg3 wgrad_bf16 $GRAFT_REPO_ROOT/tools/wgrad_one.py 16384 768 256
bash tools/pmc_any.sh wg1 wgrad_bf16 $GRAFT_REPO_ROOT/tools/wgrad_one.py 262144 256 64
for t in wg3 wg1; do echo "== $t"; python3 tools/pmc_sum.py gpurun_out/pmc_$t wgrad 5; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/wgt -o wgt -- python3 $GRAFT_REPO_ROOT/tools/wgrad_one.py 16384 768 256 > /dev/null 2>&1
cat $(find $GRAFT_REPO_ROOT/gpurun_out/wgt -name '*kernel_stats.csv') | cut -d, -f1-8 | head -5
