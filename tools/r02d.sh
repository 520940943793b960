set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 bash tools/pmc_any.sh wg1 wgrad_tile $R/tools/wgrad_one.py 16384 1024 256 0 0 16
for i in 1 2 3 4; do python3 tools/pmc_sum.py gpurun_out/pmc_wg1/p$i wgrad_tile; done
cd /tmp && timeout -k 10 100 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r02d -o kt -- python3 $R/tools/wgrad_one.py 16384 1024 256 0 0 16 > /dev/null 2>&1
cat $R/gpurun_out/r02d/kt_kernel_stats.csv | cut -c1-200
