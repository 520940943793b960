set -e
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_lin -o kt -- python3 $R/tools/linear_probe.py > $R/gpurun_out/kt_lin.log 2>&1
