cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1 || true
