#!/bin/bash
# gpurun, re-submitted only while the pool has no box free (exit code 3: nothing ran, nothing charged).
# Any other outcome -- success, a failure of the command, a refusal -- is returned as is.
# usage: tools/gpuwait.sh <timeout-seconds> <command string>
T=$1; shift
for i in $(seq 1 40); do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
    rc=$?
    [ $rc -ne 3 ] && exit $rc
    echo "[gpuwait] no box (attempt $i), waiting 120 s"
    sleep 120
done
exit 3
