# round-4 final validation: the whole GPU suite + smoke, then the 512 headline bench with its rocprofv3 trace
set -o pipefail
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo SUITE_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
T=r06z timeout -k 10 600 bash tools/quick_cswin.sh > $O/quick.log 2>&1 || { echo QUICK_FAIL; tail -20 $O/quick.log; exit 1; }
echo ALL_OK
