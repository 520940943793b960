# round-4 closing evidence at HEAD: GPU suite + smoke, 512 B16 bench + rocprofv3 trace, PMC passes (512 B16, 1024 B4 bf16 / fp8)
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo SUITE_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
T=r06y timeout -k 10 600 bash tools/quick_cswin.sh > $O/quick.log 2>&1 || { echo QUICK_FAIL; tail -20 $O/quick.log; exit 1; }
cat $O/quick.log
T=r06y CFGS="c512:--img 512 --batch 16|c1024:--img 1024 --batch 4|c1024fp8:--img 1024 --batch 4 --dtype fp8" timeout -k 10 900 bash tools/pmc_head.sh > $O/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $O/pmc.log; exit 1; }
grep -E "pass 3 done" $O/pmc.log
echo ALL_OK
