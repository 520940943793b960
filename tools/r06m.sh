# round-4: CARAFE encoder-gradient reduce-scatter + batched BCE partial loads -- their tests, then the 512 trace
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "carafe or bce" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
T=r06m timeout -k 10 600 bash tools/quick_cswin.sh > $O/quick.log 2>&1 || { echo QUICK_FAIL; tail -20 $O/quick.log; exit 1; }
cat $O/quick.log
grep -E "carafe_bwd_enc|bce_partial" $O/step_breakdown_cswin.txt
echo ALL_OK
