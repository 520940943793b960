# round-4: v2 conv weight gradient for N % 8 == 4 (CARAFE encoders) -- conv tests, the probe on those shapes, the 512 trace
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or carafe or bce" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ONLY=carafe CFGS=-1,0 timeout -k 10 300 python -u tools/conv_wgrad_probe.py > $O/wgrad_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wgrad_probe.txt; exit 1; }
cat $O/wgrad_probe.txt
T=r06n timeout -k 10 600 bash tools/quick_cswin.sh > $O/quick.log 2>&1 || { echo QUICK_FAIL; tail -20 $O/quick.log; exit 1; }
cat $O/quick.log
grep -E "carafe_bwd_enc|bce_partial|conv_wgrad|colsum" $O/step_breakdown_cswin.txt
echo ALL_OK
