# round 3 checkpoint: the whole GPU suite, then the HEAD profile (T=r03i)
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/r03i_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03i_gpu_tests.log; echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
T=r03i bash tools/r03prof.sh
