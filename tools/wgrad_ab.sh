set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "wgrad or linear or fused_mlp" > gpurun_out/tw.log 2>&1 || { tail -30 gpurun_out/tw.log; exit 1; }
tail -1 gpurun_out/tw.log
echo "== T=128 default"; timeout -k 10 200 python -u tools/linear_probe.py 2>&1 | grep wgrad
echo "== T=64"; CSU_WGRAD_T=64 timeout -k 10 200 python -u tools/linear_probe.py 2>&1 | grep wgrad
