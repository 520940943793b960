set -e
mkdir -p gpurun_out/r02h
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or linear" > gpurun_out/r02h/pytest.log 2>&1 || { tail -40 gpurun_out/r02h/pytest.log; exit 1; }
tail -2 gpurun_out/r02h/pytest.log
for D in 2 3 4; do
CSU_WGRAD_DEPTH=$D timeout -k 10 400 python -u tools/wgrad_bench.py --plans c0.5,c1,c2,t64x64:c1,t64x64:c2 > gpurun_out/r02h/wgrad_bench_$D.txt 2>&1 || { tail -30 gpurun_out/r02h/wgrad_bench_$D.txt; exit 1; }
echo "== depth $D"; cat gpurun_out/r02h/wgrad_bench_$D.txt
done
