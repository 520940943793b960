set -e
mkdir -p gpurun_out/r02c
timeout -k 10 400 python -u tools/wgrad_bench.py --plans torch,auto,c1,t64x64:c1,t64x64:c2 > gpurun_out/r02c/wgrad_bench.txt 2>&1 || { tail -30 gpurun_out/r02c/wgrad_bench.txt; exit 1; }
cat gpurun_out/r02c/wgrad_bench.txt
