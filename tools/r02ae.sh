#!/bin/bash
set -e
O=gpurun_out/r02ae; mkdir -p $O
CFGS=11,16,17,13 timeout -k 10 200 python -u tools/gemm_graph_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu $O/probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
