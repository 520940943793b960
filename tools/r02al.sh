#!/bin/bash
# 8-wave gemm4 workgroups (cfgs 16-19): tile-config parity tests, graph-timed probe on the 512 step's
# token-GEMM shapes, then the every-config HEAD bench sweep (tools/r02ak_configs.sh)
set -e
O=gpurun_out/r02al; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "tile_configs or gemm" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
CFGS=11,16,17,18,19 timeout -k 10 300 python -u tools/gemm_graph_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
bash tools/r02ak_configs.sh
