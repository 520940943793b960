#!/bin/bash
set -e
O=gpurun_out/r02ac; mkdir -p $O
CFGS=0,1,2,3 timeout -k 10 200 python -u tools/gemm_cfgs.py > $O/gemm_cfgs.txt 2>&1 || { tail -20 $O/gemm_cfgs.txt; exit 1; }
grep -v amdgpu $O/gemm_cfgs.txt
