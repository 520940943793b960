#!/bin/bash
set -e
O=gpurun_out/r02ad; mkdir -p $O
CSU_LIB_PATH=$GRAFT_REPO_ROOT/cswin-simam-unet_amd/csu/_lib/libcsu_hip_dbg.so timeout -k 10 200 python -u tools/g4_timing.py > $O/g4.txt 2>&1 || { tail -20 $O/g4.txt; exit 1; }
grep -v amdgpu $O/g4.txt
