#!/bin/bash
# side-stream weight gradients inside the HIP graph: reproducible? (a) side in graph, (b) side in
# graph joined right after each launch, (c) default (no side in graph)
set -e
O=gpurun_out/r02z; mkdir -p $O
export IMG=512 K=6 REPS=3 GRADS=1
CSU_SIDE_IN_GRAPH=1 timeout -k 10 300 python -u tools/det_graph.py > $O/side_graph.txt 2>&1 || { tail -20 $O/side_graph.txt; exit 1; }
cat $O/side_graph.txt | grep -v amdgpu.ids | cut -c1-300
CSU_SIDE_IN_GRAPH=1 CSU_SIDE_JOIN_NOW=1 timeout -k 10 300 python -u tools/det_graph.py > $O/side_graph_joinnow.txt 2>&1 || { tail -20 $O/side_graph_joinnow.txt; exit 1; }
cat $O/side_graph_joinnow.txt | grep -v amdgpu.ids | cut -c1-300
timeout -k 10 300 python -u tools/det_graph.py > $O/default.txt 2>&1 || { tail -20 $O/default.txt; exit 1; }
cat $O/default.txt | grep -v amdgpu.ids | cut -c1-300
timeout -k 10 400 bash tools/pm_attn.sh > $O/pm_attn.txt 2>&1 || { tail -20 $O/pm_attn.txt; exit 1; }
cat $O/pm_attn.txt
