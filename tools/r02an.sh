#!/bin/bash
# two ranks on cuda:0 over gloo with the real csu model + GradAllReduce vs the single-process batch
set -e
O=gpurun_out/r02an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -4 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
