#!/bin/bash
# step glue on csu kernels (head folding, shared casts, LN-bwd bf16 copies, conv dW in OIHW): full GPU
# suite, torch-op census of an eager step, 512 bench
set -e
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TREE=1 timeout -k 10 200 python -u tools/torch_ops_profile.py > $O/torch_ops_tree.txt 2>&1 || { tail -20 $O/torch_ops_tree.txt; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-baseline off > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
