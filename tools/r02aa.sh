#!/bin/bash
set -e
O=gpurun_out/r02aa; mkdir -p $O
for w in 1024 512 256 2048; do echo "WGS $w"; CSU_ATTN_WGS=$w timeout -k 10 120 python -u tools/attn_time.py 2>&1 | grep reso; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -k "bitwise" tests/test_gpu_kernels.py -k "simam or bitwise" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/bench_a.json 2> $O/bench_a.err || { tail -30 $O/bench_a.err; exit 1; }
CSU_SIDE_IN_GRAPH=1 timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/bench_side.json 2> $O/bench_side.err || { tail -30 $O/bench_side.err; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/bench_b.json 2> $O/bench_b.err || { tail -30 $O/bench_b.err; exit 1; }
CSU_SIDE_IN_GRAPH=1 timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/bench_side2.json 2> $O/bench_side2.err || { tail -30 $O/bench_side2.err; exit 1; }
for f in bench_a bench_side bench_b bench_side2; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
timeout -k 10 300 python -u bench.py --simam --cpu-baseline off > $O/bench_simam.json 2> $O/bench_simam.err || { tail -30 $O/bench_simam.err; exit 1; }
python tools/bench_summary.py $O/bench_simam.json | head -3
