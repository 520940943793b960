#!/bin/bash
# A/B of the gemm4 tile pick (ab/a.so = 128x64 everywhere, ab/b.so = 8-wave 256x128 for wide outputs):
# GEMM parity tests on b, then 3 interleaved 512 B16 bench pairs and one 1024 B4 pair
set -e
O=gpurun_out/r02am; mkdir -p $O
CSU_LIB_PATH=ab/b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for lib in a b; do
    CSU_LIB_PATH=ab/$lib.so timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline > $O/$lib$rep.json 2> $O/$lib$rep.err || { tail -20 $O/$lib$rep.err; exit 1; }
    echo "$lib rep$rep $(python -c "import json; print(json.loads(open('$O/$lib$rep.json').read().strip().splitlines()[-1])['value'])")"
  done
done
for lib in a b; do
  CSU_LIB_PATH=ab/$lib.so timeout -k 10 200 python -u bench.py --img 1024 --batch 4 --cpu-baseline off --no-roofline > $O/${lib}_1024.json 2> $O/${lib}_1024.err || { tail -20 $O/${lib}_1024.err; exit 1; }
  echo "$lib 1024 $(python -c "import json; print(json.loads(open('$O/${lib}_1024.json').read().strip().splitlines()[-1])['value'])")"
done
