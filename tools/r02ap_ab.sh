#!/bin/bash
# LayerNorm forward row groups per wave: ab/a.so vs ab/b.so (r02ap: 4 vs 1; r02aq: 4 vs 8): LN / model GPU
# tests on b, then 3 interleaved 512 B16 bench pairs
set -e
O=gpurun_out/${T:-r02ap}; mkdir -p $O
CSU_LIB_PATH=ab/b.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -k "layernorm or block or whole_model or graph" -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for lib in a b; do
    CSU_LIB_PATH=ab/$lib.so timeout -k 10 200 python -u bench.py --cpu-baseline off > $O/$lib$rep.json 2> $O/$lib$rep.err || { tail -20 $O/$lib$rep.err; exit 1; }
    python -c "
import json; r = json.loads(open('$O/$lib$rep.json').read().strip().splitlines()[-1])
k = {x['kernel']: x for x in r['roofline']['kernels']}
print('$lib rep$rep', r['value'], 'ln_fwd', k['layernorm_fwd']['us_per_step'], 'us/step frac', k['layernorm_fwd']['frac'])"
  done
done
