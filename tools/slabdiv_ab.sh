#!/bin/bash
# Interleaved 512 B16 benches over CSU_WGRAD_SLAB_DIV (grouped weight-gradient token chunks: slab bytes
# <= operand bytes * 2 / div).  DIVS="32 16 ...", T=<tag>.
set -e
T=${T:-slabdiv}; O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  for d in ${DIVS:-32 16}; do
    CSU_WGRAD_SLAB_DIV=$d timeout -k 10 300 python -u bench.py --cpu-baseline off --no-roofline > $O/b_${d}_$rep.json 2> $O/b_${d}_$rep.err || { tail -20 $O/b_${d}_$rep.err; exit 1; }
    echo "div $d rep $rep: $(python -c "import json,sys; d=json.loads([l for l in open('$O/b_${d}_$rep.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
  done
done
