# which side-stream call site makes the graphed step non-reproducible (tools/det_graph.py)
for s in lin res mlp1 mlp2 cat conv; do
  echo "== $s: $(CSU_SIDE_SITES=$s REPS=3 timeout -k 10 200 python -u tools/det_graph.py 2>&1 | grep rep | tr '\n' ' ')"
done
