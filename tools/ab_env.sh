# A/B of an environment setting on the default bench: bash tools/ab_env.sh "VAR=a" "VAR=b" ...  (each twice, interleaved)
set -e
for rep in 1 2; do
  for e in "$@"; do
    v=$(env $e timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$e -> $v img/s"
  done
done
