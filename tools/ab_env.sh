# A/B of an environment setting on the default bench: bash tools/ab_env.sh "VAR=a" "VAR=b" ...  (each AB_REPS
# times, default 2, interleaved; AB_ARGS: extra bench.py arguments, e.g. "--steps 60")
set -e
for rep in $(seq ${AB_REPS:-2}); do
  for e in "$@"; do
    v=$(env $e timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline ${AB_ARGS:-} 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$e -> $v img/s"
  done
done
