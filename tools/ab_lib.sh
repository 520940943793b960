# A/B of library builds: bash tools/ab_lib.sh ab/a.so ab/b.so ...  (wgrad probe once each, bench twice each, interleaved)
set -e
for lib in "$@"; do
  echo "== $lib"; CSU_LIB_PATH=$lib timeout -k 10 200 python -u tools/linear_probe.py 2>&1 | grep -E "^wgrad|totals"
done
for rep in 1 2; do
  for lib in "$@"; do
    v=$(CSU_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "$lib -> $v img/s"
  done
done
