set -e
for cfg in "128 1024" "64 1024" "64 512" "128 512" "64 256" "128 256"; do
  set -- $cfg
  v=$(CSU_WGRAD_T=$1 CSU_WGRAD_WGS=$2 timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "T=$1 WGS=$2 -> $v img/s"
done
