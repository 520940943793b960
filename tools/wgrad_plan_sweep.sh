# bench img/s under split-K plans of the weight-gradient GEMM: CSU_WGRAD_WGS (target workgroups) x
# CSU_WGRAD_MINTOK (minimum tokens per chunk)
set -e
for cfg in "1024 512" "1024 1024" "1024 2048" "512 1024" "2048 1024" "1024 4096"; do
  set -- $cfg
  v=$(CSU_WGRAD_WGS=$1 CSU_WGRAD_MINTOK=$2 timeout -k 10 200 python -u bench.py --cpu-baseline off --no-roofline 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "WGS=$1 MINTOK=$2 -> $v img/s"
done
