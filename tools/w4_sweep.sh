set -e
for c in 0 1 2; do echo "== CSU_W4CFG=$c"; CSU_W4CFG=$c timeout -k 10 200 python -u tools/linear_probe.py 2>&1 | grep wgrad; done
echo "== old kernel"; CSU_WGRAD4=0 timeout -k 10 200 python -u tools/linear_probe.py 2>&1 | grep wgrad
