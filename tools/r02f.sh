set -e
timeout -k 10 200 python -u tools/wgrad_timing.py
