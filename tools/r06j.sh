# round-4: conv weight-gradient configurations on the CSWin merge / CARAFE / patch-embed shapes
set -o pipefail
R=$(pwd); O=gpurun_out/r06j; mkdir -p $O; export TMPDIR=/tmp
ONLY=merge,carafe,embed CFGS=-1,0,1,2,3,4,5 timeout -k 10 400 python -u tools/conv_wgrad_probe.py > $O/wgrad_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wgrad_probe.txt; exit 1; }
echo ALL_OK
