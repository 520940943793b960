# round-4: conv weight-gradient configurations on the CSWin merge / CARAFE / patch-embed shapes; 1024 B4 lines
set -o pipefail
R=$(pwd); O=gpurun_out/r06j; mkdir -p $O; export TMPDIR=/tmp
ONLY=merge,carafe,embed CFGS=-1,0,1,2,3,4,5 timeout -k 10 400 python -u tools/conv_wgrad_probe.py > $O/wgrad_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/wgrad_probe.txt; exit 1; }
timeout -k 10 400 python bench.py --img 1024 --batch 4 > $O/bench_c1024.json 2> $O/bench_c1024.err || { echo B_FAIL; tail -20 $O/bench_c1024.err; exit 1; }
timeout -k 10 400 python bench.py --img 1024 --batch 4 --dtype fp8 > $O/bench_c1024fp8.json 2> $O/bench_c1024fp8.err || { echo B_FAIL; tail -20 $O/bench_c1024fp8.err; exit 1; }
echo ALL_OK
