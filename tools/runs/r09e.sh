# HIP runtime settings for the replayed step graph: kernel arguments in device memory, AQL packet capture
O=gpurun_out/r09e; mkdir -p $O
run() { local n=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch --no-roofline > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }; python tools/bench_summary.py $O/$n.json | grep images; }
for i in 1 2; do
  run base_$i X=1 || exit 1
  run kernarg_$i HIP_FORCE_DEV_KERNARG=1 || exit 1
  run pkt1_$i DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
  run pkt0_$i DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
done
