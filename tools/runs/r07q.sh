# gemm_ws stage-1 shapes: isolated probe (stage 1-3 shapes) + in-step per-launch ledger
O=gpurun_out/r07q; mkdir -p $O
SHAPES=s1 timeout -k 10 200 python tools/probes/gemm_ws_time.py > $O/ws_s1.txt 2>&1 || exit 1
timeout -k 10 200 python tools/probes/gemm_ws_time.py > $O/ws.txt 2>&1 || exit 1
cat $O/ws_s1.txt $O/ws.txt | grep -v amdgpu.ids
CSU_LEDGER_DUMP=$O/launches.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-ref-arch > $O/bench.json 2> $O/bench.err || exit 1
python tools/bench_summary.py $O/bench.json | grep images
