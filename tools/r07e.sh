# headline bench with the per-launch ledger dump (shape tags) -> gpurun_out/r07e/
O=gpurun_out/r07e; mkdir -p $O
CSU_LEDGER_DUMP=$O/launches.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $O/bench.json
