# A/B: early side-stream flush of the deferred weight gradients (CSU_WGRAD_EARLY_GFLOP), 512 B16
mkdir -p gpurun_out/r03n
for rep in 1 2; do
for g in 0 m16384 m65536; do
  CSU_WGRAD_EARLY_M=${g#m} timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off --no-roofline > gpurun_out/r03n/b_${g}_$rep.json 2> gpurun_out/r03n/b_${g}_$rep.err || { tail -20 gpurun_out/r03n/b_${g}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r03n/b_${g}_$rep.json'));print('gflop=$g rep=$rep', d['value'], d['ms_per_step'])"
done
done
