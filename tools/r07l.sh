# fused norm1 backward in the qkv dgrad: kernel tests, model / train / dropout parity, bench
O=gpurun_out/r07l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -k "ln_linear_ws or gemm_ws or layernorm" > $O/t1.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py tests/test_gpu_dropout.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/t2.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -3 $O/t2.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline off > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; python -c "
import json;r=json.loads(open('$O/bench.json').read().splitlines()[-1]);print(r['value'],r['ms_per_step'],r['roofline']['step_frac'])
ks=r['roofline']['kernels']
for k in ks[:10]: print(k['kernel'],k['us_per_step'],k['launches_per_step'])"
