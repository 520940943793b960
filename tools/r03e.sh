# round 3: parity (fused attention backward + norm2-in-Mlp) then the HEAD profile
mkdir -p gpurun_out
run() {  # name, timeout, pytest args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -u -m pytest -v --timeout 400 --timeout-method thread "$@" > gpurun_out/r03e_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 gpurun_out/r03e_$name.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run kern 400 tests/test_gpu_kernels.py -k "stripe or two_branch or bce or mlp"
run model 500 tests/test_gpu_dropout.py tests/test_gpu_model.py
run train 900 tests/test_gpu_train.py tests/test_gpu_dist.py
T=r03e bash tools/r03prof.sh
