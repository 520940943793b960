# round-4 A/B: gemm4 auto pick 128x64 (shipped) vs the 8-wave 256x128 tile for the wide-output forwards (N >= 2K, K >= 128)
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
AB=$(pwd)/tools/ab_lib/libcsu_hip_g4wide.so
CSU_LIB_PATH=$AB timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "linear or gemm" > $O/tests_wide.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests_wide.log; exit 1; }
tail -1 $O/tests_wide.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --cpu-baseline off --no-roofline > $O/a512_$i.json 2>/dev/null || { echo A_FAIL; exit 1; }
  CSU_LIB_PATH=$AB timeout -k 10 200 python bench.py --cpu-baseline off --no-roofline > $O/b512_$i.json 2>/dev/null || { echo B_FAIL; exit 1; }
  echo "512 pair $i: $(python -c "import json;print(json.load(open('$O/a512_$i.json'))['value'])") vs $(python -c "import json;print(json.load(open('$O/b512_$i.json'))['value'])")"
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --img 1024 --batch 4 --cpu-baseline off --no-roofline > $O/a1024_$i.json 2>/dev/null || { echo A_FAIL; exit 1; }
  CSU_LIB_PATH=$AB timeout -k 10 200 python bench.py --img 1024 --batch 4 --cpu-baseline off --no-roofline > $O/b1024_$i.json 2>/dev/null || { echo B_FAIL; exit 1; }
  echo "1024 pair $i: $(python -c "import json;print(json.load(open('$O/a1024_$i.json'))['value'])") vs $(python -c "import json;print(json.load(open('$O/b1024_$i.json'))['value'])")"
done
echo ALL_OK
