for v in default noflag; do
  if [ $v = default ]; then unset CSU_LIB_PATH; else export CSU_LIB_PATH=$PWD/cswin-simam-unet_amd/csu/_lib/exp/lib_$v.so; fi
  echo "== $v"; timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 120 --timeout-method thread -k "stripe" 2>&1 | tail -3
done
