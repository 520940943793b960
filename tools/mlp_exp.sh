# fused-Mlp timing under experiment builds of the library (csu/_lib/exp/lib_<V>.so)
set -e
for v in base NOGELU NODMA NOBAR; do
  if [ $v = base ]; then unset CSU_LIB_PATH; else export CSU_LIB_PATH=$PWD/cswin-simam-unet_amd/csu/_lib/exp/lib_$v.so; fi
  echo "== $v"; timeout -k 10 120 python -u tools/mlp_probe.py 2>&1 | grep "C="
done
