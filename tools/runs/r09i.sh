# final HEAD: GPU suite + smoke + bench + rocprof groups, then every other BASELINE config
bash tools/gpu_check.sh r09i tests || exit 1
bash tools/configs_bench.sh r09i_cfg
