# closing HEAD (after the conv weight-gradient XCD order and the 4096-token GEMM tiles): GPU suite +
# smoke + bench + rocprof groups, then every other BASELINE config line
bash tools/gpu_check.sh r09z tests || exit 1
bash tools/configs_bench.sh r09z_cfg
