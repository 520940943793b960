# closing HEAD (after the fp32 GEMM tiles): GPU suite +
# smoke + bench + rocprof groups, then every other BASELINE config line
bash tools/gpu_check.sh r0ze tests || exit 1
bash tools/configs_bench.sh r0ze_cfg
