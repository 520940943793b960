# closing HEAD (after the fp32 weight-gradient split depth): GPU suite + smoke + bench + rocprof groups,
# and the fp32 config line
bash tools/gpu_check.sh r0zj tests || exit 1
mkdir -p gpurun_out/r0zj_cfg
timeout -k 10 420 python -u bench.py --img 256 --batch 8 --dtype fp32 --no-ref-arch > gpurun_out/r0zj_cfg/cfg1_256_fp32.json 2> gpurun_out/r0zj_cfg/cfg1.err || exit 1
python tools/bench_summary.py gpurun_out/r0zj_cfg/cfg1_256_fp32.json | grep images
