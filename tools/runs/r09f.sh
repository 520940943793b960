# closing HEAD after the LayerNorm change: GPU suite + smoke + bench + rocprof groups of the timed replays
bash tools/gpu_check.sh r09f tests
