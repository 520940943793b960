# round 6 closing HEAD, part 1: the whole GPU suite + smoke + bench + rocprof kernel trace of the timed replays
bash tools/gpu_check.sh r08x tests
