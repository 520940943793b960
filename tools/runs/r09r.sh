# final HEAD (after the branch-free dQ loop and the 128x128 wgrad barrier): GPU suite + smoke + bench + rocprof groups
bash tools/gpu_check.sh r09r tests
