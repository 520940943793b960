# final HEAD (after the attention-prologue change): GPU suite + smoke + bench + rocprof groups
bash tools/gpu_check.sh r09l tests
