# grouped 128 x 128 weight gradients: a scheduling barrier per k-step (WG_SB128 1: 240 VGPRs, no spill)
# vs every k-step's fragments hoisted (256 VGPRs + 4 spilled; the reload waits vmcnt(0); libcsu_hip_ab.so)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wgrad or linear or model" > gpurun_out/r09q_tests.log 2>&1 || { tail -30 gpurun_out/r09q_tests.log; exit 1; }
tail -2 gpurun_out/r09q_tests.log
bash tools/ab_lib.sh r09q linear_wgrad || exit 1
bash tools/ab_1024.sh r09q linear_wgrad
