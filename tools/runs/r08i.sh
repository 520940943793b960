# round 6 evidence at HEAD (8-wave C = 256 Mlp, e4m3 weight streaming in the fp8 format): GPU suite +
# smoke + bench + rocprof groups of the timed replays; PMC passes (graph-matched eager steps) of the SimAM
# headline, the reference architecture and 1024x1024 B4 (traffic keys); the other BASELINE configs
bash tools/gpu_check.sh r08i tests || exit 1
T=r08i_pmc CFGS="c512s:--img 512 --batch 16 --no-ref-arch|c512n:--img 512 --batch 16 --no-simam --no-ref-arch|c1024s:--img 1024 --batch 4 --no-ref-arch" bash tools/pmc_head.sh > gpurun_out/r08i_pmc.log 2>&1 || { tail -20 gpurun_out/r08i_pmc.log; exit 1; }
echo pmc done
bash tools/configs_bench.sh r08i_cfg
