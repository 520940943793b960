B="python -u bench.py --steps 3 --warmup 2 --img 256 --batch 4 --no-roofline --cpu-baseline off"
run() { v=$(env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 timeout -k 10 120 $B 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['final_loss'])"); echo "$* -> $v"; }
run X=1; run X=2
run X=3 --dp-force 2>/dev/null || true
run CSU_CONV_WGRAD_V1=1 X=1; run CSU_CONV_WGRAD_V1=1 X=2
run CSU_CONV_PHASE_LAUNCHES=1 X=1
run CSU_PAD_CHANNELS=0 X=1
run CSU_SIDE_CONV=0 X=1; run CSU_SIDE_CONV=0 X=2
