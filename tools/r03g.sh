# attention backward: per-stage times (regular build) and per-workgroup phases (WG_TIMING build)
set -e
timeout -k 10 120 python tools/attn_time.py
for st in 1 2 3 4; do CSU_LIB_PATH=cswin-simam-unet_amd/csu/_lib/libcsu_hip_dbg.so timeout -k 10 60 python tools/attn_wg_timeline.py $st | head -2; done
