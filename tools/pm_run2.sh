set -e
bash tools/pmc_any.sh w4_qkv256 wgrad4 $GRAFT_REPO_ROOT/tools/wgrad_one.py 16384 768 256
CSU_WGRAD4=0 bash tools/pmc_any.sh wold_qkv256 wgrad_bf16 $GRAFT_REPO_ROOT/tools/wgrad_one.py 16384 768 256
