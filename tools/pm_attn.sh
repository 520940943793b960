set -e
bash tools/pmc_any.sh attn3 stripe $GRAFT_REPO_ROOT/tools/attn_one.py
