set -e
bash tools/pmc_any.sh attn4 stripe $GRAFT_REPO_ROOT/tools/attn_one.py
for k in stripe_fwd_w stripe_bwd_dq_w stripe_bwd_dkdv_w; do echo "== $k"; python3 tools/pmc_sum.py gpurun_out/pmc_attn4 $k 5 | tr '\n' ';' | sed 's/  */ /g'; echo; done
