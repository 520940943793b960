set -e
bash tools/pmc_any.sh mlp mlp_ $GRAFT_REPO_ROOT/tools/mlp_one.py
for k in "mlp_fwd_kernel<64>" "mlp_fwd_kernel<128>" "mlp_fwd_kernel<256>" "mlp_bwd_kernel<64>" "mlp_bwd_kernel<128>" "mlp_bwd_kernel<256>"; do
  echo "== $k"; python3 tools/pmc_sum.py gpurun_out/pmc_mlp "$k" 1
done
