set -e
bash tools/pmc_gemm.sh 16384 256 768 12 qkv256_c12
bash tools/pmc_gemm.sh 16384 256 768 2 qkv256_c2
ls -R gpurun_out/pmc_qkv256_c12 | head -30
