# PMC passes over one GEMM shape: bash tools/pmc_gemm.sh M K N cfg tag
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_$5; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE TA_BUSY_avr TA_ADDR_STALL_CYCLES_sum" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --kernel-include-regex gemm --output-format csv -d $O/p$i -o p$i -- python3 $R/tools/gemm_one.py $1 $2 $3 $4 > $O/p$i.log 2>&1
done
